# r03ad: ParseFloatPercentage fast path (one double division for <= 8 decimals, bytes from dword
# loads, loop bounded by the wave's longest string): parser parity + pdict times
set -uo pipefail
O=gpurun_out/r03ad; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    -k "not full_size" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python3 tools/stage_run.py --reps 10 --stages run > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
