# r03f: encoder rewrite (dword-assembling writer, entry-parallel wire sizing, 16-B string loads)
# and the fan-out stamp fix: encoder/fan-out parity tests, then per-stage kernel times
set -uo pipefail
O=gpurun_out/r03f; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_multishard_gpu.py tests/test_configs_gpu.py -k "wire or remote or fanout or tc_argv or reach or config" \
    > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
