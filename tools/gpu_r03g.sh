# r03g: single-pass wire writer (look-back scan, two-pass fallback); RemotePod messages and the receiving daemon's tc argv in add-list order (sizes per add
# entry gathered into fan-out order; writer stores each message at its fan-out position)
set -uo pipefail
O=gpurun_out/r03g; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_multishard_gpu.py tests/test_configs_gpu.py -k "wire or remote or fanout or tc_argv or reach or config" \
    > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
