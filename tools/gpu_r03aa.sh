# r03aa: RemotePod / tc segment writers in one 64-lane round when the wave's messages fit
# (10 KB image for k_remote_write): parity of the output stages + stage times
set -uo pipefail
O=gpurun_out/r03aa; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_multishard_gpu.py \
    -k "remote or tc or fanout or wire or reach" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python3 tools/stage_run.py --reps 5 --stages run,fanout,remote,tc > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
