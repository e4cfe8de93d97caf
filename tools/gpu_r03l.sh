# r03l: kdtn_vni_contested (order-dependent VxlanManager keys), 8-B string table again, fan-out
# prefetch: VXLAN / encoder / fan-out parity, then stage times
set -uo pipefail
O=gpurun_out/r03l; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_vni_state_gpu.py \
    tests/test_parity_gpu.py tests/test_multishard_gpu.py -k "vni or wire or remote or fanout or tc_argv or reach or shard" \
    > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
