# r03j: 32-ary wave-cooperative entry -> topology search (reach, VXLAN ops, wire sizes, RemotePod):
# parity of every path that uses it, then stage times
set -uo pipefail
O=gpurun_out/r03j; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_multishard_gpu.py tests/test_configs_gpu.py tests/test_state_gpu.py tests/test_vni_state_gpu.py \
    -k "wire or remote or fanout or tc_argv or reach or config or state or vni or kubedtn" > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
