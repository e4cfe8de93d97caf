# r03u: A/B of the pod-table side stream (KDTN_SIDE 0-3) + the product default's parity subset
set -uo pipefail
O=gpurun_out/r03u; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/side_ab.py --reps 40 --cache /tmp/kdtn_cache > $O/side_ab.json 2> $O/side_ab.err || { tail -5 $O/side_ab.err; exit 1; }
cat $O/side_ab.json | head -12
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_multishard_gpu.py tests/test_state_gpu.py \
    tests/test_parity_gpu.py -k "not full_size" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
exit $rc
