# r03n: key-string predicates — ParseCIDR shortcut for '/'-less strings and register (SWAR)
# ParseMAC for the 17/23-byte colon / hyphen layouts: predicate fuzz + parity, then stage times
set -uo pipefail
O=gpurun_out/r03n; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_ingest_gpu.py -k "predicate or cidr or golden or random or synthetic or hub or ingest" > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 5 --stages run > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
