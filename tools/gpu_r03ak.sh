# r03ak: repeated strings later than their inserter skip the first-occurrence read: ingest parity + stage times
set -uo pipefail
O=gpurun_out/r03ak; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_ingest_gpu.py tests/test_ingest_shard_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 500 python -u bench.py --no-wire --no-e2e --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg2.json')); i=d['ingest_stage']; print(i['gpu_ms'], i['roofline']['frac'], i['kernels_ms'])"
