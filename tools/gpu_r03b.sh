# r03b: encoder / fan-out / sharded VXLAN tests after the string-table and multisplit changes,
# then bench lines for configs 2 and 3 (wire + remote stages, resident chain)
set -uo pipefail
O=gpurun_out/r03b; mkdir -p $O
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
    tests/test_multishard_gpu.py tests/test_parity_gpu.py -k "wire or remote or fanout or tc_argv or reach or multishard or shard or vni" \
    > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; ok $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest > $O/bench_cfg2.json 2> $O/bench_cfg2.err; rc=$?
tail -c 300 $O/bench_cfg2.json; ok $rc
timeout -k 10 600 python -u bench.py --config 3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err; rc=$?
tail -c 1500 $O/bench_cfg3.json; exit $rc
