# r03a: the round's new GPU tests first, then the whole suite, then the default bench line.
# A test failure (pytest rc 1) does not stop the script; a timeout, abort or crash does.
set -uo pipefail
O=gpurun_out/r03a; mkdir -p $O
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
    tests/test_state_gpu.py tests/test_bench_gpu.py tests/test_vni_state_gpu.py tests/test_ingest_shard_gpu.py \
    "tests/test_parity_gpu.py::test_remote_pod_messages" "tests/test_configs_gpu.py::test_config2_sharded_8_full_size" \
    > $O/new_tests.log 2>&1; rc=$?
tail -5 $O/new_tests.log; ok $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; ok $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg2.json 2> $O/bench_cfg2.err; rc=$?
tail -c 600 $O/bench_cfg2.json; exit $rc
