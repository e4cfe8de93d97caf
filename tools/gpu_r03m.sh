# r03m: GPU record at HEAD — whole -m gpu suite, smoke, bench lines for configs 2, 3, 4
set -uo pipefail
O=gpurun_out/r03m; mkdir -p $O
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; ok $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
tail -c 300 $O/bench_cfg2.json; echo
timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit $?
tail -c 300 $O/bench_cfg3.json; echo
timeout -k 10 200 python -u bench.py --config 4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit $?
tail -c 300 $O/bench_cfg4.json
