# r03e: GPU record at HEAD after the container restore: whole -m gpu suite, smoke, default bench line
set -uo pipefail
O=gpurun_out/r03e; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/ablate.py --pods 1000000 --reps 10 --masks ALL --variants 16899,25091 > $O/ab_pct_lds.json 2> $O/ab.err || exit $?
cat $O/ab_pct_lds.json
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc"; exit $rc; }; }
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; ok $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err; rc=$?
tail -c 600 $O/bench_cfg2.json; exit $rc
