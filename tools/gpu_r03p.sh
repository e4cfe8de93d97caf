# r03p: GPU record at HEAD after the container restore: full parity suite, smoke, default
# bench line, rocprofv3 kernel stats + FETCH/WRITE passes of config 2
set -uo pipefail
O=gpurun_out/r03p; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
cat $O/bench_cfg2.json
bash tools/gpu_profile_round.sh r03p "2"
