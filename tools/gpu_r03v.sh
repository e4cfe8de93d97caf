# r03v: fused epoch front (pod tables inside the dictionary-parse launches): A/B, full GPU
# suite, smoke, default bench line
set -uo pipefail
O=gpurun_out/r03v; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/side_ab.py --reps 40 --knob KDTN_FUSE --modes 0,1 --cache /tmp/kdtn_cache > $O/fuse_ab.json 2> $O/fuse_ab.err || { tail -5 $O/fuse_ab.err; exit 1; }
head -12 $O/fuse_ab.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --no-ingest > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg2.json'))
print(d['value']/1e9, d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d['kernels_ms'])"
