# r03fin: closing GPU record of the session at HEAD: full parity suite, smoke, bench lines for
# 3 and 4
set -uo pipefail
O=gpurun_out/r03fin; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
timeout -k 10 500 python -u bench.py --config 3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit $?
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit $?
for c in 2 3 4; do python3 -c "
import json; d=json.load(open('$O/bench_cfg$c.json'))
print($c, round(d['value']/1e9,3), round(d['ms_per_step'],4), d['roofline'].get('avg_ms'), round(d['roofline']['frac'],4))"; done
