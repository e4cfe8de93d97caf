# r03ag: buffer growth headroom + commit fast path before the mask upload: full suite, config-3
# resident chain, config-2 line
set -uo pipefail
O=gpurun_out/r03ag; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 500 python -u bench.py --config 3 --no-cpu-baseline --no-ingest --no-wire > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg3.json')); print(d['value']/1e9, d['ms_per_step']); print(json.dumps(d.get('resident_chain')))"
timeout -k 10 400 python -u bench.py --no-ingest --no-wire > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg2.json')); print(d['value']/1e9, d['ms_per_step'], json.dumps(d.get('e2e_pcie'))[:400])"
