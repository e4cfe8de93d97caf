# r03af: commit fast path (every Topology committed: no reassembly) and per-block commit
# counting: state parity + config-3 bench line with the resident chain
set -uo pipefail
O=gpurun_out/r03af; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_state_gpu.py tests/test_vni_state_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 500 python -u bench.py --config 3 --no-cpu-baseline --no-ingest --no-wire > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg3.json')); print(d['value']/1e9, d['ms_per_step']); print(json.dumps(d.get('resident_chain')))"
