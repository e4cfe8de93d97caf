# r03w: timing events without the system-scope fence; HIP-event totals read once per timed loop
# parity subset
set -uo pipefail
O=gpurun_out/r03x; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --no-ingest --no-wire --no-e2e > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg2.json'))
print(d['value']/1e9, d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d['kernels_ms'])"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_state_gpu.py \
    -k "not full_size" > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
exit $rc
