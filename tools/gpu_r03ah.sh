# r03ah: kdtn_epoch_sync polls the epoch's completion event: config-2 step time (two lines)
set -uo pipefail
O=gpurun_out/r03ah; mkdir -p $O
for i in 1 2; do
timeout -k 10 400 python -u bench.py --no-ingest --no-wire --no-e2e --no-cpu-baseline --steps 50 > $O/bench_cfg2_$i.json 2> $O/bench_cfg2_$i.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_cfg2_$i.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline']['avg_ms'])"
done
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_parity_gpu.py -k "random or golden" > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
exit $rc
