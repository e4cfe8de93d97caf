# r02o: parity of split bulk chunks (k_reconcile) and the XCD-contiguous ingest blocks; benches
set -euo pipefail
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/bench4.json 2> $O/bench4.err
python -c "import json; d=json.load(open('$O/bench4.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-wire --no-e2e > $O/bench2.json 2> $O/bench2.err
python -c "import json; d=json.load(open('$O/bench2.json')); print(d['value'], d['ms_per_step'], d['kernels_ms']); i=d['ingest_stage']; print(i['gpu_ms'], i['kernels_ms'], i['epoch_on_ingest_tables']['ms_per_step'])"
