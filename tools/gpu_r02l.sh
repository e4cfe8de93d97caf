# r02l: parity of the deferred placement (k_place) and the grid-stride k_full_prefix; config 2/3 timing
set -euo pipefail
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_multishard_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --no-cpu-baseline > $O/bench3.json 2> $O/bench3.err
python -c "import json; d=json.load(open('$O/bench3.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'], d['diff_only_reconcile_ms'])"
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-ingest --no-wire --no-e2e > $O/bench2.json 2> $O/bench2.err
python -c "import json; d=json.load(open('$O/bench2.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
