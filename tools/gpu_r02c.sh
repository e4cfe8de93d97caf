set -euo pipefail
mkdir -p gpurun_out/r02c; python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c/smoke.log 2>&1; tail -1 gpurun_out/r02c/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_multishard_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c/pytest.log 2>&1
tail -3 gpurun_out/r02c/pytest.log
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --no-cpu-baseline > gpurun_out/r02c/bench3.json 2> gpurun_out/r02c/bench3.err
python -c "import json; d=json.load(open('gpurun_out/r02c/bench3.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'], d['diff_only_reconcile_ms'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-wire --no-ingest --no-e2e > gpurun_out/r02c/bench2.json 2> gpurun_out/r02c/bench2.err
python -c "import json; d=json.load(open('gpurun_out/r02c/bench2.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 400 python -u tools/ablate.py --pods 1000000 --reps 6 --masks ALL --variants 515,547,579,611,519,643,771 > gpurun_out/r02c/variants.json 2> gpurun_out/r02c/variants.err
python -c "import json; d=json.load(open('gpurun_out/r02c/variants.json')); print({k: v for k, v in d['ms'].items() if k.startswith('variant')})"
