# r02d: parity of the changed CalcDiff window, config-3 epochs and its phase trace
set -euo pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02e/pytest.log 2>&1
tail -2 gpurun_out/r02e/pytest.log
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --no-cpu-baseline > gpurun_out/r02e/bench3.json 2> gpurun_out/r02e/bench3.err
python -c "import json; d=json.load(open('gpurun_out/r02e/bench3.json')); print(d['value'], d['ms_per_step'], d['kernels_ms']['reconcile'], d['diff_only_reconcile_ms'])"
timeout -k 10 300 python -u tools/wgtrace.py --config 3 --variant 2579 --reps 3 > gpurun_out/r02e/wgtrace3.json 2> gpurun_out/r02e/wgtrace3.err
cat gpurun_out/r02e/wgtrace3.json
