# r02f: config-3 CalcDiff with L2-warmed candidates; XCD map A/B on config 2
set -euo pipefail
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --no-cpu-baseline > $O/bench3.json 2> $O/bench3.err
python -c "import json; d=json.load(open('$O/bench3.json')); print(d['value'], d['ms_per_step'], d['kernels_ms']['reconcile'], d['diff_only_reconcile_ms'])"
timeout -k 10 300 python -u tools/wgtrace.py --config 3 --variant 2579 --reps 3 > $O/wgtrace3.json 2> $O/wgtrace3.err
python -c "import json; d=json.load(open('$O/wgtrace3.json')); print({k: d[k] for k in ('kernel_ms_event','lifetime_us','diff_phaseA_us','diff_phaseB_us','diff_rest_to_counts_us')})"
