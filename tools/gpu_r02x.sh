# r02x: topology rows loaded with the first-partial read; gathers before the next segment search
set -euo pipefail
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/ablate.py --pods 1000000 --reps 10 --masks ALL,DIFF > $O/ablate_1m.json 2>&1
timeout -k 10 300 python -u tools/epoch_overhead.py --pods 1000000,125000 > $O/overhead.jsonl 2> $O/overhead.err
cat $O/overhead.jsonl
timeout -k 10 500 python -u bench.py --config 3 --steps 5 --no-cpu-baseline > $O/bench3.json 2> $O/bench3.err
python -c "import json; d=json.load(open('$O/bench3.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['kernels_ms'])"
grep -A12 '"ALL"\|"DIFF"' $O/ablate_1m.json | grep "reconcile\|ALL\|DIFF"
