# r02am: entry-parallel reach rule (fan-out, tc): full parity suite, config-2 bench (wire / fan-out stage)
set -euo pipefail
O=gpurun_out/r02am; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err
python -c "import json; d=json.load(open('$O/bench_cfg2.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['traffic'], d['wire_stage']['fanout'])"
