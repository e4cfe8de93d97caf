# r02z3: HEAD record — full parity suite, config-3 bench line, then rocprofv3 stats + PMC traffic for configs 2-4
set -euo pipefail
O=gpurun_out/r02z3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python -u bench.py --config 3 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
python -c "import json; d=json.load(open('$O/bench_cfg3.json')); print(3, d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'])"
bash tools/gpu_profile_round.sh r02zp2 "2 3 4"
