# r02ao: product default with the first-record prefetch: full parity suite, smoke, config-2 / config-4 benches
set -euo pipefail
O=gpurun_out/r02ao; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python -u bench.py --config 4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
for c in 2 4; do python -c "import json; d=json.load(open('$O/bench_cfg$c.json')); print($c, d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'])"; done
timeout -k 10 300 python -u tools/shard_epoch.py --nshards 8 > $O/shard_n8.json 2> $O/shard_n8.err
python -c "import json; d=json.load(open('$O/shard_n8.json')); print(8, d['L0']['ms_epoch'], d['projected_links_per_s_at_N'])"
