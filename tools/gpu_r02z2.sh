# r02z2: the round's GPU record — full parity suite, smoke, bench lines for configs 2 / 3 / 4
set -euo pipefail
O=gpurun_out/r02z2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 500 python -u bench.py --config 3 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python -u bench.py --config 4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
for c in 2 3 4; do python -c "import json; d=json.load(open('$O/bench_cfg$c.json')); print($c, d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'])"; done
for N in 8 4 2; do
  timeout -k 10 300 python -u tools/shard_epoch.py --nshards $N > $O/shard_n$N.json 2> $O/shard_n$N.err
  python -c "import json; d=json.load(open('$O/shard_n$N.json')); print($N, d['L0']['ms_epoch'], d['projected_links_per_s_at_N'])"
done
