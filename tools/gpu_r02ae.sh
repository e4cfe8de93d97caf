# r02ae: epoch-begin launch (zero + pod rows) and verify+prefix fusion: parity, fixed costs, N-rank proxies
set -euo pipefail
O=gpurun_out/r02ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/epoch_overhead.py --pods 1000000,125000 > $O/overhead.jsonl 2> $O/overhead.err
cat $O/overhead.jsonl
for N in 8 4 2; do
  timeout -k 10 300 python -u tools/shard_epoch.py --nshards $N > $O/shard_n$N.json 2> $O/shard_n$N.err
  python -c "import json; d=json.load(open('$O/shard_n$N.json')); print($N, d['L0']['ms_epoch'], d['L1']['ms_epoch'], d['L2']['kernels_ms'])"
done
