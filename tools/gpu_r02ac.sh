# r02ac: one rank of the N = 2 / 4 / 8 strong-scaling run measured on one GPU (host-imported pod table)
set -euo pipefail
O=gpurun_out/r02ac; mkdir -p $O
for N in 8 4 2; do
  timeout -k 10 300 python -u tools/shard_epoch.py --nshards $N > $O/shard_n$N.json 2> $O/shard_n$N.err
  python -c "import json; d=json.load(open('$O/shard_n$N.json')); print($N, d['links_rank'], d['kdict'], d['pdict'], d['L0']['ms_epoch'], d['L1']['ms_epoch'], d['L2']['kernels_ms'])"
done
