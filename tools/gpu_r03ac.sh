# r03ac: one rank of the N = 2 / 4 / 8 strong-scaling run on one GPU at HEAD (tools/shard_epoch.py)
set -uo pipefail
O=gpurun_out/r03ac; mkdir -p $O
for N in 2 4 8; do
  timeout -k 10 300 python -u tools/shard_epoch.py --nshards $N > $O/shard_n$N.json 2> $O/shard_n$N.err || exit $?
  tail -c 600 $O/shard_n$N.json; echo
done
