# r02as: rank-interleaved pod-table order: full parity suite, one-rank epochs at N = 8 / 4 / 2
set -euo pipefail
O=gpurun_out/r02as; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for N in 8 4 2; do
  timeout -k 10 300 python -u tools/shard_epoch.py --nshards $N > $O/shard_n$N.json 2> $O/shard_n$N.err
  python -c "import json; d=json.load(open('$O/shard_n$N.json')); print($N, d['L0']['ms_epoch'], d['projected_links_per_s_at_N'], d['L2']['kernels_ms'])"
done
