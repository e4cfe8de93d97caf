# r02at: bench.py's multi-rank path on one GPU: 2 ranks with the host transport (gloo all-gather)
set -euo pipefail
O=gpurun_out/r02at; mkdir -p $O
export KDTN_BENCH_HOST_XCHG=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 5 --warmup 1 --pods 200000 > $O/bench2_n2.json 2> $O/bench2_n2.err
cat $O/bench2_n2.json | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
    bench.py --gpus 2 --config 3 --steps 2 --warmup 1 --pods 200000 > $O/bench3_n2.json 2> $O/bench3_n2.err
cat $O/bench3_n2.json | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['exchange'])"
