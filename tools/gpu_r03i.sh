# r03i: vector-memory pipe probe (per-instruction vs per-byte costs) and the 16-B qdisc store
# variant of k_reconcile (A/B against the default in one process)
set -uo pipefail
O=gpurun_out/r03i; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 tools/vmem_probe > $O/vmem_probe.jsonl 2> $O/vmem_probe.err || exit $?
cat $O/vmem_probe.jsonl
timeout -k 10 300 python -u tools/ablate.py --pods 1000000 --reps 10 --masks ALL \
    --variants 16899,49667 > $O/ab_q16.json 2> $O/ab.err || exit $?
cat $O/ab_q16.json
