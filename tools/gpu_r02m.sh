# r02m: random-gather ceiling probe, k_reconcile gather ablations (config 2), ingest HBM traffic
set -euo pipefail
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 120 kube-dtn_amd/bin/gather_probe 10000000 10 > $O/gather_probe.jsonl 2> $O/gather_probe.err
cat $O/gather_probe.jsonl
timeout -k 10 400 python -u tools/ablate.py --variants 515,523,547,579,611 --reps 10 > $O/ablate_cfg2.json 2> $O/ablate_cfg2.err
cat $O/ablate_cfg2.json
bash tools/ingest_pmc_traffic.sh r02m
