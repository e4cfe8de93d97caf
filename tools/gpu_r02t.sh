# r02t: A/B of the property-parse split and of k_reconcile's workgroups per chunk (profiling build)
set -euo pipefail
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 200 python -u tools/ablate.py --pods 125000 --reps 20 --masks none --env KDTN_PD_SPLIT=0,1 > $O/pdsplit_125k.json 2>&1
timeout -k 10 300 python -u tools/ablate.py --pods 1000000 --reps 10 --masks none --env KDTN_PD_SPLIT=0,1 > $O/pdsplit_1m.json 2>&1
timeout -k 10 200 python -u tools/ablate.py --pods 125000 --reps 20 --masks none --env KDTN_SPLIT=1,2,3,4,6,8 > $O/split_125k.json 2>&1
timeout -k 10 200 python -u tools/ablate.py --config 4 --pods 12500 --reps 20 --masks none --env KDTN_SPLIT=1,2,3,4,6,8 > $O/split_cfg4_12k.json 2>&1
cat $O/*.json
