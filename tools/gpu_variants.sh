#!/bin/bash
# Variant A/B of k_reconcile (times, then FETCH_SIZE / WRITE_SIZE per variant, one pass each).
# Usage (GPU box, repo root): bash tools/gpu_variants.sh <tag> <variants> [pods]
set -euo pipefail
TAG=$1; VARS=$2; PODS=${3:-1000000}
R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
CACHE=/tmp/kdtn_cache
timeout -k 10 300 python3 $R/tools/ablate.py --pods $PODS --reps 10 --masks ALL --variants $VARS --cache $CACHE > $OUT/times.json 2> $OUT/times.err
cat $OUT/times.json
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run \
      -- python3 $R/tools/ablate.py --pods $PODS --reps 1 --masks ALL --variants $VARS --cache $CACHE > $OUT/pmc$i.log 2>&1
done
python3 $R/tools/pmc_summary.py $OUT | grep reconcile
echo "gpu_variants $TAG done"
