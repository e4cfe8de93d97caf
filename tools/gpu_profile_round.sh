#!/bin/bash
# Profiles of the benched configs (one GPU-box pass): rocprofv3 kernel-trace stats of the
# bench command per config, then the HBM traffic of k_reconcile per config from separate
# FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md § HBM: one counter group per pass).
# Usage (on the GPU box, repo root): bash tools/gpu_profile_round.sh <tag> [configs]
set -euo pipefail
TAG=${1:-r02}
CONFIGS=${2:-"2 3 4"}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
CACHE=/tmp/kdtn_cache
cd /tmp && export TMPDIR=/tmp
for C in $CONFIGS; do
  case $C in 2) P=1000000; S=20;; 3) P=1000000; S=5;; 4) P=100000; S=20;; esac
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats$C -o run \
      -- python3 $R/bench.py --config $C --steps $S --no-cpu-baseline --no-ingest --no-wire --no-e2e \
      > $OUT/stats_bench$C.json 2> $OUT/stats$C.err
  echo "config $C stats done"
  timeout -k 10 300 python3 $R/tools/ablate.py --config $C --pods $P --reps 1 --masks DIFF --cache $CACHE \
      > $OUT/pmc_warm$C.log 2>&1
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc${C}_$i -o run \
        -- python3 $R/tools/ablate.py --config $C --pods $P --reps 3 --masks ALL --cache $CACHE \
        > $OUT/pmc${C}_$i.log 2>&1
    echo "config $C pmc $grp done"
  done
done
echo "profile round $TAG done"
