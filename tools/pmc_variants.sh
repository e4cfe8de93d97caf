#!/bin/bash
# L2 / fabric request counters for several k_reconcile variants in one process each
# (tools/ablate.py --variants, interleaved). Usage (GPU box):
#   bash tools/pmc_variants.sh <outdir> [pods] [variants]
set -e
OUT=$1; PODS=${2:-1000000}; VARS=${3:-1,33,65,97}
R=$(pwd)
mkdir -p $OUT
CACHE=/tmp/kdtn_cache
timeout -k 10 200 python3 $R/tools/ablate.py --pods $PODS --reps 1 --masks DIFF --cache $CACHE > $R/$OUT/warm.log 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$OUT/v$i -o run -- python3 $R/tools/ablate.py --pods $PODS --reps 2 --masks NONE --variants $VARS --cache $CACHE > $R/$OUT/v$i.log 2>&1
done
