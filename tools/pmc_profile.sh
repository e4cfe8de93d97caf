#!/bin/bash
# PMC passes over one reconcile epoch (tools/ablate.py, ALL stages), one rocprofv3 run per
# counter group (gfx950 TCC slots: FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage (on the GPU box): bash tools/pmc_profile.sh <outdir> [pods]
set -e
OUT=$1; PODS=${2:-1000000}
R=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/tools/ablate.py --pods $PODS --reps 2 --masks ALL > $R/$OUT/p$i.log 2>&1
done
