#!/bin/bash
# PMC passes over one reconcile epoch (tools/ablate.py), one rocprofv3 run per counter
# group (gfx950 TCC has 4 slots per pass; FETCH_SIZE and WRITE_SIZE cannot share one).
# Usage (on the GPU box): bash tools/pmc_profile.sh <outdir> [pods] [masks]
set -e
OUT=$1; PODS=${2:-1000000}; MASKS=${3:-ALL}
R=$(pwd)
mkdir -p $OUT
CACHE=/tmp/kdtn_cache
timeout -k 10 200 python3 $R/tools/ablate.py --pods $PODS --reps 1 --masks DIFF --cache $CACHE > $R/$OUT/warm.log 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_EA0_RDREQ_LEVEL_sum TCC_BUSY_sum TCC_CYCLE_sum TCC_LATENCY_FIFO_FULL_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_STALL_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/tools/ablate.py --pods $PODS --reps 2 --masks $MASKS --cache $CACHE > $R/$OUT/p$i.log 2>&1
done
