#!/bin/bash
# SQ / TA counter passes over one epoch (tools/ablate.py), one rocprofv3 run per group.
# Usage (GPU box, repo root): bash tools/pmc_sq.sh <tag>
set -euo pipefail
TAG=$1; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
CACHE=/tmp/kdtn_cache
timeout -k 10 300 python3 $R/tools/ablate.py --pods 1000000 --reps 1 --masks DIFF --cache $CACHE > $OUT/warm.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run \
      -- python3 $R/tools/ablate.py --pods 1000000 --reps 1 --masks ALL --cache $CACHE > $OUT/pmc$i.log 2>&1
done
python3 $R/tools/pmc_summary.py $OUT
echo "pmc_sq $TAG done"
