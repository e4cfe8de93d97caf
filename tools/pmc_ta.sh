#!/bin/bash
# TA / TCP utilisation passes over one epoch (tools/ablate.py). Usage: bash tools/pmc_ta.sh <tag>
set -euo pipefail
TAG=$1; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
CACHE=/tmp/kdtn_cache
timeout -k 10 300 python3 $R/tools/ablate.py --pods 1000000 --reps 1 --masks DIFF --cache $CACHE > $OUT/warm.log 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_COUNT" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run \
      -- python3 $R/tools/ablate.py --pods 1000000 --reps 1 --masks ALL --cache $CACHE > $OUT/pmc$i.log 2>&1
done
python3 $R/tools/pmc_summary.py $OUT | grep -E "reconcile|kdict"
echo "pmc_ta $TAG done"
