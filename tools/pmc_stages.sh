#!/bin/bash
# Counter passes over the config-2 output stages (tools/stage_run.py: encode, fan-out, RemotePod,
# tc), one rocprofv3 run per group; per-kernel means into <tag>/summary.txt.
# Usage (GPU box, repo root): bash tools/pmc_stages.sh <tag> [stage_run.py args]
set -euo pipefail
TAG=$1; shift; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
ARGS=${*:---reps 1}
timeout -k 10 300 python3 $R/tools/stage_run.py $ARGS > $OUT/warm.json 2> $OUT/warm.err
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run \
      -- python3 $R/tools/stage_run.py $ARGS > $OUT/pmc$i.log 2>&1
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.txt
echo "pmc_stages $TAG done"
