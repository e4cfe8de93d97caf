#!/bin/bash
# SQ / TCC counter passes over kdtn_json_ingest (tools/ingest_run.py), one rocprofv3 run per
# group. Usage (GPU box, repo root): bash tools/ingest_pmc.sh <tag>
set -euo pipefail
TAG=$1; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
DOC=/tmp/kdtn_doc.json
timeout -k 10 300 python3 $R/tools/ingest_run.py --doc $DOC --reps 1 > $OUT/warm.log 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run \
      -- python3 $R/tools/ingest_run.py --doc $DOC --reps 1 > $OUT/pmc$i.log 2>&1
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
echo "ingest_pmc $TAG done"
