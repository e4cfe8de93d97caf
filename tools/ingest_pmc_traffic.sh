#!/bin/bash
# HBM traffic of the CR-ingest kernels on the config-2 TopologyList (2.86 GB document):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over tools/ingest_run.py.
# Usage (GPU box, repo root): bash tools/ingest_pmc_traffic.sh <tag> [pods]
# IPMC_GROUPS overrides the passes: groups separated by ';', counters in a group by ',' (one
# rocprofv3 run per group, within the per-block counter limits).
set -euo pipefail
TAG=$1; PODS=${2:-1000000}; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
DOC=/tmp/kdtn_doc_$PODS.json
timeout -k 10 400 python3 $R/tools/ingest_run.py --pods $PODS --doc $DOC --reps 1 > $OUT/ingest_warm.log 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra GROUPS_ <<< "${IPMC_GROUPS:-FETCH_SIZE;WRITE_SIZE}"
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv -d $OUT/ingpmc$i -o run \
      -- python3 $R/tools/ingest_run.py --pods $PODS --doc $DOC --reps 2 > $OUT/ingpmc$i.log 2>&1
  echo "ingest pmc $grp done"
done
