#!/bin/bash
# Resident-loop diagnosis on the GPU box: page-locked H2D rates of this box, the per-epoch
# resident loop (tools/resident_run.py; MODE=--pipeline for the overlapped loop), and the same
# loop under rocprofv3 kernel + memory-copy tracing (copy and kernel timestamps).
# Usage: [MODE=--pipeline] bash tools/resident_diag.sh <tag>
set -euo pipefail
TAG=$1; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 120 python -u tools/h2d_probe.py > $OUT/h2d.jsonl 2> $OUT/h2d.err
timeout -k 10 300 python -u tools/resident_run.py --epochs 6 ${MODE:-} > $OUT/resident.jsonl 2> $OUT/resident.err
tail -1 $OUT/resident.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run \
    -- python3 $R/tools/resident_run.py --epochs 4 ${MODE:-} > $OUT/trace.log 2>&1
tail -1 $OUT/trace.log
echo "resident_diag $TAG done"
