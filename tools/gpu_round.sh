#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel-trace stats of the bench
# command, and the two HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs).
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag> [what]
#   what: comma list of tests,smoke,bench,bench3,bench4,stats,pmc (default: tests,smoke,bench,stats,pmc)
# Every GPU step has its own time limit and the script stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
WHAT=${2:-tests,smoke,bench,stats,pmc}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
has() { [[ ",$WHAT," == *",$1,"* ]]; }

if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1
  tail -3 $OUT/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
fi
if has bench; then
  timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
fi
if has bench3; then
  timeout -k 10 500 python -u bench.py --config 3 > $OUT/bench3.json 2> $OUT/bench3.err
  cat $OUT/bench3.json
fi
if has bench4; then
  timeout -k 10 300 python -u bench.py --config 4 > $OUT/bench4.json 2> $OUT/bench4.err
  cat $OUT/bench4.json
fi
cd /tmp && export TMPDIR=/tmp
if has stats; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run \
      -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/stats_bench.json 2> $OUT/stats.err
  cat $OUT/stats_bench.json
fi
if has pmc; then
  CACHE=/tmp/kdtn_cache
  timeout -k 10 300 python3 $R/tools/ablate.py --pods 1000000 --reps 1 --masks DIFF --cache $CACHE \
      > $OUT/pmc_warm.log 2>&1
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run \
        -- python3 $R/tools/ablate.py --pods 1000000 --reps 3 --masks ALL --cache $CACHE \
        > $OUT/pmc$i.log 2>&1
  done
  python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
  cat $OUT/pmc_summary.txt
fi
echo "gpu_round $TAG done"
