#!/bin/bash
# The one GPU-box runner: parity tests, smoke, bench lines, rocprofv3 kernel-trace stats and
# HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs), the one-rank strong-scaling proxy.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag> [what]
#   what: comma list of
#     tests      pytest -m gpu (all files, or the files in $TESTS, -k $K when set)
#     smoke      __graft_entry__.smoke()
#     bench      bench.py config 2 (the driver's line); bench3 / bench4 / bench1 other configs
#     stats      rocprofv3 --kernel-trace --stats of the config-2 bench; stats3 / stats4 likewise
#     pmc        k_reconcile FETCH_SIZE / WRITE_SIZE passes over config 2 (pmc3 / pmc4 likewise)
#     shard      one rank of N = 2 / 4 / 8 on this GPU (tools/shard_epoch.py); $SHARD_NS overrides
#     ingest     config-2 ingest stage with kernel times (tools/ingest_run.py)
#     ipmc       ingest FETCH_SIZE / WRITE_SIZE passes (tools/ingest_pmc_traffic.sh)
#     istats     rocprofv3 --kernel-trace --stats of the config-2 ingest (tools/ingest_run.py)
#     iab        ingest A/B of profiling variants $IAB_VARIANTS (tools/ingest_ablate.py, default 0,16)
#     stages     output-stage kernel times (tools/stage_run.py)
#     restrace   rocprofv3 kernel + memory-copy trace of the pipelined resident loop (exit check)
#     shardstats rocprofv3 kernel stats of one rank of N = $SHARD_N (default 8)
#   default: tests,smoke,bench,stats,pmc
# Every GPU step has its own time limit and the script stops at the first failure.
set -euo pipefail
TAG=${1:-r04}
WHAT=${2:-tests,smoke,bench,stats,pmc}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
has() { [[ ",$WHAT," == *",$1,"* ]]; }
CACHE=/tmp/kdtn_cache

if has tests; then
  KARG=()
  [[ -n "${K:-}" ]] && KARG=(-k "$K")
  timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
      "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1
  tail -3 $OUT/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
fi
if has iab; then
  timeout -k 10 500 python -u tools/ingest_ablate.py 1000000 ${IAB_VARIANTS:-0,16} > $OUT/ingest_ab.jsonl 2> $OUT/ingest_ab.err
  cat $OUT/ingest_ab.jsonl
fi
for C in 2 1 3 4; do
  B=bench; [[ $C != 2 ]] && B=bench$C
  if has $B; then
    timeout -k 10 500 python -u bench.py --config $C ${BENCH_ARGS:-} > $OUT/$B.json 2> $OUT/$B.err
    cat $OUT/$B.json
  fi
done
if has shard; then
  for N in ${SHARD_NS:-2 4 8}; do
    timeout -k 10 300 python -u tools/shard_epoch.py --nshards $N > $OUT/shard_n$N.json 2> $OUT/shard_n$N.err
    cat $OUT/shard_n$N.json
  done
fi
if has ingest; then
  timeout -k 10 400 python -u tools/ingest_run.py --pods 1000000 --doc /tmp/kdtn_doc_1000000.json > $OUT/ingest.json 2> $OUT/ingest.err
  tail -5 $OUT/ingest.json
fi
if has stages; then
  timeout -k 10 400 python -u tools/stage_run.py > $OUT/stages.json 2> $OUT/stages.err
  tail -5 $OUT/stages.json
fi
cd /tmp && export TMPDIR=/tmp
for C in 2 3 4; do
  S=stats; [[ $C != 2 ]] && S=stats$C
  case $C in 2) P=1000000; ST=20;; 3) P=1000000; ST=5;; 4) P=100000; ST=20;; esac
  if has $S; then
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$S -o run \
        -- python3 $R/bench.py --config $C --steps $ST --warmup 3 --no-cpu-baseline > $OUT/${S}_bench.json 2> $OUT/$S.err
    cat $OUT/${S}_bench.json
  fi
  PM=pmc; [[ $C != 2 ]] && PM=pmc$C
  if has $PM; then
    timeout -k 10 300 python3 $R/tools/ablate.py --config $C --pods $P --reps 1 --masks DIFF --cache $CACHE \
        > $OUT/${PM}_warm.log 2>&1
    i=0
    for grp in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/${PM}_$i -o run \
          -- python3 $R/tools/ablate.py --config $C --pods $P --reps 3 --masks ALL --cache $CACHE \
          > $OUT/${PM}_$i.log 2>&1
    done
    echo "$PM done"
  fi
done
if has restrace; then
  # traced pipelined resident loop (the round-4 exit-time SIGSEGV): library map written at exit
  timeout -k 10 400 rocprofv3 ${RT_FLAGS:---kernel-trace --memory-copy-trace --stats} --output-format csv -d $OUT/restrace -o run \
      -- python3 $R/tools/resident_run.py ${RT_ARGS:---epochs 4 --pipeline} --maps $OUT/restrace_maps.txt \
      > $OUT/restrace.jsonl 2> $OUT/restrace.log
  tail -2 $OUT/restrace.jsonl
fi
if has shardstats; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shardstats -o run \
      -- python3 $R/tools/shard_epoch.py --nshards ${SHARD_N:-8} > $OUT/shardstats.json 2> $OUT/shardstats.err
  cat $OUT/shardstats.json
fi
if has istats; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/istats -o run \
      -- python3 $R/tools/ingest_run.py --pods 1000000 --doc /tmp/kdtn_doc_1000000.json > $OUT/istats_ingest.json 2> $OUT/istats.err
  cat $OUT/istats_ingest.json
fi
if has ipmc; then
  (cd $R && bash tools/ingest_pmc_traffic.sh $TAG/ipmc 1000000)
fi
echo "gpu_round $TAG done"
