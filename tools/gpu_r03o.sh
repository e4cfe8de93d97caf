# r03o: delta upload (host checks over the appended suffix only, vectorised reference check,
# wave-cooperative topology search in the store assembly) and the short-wave CIDR class path:
# state / predicate parity, stage times, config-3 bench line (resident chain)
set -uo pipefail
O=gpurun_out/r03o; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_state_gpu.py \
    tests/test_parity_gpu.py tests/test_configs_gpu.py -k "state or commit or delta or resident or predicate or cidr or golden or random or synthetic or config3 or churn" > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 5 --stages run > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline --no-ingest --no-wire > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit $?
tail -c 700 $O/bench_cfg3.json
