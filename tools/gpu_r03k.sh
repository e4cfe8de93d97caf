# r03k: fan-out chunk loads prefetched; 16-B string-table entries with strings of <= 12 bytes inline (no dependent arena load),
# one-pass 1024-thread top scan: encoder parity, then stage times of the product (writers at 3
# waves/SIMD) and of the profiling build (writers held to 4 waves, spilling)
set -uo pipefail
O=gpurun_out/r03k; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_multishard_gpu.py tests/test_configs_gpu.py tests/test_state_gpu.py tests/test_vni_state_gpu.py \
    tests/test_ingest_gpu.py -k "wire or remote or fanout or tc_argv or reach or config or state or vni or kubedtn or scan or ingest" > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
timeout -k 10 300 python3 tools/stage_run.py --reps 3 --prof --stages encode,remote > $O/stages_prof.json 2> $O/stages_prof.err || exit $?
cat $O/stages_prof.json
