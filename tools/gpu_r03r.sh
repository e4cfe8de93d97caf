# r03r: leaner CIDR classifier (cidr_swar2) — predicate parity + A/B vs the round-2 classifier;
# full-size whole-epoch oracle checks (config 2, config 3 x10, 8 shards)
set -uo pipefail
O=gpurun_out/r03r; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_parity_gpu.py \
    -k "predicate or cidr or golden or synthetic or random_epochs" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/ablate.py --pods 1000000 --reps 10 --masks ALL --env KDTN_KD_SUB=1,42,1,42 \
    --cache /tmp/kdtn_cache > $O/kd_ab.json 2> $O/kd_ab.err || exit $?
python3 -c "
import json; d=json.load(open('$O/kd_ab.json'))['ms']
for k,v in d.items(): print(k, v.get('kdict_parse'), v.get('reconcile'))"
timeout -k 10 900 python -u -m pytest -v --durations=0 --timeout 400 --timeout-method thread tests/test_configs_gpu.py \
    tests/test_parity_gpu.py::test_config2_full_size_properties > $O/full.log 2>&1; rc=$?
tail -12 $O/full.log
exit $rc
