# r03s: branch-free octet windows in the CIDR classifier: predicate parity + kdict A/B
set -uo pipefail
O=gpurun_out/r03s; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_parity_gpu.py \
    -k "predicate or cidr or golden or synthetic or random_epochs" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/ablate.py --pods 1000000 --reps 10 --masks ALL --env KDTN_KD_SUB=1,42,1,42 \
    --cache /tmp/kdtn_cache > $O/kd_ab.json 2> $O/kd_ab.err || exit $?
python3 -c "
import json; d=json.load(open('$O/kd_ab.json'))['ms']
for k,v in d.items(): print(k, v.get('kdict_parse'), v.get('reconcile'))"
exit 0
