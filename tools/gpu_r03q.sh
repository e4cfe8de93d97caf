# r03q: k_kdict_flags A/B — launch floor (40), load floor (41), 1/2/4 strings per thread,
# persistent software-pipelined waves at 8/16 workgroups per CU (32/33)
set -uo pipefail
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 400 python3 tools/ablate.py --pods 1000000 --reps 10 --masks ALL --env KDTN_KD_SUB=1,2,4,32,33,40,41 \
    --cache /tmp/kdtn_cache > $O/kd_ab.json 2> $O/kd_ab.err || exit $?
python3 -c "
import json; d=json.load(open('$O/kd_ab.json'))['ms']
for k,v in d.items(): print(k, v.get('kdict_parse'), v.get('reconcile'))"
