# r02ai: duration fast path (parity + per-interpretation timing) and the wave-staged kdict A/B
set -euo pipefail
O=gpurun_out/r02ai; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 250 python -u tools/ablate.py --pods 1000000 --reps 20 --masks none --env KDTN_PD_ONLY=0,1,2,4 > $O/pd_1m.json 2>&1
timeout -k 10 250 python -u tools/ablate.py --pods 1000000 --reps 20 --masks none --env KDTN_KD_SUB=1,16 > $O/kd_1m.json 2>&1
timeout -k 10 200 python -u tools/ablate.py --pods 125000 --reps 30 --masks none --env KDTN_KD_SUB=1,16 > $O/kd_125k.json 2>&1
grep "PD_ONLY\|pdict\|KD_SUB\|kdict" $O/pd_1m.json $O/kd_*.json
