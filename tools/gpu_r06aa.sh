set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --config 2 --env KDTN_KD_SUB=1,43 --reps 20 > $O/kd_ab.json 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -v --timeout 240 --timeout-method thread -k "cidr or key or kdict or predicate or go_stdlib" > $O/pytest.log 2>&1
