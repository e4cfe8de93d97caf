set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --config 4 --pods 100000 --env KDTN_SPLIT=1,2,3,4,6,8,12 --reps 20 > $O/split_cfg4.json 2>&1 &&
timeout -k 10 300 python -u tools/ablate.py --config 1 --pods 10000 --env KDTN_SPLIT=1,2,4,8,16 --reps 20 > $O/split_cfg1.json 2>&1
