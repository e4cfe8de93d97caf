set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
KDTN_VARIANT=2116099 timeout -k 10 300 python -u tools/ablate.py --config 1 --pods 10000 --env KDTN_SPLIT=1,2,3,4 --reps 30 --wall > $O/split_cfg1_diff.json 2>&1
