set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ad; mkdir -p $O
export KDTN_VARIANT=2116099
timeout -k 10 400 python -u tools/ablate.py --churn 4 --env KDTN_FUSE=0,1 --reps 15 > $O/fuse_churn.json 2>&1 &&
timeout -k 10 400 python -u tools/ablate.py --churn 4 --env KDTN_LOOKUP_SIDE=0,1,2 --reps 15 > $O/side_churn.json 2>&1
