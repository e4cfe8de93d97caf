set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ae; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --config 2 --env KDTN_FUSE=0,1 --wall --reps 30 --masks ALL > $O/fuse_cfg2.json 2>&1 &&
timeout -k 10 300 python -u tools/ablate.py --config 4 --pods 100000 --env KDTN_FUSE=0,1 --wall --reps 30 --masks ALL > $O/fuse_cfg4.json 2>&1 &&
KDTN_VARIANT=2116099 timeout -k 10 300 python -u tools/ablate.py --config 1 --pods 10000 --env KDTN_FUSE=0,1 --wall --reps 30 --masks ALL > $O/fuse_cfg1.json 2>&1
