set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ac; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --config 3 --pods 1000000 --env KDTN_FUSE=0,1 --wall --reps 20 > $O/fuse_cfg3.json 2>&1 &&
timeout -k 10 300 python -u tools/ablate.py --config 3 --pods 1000000 --env KDTN_LOOKUP_SIDE=0,1 --wall --reps 20 > $O/side_cfg3.json 2>&1
