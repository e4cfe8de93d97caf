set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --variants 16899,4211203,16931 --reps 20 --masks ALL > $O/ablate.json 2>&1
