set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u tools/variant_check.py --variants 49667 --configs 2,4:100000,1 --random 4 > $O/variant_check.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/ablate.py --variants 16899,49667 --reps 30 --masks ALL > $O/ablate.json 2>&1 &&
timeout -k 10 300 python -u tools/ablate.py --config 4 --pods 100000 --variants 16899,49667 --reps 30 --masks ALL > $O/ablate4.json 2>&1
