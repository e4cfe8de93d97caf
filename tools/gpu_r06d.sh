set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 400 python -u tools/ablate.py --churn 5 --variants 18947,281091,16899 --reps 8 > $O/ablate_churn.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 2579 > $O/wgtrace_2579.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 264723 > $O/wgtrace_264723.json 2>&1
