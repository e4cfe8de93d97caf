set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 300 python -u tools/variant_check.py --variants 2116099 --configs 3,1 --random 8 > $O/variant_check.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/ablate.py --churn 5 --variants 18947,2116099 --reps 8 > $O/ablate_churn.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 2579 > $O/wgtrace_2579.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 2099731 > $O/wgtrace_2099731.json 2>&1
