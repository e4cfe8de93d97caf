# closing parity run and bench lines at the final sources (PMC summaries committed first)
set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06o tests,smoke,bench,bench3,bench4,bench1
