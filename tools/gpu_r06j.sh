# closing parity and bench lines (after the PMC summaries of these kernel sources are committed)
set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06j tests,smoke,bench,bench3,bench4,bench1
