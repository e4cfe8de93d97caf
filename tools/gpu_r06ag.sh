# final bench lines (after the PMC summaries of the final sources are committed)
set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06ag bench,bench3,bench4,bench1
