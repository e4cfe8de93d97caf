# closing counters at the round's final kernel sources (see tools/gpu_r06i.sh)
set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06n stats,pmc,stats3,pmc3,stats4,pmc4
