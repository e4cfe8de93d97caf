# final sources: the whole GPU suite, smoke, kernel stats and PMC passes of configs 2 / 3 / 4
set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06af tests,smoke,stats,pmc,stats3,pmc3,stats4,pmc4
