# closing counters at the round's last kernel sources: rocprofv3 kernel stats and the
# FETCH_SIZE / WRITE_SIZE passes of configs 2 / 3 / 4, then the SQ / TA passes of config 2
set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06i stats,pmc,stats3,pmc3,stats4,pmc4
bash tools/pmc_sq.sh r06i_sq
