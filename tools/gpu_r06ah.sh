set -euo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r06ah shard
