# closing proxies and stage reports: one rank of N = 2 / 4 / 8, output stages, CR ingest, and the
# pipelined resident loop under rocprofv3 --kernel-trace --stats (the SDMA download path traced)
set -euo pipefail
cd $GRAFT_REPO_ROOT
RT_FLAGS="--kernel-trace --stats" bash tools/gpu_round.sh r06p shard,stages,ingest,restrace
