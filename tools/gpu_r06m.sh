set -euo pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_state_gpu.py" bash tools/gpu_round.sh r06m tests,bench1
