set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python -u tools/resident_run.py --epochs 6 --both --sdma-engines 2,6,2,6 > $O/resident_engines.jsonl 2> $O/resident_engines.err &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_state_gpu.py -k "download or resident or pipelined or async" > $O/pytest.log 2>&1
