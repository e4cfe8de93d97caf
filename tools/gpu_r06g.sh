set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 300 python -u tools/ablate.py --variants 16899,541187,1065475,16931,16963 --reps 20 --masks ALL > $O/ablate.json 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "go_stdlib" > $O/pytest.log 2>&1
