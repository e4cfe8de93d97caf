set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06a
timeout -k 10 300 python -u tools/variant_check.py --variants 66051,65539 > gpurun_out/r06a/variant_check.jsonl 2>&1 &&
timeout -k 10 240 python -u tools/ablate.py --variants 16899,66051,65539,515 --reps 20 --masks ALL > gpurun_out/r06a/ablate.json 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "registered or without_sync or page_locked" tests/test_ingest_gpu.py > gpurun_out/r06a/pytest.log 2>&1
