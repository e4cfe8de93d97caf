set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 300 python -u tools/variant_check.py --variants 281091 --configs 3,1 --random 8 > $O/variant_check.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/ablate.py --config 3 --variants 18947,281091 --reps 20 --masks ALL > $O/ablate_cfg3.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 2579 > $O/wgtrace_2579.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 264723 > $O/wgtrace_264723.json 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ingest_gpu.py -k "escape or separator or grow" > $O/pytest.log 2>&1
