set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python -u tools/variant_check.py --variants 281091 --configs 3 --random 4 > $O/variant_check.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/ablate.py --churn 5 --variants 18947,281091 --reps 8 > $O/ablate_churn.json 2>&1 &&
timeout -k 10 200 python -u tools/wgtrace.py --config 3 --variant 264723 > $O/wgtrace_264723.json 2>&1 &&
timeout -k 10 120 ./tools/sdma_probe 48 20 > $O/sdma_probe.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/resident_run.py --epochs 6 --both --sdma-engines 2,1,4 > $O/resident_engines.jsonl 2> $O/resident_engines.err
