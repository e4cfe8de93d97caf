# r03ae: kernel trace of the config-3 resident chain (delta upload, run, download, commit) and
# the new timer-totals test
set -uo pipefail
R=$(pwd); O=$R/gpurun_out/r03ae; mkdir -p $O
export PYTHONUNBUFFERED=1
true


cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/stats -o run \
    -- python3 $R/bench.py --config 3 --steps 2 --warmup 1 --resident-epochs 5 --no-cpu-baseline --no-ingest --no-wire \
    > $O/bench3.json 2> $O/bench3.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench3.json')); print(json.dumps(d.get('resident_chain')))"
