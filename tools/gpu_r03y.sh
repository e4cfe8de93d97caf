# r03y: rocprofv3 kernel stats of the output stages (fan-out, wire, RemotePod, tc) at HEAD
set -uo pipefail
O=$(pwd)/gpurun_out/r03y; mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
    -- python3 $R/tools/stage_run.py --reps 3 --stages run,fanout,encode,remote,tc > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json | head -60
