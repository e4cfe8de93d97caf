# r02au: the driver's default bench command at HEAD (N = 1)
set -euo pipefail
O=gpurun_out/r02au; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['config']['exchange'], d['cpu_baseline']['value'])"
