# r02n: workgroup trace of config 4 (bulk path, power-law degrees); rocprof stats + HBM traffic of config 3
set -euo pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 300 python -u tools/wgtrace.py --config 4 --pods 100000 --variant 531 --reps 3 > $O/wgtrace4.json 2> $O/wgtrace4.err
python -c "import json; d=json.load(open('$O/wgtrace4.json')); print(d['kernel_ms_event'], d['span_us'], d['lifetime_us'], d['mean_resident_wgs'])"
bash tools/gpu_profile_round.sh r02n 3
