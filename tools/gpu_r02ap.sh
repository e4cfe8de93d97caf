# r02ap: VNI apply visibility kept from the count pass: parity and the config-4 apply stage
set -euo pipefail
O=gpurun_out/r02ap; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vni_state_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_vni.log 2>&1 || { tail -30 $O/pytest_vni.log; exit 1; }
tail -1 $O/pytest_vni.log
timeout -k 10 300 python -u bench.py --config 4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
python -c "import json; d=json.load(open('$O/bench_cfg4.json')); print(d['value'], d['ms_per_step'], d['vni_apply_stage'])"
