# r02v: VNI state apply parity first, then the full GPU suite and the benches
set -euo pipefail
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vni_state_gpu.py tests/test_host_cpp.py -x -v --timeout 120 --timeout-method thread > $O/pytest_vni.log 2>&1 || { tail -40 $O/pytest_vni.log; exit 1; }
tail -2 $O/pytest_vni.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench2.json 2> $O/bench2.err
python -c "import json; d=json.load(open('$O/bench2.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['kernels_ms'])"
timeout -k 10 300 python -u bench.py --pods 125000 --no-cpu-baseline --no-wire --no-e2e --no-ingest > $O/bench2_125k.json 2> $O/bench2_125k.err
python -c "import json; d=json.load(open('$O/bench2_125k.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['kernels_ms'])"
