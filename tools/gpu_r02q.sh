# r02q: full GPU parity (incl. the one-rank RCCL communicator), smoke, config-2 bench, and a
# 125k-pod config-2 epoch (the per-rank size of the N = 8 strong-scaling run) for the fixed costs
set -euo pipefail
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench2.json 2> $O/bench2.err
python -c "import json; d=json.load(open('$O/bench2.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 300 python -u bench.py --pods 125000 --no-cpu-baseline --no-wire --no-e2e --no-ingest > $O/bench2_125k.json 2> $O/bench2_125k.err
python -c "import json; d=json.load(open('$O/bench2_125k.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
