# r03d: parity of the changed encoder / fan-out / state paths, then kernel stats and counters
# of the epoch + output stages (config 2) and of the gather probe
set -uo pipefail
R=$(pwd); O=$R/gpurun_out/r03d; mkdir -p $O
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_state_gpu.py \
    tests/test_multishard_gpu.py tests/test_vni_state_gpu.py tests/test_parity_gpu.py \
    -k "state or commit or delta or resident or wire or remote or fanout or tc_argv or reach or shard or vni" \
    > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log; ok $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/tools/stage_run.py --reps 3 > $O/stats.log 2>&1 || exit $?
i=0
for grp in "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc$i -o run \
      -- python3 $R/tools/stage_run.py --reps 1 > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv \
    -d $O/probe_pmc -o run -- $R/kube-dtn_amd/bin/gather_probe 10000000 3 > $O/probe_pmc.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv \
    -d $O/probe_pmc2 -o run -- $R/kube-dtn_amd/bin/gather_probe 10000000 3 > $O/probe_pmc2.log 2>&1 || exit $?
python3 $R/tools/pmc_summary.py $O > $O/summary.txt
echo done
