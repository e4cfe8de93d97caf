# r03h: two-pass wire writer again; RemotePod/tc-remote writers store per-daemon runs through the
# wave's LDS image (wave_segments_write); reach status fused into the cut pass; faster string
# table. Parity of the encoder / fan-out paths, stage times, and a k_reconcile phase trace (config 2)
set -uo pipefail
O=gpurun_out/r03h; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_multishard_gpu.py tests/test_configs_gpu.py tests/test_state_gpu.py -k "wire or remote or fanout or tc_argv or reach or config or state" \
    > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/stage_run.py --reps 3 > $O/stages.json 2> $O/stages.err || exit $?
cat $O/stages.json
timeout -k 10 300 python3 tools/wgtrace.py --variant 16915 --reps 3 > $O/wgtrace_cfg2.json 2> $O/wgtrace.err || echo "wgtrace rc $?"
cat $O/wgtrace_cfg2.json
timeout -k 10 300 python -u tools/ablate.py --pods 1000000 --reps 10 --masks ALL \
    --variants 16899,16963,16931,16995,16903 > $O/ab_gathers.json 2> $O/ab.err || exit $?
cat $O/ab_gathers.json
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/$O/list_avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$O/pmc$i -o run \
      -- python3 $R/tools/ablate.py --pods 1000000 --reps 2 --masks ALL --cache /tmp/kdtn_cache > $R/$O/pmc$i.log 2>&1 || { echo "pmc pass $i rc $?"; break; }
done
echo done
