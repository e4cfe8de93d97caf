# r03ai: SQ counters of the epoch front (k_kdict_flags VALU-bound claim) — one --pmc pass per group
set -uo pipefail
R=$(pwd); O=$R/gpurun_out/r03aj/sq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/stage_run.py --reps 1 --stages run > $O/warm.log 2>&1 || exit $?
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc$i -o run \
      -- python3 $R/tools/stage_run.py --reps 2 --stages run > $O/pmc$i.log 2>&1 || exit $?
  echo "pass $i done"
done
