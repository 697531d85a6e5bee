# Round 6: SQ counters of the C2 fp64 fast kernels on the final build -- the
# per-launch k_iter (policy flow=0) and the dataflow k_iter_flow (default) --
# over prof_iter.py 50 iterations (every dispatch then runs 50 iterations:
# divide the flow rows by 50 for per-iteration values).  One rocprofv3
# --pmc pass per counter group, each under its own time limit.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_c2; mkdir -p $OUT
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_IFETCH GRBM_GUI_ACTIVE"
PB="SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_INST_LEVEL_VMEM"
PC="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"
PD="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
PE="TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT"
for cfg in kiter:flow=0 flow:flow=1; do
  n=${cfg%%:*}; pol=${cfg#*:}
  i=0
  for P in "$PA" "$PB" "$PC" "$PD" "$PE"; do
    i=$((i+1))
    GQMAP_POLICY=$pol timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${n}_p$i -o run --output-format csv \
      -- python3 scripts/prof_iter.py 50 fp64 > $OUT/${n}_p$i.log 2>&1
    rc=$?; echo "$n p$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/pmc_table.py $OUT kiter flow > $OUT/table.txt
cat $OUT/table.txt
