# SQ-level counters of the fused iteration kernel over a short C2 run
# (scripts/prof_iter.py), one rocprofv3 --pmc pass per group (no multi-pass
# splitting on this pool).  VARS: libraries in build/var; PRECS: fp64 fp32.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_sq; mkdir -p $OUT
VARS=${VARS:-new}; PRECS=${PRECS:-"fp64 fp32"}; ITS=${ITS:-30}
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_IFETCH GRBM_GUI_ACTIVE"
PB="SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_INST_LEVEL_VMEM"
PC="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"
PE="TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT"
PD="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
for v in $VARS; do
  for prec in $PRECS; do
    i=0
    for P in "$PA" "$PB" "$PC" "$PD" "$PE"; do
      i=$((i+1))
      GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -s KILL 90 rocprofv3 --pmc $P \
        -d $OUT/${v}_${prec}_p$i -o run --output-format csv -- python3 scripts/prof_iter.py $ITS $prec ${ENGINE:-mixture} \
        > $OUT/${v}_${prec}_p$i.log 2>&1
      rc=$?; echo "$v $prec p$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
python3 scripts/pmc_table.py $OUT $(for v in $VARS; do for p in $PRECS; do printf "%s_%s " $v $p; done; done) > $OUT/table.txt
cat $OUT/table.txt
