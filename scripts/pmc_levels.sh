# SQ / TA counters of the small-grid iteration kernels (C3's 240x320 and
# 120x160 levels, the 8-way strip 388x75 at Q=4): one rocprofv3 --pmc pass
# per counter group, scripts/level_prof.py CASE 50 (per-dispatch values).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_levels; mkdir -p $OUT
CASES=${CASES:-"l240 l120 strip8"}; PREC=${PREC:-fp64}
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
PB="SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM"
PE="TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT"
for c in $CASES; do
  i=0
  for P in "$PA" "$PB" "$PE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${c}_p$i -o run --output-format csv -- \
      python3 scripts/level_prof.py $c 50 $PREC > $OUT/${c}_p$i.log 2>&1
    rc=$?; echo "$c p$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/pmc_table.py $OUT $CASES > $OUT/table.txt
cat $OUT/table.txt
