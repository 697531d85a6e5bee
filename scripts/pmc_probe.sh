# Counter passes over a short C2 run (scripts/prof_iter.py) for the variant
# libraries named in $VARS (build/var/libgqmap_<v>.so); one rocprofv3 --pmc
# run per pass (MI355X_MICROARCH.md: no multi-pass splitting).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_probe; mkdir -p $OUT
VARS=${VARS:-"vv patch"}; PREC=${PREC:-fp64}; ITS=${ITS:-30}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
P3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P4="TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_STALL_MULTI_MISS_sum SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_ANY"
for v in $VARS; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -s KILL 90 rocprofv3 --pmc $P \
      -d $OUT/${v}_p$i -o run --output-format csv -- python3 scripts/prof_iter.py $ITS $PREC ${ENGINE:-mixture} > $OUT/${v}_p$i.log 2>&1
    rc=$?; echo "$v p$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/pmc_table.py $OUT $VARS > $OUT/table.txt; cat $OUT/table.txt
