set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/c4probe; mkdir -p $OUT
timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 > $OUT/phase.log 2>&1 || exit 1
for sp in 4 1; do GQMAP_SPLIT=$sp timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 >> $OUT/phase.log 2>&1 || exit 1; done
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
P4="TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_ANY"
i=0
for P in "$P1" "$P2" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/c4_p$i -o run --output-format csv -- python3 scripts/prof_iter.py 10 fp64 super > $OUT/c4_p$i.log 2>&1 || exit 1
  i2=$i; timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/c2_p$i -o run --output-format csv -- python3 scripts/prof_iter.py 30 fp64 mixture > $OUT/c2_p$i.log 2>&1 || exit 1
done
echo done
