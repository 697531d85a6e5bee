# One PMC pass (P1 SQ counters) over a short run: ENGINE=super|mixture PREC=fp64 ITS=10
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_quick; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $OUT/${TAG:-q}_p1 -o run --output-format csv -- python3 scripts/prof_iter.py ${ITS:-10} ${PREC:-fp64} ${ENGINE:-super} > $OUT/${TAG:-q}_p1.log 2>&1
