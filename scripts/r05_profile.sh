# Round-5 profiles of the driver's command (bench.py --steps 20, default
# warm-up): rocprofv3 kernel trace + stats, then the round profile of C2 fp64
# (FETCH_SIZE / WRITE_SIZE passes -> profiles/traffic_c2_fp64.json).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05prof/bench20 -o run --output-format csv -- \
  python3 bench.py --steps 20 > gpurun_out/r05prof/bench20.json 2> gpurun_out/r05prof/bench20.err || exit $?
python3 scripts/trace_segments.py gpurun_out/r05prof/bench20/run_kernel_trace.csv > gpurun_out/r05prof/bench20_segments.txt || exit $?
CFG=c2 PREC=fp64 TAG=r05 STEPS=200 bash scripts/profile_round.sh
