# Round 6 profile of C2 fp64 on the dataflow launch: rocprofv3
# --kernel-trace --stats of the driver's command (bench.py --steps 20),
# then FETCH_SIZE / WRITE_SIZE passes over scripts/prof_iter.py 200 (every
# k_iter_flow dispatch runs 50 iterations there) and the calibration
# kernels; summaries into profiles/ (pmc_summary.py, trace_segments.py).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG/c2_fp64
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || exit $?
echo "trace ok"
for ctr in FETCH_SIZE WRITE_SIZE; do
  low=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/$low -o run --output-format csv -- \
    python3 scripts/prof_iter.py 200 fp64 > $OUT/$low.log 2>&1 || exit $?
  echo "$ctr ok"
done
[ -x scripts/micro/fetch_calib ] || hipcc --offload-arch=gfx950 -O2 scripts/micro/fetch_calib.hip -o scripts/micro/fetch_calib || exit $?
for ctr in FETCH_SIZE WRITE_SIZE; do
  low=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/$TAG/calib_$low -o run --output-format csv -- \
    scripts/micro/fetch_calib > gpurun_out/$TAG/calib_$low.log 2>&1 || exit $?
done
FLOW_ITS=50 python3 scripts/pmc_summary.py gpurun_out/$TAG c2 fp64 > /dev/null || exit $?
python3 scripts/trace_segments.py $(find $OUT/trace -name "*kernel_trace.csv" | head -1) --its 20 > $OUT/segments.txt || exit $?
echo "profile ok"
