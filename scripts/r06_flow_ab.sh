# Round 6: the dataflow launch (policy flow, k_iter_flow) on C2 -- GPU
# bit-exactness against the per-launch path, then an interleaved A/B of
# scripts/prof_iter.py (C2 fp64 and fp32, 200 iterations: k_iter / dataflow
# kernel sum from HIP events, and the graph-replay wall clock).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_flow.py \
    > gpurun_out/r06_flow_tests.txt 2>&1 || exit $?
  echo "tests ok"
fi
if [ "$STEP" = all ] || [ "$STEP" = ab ]; then
  : > gpurun_out/r06_flow_ab.txt
  for r in 1 2 3; do
    for prec in ${PRECS:-fp64 fp32}; do
      for pol in flow=0 flow=1; do
        GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py ${ITS:-200} $prec \
          | sed "s/^/$pol r$r /" >> gpurun_out/r06_flow_ab.txt || exit $?
      done
    done
  done
  echo "ab ok"
fi
