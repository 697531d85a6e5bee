# Round 6: (1) the dataflow tests on the default build (lag 2) and the stop /
# fault tests on the lag-6 variant (build/var/libgqmap_l6.so: overshoot ->
# ovr_recover); (2) the literal engine with the padded frame stored as
# double (policy vv_float=0: no per-tap conversion) against float, C2 fp64,
# 200 iterations, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_flow.py \
    > gpurun_out/r06_flow_tests_lag2.txt 2>&1 || exit $?
  echo "tests lag2 ok"
  GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_l6.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_flow.py -k "stop or failed or decay or c2_bit" \
    > gpurun_out/r06_flow_tests_lag6.txt 2>&1 || exit $?
  echo "tests lag6 ok"
fi
if [ "$STEP" = all ] || [ "$STEP" = ab ]; then
  : > gpurun_out/r06_lit_vv_ab.txt
  for r in 1 2 3; do
    for pol in vv_float=1 vv_float=0; do
      GQMAP_ARITH=literal GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 \
        | sed "s/^/$pol r$r /" >> gpurun_out/r06_lit_vv_ab.txt || exit $?
    done
  done
  echo "ab ok"
fi
