# GPU parity subset, then an interleaved A/B of the variant libraries in
# gqmap-opticalflow_amd/build/var (scripts/variants.py) and per-phase timing.
#   TESTS="..." PRECS=fp64,fp32 ITS=100 ROUNDS=3 bash scripts/ab_kernel.sh
set -u
mkdir -p gpurun_out
TESTS=${TESTS:-}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; echo tests=$rc
  tail -3 gpurun_out/ab_tests.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab_tests.log | head -30; exit $rc; fi
fi
ROUNDS=${ROUNDS:-3} timeout -k 10 900 python -u scripts/variants.py ${ITS:-100} ${PRECS:-fp64,fp32} ${ENGINE:-mixture} > gpurun_out/ab_variants.log 2>&1; rc=$?; echo variants=$rc
cat gpurun_out/ab_variants.log
[ $rc -eq 0 ] || exit $rc
for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
  for p in ${PHASE_PRECS:-fp64}; do
    GQMAP_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/phase_time.py $p 20 ${PHASE_CFG:-c2} || exit $?
  done
done
