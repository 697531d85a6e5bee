# Round 6: the literal-order engine's execution forms (GQ_LIT_FORM 0/1/2,
# gqmap_math.h) -- GPU bit-exactness of the default build, interleaved A/B of
# the variants (scripts/variants.py, C2 fp64 arith=literal, 200 its), SQ
# counters of f0 (round 5's form) and f2; then the C3 line and the RCCL
# self-send probe with capture (last: it may time out).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_legacy.py tests/test_gpu_literal.py > gpurun_out/r06_lit_tests.txt 2>&1 || exit $?
  echo "tests ok"
fi
if [ "$STEP" = all ] || [ "$STEP" = ab ]; then
  GQMAP_ARITH=literal ROUNDS=3 timeout -k 10 400 python -u scripts/variants.py 200 fp64 > gpurun_out/r06_lit_ab.txt 2>&1 || exit $?
  echo "ab ok"
fi
if [ "$STEP" = all ] || [ "$STEP" = pmc ]; then
  VARS="f0 f2" PRECS=fp64 GQMAP_ARITH=literal ITS=30 timeout -k 10 500 bash scripts/pmc_sq.sh > gpurun_out/r06_lit_pmc.txt 2>&1 || exit $?
  echo "pmc ok"
fi
