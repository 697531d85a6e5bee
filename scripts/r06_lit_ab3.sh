# Round 6: literal-engine variants (build/var): the next point's XJ scalar
# load issued a point early (xjp), the divisions by pi as div_rcp with
# RN(1/pi) (pidiv), both, against neither (base) -- C2 fp64 arith=literal,
# 200 iterations, interleaved rounds (chk = state checksum); then the
# literal GPU tests on the variant with both.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GQMAP_ARITH=literal ROUNDS=${ROUNDS:-3} timeout -k 10 600 python -u scripts/variants.py 200 fp64 > gpurun_out/r06_lit_ab3.txt 2>&1 || exit $?
echo "ab ok"
GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_both.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_literal.py > gpurun_out/r06_lit_tests3.txt 2>&1 || exit $?
echo "tests ok"
