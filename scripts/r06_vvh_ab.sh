# Round 6: the padded frame (VV) stored as binary16 (exact for the integer
# frames of C2: values in [-510, 765]) -- half the tap-gather bytes of float
# storage.  build/var: base (float), h16 (GQ_VVS_HALF); C2 fp64 fast
# (dataflow launch) and literal arithmetic, 200 iterations, interleaved;
# then the literal / dataflow GPU tests on the default build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > gpurun_out/r06_vvh_ab.txt 2>&1 || exit $?
GQMAP_ARITH=literal ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 >> gpurun_out/r06_vvh_ab.txt 2>&1 || exit $?
echo "ab ok"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_literal.py \
  tests/test_gpu_flow.py > gpurun_out/r06_lit_tests2.txt 2>&1 || exit $?
echo "tests ok"
