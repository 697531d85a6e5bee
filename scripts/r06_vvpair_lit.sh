# Round 6 (late): the literal-order engine on the binary16 column-pair frame
# store -- its GPU tests (bit-exact vs the restatement at 20 / 500
# iterations), the dataflow tests, then C2 fp64 arith=literal vv_pair=1 vs 0
# (200 its, 3 interleaved rounds; the same checksum expected).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_literal.py \
  tests/test_gpu_flow.py > gpurun_out/r06_vvpair_lit_tests.txt 2>&1 || exit $?
echo "tests ok"
OUT=gpurun_out/r06_vvpair_lit_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in vv_pair=0 vv_pair=1; do
    GQMAP_ARITH=literal GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
