# Round 6: the literal-order engine on the dataflow launch -- its GPU tests
# (bit-exact against the restatement, on the default policy), then flow off /
# on interleaved (prof_iter.py 200, arith=literal).
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_literal.py \
  > gpurun_out/r06_lit_flow_tests.txt 2>&1 || exit $?
echo "tests ok"
OUT=gpurun_out/r06_lit_flow_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_ARITH=literal GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
