# Round 6: the dataflow launch on the super engine (C4) -- its GPU tests,
# then flow off / on interleaved (prof_iter.py 100 fp64 super).
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_flow.py \
  > gpurun_out/r06_flow_tests3.txt 2>&1 || exit $?
echo "tests ok"
OUT=gpurun_out/r06_super_flow_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_POLICY=$pol timeout -k 5 200 python3 scripts/prof_iter.py 100 fp64 super | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
