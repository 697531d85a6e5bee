# Round 6 (late): the literal-order dataflow launch allowed 2 waves per SIMD
# (GQ_FLOW_LIT_WAVES=2, build/var/libgqmap_lw2.so: no spills, 512 slots)
# against the per-launch literal kernel -- C2 fp64 arith=literal, 200
# iterations, 3 interleaved rounds; then the literal flow test.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_lit_flow_ab3.txt
: > $OUT
L=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_lw2.so
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_LIB=$L GQMAP_ARITH=literal GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
GQMAP_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_flow.py \
  -k literal > gpurun_out/r06_lit_flow_test3.txt 2>&1 || exit $?
echo "test ok"
