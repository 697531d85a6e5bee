# Round 6: the dataflow launch on the coarse-to-fine levels -- GPU
# bit-exactness (tests/test_gpu_flow.py), then the level kernels with
# policy flow=0 / flow=1 interleaved (scripts/ctf_level_ab.py: HIP-event
# kernel sum and graph-replay wall clock per iteration).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_flow.py \
  > gpurun_out/r06_flow_tests2.txt 2>&1 || exit $?
echo "tests ok"
OUT=gpurun_out/r06_flow_ctf_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_POLICY=$pol timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5,0.25 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ctf ab ok"
