# Round 6 (last): the column-pair store for the fp32 engine -- the parity /
# dataflow / logP GPU tests, then C2 fp32 vv_pair=0 vs 1 (200 its, 3 rounds).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_flow.py tests/test_gpu_vv.py tests/test_gpu_logp.py > gpurun_out/r06_vvpair_fp32_tests.txt 2>&1 || exit $?
echo "tests ok"
OUT=gpurun_out/r06_vvpair_fp32_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in vv_pair=0 vv_pair=1; do
    GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp32 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
