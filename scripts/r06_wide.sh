# Round 6 (late): the 3-wave instantiation for large frames (GQ_FLOW_WIDE_ITEMS)
# -- the dataflow tests, then the C5 line and the driver's C2 line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_flow.py \
  > gpurun_out/r06_flow_tests_wide.txt 2>&1 || exit $?
echo "tests ok"
timeout -k 10 600 python -u bench.py --config c5 --steps 20 > gpurun_out/r06_c5_wide.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c2_wide.txt 2>&1 || exit $?
echo "bench ok"
