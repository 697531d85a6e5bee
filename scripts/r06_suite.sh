# Round 6: the whole GPU suite, the ctf levels with flow off / on, and the
# C2 / C3 bench lines on the default policies.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = suite ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/r06_gpu_suite.txt 2>&1 || exit $?
  echo "suite ok"
fi
if [ "$STEP" = all ] || [ "$STEP" = ctf ]; then
  OUT=gpurun_out/r06_flow_ctf_ab2.txt
  : > $OUT
  for r in 1 2 3; do
    for pol in flow=0 flow=1; do
      GQMAP_POLICY=$pol timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5,0.25 | sed "s/^/$pol r$r /" >> $OUT || exit $?
    done
  done
  echo "ctf ok"
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_c2.txt 2>&1 || exit $?
  timeout -k 10 400 python -u bench.py --config c3 --steps 100 --warmup 2 > gpurun_out/r06_bench_c3.txt 2>&1 || exit $?
  echo "bench ok"
fi
