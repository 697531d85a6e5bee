# Round 6 final measurements on one box: the GPU suite, the driver's C2
# command twice and the default 500-step line, then the rocprofv3 trace of
# the driver's command and the FETCH/WRITE passes (r06_profile_c2.sh) --
# STEP=suite|bench|profile|configs (default: all but configs).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEP=${STEP:-main}
if [ "$STEP" = main ] || [ "$STEP" = suite ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/r06_gpu_suite_final.txt 2>&1 || exit $?
  echo "suite ok"
fi
if [ "$STEP" = main ] || [ "$STEP" = bench ]; then
  : > gpurun_out/r06_final_c2.jsonl
  for k in 1 2; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_final_c2_$k.txt 2>&1 || exit $?
    grep '^{' gpurun_out/r06_final_c2_$k.txt >> gpurun_out/r06_final_c2.jsonl
  done
  timeout -k 10 600 python -u bench.py > gpurun_out/r06_final_c2_500.txt 2>&1 || exit $?
  echo "bench ok"
fi
if [ "$STEP" = main ] || [ "$STEP" = profile ]; then
  TAG=${TAG:-r06} timeout -k 10 900 bash scripts/r06_profile_c2.sh || exit $?
fi
if [ "$STEP" = configs ]; then
  : > gpurun_out/r06_final_configs.jsonl
  for args in "--config c3" "--config c4 --steps 20" "--config c5 --steps 20" "--config c1" "--precision fp32 --steps 500"; do
    timeout -k 10 600 python -u bench.py $args > gpurun_out/r06_cfg.txt 2>&1 || exit $?
    grep '^{' gpurun_out/r06_cfg.txt >> gpurun_out/r06_final_configs.jsonl
    echo "$args ok"
  done
fi
