# Round 6 closing run on the final build: the whole GPU suite, the driver's
# C2 line twice, the fp32 and C5 lines.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r06_gpu_suite_closing.txt 2>&1 || exit $?
echo "suite ok"
: > gpurun_out/r06_closing_lines.jsonl
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--precision fp32 --steps 500" "--config c5 --steps 20"; do
  timeout -k 10 600 python -u bench.py $args > gpurun_out/r06_closing.txt 2>&1 || exit $?
  grep '^{' gpurun_out/r06_closing.txt >> gpurun_out/r06_closing_lines.jsonl
  echo "$args ok"
done
