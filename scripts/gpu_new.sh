# Run a chosen subset of GPU tests, then optional bench lines; each step
# time-limited, stop at the first failure.
#   bash scripts/gpu_new.sh "<pytest -k expr or file list>" "<bench args>;<bench args>..."
set -u
mkdir -p gpurun_out
TESTS="$1"
BENCHES="${2:-}"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpunew.log 2>&1; rc=$?; echo tests=$rc
tail -5 gpurun_out/gpunew.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpunew.log | head -30; exit $rc; fi
IFS=';'
i=0
for b in $BENCHES; do
  i=$((i+1))
  IFS=' '
  timeout -k 10 600 python bench.py $b > gpurun_out/bench_$i.log 2>&1; rc=$?; echo "bench[$b]=$rc"
  tail -1 gpurun_out/bench_$i.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$i.log; exit $rc; fi
  IFS=';'
done
