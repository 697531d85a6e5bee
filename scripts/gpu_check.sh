# Round GPU check: smoke, the GPU test suite, a short bench.  Each step under
# its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke=$rc
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?; echo tests=$rc
if [ $rc -ne 0 ]; then tail -30 gpurun_out/gputests.log; exit $rc; fi
timeout -k 10 400 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1; echo bench=$?
