set -u
timeout -k 10 200 python -u -m pytest tests/test_gpu_tiles.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tiles2.log 2>&1; echo tiles=$?; tail -1 gpurun_out/tiles2.log
for n in 1 2 4 8; do timeout -k 10 120 python scripts/strip_time.py $n 200 || exit 1; done
