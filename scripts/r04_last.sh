#!/bin/bash
# Last check of the round: the -m gpu suite, smoke, the driver's C2 line.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_last_tests.txt 2>&1 || { tail -30 gpurun_out/r04_last_tests.txt; exit 1; }
tail -2 gpurun_out/r04_last_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 2
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_last.jsonl 2> gpurun_out/r04_last.err || exit 3
echo done
