#!/bin/bash
# Round-4 GPU check: the -m gpu suite (or the files given as arguments), then
# the driver's bench line and the default (500-step) C2 line.  Every GPU step
# under its own time limit.
set -u
mkdir -p gpurun_out
T=${*:-tests}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_gputests.txt 2>&1 || { tail -30 gpurun_out/r04_gputests.txt; exit 1; }
tail -3 gpurun_out/r04_gputests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench20.jsonl 2> gpurun_out/r04_bench20.err || exit 2
timeout -k 10 400 python bench.py > gpurun_out/r04_bench500.jsonl 2> gpurun_out/r04_bench500.err || exit 3
echo done
