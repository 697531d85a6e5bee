#!/bin/bash
# Round-4 bench lines of every config (fp64, 1 GPU) into gpurun_out/r04_all.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_all.jsonl
: > $out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $out 2>> gpurun_out/r04_all.err || exit 2
timeout -k 10 300 python bench.py >> $out 2>> gpurun_out/r04_all.err || exit 3
timeout -k 10 300 python bench.py --config c1 >> $out 2>> gpurun_out/r04_all.err || exit 4
timeout -k 10 400 python bench.py --config c4 >> $out 2>> gpurun_out/r04_all.err || exit 5
timeout -k 10 300 python bench.py --config c3 >> $out 2>> gpurun_out/r04_all.err || exit 6
timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline >> $out 2>> gpurun_out/r04_all.err || exit 7
echo done
