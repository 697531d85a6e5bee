#!/bin/bash
# The driver's C2 command with and without clock settling, C4 and C5 lines.
set -u
mkdir -p gpurun_out/r04settle
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04settle/c2_settle.jsonl 2> gpurun_out/r04settle/c2_settle.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-settle --no-cpu-baseline > gpurun_out/r04settle/c2_nosettle.jsonl 2> gpurun_out/r04settle/c2_nosettle.err || exit 2
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04settle/c2_settle_b.jsonl 2>> gpurun_out/r04settle/c2_settle.err || exit 3
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --no-parity > gpurun_out/r04settle/c4.jsonl 2> gpurun_out/r04settle/c4.err || exit 4
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-parity > gpurun_out/r04settle/c5.jsonl 2> gpurun_out/r04settle/c5.err || exit 5
echo done
