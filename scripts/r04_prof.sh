#!/bin/bash
# Round-4 profiles: kernel time vs tile count (C2), then rocprofv3 stats and
# HBM passes of the driver's C2 window (20 steps) and of a 500-step run.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/tile_count_sweep.py fp64 > gpurun_out/r04_tile_sweep.txt 2>&1 || exit 1
cat gpurun_out/r04_tile_sweep.txt
CFG=c2 PREC=fp64 TAG=r04s20 STEPS=20 bash scripts/profile_round.sh || exit 2
CFG=c2 PREC=fp64 TAG=r04 STEPS=500 bash scripts/profile_round.sh || exit 3
echo done
