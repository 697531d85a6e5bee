#!/bin/bash
# 16x12 vs 16x16 tiles (GQMAP_TILE_SHAPE) on C2 fp64/fp32: k_iter us/it early /
# mid / late, then the tile-count sweep with the default policy, then the
# GPU suite.
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_shape_ab.txt
: > $out
for p in fp64 fp32; do
  for v in 16 12; do
    echo "GQMAP_TILE_SHAPE=$v" >> $out
    GQMAP_TILE_SHAPE=$v timeout -k 10 120 python scripts/phase_time.py $p 20 c2 >> $out 2>&1 || exit 1
  done
done
cat $out
timeout -k 10 300 python scripts/tile_count_sweep.py fp64 > gpurun_out/r04_tile_sweep_policy.txt 2>&1 || exit 2
cat gpurun_out/r04_tile_sweep_policy.txt
