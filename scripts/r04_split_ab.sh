#!/bin/bash
# Phase-split iteration A/B (GQMAP_PHASE_SPLIT): C2 k_iter us/it early / mid /
# late, fp64 and fp32, then the C2-sized parity tests with the split on.
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_split_ab.txt
: > $out
for p in fp64 fp32; do
  for v in 0 1; do
    echo "GQMAP_PHASE_SPLIT=$v" >> $out
    GQMAP_PHASE_SPLIT=$v timeout -k 10 120 python scripts/phase_time.py $p 20 c2 >> $out 2>&1 || exit 1
  done
done
cat $out
GQMAP_PHASE_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_longrun.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_split_tests.txt 2>&1
tail -3 gpurun_out/r04_split_tests.txt
