#!/bin/bash
# A/B of the staged-tap window (GQ_TAP_LDS) on the C2 kernel: k_iter us/it
# early / mid / late (scripts/phase_time.py) for the library and the
# variants under gqmap-opticalflow_amd/build/var.
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_lds_ab2.txt
: > $out
for lib in libgqmap.so $(cd gqmap-opticalflow_amd && ls build/var/*.so); do
  GQMAP_LIB=$PWD/gqmap-opticalflow_amd/$lib timeout -k 10 120 python scripts/phase_time.py ${PREC:-fp64} 20 c2 >> $out 2>&1 || exit 1
done
cat $out
