# C3 middle levels: lanes per node Q = 2, 4, 8, 16 for each libgqmap variant
# in build/var (waves/SIMD bound, edge-job prefetch on/off).
set -u
mkdir -p gpurun_out
for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
  n=$(basename $lib .so); n=${n#libgqmap_}
  GQMAP_LIB=$PWD/$lib QS=${QS:-2,4,8,16} timeout -k 10 200 python -u scripts/level_sweep.py fp64 | sed "s/^/$n /" || exit $?
done
