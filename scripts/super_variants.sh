# C4-shaped (Urban3, super L=3 K=11) timings of variant libraries: k_iter us/it.
set -u
for r in 1 2; do
for v in ${VARS:-base}; do
  GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 10 120 python scripts/prof_iter.py 40 fp64 super 2>&1 | sed "s/^/$v /" || exit 1
done
done
