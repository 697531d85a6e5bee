# Interleaved C4 phase timings of variant libraries build/var/libgqmap_<v>.so
set -u
for r in 1 2; do
for v in ${VARS:-cur}; do
  for p in ${PRECS:-fp64}; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 10 120 python scripts/phase_time.py $p 20 c4 2>&1 || exit 1
  done
done
done
