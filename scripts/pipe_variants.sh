# Interleaved C2 phase timings (scripts/phase_time.py) of variant libraries
# build/var/libgqmap_<v>.so; VARS and PRECS select them.
set -u
for r in 1 2; do
for v in ${VARS:-base}; do
  for p in ${PRECS:-fp64}; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 10 90 python scripts/phase_time.py $p 20 2>&1 || exit 1
  done
done
done
