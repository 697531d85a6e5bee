# Pipelined-kernel variants (build/var/libgqmap_<v>.so): phase timings on C2.
set -u
for v in ${VARS:-stats statsf1}; do
  for p in fp64; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 10 90 python scripts/phase_time.py $p 20 2>&1 || exit 1
  done
done
