# Interleaved phase timing (scripts/phase_time.py) of the variant libraries
# build/var/libgqmap_<v>.so named in $VARS (default: all), fp64 and fp32.
set -u
VARS=${VARS:-$(ls gqmap-opticalflow_amd/build/var/ | sed -n 's/^libgqmap_\(.*\)\.so$/\1/p')}
PRECS=${PRECS:-"fp64 fp32"}
for r in 1 2; do
  for v in $VARS; do
    for p in $PRECS; do
      GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 10 120 python scripts/phase_time.py $p 20 || exit 1
    done
  done
done
