# VV of the fp64 engines stored as _Float16 (exact for integer frames: cubic
# padding stays in [-510, 765]) vs float: half the gather bytes, two
# conversions per tap.
set -u
for r in 1 2; do
  for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
    GQMAP_LIB=$PWD/$lib timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 || exit 1
    GQMAP_LIB=$PWD/$lib timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 || exit 1
  done
done
