# Literal-order engine (C2 fp64, scripts/prof_iter.py 200, arith=literal):
# library variants in gqmap-opticalflow_amd/build/var (VARS), interleaved,
# 3 rounds; the checksum must match across variants.
set -u
V=$PWD/gqmap-opticalflow_amd/build/var
for r in 1 2 3; do
  for lib in ${VARS:-base}; do
    GQMAP_LIB=$V/libgqmap_$lib.so GQMAP_ARITH=literal timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$lib r$r /" || exit 1
  done
done
