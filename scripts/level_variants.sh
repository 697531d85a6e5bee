# Interleaved k_iter timing of the small-grid cases (scripts/level_prof.py)
# for the library variants in gqmap-opticalflow_amd/build/var (VARS).
set -u
for r in 1 2 3; do
  for v in ${VARS:-base}; do
    for c in ${CASES:-l240 l120 strip8}; do
      GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 5 120 python3 scripts/level_prof.py $c 200 fp64 | sed "s/^/$v r$r /" || exit 1
    done
  done
done
