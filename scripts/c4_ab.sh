# C4 (super engine) k_iter A/B of build/var/libgqmap_*.so, interleaved rounds
set -u
for r in 1 2 3; do
  for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
    GQMAP_LIB=$PWD/$lib timeout -k 10 120 python scripts/phase_time.py ${PREC:-fp64} 20 c4 || exit 1
  done
done
