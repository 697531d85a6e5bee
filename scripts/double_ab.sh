# A/B: one block per slot with a second tile for the first blocks (default)
# vs one block per tile (GQMAP_ONE_TILE_PER_BLOCK=1), and the previous library.
set -u
L=$PWD/gqmap-opticalflow_amd/build/var
for r in 1 2; do
  for v in prev cur cur1; do
    lib=$L/libgqmap_${v%1}.so
    if [ $v = cur1 ]; then export GQMAP_ONE_TILE_PER_BLOCK=1; else unset GQMAP_ONE_TILE_PER_BLOCK; fi
    echo "variant $v"
    GQMAP_LIB=$lib timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 || exit 1
    GQMAP_LIB=$lib timeout -k 10 120 python scripts/phase_time.py fp32 20 c2 || exit 1
  done
done
