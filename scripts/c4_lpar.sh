# C4 k_iter time per iteration: component-parallel blocks (default) vs one
# block per tile (GQMAP_LPAR=1), for lanes-per-node Q = 16, 4, 1.
set -u
for sp in 16 4 1; do
  GQMAP_SPLIT=$sp timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 || exit 1
  GQMAP_LPAR=1 GQMAP_SPLIT=$sp timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 || exit 1
done
