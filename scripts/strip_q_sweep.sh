# One rank's strip of the N-way strong-scaling layout (RubberWhale 388 x
# 584/N, mixture K=9 fp64, scripts/level_prof.py 200): k_iter against lanes
# per node forced with GQMAP_SPLIT, interleaved, 2 rounds.
set -u
CASES=${CASES:-"strip2:1 strip2:2 strip2:4 strip4:1 strip4:2 strip4:4 strip8:1 strip8:2 strip8:4 strip16:1 strip16:2 strip16:4 strip32:2 strip32:4 strip32:8"}
for r in 1 2; do
  for c in $CASES; do
    GQMAP_SPLIT=${c#*:} timeout -k 5 120 python3 scripts/level_prof.py ${c%%:*} 200 fp64 | sed "s/^/r$r /" || exit 1
  done
done
