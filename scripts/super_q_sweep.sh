# C4 super engine fp64 (Urban3 480x640, L=3, K=11): k_iter against the lanes
# per node forced through GQMAP_SPLIT (scripts/prof_iter.py 200 super),
# interleaved, 2 rounds.  The policy picks Q=4 (19,200 super-nodes).
set -u
for r in 1 2; do
  for q in 4 8 16; do
    GQMAP_SPLIT=$q timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 super | sed "s/^/r$r Q=$q /" || exit 1
  done
done
