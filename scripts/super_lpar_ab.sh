# C4 super engine (Urban3 480x640, L=3, K=11, fp64, scripts/prof_iter.py 200
# super): one block per tile and component (default, lpar=3) against one
# block per tile running the three components in turn (policy lpar=1), and
# lpar=3 without the per-XCD component placement (lpar_xcd=0); 2 rounds.
set -u
for r in 1 2; do
  for pol in "" lpar=1 lpar_xcd=0; do
    GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 super | sed "s/^/r$r [${pol:-default}] /" || exit 1
  done
done
