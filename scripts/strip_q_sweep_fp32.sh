# scripts/strip_q_sweep.sh for fp32 (scripts/level_prof.py stripN 200 fp32, GQMAP_SPLIT forced).
set -u
for r in 1 2; do
  for c in strip2:1 strip2:2 strip4:1 strip4:2 strip4:4 strip8:2 strip8:4 strip16:2 strip16:4; do
    GQMAP_SPLIT=${c#*:} timeout -k 5 120 python3 scripts/level_prof.py ${c%%:*} 200 fp32 | sed "s/^/r$r /" || exit 1
  done
done
