# C3 pyramid levels (Grove3 full size / resized, ctf K=11 fp64,
# scripts/level_prof.py 200): k_iter against lanes per node forced with
# GQMAP_SPLIT, interleaved, 2 rounds (the persistent small-grid path is not
# on run_timed's per-launch timing: k_iter is the plain launch).
set -u
CASES=${CASES:-"l480:1 l480:2 l240:1 l240:2 l240:4 l120:2 l120:4 l120:8 l60:4 l60:8 l60:16 l30:8 l30:16 l30:64"}
for r in 1 2; do
  for c in $CASES; do
    GQMAP_SPLIT=${c#*:} timeout -k 5 120 python3 scripts/level_prof.py ${c%%:*} 200 fp64 | sed "s/^/r$r /" || exit 1
  done
done
