# Literal-order engine (C2 fp64, scripts/prof_iter.py 200): padded frame
# stored as float (default for integer frames) against double
# (gqmap_debug_policy vv_float=0), interleaved, 3 rounds.
set -u
for r in 1 2 3; do
  for pol in vv_float=1 vv_float=0; do
    GQMAP_ARITH=literal GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" || exit 1
  done
done
