# Execution policies (gqmap_debug_policy, GQMAP_POLICY=name=value) on C2
# (scripts/prof_iter.py 200 fp64 / fp32) and the ctf 480x640 level
# (scripts/level_prof.py l480 200), interleaved, 2 rounds.
set -u
POLS=${POLS:-"default band_rows=1 cu_group=0 cu_group=1 cu_group=2 cu_group=4"}
for r in 1 2; do
  for pol in $POLS; do
    p=$pol; [ "$p" = default ] && p=""
    for prec in fp64 fp32; do
      GQMAP_POLICY=$p timeout -k 5 120 python3 scripts/prof_iter.py 200 $prec | sed "s/^/r$r [$pol] /" || exit 1
    done
    GQMAP_POLICY=$p timeout -k 5 120 python3 scripts/level_prof.py l480 200 fp64 | sed "s/^/r$r [$pol] /" || exit 1
  done
done
