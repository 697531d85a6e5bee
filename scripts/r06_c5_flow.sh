# Round 6: the dataflow launch on a C5 frame (RubberWhale x4, 1552x2336,
# state 2 x 261 MB: non-temporal stores and the band-row walk on the
# per-launch path) -- flow off / on, interleaved, 50 iterations each.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_c5_flow.txt
: > $OUT
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_SCALE=4 GQMAP_POLICY=$pol timeout -k 5 200 python3 scripts/prof_iter.py 50 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "c5 ok"
