# Round 6 (last): with the column-pair store -- C2 fp64 per launch (flow=0)
# vs the dataflow launch (default), 3 rounds; and C5 with the 3-wave wide
# instantiation (base) vs 2 waves everywhere (nowide, build/var).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_last_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in flow=0 flow=-1; do
    GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "c2 ok"
for v in base nowide; do
  GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so GQMAP_SCALE=4 timeout -k 5 200 python3 scripts/prof_iter.py 50 fp64 \
    | sed "s/^/c5 $v /" >> $OUT || exit $?
  GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so GQMAP_SCALE=4 timeout -k 5 200 python3 scripts/prof_iter.py 50 fp64 \
    | sed "s/^/c5 $v /" >> $OUT || exit $?
done
echo "c5 ok"
