# Round 6 (late): the padded frame stored as double (policy vv_float=0: no tap
# conversions, twice the gather bytes) on the 2-wave dataflow launch -- C2
# fp64, 200 iterations, 3 interleaved rounds; then the 480x640 / 240x320 levels.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_vvd2w_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in vv_float=1 vv_float=0; do
    GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
