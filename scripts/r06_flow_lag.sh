# Round 6: the dataflow launch's finalize lag (GQ_FLOW_LAG 2/4/6/8, build/var)
# -- interleaved C2 fp64 and C3 480x640 / 240x320 level timings (policy
# flow=1), then the item timeline of the lag-6 form (libgqmap_tl6.so).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_flow_lag.txt
: > $OUT
for r in 1 2 3; do
  for v in ${VARS:-l2 l4 l6 l8}; do
    lib=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so
    GQMAP_LIB=$lib GQMAP_POLICY=flow=1 timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$v r$r /" >> $OUT || exit $?
    GQMAP_LIB=$lib GQMAP_POLICY=flow=1 timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 | sed "s/^/$v r$r /" >> $OUT || exit $?
  done
done
echo "lag ab ok"
if [ -f gqmap-opticalflow_amd/build/var/libgqmap_tl6.so ]; then
  GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_tl6.so timeout -k 5 120 python3 scripts/flow_timeline.py \
    > gpurun_out/r06_flow_timeline_lag6.txt 2>&1 || exit $?
  echo "timeline ok"
fi
