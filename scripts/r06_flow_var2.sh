# Round 6: dataflow-kernel variants (build/var) on C2 fp64 and the ctf
# 480x640 / 240x320 levels, policy flow=1, interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_flow_var2.txt
: > $OUT
for r in 1 2 3; do
  for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
    n=$(basename $lib .so); n=${n#libgqmap_}
    GQMAP_LIB=$PWD/$lib GQMAP_POLICY=flow=1 timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$n r$r /" >> $OUT || exit $?
    GQMAP_LIB=$PWD/$lib GQMAP_POLICY=flow=1 timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 | sed "s/^/$n r$r /" >> $OUT || exit $?
  done
done
echo "var2 ok"
