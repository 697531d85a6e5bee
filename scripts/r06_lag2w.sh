# Round 6 (late): the finalize lag again on the 2-wave dataflow launch (l4,
# l6 vs base = lag 2): C2 fp64 fast and literal (variants.py, 200 its, 3
# rounds) and the ctf levels; then the item timeline of the 2-wave build
# (tl, GQ_FLOW_TL) with the wait attribution.  (tl is excluded from the A/B.)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out gpurun_out/tlbuild
mv gqmap-opticalflow_amd/build/var/libgqmap_tl.so gpurun_out/tlbuild/ || exit 1
OUT=gpurun_out/r06_lag2w_ab.txt
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > $OUT 2>&1 || exit $?
GQMAP_ARITH=literal ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 >> $OUT 2>&1 || exit $?
for r in 1 2; do
  for v in base l4 l6; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 \
      | sed "s/^/$v r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
GQMAP_LIB=$PWD/gpurun_out/tlbuild/libgqmap_tl.so FLOW_TL_OUT=gpurun_out/flow_tl_2w.npz timeout -k 5 180 python3 scripts/flow_timeline.py \
  > gpurun_out/r06_flow_timeline_2w.txt 2>&1 || exit $?
rm -f gpurun_out/tlbuild/libgqmap_tl.so
echo "timeline ok"
