# Round 6 (late): the fast dataflow kernels at 2 waves per SIMD (fw2,
# GQ_FLOW_WAVES=2) against 3 (base): C2 fp64 (variants.py, 200 its, 5
# rounds) and the ctf 480x640 / 240x320 levels (3 rounds).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_fw2_ab.txt
ROUNDS=5 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > $OUT 2>&1 || exit $?
echo "c2 ok"
for r in 1 2 3; do
  for v in base fw2; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 \
      | sed "s/^/$v r$r /" >> $OUT || exit $?
  done
done
echo "ctf ok"
