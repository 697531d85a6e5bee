# Round 6 (late): 2 waves per SIMD for the dataflow launch.  build/var:
# base (literal flow at 2 waves, the default now), fw2 (the fast C2 / ctf
# flow kernels at 2 waves too), lm / lx / lu2 (literal node-loop mirror,
# XJ prefetch, unroll 2 -- with the 2-wave register budget).  C2 fp64 fast
# and literal (variants.py, 200 its, 3 rounds), the ctf 480x640 / 240x320
# levels for base and fw2.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_w2_ab.txt
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > $OUT 2>&1 || exit $?
GQMAP_ARITH=literal ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 >> $OUT 2>&1 || exit $?
echo "c2 ok"
for r in 1 2; do
  for v in base fw2; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 \
      | sed "s/^/$v r$r /" >> $OUT || exit $?
  done
done
echo "ctf ok"
