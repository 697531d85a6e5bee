# Round 6 (late): claim prefetch (pf) and claim-with-ticket (pair) on the
# 2-wave dataflow launch against the build (base): C2 fp64 fast and literal
# (variants.py, 200 its, 3 rounds) and the ctf levels.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_pf2w_ab.txt
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > $OUT 2>&1 || exit $?
GQMAP_ARITH=literal ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 >> $OUT 2>&1 || exit $?
for r in 1 2; do
  for v in base pf pair; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 \
      | sed "s/^/$v r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
