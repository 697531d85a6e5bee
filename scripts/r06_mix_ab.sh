# Round 6 (late), 2-wave dataflow launches: the node-first / edge-first
# alternation off (mix0) and on for the literal kernel too (litmix) against
# the build (base) -- C2 fp64 fast and literal (variants.py, 200 its, 3
# rounds); then fp32 C2 per launch vs as items on the build (flow=0/1).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_mix_ab.txt
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > $OUT 2>&1 || exit $?
GQMAP_ARITH=literal ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 >> $OUT 2>&1 || exit $?
echo "c2 ok"
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp32 | sed "s/^/fp32 $pol r$r /" >> $OUT || exit $?
  done
done
echo "fp32 ok"
