# Round 6 (late): the literal-order engine per launch (flow=0) against the
# dataflow launch (flow=1, forced) after the mirror / clamp changes -- C2
# fp64 arith=literal, 200 iterations, 3 interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_lit_flow_ab2.txt
: > $OUT
for r in 1 2 3; do
  for pol in flow=0 flow=1; do
    GQMAP_ARITH=literal GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
