# Round 6: how much the co-resident tile grouping (policy cu_group: the
# workgroups that start on one CU take vertically adjacent tiles) is worth
# on the per-launch path -- C2 fp64 (prof_iter.py) and the ctf levels
# (ctf_level_ab.py) with cu_group=0 against the default, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_cugroup_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in cu_group=-1 cu_group=0; do
    GQMAP_POLICY=$pol timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$pol r$r /" >> $OUT || exit $?
    GQMAP_POLICY=$pol timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1,0.5 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "cugroup ok"
