# C4 super engine (fp64) with the lanes-per-node split forced (GQMAP_SPLIT), prof_iter.py: k_iter us/it.
set -u
mkdir -p gpurun_out
: > gpurun_out/super_split.log
for r in 1 2; do for q in 2 4; do
  GQMAP_SPLIT=$q timeout -k 10 120 python -u scripts/prof_iter.py 100 fp64 super | sed "s/^/r$r Q=$q /" >> gpurun_out/super_split.log 2>&1 || exit $?
done; done
cat gpurun_out/super_split.log
