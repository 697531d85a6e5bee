# fp32 C2 with the lanes-per-node split forced (GQMAP_SPLIT), prof_iter.py: k_iter us/it.
set -u
mkdir -p gpurun_out
for q in 1 2 4; do
  GQMAP_SPLIT=$q timeout -k 10 120 python -u scripts/prof_iter.py 100 fp32 | sed "s/^/fp32 Q=$q /" >> gpurun_out/fp32_split.log 2>&1 || exit $?
done
cat gpurun_out/fp32_split.log
