# Q=2 / 3-wave-bound experiment: interleaved A/B of the build/var libraries,
# C2 with two lanes per node on each, and the C3 per-level Q sweep.
set -u
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 100 fp64,fp32 > gpurun_out/q2_variants.log 2>&1 || exit $?
cat gpurun_out/q2_variants.log
for v in base w3; do
  for q in 1 2; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so GQMAP_SPLIT=$q timeout -k 10 120 python -u scripts/prof_iter.py 100 fp64 | sed "s/^/$v Q=$q /" || exit $?
  done
done
GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_w3.so timeout -k 10 300 python -u scripts/level_sweep.py fp64 | sed "s/^/w3 /" || exit $?
GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_base.so timeout -k 10 300 python -u scripts/level_sweep.py fp64 | sed "s/^/base /" || exit $?
