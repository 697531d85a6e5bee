# Interleaved A/B of LLVM scheduler variants (build/var/libgqmap_*.so): C2 fp64/fp32 and the C3 full level.
set -u
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 900 python -u scripts/variants.py 100 fp64,fp32 > gpurun_out/sched_c2.log 2>&1 || exit $?
cat gpurun_out/sched_c2.log
SCALES=1.0,0.5 bash scripts/ctf_level_ab.sh
