# Interleaved A/B of build/var/libgqmap_*.so on the C4 super engine (fp64, variants.py).
set -u
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 900 python -u scripts/variants.py 100 fp64 super > gpurun_out/super_sched.log 2>&1 || exit $?
cat gpurun_out/super_sched.log
