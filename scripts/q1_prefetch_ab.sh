# Interleaved A/B of edge-job prefetch / unroll on the Q=1 kernels: C2 (variants.py) and the C3 full level.
set -u
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 100 fp64,fp32 > gpurun_out/q1pf_c2.log 2>&1 || exit $?
cat gpurun_out/q1pf_c2.log
SCALES=1.0 bash scripts/ctf_level_ab.sh
