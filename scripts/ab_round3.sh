set -u
mkdir -p gpurun_out
SCALES=0.0625,0.125,0.25,0.5,1.0 bash scripts/ctf_level_ab.sh > gpurun_out/ab1.log 2>&1 || exit 1
ROUNDS=3 timeout -k 10 300 python scripts/variants.py 100 fp64 > gpurun_out/ab2.log 2>&1 || exit 2
QS=16,64 timeout -k 10 200 python -u scripts/level_sweep.py fp64 > gpurun_out/ab3.log 2>&1 || exit 3
GQMAP_SPLIT=64 TL_CFGS="ctf:0.0625" bash scripts/tl_levels.sh > gpurun_out/ab4.log 2>&1 || exit 4
