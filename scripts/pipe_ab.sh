# software-pipelined node gathers in the fp64 single-scale loop (variant removed after this A/B,
# (GQ_NODE_PIPE=1: next point's 16 taps loaded before the current bicubic)
# vs the plain loop; the pipelined C2 kernel needs 182 VGPRs (2 waves/SIMD).
set -u
for r in 1 2; do
  for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
    GQMAP_LIB=$PWD/$lib timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 || exit 1
  done
done
