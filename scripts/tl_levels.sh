# Per-phase k_iter timelines (scripts/timeline.py) of the C3 levels and C2
# from the GQ_TIMELINE=20 build: make -C gqmap-opticalflow_amd variants VARS="tl:-DGQ_TIMELINE=20"; mv build/var/libgqmap_tl.so build/tl/
set -e
L=${TL_LIB:-$PWD/gqmap-opticalflow_amd/build/tl/libgqmap_tl.so}
for c in ${TL_CFGS:-ctf:0.0625 ctf:0.125 ctf:0.25 ctf:0.5 c2}; do
  GQMAP_LIB=$L timeout -k 10 120 python -u scripts/timeline.py ${TL_PREC:-fp64} $c
done
