# Interleaved A/B of build/var/libgqmap_*.so on the C3 levels (scripts/ctf_level_ab.py).
set -u
mkdir -p gpurun_out
: > gpurun_out/ctf_ab.log
for r in 1 2 3; do
  for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
    n=$(basename $lib .so); n=${n#libgqmap_}
    GQMAP_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/ctf_level_ab.py fp64 ${SCALES:-0.5,0.25} | sed "s/^/$n r$r /" >> gpurun_out/ctf_ab.log || exit $?
  done
done
cat gpurun_out/ctf_ab.log
