# strip_time.py (rccl1 = one-rank RCCL tile) for each build/var/libgqmap_*.so
set -u
timeout -k 10 200 python -u -m pytest tests/test_gpu_tiles.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tiles3.log 2>&1; echo tiles=$?; tail -1 gpurun_out/tiles3.log
for r in 1 2; do
  for lib in gqmap-opticalflow_amd/build/var/libgqmap_*.so; do
    n=$(basename $lib .so); n=${n#libgqmap_}
    for s in 8 2; do
      GQMAP_LIB=$PWD/$lib timeout -k 10 120 python scripts/strip_time.py $s 200 2>/dev/null | grep rccl1 | sed "s/^/$n /" || exit 1
    done
  done
done
