# C5 (the eight pairs upsampled 4x, bench.py --config c5, no CPU baseline / parity
# legs) for the library variants in gqmap-opticalflow_amd/build/var (VARS), 2 rounds.
set -u
V=$PWD/gqmap-opticalflow_amd/build/var
for r in 1 2; do
  for lib in ${VARS:-base}; do
    GQMAP_LIB=$V/libgqmap_$lib.so timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-parity \
      > gpurun_out/c5_$lib.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/c5_$lib.json').read().strip().splitlines()[-1]); print('$lib r$r', round(d['value'], 4), round(d['ms_per_step'], 3), round(d['roofline']['frac'], 4))"
  done
done
