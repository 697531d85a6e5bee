# A/B of the LDS-parking variants (GQ_PARK) on C2 (fp64, fp32) and C3.
set -u
L=$PWD/gqmap-opticalflow_amd/build/var
for r in 1 2; do
  for v in cur park park4; do
    GQMAP_LIB=$L/libgqmap_$v.so timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 || exit 1
    GQMAP_LIB=$L/libgqmap_$v.so timeout -k 10 120 python scripts/phase_time.py fp32 20 c2 || exit 1
  done
done
for v in cur park; do
  echo "c3 $v"; GQMAP_LIB=$L/libgqmap_$v.so timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline | grep -o '"value": [0-9.]*' || exit 1
done
