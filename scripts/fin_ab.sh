# A/B of the fused finalize reduction (GQ_FIN_GROUP) on C2; also the unfused form.
set -u
L=$PWD/gqmap-opticalflow_amd/build/var
for r in 1 2; do
  for v in cur fing; do
    GQMAP_LIB=$L/libgqmap_$v.so timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 || exit 1
    GQMAP_LIB=$L/libgqmap_$v.so timeout -k 10 120 python scripts/phase_time.py fp32 20 c2 || exit 1
  done
  echo unfused; GQMAP_NO_FUSED_FINALIZE=1 GQMAP_LIB=$L/libgqmap_cur.so timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 || exit 1
done
