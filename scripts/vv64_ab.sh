# VV stored as double (GQMAP_VV64=1: no per-tap f32->f64 conversion, 2x gather
# bytes) vs float (default) on C4 and C2; C4 at Q = 4 and 8.
set -u
for r in 1 2; do
  timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 | sed 's/^/vv32 /' || exit 1
  GQMAP_VV64=1 timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 | sed 's/^/vv64 /' || exit 1
  GQMAP_SPLIT=8 timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 | sed 's/^/vv32 /' || exit 1
  timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 | sed 's/^/vv32 /' || exit 1
  GQMAP_VV64=1 timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 | sed 's/^/vv64 /' || exit 1
done
