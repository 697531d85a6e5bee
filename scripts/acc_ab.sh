# A/B of the atomic limb-sum finalize (default) against the row reduction
# (GQMAP_NO_ATOMIC_SUMS=1) on C2, both dtypes; then the round GPU check.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for dt in fp64 fp32; do
    echo "atomic $dt"; timeout -k 10 120 python scripts/phase_time.py $dt 20 c2 || exit 1
    echo "rows $dt"; GQMAP_NO_ATOMIC_SUMS=1 timeout -k 10 120 python scripts/phase_time.py $dt 20 c2 || exit 1
  done
done
