# Literal-order engine (C2 fp64, scripts/prof_iter.py 200): the library's
# IEEE division sequence against div_rcp's reciprocal + two corrections
# (variant build mdiv: -DGQ_LIT_MDIV=1), interleaved, 3 rounds; then the
# literal GPU tests (bit-exact against the restatement) on the variant.
set -u
V=$PWD/gqmap-opticalflow_amd/build/var
for r in 1 2 3; do
  for lib in base mdiv; do
    GQMAP_LIB=$V/libgqmap_$lib.so GQMAP_ARITH=literal timeout -k 5 120 python3 scripts/prof_iter.py 200 fp64 | sed "s/^/$lib r$r /" || exit 1
  done
done
GQMAP_LIB=$V/libgqmap_mdiv.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_literal.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
