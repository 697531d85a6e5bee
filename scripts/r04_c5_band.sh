#!/bin/bash
# C5 with the row-by-row band walk off (GQMAP_BAND_ROWS=0) and as built (on
# for C5's frames): rocprofv3 FETCH_SIZE pass and timing of bench.py --config
# c5, interleaved twice; then the GPU tests of the walk's bit-identity.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04band
for r in 1 2; do
for v in off on; do
  e="GQMAP_BAND_ROWS=1"; [ $v = off ] && e="GQMAP_BAND_ROWS=0"
  if [ $r = 1 ]; then
    env $e timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r04band/${v}_FETCH_SIZE -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r04band/${v}_FETCH_SIZE.log 2>&1 || exit 1
  fi
  env $e timeout -k 10 300 python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04band/${v}_time_r$r.jsonl 2>&1 || exit 2
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "band_row or nontemporal" > gpurun_out/r04band/test.txt 2>&1
rc=$?
tail -2 gpurun_out/r04band/test.txt
exit $rc
