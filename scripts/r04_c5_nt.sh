#!/bin/bash
# C5 HBM bytes with and without non-temporal state stores (build/var/libgqmap_nts.so):
# rocprofv3 FETCH_SIZE and WRITE_SIZE passes of bench.py --config c5 --steps 10, then timing.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c5
for v in base nts; do
  lib=$PWD/gqmap-opticalflow_amd/libgqmap.so
  [ $v = nts ] && lib=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_nts.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    GQMAP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/r04c5/${v}_$ctr -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r04c5/${v}_$ctr.log 2>&1 || exit 1
  done
  GQMAP_LIB=$lib timeout -k 10 300 python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04c5/${v}_time.jsonl 2>&1 || exit 2
done
echo done
