#!/bin/bash
# C5 HBM bytes and time: the library (NT state stores) vs + NT own-state loads (build/var/libgqmap_ntown.so)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c5d
for v in lib ntown; do
  lib=$PWD/gqmap-opticalflow_amd/libgqmap.so
  [ $v = ntown ] && lib=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_ntown.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    GQMAP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/r04c5d/${v}_$ctr -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r04c5d/${v}_$ctr.log 2>&1 || exit 1
  done
  GQMAP_LIB=$lib timeout -k 10 300 python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04c5d/${v}_time.jsonl 2>&1 || exit 2
done
echo done
