#!/bin/bash
# C5 HBM bytes: NT state stores (the library) vs + NT own-state loads (build/var/libgqmap_ntl.so);
# then C2 timing of both with the NT policy forced on (GQMAP_NT_STATE=1) and off.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c5b
for v in nts ntl; do
  lib=$PWD/gqmap-opticalflow_amd/libgqmap.so
  [ $v = ntl ] && lib=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_ntl.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    GQMAP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/r04c5b/${v}_$ctr -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r04c5b/${v}_$ctr.log 2>&1 || exit 1
  done
  GQMAP_LIB=$lib timeout -k 10 300 python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04c5b/${v}_time.jsonl 2>&1 || exit 2
done
for v in 0 1; do
  GQMAP_NT_STATE=$v timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 >> gpurun_out/r04c5b/c2_nt.txt 2>&1 || exit 3
  GQMAP_NT_STATE=$v GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_ntl.so timeout -k 10 120 python scripts/phase_time.py fp64 20 c2 >> gpurun_out/r04c5b/c2_nt.txt 2>&1 || exit 4
done
cat gpurun_out/r04c5b/c2_nt.txt
