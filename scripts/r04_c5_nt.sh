#!/bin/bash
# C5 HBM bytes with the state_nt policy off (GQMAP_NT_STATE=0) and as built
# (non-temporal state stores for C5's frames): rocprofv3 FETCH_SIZE and
# WRITE_SIZE passes of bench.py --config c5 --steps 10, then timing; then the
# GPU test of the policy's bit-identity.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c5c
for v in off on; do
  e=""; [ $v = off ] && e="GQMAP_NT_STATE=0"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env $e timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/r04c5c/${v}_$ctr -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r04c5c/${v}_$ctr.log 2>&1 || exit 1
  done
  env $e timeout -k 10 300 python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04c5c/${v}_time.jsonl 2>&1 || exit 2
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "nontemporal" > gpurun_out/r04c5c/test.txt 2>&1
tail -2 gpurun_out/r04c5c/test.txt
