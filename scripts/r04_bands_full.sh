#!/bin/bash
# The -m gpu suite on the current tree, then the banded-pipeline checks.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_suite3.txt 2>&1 || { tail -30 gpurun_out/r04_suite3.txt; exit 1; }
tail -2 gpurun_out/r04_suite3.txt
bash scripts/r04_bands.sh
