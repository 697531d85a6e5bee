#!/bin/bash
# The banded-pipeline checks, then the rest of the -m gpu suite.
set -u
mkdir -p gpurun_out
bash scripts/r04_bands.sh || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_suite3.txt 2>&1 || { tail -30 gpurun_out/r04_suite3.txt; exit 1; }
tail -2 gpurun_out/r04_suite3.txt
