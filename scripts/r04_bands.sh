#!/bin/bash
# Banded pipeline: graph-capture smoke (runs of 1, 2, 4, 50 iterations), C2
# timing for B = 0 (one launch per iteration), 3, 4, 6, 8, then its
# bit-identity GPU tests.
set -u
mkdir -p gpurun_out
GQMAP_BANDS=4 timeout -k 10 120 python -X faulthandler scripts/bands_graph_diag.py > gpurun_out/bands_diag.txt 2>&1 || { cat gpurun_out/bands_diag.txt; exit 1; }
cat gpurun_out/bands_diag.txt
timeout -k 10 500 python -u scripts/bands_probe.py > gpurun_out/bands_probe.txt 2>&1 || { cat gpurun_out/bands_probe.txt; exit 2; }
cat gpurun_out/bands_probe.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k banded > gpurun_out/bands_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/bands_tests.txt
exit $rc
