#!/bin/bash
# Round-4 end-of-session check: the -m gpu suite, smoke, and a bench line for
# every config (fp64; C2 also fp32) into gpurun_out/r04_final2.jsonl.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_final2_tests.txt 2>&1 || { tail -30 gpurun_out/r04_final2_tests.txt; exit 1; }
tail -2 gpurun_out/r04_final2_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final2_smoke.txt 2>&1 || exit 2
cat gpurun_out/r04_final2_smoke.txt
out=gpurun_out/r04_final2.jsonl
: > $out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $out 2>> gpurun_out/r04_final2.err || exit 3
timeout -k 10 300 python bench.py >> $out 2>> gpurun_out/r04_final2.err || exit 4
timeout -k 10 300 python bench.py --precision fp32 --no-cpu-baseline >> $out 2>> gpurun_out/r04_final2.err || exit 5
timeout -k 10 300 python bench.py --config c1 >> $out 2>> gpurun_out/r04_final2.err || exit 6
timeout -k 10 400 python bench.py --config c4 >> $out 2>> gpurun_out/r04_final2.err || exit 7
timeout -k 10 300 python bench.py --config c3 >> $out 2>> gpurun_out/r04_final2.err || exit 8
timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline >> $out 2>> gpurun_out/r04_final2.err || exit 9
echo done
