set -u
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "prepared or graph_replay or stop_inside" > gpurun_out/ab/tests.log 2>&1; rc=$?; echo tests=$rc; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab/tests.log; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab/c2_$i.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --precision fp32 > gpurun_out/ab/c2f_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --config c4 > gpurun_out/ab/c4.log 2>&1 || exit 1
echo done
