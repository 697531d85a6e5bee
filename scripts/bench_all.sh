# End-of-round bench lines for every config (default steps), fp64 and the fp32 headline.
set -u
mkdir -p gpurun_out/bench_all
for c in c2 c1 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_all/$c.log 2>&1 || { echo "$c failed"; exit 1; }
  echo "$c done"
done
timeout -k 10 300 python bench.py --config c2 --precision fp32 > gpurun_out/bench_all/c2_fp32.log 2>&1 || exit 1
echo all done
