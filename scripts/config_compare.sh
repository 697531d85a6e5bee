# bench.py on every config for the variant libraries in $VARS (no CPU
# baseline): one JSON line each, prefixed with the variant name.
set -u
mkdir -p gpurun_out
for v in ${VARS:-cur}; do
  for c in ${CFGS:-c2 c3 c4 c5}; do
    GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_$v.so timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --warmup 5 > gpurun_out/cmp_${v}_$c.json 2> gpurun_out/cmp_${v}_$c.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/cmp_${v}_$c.json')); print('$v', '$c', round(d['value'],4), d['unit'], 'aepe', round(d['aepe'],4), 'frac', round(d['roofline']['frac'],3))"
  done
done
