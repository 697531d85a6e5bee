# Time-limited GPU steps by name, for one gpurun call; each step's output goes
# to gpurun_out/steps/<name>.*, the chain stops at the first failing step.
#   bash scripts/gpu_steps.sh smoke tests bench20 bench
#   bash scripts/gpu_steps.sh tests:tests/test_gpu_tiles.py configs profile:c2:fp64:r05:200
# steps:
#   smoke                 __graft_entry__.smoke()
#   tests[:PATHS]         pytest -m gpu (default: tests/)
#   bench20 / bench       bench.py --steps 20 (the driver's window) / its defaults
#   configs               bench.py --config c1 c3 c4 c5 and c2 fp32, one line each
#   profile:CFG:PREC:TAG:STEPS   scripts/profile_round.sh (kernel trace + FETCH/WRITE passes)
#   trace20:TAG           rocprofv3 --kernel-trace --stats of bench.py --steps 20 + per-segment k_iter means
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/steps; mkdir -p $O
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  case $name in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    tests) timeout -k 10 900 python -u -m pytest ${arg:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 \
             --timeout-method thread > $O/tests.log 2>&1 ;;
    bench20) timeout -k 10 400 python bench.py --steps 20 > $O/bench20.json 2> $O/bench20.err ;;
    bench) timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err ;;
    configs) : > $O/configs.jsonl
      for c in c1 c3 c4 c5; do
        timeout -k 10 400 python bench.py --config $c >> $O/configs.jsonl 2>> $O/configs.err || break
      done && timeout -k 10 400 python bench.py --precision fp32 >> $O/configs.jsonl 2>> $O/configs.err ;;
    profile) IFS=: read -r CFG PREC TAG STEPS <<< "$arg"
      CFG=$CFG PREC=$PREC TAG=$TAG STEPS=$STEPS bash scripts/profile_round.sh > $O/profile_$CFG.log 2>&1 ;;
    trace20) d=gpurun_out/${arg:-rNN}prof; mkdir -p $d
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/bench20 -o run --output-format csv -- \
        python3 bench.py --steps 20 > $d/bench20.json 2> $d/bench20.err &&
      python3 scripts/trace_segments.py $d/bench20/run_kernel_trace.csv > $d/bench20_segments.txt ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  rc=$?; echo "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
