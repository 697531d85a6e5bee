# Round 6: the C5 line with the dataflow launch (default) and with one launch
# per iteration (--policy flow=0), interleaved, 2 rounds.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_c5_ab.jsonl
: > $OUT
for r in 1 2; do
  for pol in "" "--policy flow=0"; do
    timeout -k 10 500 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-parity $pol > gpurun_out/r06_c5_run.txt 2>&1 || exit $?
    grep '^{' gpurun_out/r06_c5_run.txt >> $OUT
    echo "r$r $pol ok"
  done
done
