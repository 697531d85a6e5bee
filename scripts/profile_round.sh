# Round profile of one bench configuration: rocprofv3 kernel trace + stats,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md
# HBM section), plus the FETCH/WRITE calibration micro-kernels; summarised by
# scripts/pmc_summary.py into profiles/.
# usage (GPU box): CFG=c2 PREC=fp64 TAG=r01 bash scripts/profile_round.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-c2}; PREC=${PREC:-fp64}; TAG=${TAG:-r01}; STEPS=${STEPS:-200}
OUT=gpurun_out/$TAG/${CFG}_${PREC}
mkdir -p $OUT
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- \
    python3 bench.py --config $CFG --precision $PREC --steps $STEPS --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/$name.log 2>&1
  local rc=$?; echo "$name=$rc"
  return $rc
}
run trace --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
if [ ! -f gpurun_out/$TAG/calib_fetch/run_counter_collection.csv ]; then
  [ -x scripts/micro/fetch_calib ] || hipcc --offload-arch=gfx950 -O2 scripts/micro/fetch_calib.hip -o scripts/micro/fetch_calib || exit $?
  for ctr in FETCH_SIZE WRITE_SIZE; do
    low=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
    timeout -k 10 120 rocprofv3 --pmc $ctr -d gpurun_out/$TAG/calib_$low -o run --output-format csv -- \
      scripts/micro/fetch_calib > gpurun_out/$TAG/calib_$low.log 2>&1 || exit $?
  done
fi
python3 scripts/pmc_summary.py gpurun_out/$TAG $CFG $PREC
