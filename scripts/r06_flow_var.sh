# Round 6: variants of the dataflow kernel (build/var, GQ_FLOW_* flags) with
# policy flow=1, interleaved (scripts/variants.py), then the per-launch path
# (flow=0) on the first variant's library for reference.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/r06_flow_var.txt
GQMAP_POLICY=flow=1 ROUNDS=${ROUNDS:-3} timeout -k 10 900 python3 -u scripts/variants.py ${ITS:-200} ${PRECS:-fp64,fp32} > $OUT 2>&1 || exit $?
BASE=$(ls gqmap-opticalflow_amd/build/var/libgqmap_*.so | head -1)
for r in 1 2 3; do
  for prec in $(echo ${PRECS:-fp64,fp32} | tr ',' ' '); do
    GQMAP_LIB=$BASE GQMAP_POLICY=flow=0 timeout -k 5 120 python3 scripts/prof_iter.py ${ITS:-200} $prec | sed "s/^/per-launch r$r /" >> $OUT || exit $?
  done
done
echo "var ok"
