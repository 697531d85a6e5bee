# Round 6: the dataflow launch's item timeline with the wait attributed to
# the dependency that released it (scripts/flow_timeline.py; GQ_FLOW_TL=1
# build in build/var; raw data -> gpurun_out/flow_tl.npz).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GQMAP_LIB=$PWD/gqmap-opticalflow_amd/build/var/libgqmap_tl.so timeout -k 5 180 python3 scripts/flow_timeline.py \
  > gpurun_out/r06_flow_timeline2.txt 2>&1 || exit $?
echo "timeline ok"
