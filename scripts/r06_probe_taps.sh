# Round 6 (late) timing probes (GQ_PROBE_HALF_TAPS, GQ_PROBE_H2): the fast kernels with half the tap-column
# loads (GQ_PROBE_HALF_TAPS: columns 2, 3 re-read 0, 1 -- wrong values,
# timing only) against the build -- is the node loop bound by its gathers?
# C2 fp64, 200 its, 3 rounds (variants.py; the checksums differ by design).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 600 python -u scripts/variants.py 200 fp64 > gpurun_out/${OUTF:-r06_probe_taps.txt} 2>&1 || exit $?
echo "ok"
