# A/B of the software-pipelined ctf node loop (GQ_CTF_PIPE_MIN_Q) on the C3
# middle levels (240x320 at Q = 2, 120x160 at Q = 4), then the GPU suite on
# the default build.
set -u
mkdir -p gpurun_out
SCALES=0.5,0.25,1.0 timeout -k 10 400 bash scripts/ctf_level_ab.sh > gpurun_out/pipe_ab.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/pipe_tests.txt
exit $rc
