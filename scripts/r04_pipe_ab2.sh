# A/B of the software-pipelined ctf node loop at Q = 2 (the 240x320 level, taps
# stored as double: resampled frames), then the ctf GPU tests on the default build.
set -u
mkdir -p gpurun_out
SCALES=0.5 timeout -k 10 400 bash scripts/ctf_level_ab.sh > gpurun_out/pipe_ab2.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ctf or pyramid or persist" > gpurun_out/pipe_tests2.txt 2>&1
rc=$?
tail -3 gpurun_out/pipe_tests2.txt
exit $rc
