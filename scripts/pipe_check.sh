# Pipelined vs per-iteration kernel on C2 (phase timings), then the GPU check.
set -u
mkdir -p gpurun_out
GQMAP_PIPE=1 timeout -k 10 90 python scripts/phase_time.py fp64 20 || exit $?
GQMAP_PIPE=0 timeout -k 10 90 python scripts/phase_time.py fp64 20 || exit $?
GQMAP_PIPE=1 timeout -k 10 90 python scripts/phase_time.py fp32 20 || exit $?
GQMAP_PIPE=0 timeout -k 10 90 python scripts/phase_time.py fp32 20 || exit $?
bash scripts/gpu_check.sh
