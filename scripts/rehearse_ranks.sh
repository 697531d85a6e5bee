# Multi-rank bench rehearsal on a one-GPU box: N ranks share cuda:0 through the
# gloo backend (GQMAP_BENCH_BACKEND=gloo), frame-parallel C2 and tiled C2
# (host-staged tiles are not used by bench; tiled RCCL needs one GPU per rank,
# so only the frame-parallel mode runs here).
set -u
mkdir -p gpurun_out
N=${N:-2}
GQMAP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/rehearse_c2_n$N.log 2>&1; rc=$?; echo "c2 n=$N rc=$rc"; tail -1 gpurun_out/rehearse_c2_n$N.log
exit $rc
