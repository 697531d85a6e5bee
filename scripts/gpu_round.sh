set -u
bash scripts/gpu_check.sh || exit $?
CFG=c2 PREC=fp64 TAG=r02 STEPS=200 bash scripts/profile_round.sh
