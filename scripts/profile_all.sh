# Round profile of the measured configs: rocprofv3 kernel trace + stats and
# FETCH_SIZE / WRITE_SIZE passes (scripts/profile_round.sh) per config.
set -u
TAG=${TAG:-r02}
for spec in "c2 fp64 200" "c2 fp32 200" "c4 fp64 100" "c5 fp64 20" "c3 fp64 100"; do
  set -- $spec
  CFG=$1 PREC=$2 STEPS=$3 TAG=$TAG bash scripts/profile_round.sh || exit $?
done
