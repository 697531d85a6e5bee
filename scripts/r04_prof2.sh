#!/bin/bash
# Round-4 profiles after the band walk: rocprofv3 stats + FETCH/WRITE passes of
# C5 (100 steps, the bench default), C3 and C4 (fp64).
set -u
CFG=c5 PREC=fp64 TAG=r04 STEPS=100 bash scripts/profile_round.sh || exit 1
CFG=c3 PREC=fp64 TAG=r04 STEPS=500 bash scripts/profile_round.sh || exit 2
CFG=c4 PREC=fp64 TAG=r04 STEPS=200 bash scripts/profile_round.sh || exit 3
echo done
