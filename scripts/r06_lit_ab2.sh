# Round 6: literal-engine variants (build/var): bare v_min/v_max clamp (mm),
# column-stride tap addresses (ad), both (mmad), node loop unrolled 2 / 3
# (u2, u3; with mm + ad) against neither (b0) -- C2 fp64 arith=literal, 200
# iterations, interleaved rounds (scripts/variants.py; chk = state checksum).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GQMAP_ARITH=literal ROUNDS=${ROUNDS:-3} timeout -k 10 600 python -u scripts/variants.py 200 fp64 > gpurun_out/r06_lit_ab2.txt 2>&1 || exit $?
echo "ab ok"
