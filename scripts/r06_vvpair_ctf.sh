# Round 6 (late): the column-pair store on the ctf levels at one lane per
# node (C3's 480x640 level: integer frames) -- the whole GPU suite, the
# 480x640 level with vv_pair=0 / 1 (3 interleaved rounds, same checksum
# expected), then the C3 line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r06_gpu_suite_vvctf.txt 2>&1 || exit $?
echo "suite ok"
OUT=gpurun_out/r06_vvpair_ctf_ab.txt
: > $OUT
for r in 1 2 3; do
  for pol in vv_pair=0 vv_pair=1; do
    GQMAP_POLICY=$pol timeout -k 5 200 python3 scripts/ctf_level_ab.py fp64 1 | sed "s/^/$pol r$r /" >> $OUT || exit $?
  done
done
echo "ab ok"
for pol in vv_pair=0 vv_pair=1; do
  timeout -k 10 600 python -u bench.py --config c3 --policy $pol > gpurun_out/r06_c3_$pol.txt 2>&1 || exit $?
done
echo "c3 ok"
