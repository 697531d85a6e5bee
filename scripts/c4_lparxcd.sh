# C4: a tile's L components on one XCD back to back (default) vs component-major
# (GQMAP_NO_LPAR_XCD=1): k_iter time and FETCH_SIZE per launch
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lx
for r in 1 2; do
  timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 | sed 's/^/xcd /' || exit 1
  GQMAP_NO_LPAR_XCD=1 timeout -k 10 120 python scripts/phase_time.py fp64 20 c4 | sed 's/^/cmaj /' || exit 1
done
for v in xcd cmaj; do
  if [ $v = cmaj ]; then export GQMAP_NO_LPAR_XCD=1; else unset GQMAP_NO_LPAR_XCD; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/lx/f_$v -o run --output-format csv -- python3 scripts/phase_time.py fp64 5 c4 > gpurun_out/lx/f_$v.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/lx/w_$v -o run --output-format csv -- python3 scripts/phase_time.py fp64 5 c4 > gpurun_out/lx/w_$v.log 2>&1 || exit 3
done
python3 - <<'PY'
import csv, glob, statistics
for v in ("xcd", "cmaj"):
    for c in ("f", "w"):
        f = glob.glob(f"gpurun_out/lx/{c}_{v}/**/*counter_collection.csv", recursive=True)[0]
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_iter" in r["Kernel_Name"]]
        print(v, c, len(vals), "median KB", statistics.median(vals))
PY
