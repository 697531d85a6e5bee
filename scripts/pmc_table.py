"""Per-launch k_iter averages of the counters collected by pmc_probe.sh."""
import csv
import glob
import os
import sys
from collections import defaultdict

out, variants = sys.argv[1], sys.argv[2:]
rows = {}
for v in variants:
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(out, f"{v}_p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_iter" not in r.get("Kernel_Name", ""):
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows[v] = {k: sum(x) / len(x) for k, x in acc.items()}
names = sorted({k for r in rows.values() for k in r})
print("counter".ljust(40) + "".join(v.rjust(16) for v in variants))
for n in names:
    print(n.ljust(40) + "".join(f"{rows[v].get(n, float('nan')):16.4g}" for v in variants))
