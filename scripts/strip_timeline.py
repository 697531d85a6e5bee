"""Per-iteration timeline of one rank's RCCL strip from a rocprofv3 kernel
trace of scripts/strip_time.py (rccl1 mode): for each k_unpack_advance, the
two k_iter launches before it -- start offsets, durations and the gaps
between them.  usage: strip_timeline.py run_kernel_trace.csv"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
it = []
for i, r in enumerate(rows):
    if "unpack_advance" not in r["Kernel_Name"] or i < 2:
        continue
    a, b = rows[i - 2], rows[i - 1]
    if "k_iter" not in a["Kernel_Name"] or "k_iter" not in b["Kernel_Name"]:
        continue
    nxt = next((x for x in rows[i + 1:] if "k_iter" in x["Kernel_Name"]), None)
    t = lambda x, k: int(x[k]) / 1000.0
    end2 = max(t(a, "End_Timestamp"), t(b, "End_Timestamp"))
    it.append(dict(k1=t(a, "End_Timestamp") - t(a, "Start_Timestamp"), k2=t(b, "End_Timestamp") - t(b, "Start_Timestamp"),
                   stagger=t(b, "Start_Timestamp") - t(a, "Start_Timestamp"), to_ua=t(r, "Start_Timestamp") - end2,
                   ua=t(r, "End_Timestamp") - t(r, "Start_Timestamp"),
                   ua_to_next=(t(nxt, "Start_Timestamp") - t(r, "End_Timestamp")) if nxt else float("nan"),
                   period=(t(nxt, "Start_Timestamp") - t(a, "Start_Timestamp")) if nxt else float("nan")))
print(f"{len(it)} iterations (medians, us)")
for k in ("k1", "k2", "stagger", "to_ua", "ua", "ua_to_next", "period"):
    v = [x[k] for x in it if x[k] == x[k]]
    print(f"  {k:11s} {statistics.median(v):7.2f}")
