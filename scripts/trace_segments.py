"""Per-segment k_iter durations of a rocprofv3 kernel trace of bench.py: the
launches between two k_init_state dispatches form one segment (warm-up,
clock-settle chunks, the timed steps, the instrumented replay, ...), so the
timed window's rocprofv3 mean can be set beside the line's HIP-event mean.
A dataflow segment (k_iter_flow: one dispatch per <= 50 iterations) is
reported as its total duration divided by the segment's iterations (--its,
the bench's steps; a segment of that many single-iteration dispatches counts
one per dispatch).
usage: trace_segments.py <run_kernel_trace.csv> [--its N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ITS = int(sys.argv[sys.argv.index("--its") + 1]) if "--its" in sys.argv else 20
segs, cur = [], []
for r in rows:
    n = r["Kernel_Name"]
    if "k_init_state" in n:
        segs.append(cur)
        cur = []
    elif "k_iter" in n:
        kind = "k_iter_lit" if "k_iter_lit" in n else "k_iter_flow" if "k_iter_flow" in n else "k_iter"
        cur.append((kind, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
segs.append(cur)
print(f"{'segment':>7s} {'kernel':>11s} {'launches':>8s} {'mean_us':>8s} {'min_us':>7s} {'max_us':>7s} "
      f"{'us/iteration':>12s}")
for i, s in enumerate(segs):
    if s:
        d = [x for _, x in s]
        its = len(d) if (s[0][0] != "k_iter_flow" or len(d) >= ITS) else ITS
        print(f"{i:7d} {s[0][0]:>11s} {len(d):8d} {sum(d) / len(d):8.1f} {min(d):7.1f} {max(d):7.1f} "
              f"{sum(d) / its:12.1f}")
