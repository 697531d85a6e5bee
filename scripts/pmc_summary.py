"""Summarise a profile_round.sh run into profiles/:
  profiles/<tag>_<cfg>_<prec>_kernel_stats.csv   rocprofv3 --stats table (copied)
  profiles/<tag>_<cfg>_<prec>_summary.txt        per-kernel avg duration, FETCH/WRITE per dispatch
  profiles/traffic_<cfg>_<prec>.json             corrected HBM bytes per k_iter launch (bench.py)
FETCH_SIZE is scaled by the factor measured on the calibration kernels for
the same access width (8-B lanes for fp64 state, 4-B for fp32) against their
known byte counts; WRITE_SIZE likewise.
usage: python3 scripts/pmc_summary.py gpurun_out/<tag> <cfg> <prec>"""
import csv
import json
import re
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# iterations per k_iter_flow dispatch in the profiled run (FLOW_ITS=50 with
# scripts/prof_iter.py and a multiple of 50 iterations; 0: not a flow profile)
FLOW_ITS = int(os.environ.get("FLOW_ITS", "0"))


def rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def find(d, name):
    for dp, _, fs in os.walk(d):
        for f in fs:
            if f.endswith(name):
                return os.path.join(dp, f)
    return None


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in rows(path):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    base, cfg, prec = sys.argv[1], sys.argv[2], sys.argv[3]
    tag = os.path.basename(base.rstrip("/"))
    d = os.path.join(base, f"{cfg}_{prec}")
    stats = find(os.path.join(d, "trace"), "kernel_stats.csv")
    fetch = per_kernel(find(os.path.join(d, "fetch"), "counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(find(os.path.join(d, "write"), "counter_collection.csv"), "WRITE_SIZE")
    cal_f = per_kernel(find(os.path.join(base, "calib_fetch"), "counter_collection.csv"), "FETCH_SIZE")
    cal_w = per_kernel(find(os.path.join(base, "calib_write"), "counter_collection.csv"), "WRITE_SIZE")
    GiB = float(1 << 30)
    width = "double" if prec == "fp64" else "float"
    pick = lambda tab, kind: next((v for k, v in tab.items() if kind in k and width in k), None)
    f_read = pick(cal_f, "k_read")    # FETCH_SIZE units are KB (rocprofv3 derived counter)
    f_write = pick(cal_w, "k_write")
    fcorr = GiB / (f_read * 1024) if f_read else None
    wcorr = GiB / (f_write * 1024) if f_write else None
    out_stats = os.path.join(ROOT, "profiles", f"{tag}_{cfg}_{prec}_kernel_stats.csv")
    shutil.copy(stats, out_stats)
    lines = [f"profile {tag} config {cfg} precision {prec} (bench.py --warmup 5 under rocprofv3; steps in the .log)",
             f"calibration ({width} lanes, 1 GiB): FETCH_SIZE x{fcorr:.3f}, WRITE_SIZE x{wcorr:.3f}"
             if fcorr and wcorr else "calibration: missing", ""]
    lines.append(f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'FETCH_KB':>12s} {'WRITE_KB':>12s} {'HBM_MB(corr)':>13s}")
    traffic = None
    for r in rows(stats):
        name = r["Name"]
        f = fetch.get(name)
        w = write.get(name)
        corr = (f * 1024 * fcorr + w * 1024 * wcorr) if (f is not None and w is not None and fcorr) else None
        lines.append(f"{name[:70]:70s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:10.2f} "
                     f"{f if f is not None else float('nan'):12.1f} {w if w is not None else float('nan'):12.1f} "
                     f"{(corr or float('nan')) / 1e6:13.3f}")
        if cfg != "c1" and "k_iter_flow" in name and corr is not None and FLOW_ITS:
            # the dataflow launch runs FLOW_ITS iterations per dispatch in the
            # profiled driver (scripts/prof_iter.py with a multiple of 50):
            # per-iteration figures, comparable with a per-launch k_iter's
            # (durations: the stats come from the bench trace, whose dispatches
            # run different iteration counts -- per-iteration times are in the
            # trace_segments.py table instead)
            traffic = dict(kernel=name, iterations_per_launch=FLOW_ITS, avg_us=None, fetch_kb=f / FLOW_ITS,
                           write_kb=w / FLOW_ITS, fetch_corr=fcorr, write_corr=wcorr,
                           hbm_bytes_per_launch=corr / FLOW_ITS, unit="HBM bytes per iteration",
                           source=f"profiles/{tag}_{cfg}_{prec}_summary.txt")
            lines.append(f"  -> counters per iteration ({FLOW_ITS} iterations per dispatch in the counter passes): "
                         f"FETCH {f / FLOW_ITS:.1f} KB, WRITE {w / FLOW_ITS:.1f} KB, HBM {corr / FLOW_ITS / 1e6:.3f} MB "
                         f"(the avg_us column: the bench trace's dispatches, of mixed iteration counts)")
        elif cfg != "c1" and "k_iter" in name and "k_iter_flow" not in name and traffic is None and corr is not None:
            traffic = dict(kernel=name, avg_us=float(r["AverageNs"]) / 1e3, fetch_kb=f, write_kb=w,
                           fetch_corr=fcorr, write_corr=wcorr, hbm_bytes_per_launch=corr,
                           source=f"profiles/{tag}_{cfg}_{prec}_summary.txt")
        if cfg == "c1" and "k_legacy" in name and "sigma0" not in name and corr is not None:
            # C1: one iteration = k_legacy_grad + k_legacy_update + k_legacy_ctl
            if traffic is None:
                traffic = dict(kernel="k_legacy_grad + k_legacy_update + k_legacy_ctl (bytes per iteration)",
                               avg_us=0.0, fetch_corr=fcorr, write_corr=wcorr, hbm_bytes_per_launch=0.0,
                               per_kernel={}, source=f"profiles/{tag}_{cfg}_{prec}_summary.txt")
            traffic["avg_us"] += float(r["AverageNs"]) / 1e3
            traffic["hbm_bytes_per_launch"] += corr
            traffic["per_kernel"][re.search(r"k_legacy_\w+", name).group(0)] = corr
    txt = "\n".join(lines) + "\n"
    open(os.path.join(ROOT, "profiles", f"{tag}_{cfg}_{prec}_summary.txt"), "w").write(txt)
    if traffic:
        json.dump(traffic, open(os.path.join(ROOT, "profiles", f"traffic_{cfg}_{prec}.json"), "w"), indent=1)
    print(txt)


if __name__ == "__main__":
    main()
