#!/usr/bin/env python3
"""Summarise a scripts/gpu_profile.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>/.

Writes kernel_stats.csv (rocprofv3 --stats), kernel_gaps.txt (step-kernel launch cadence from the
kernel trace) and one pmc_<pass>_zb_step_kernel.csv per PMC pass with the per-dispatch mean of
each counter over the zb_step_kernel dispatches (FETCH_SIZE / WRITE_SIZE are KiB per dispatch).
Usage: python scripts/prof_summary.py <tag>
"""
import csv
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = os.environ.get("KERNEL", "zb_step_kernel")


def main(tag: str) -> None:
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    trace = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        rows = [r for r in csv.DictReader(open(trace)) if KERNEL in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        per = [(int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
        with open(os.path.join(dst, "kernel_gaps.txt"), "w") as f:
            f.write(f"{KERNEL}: {len(rows)} dispatches, grid {rows[0]['Grid_Size_X']} x wg {rows[0]['Workgroup_Size_X']}\n")
            f.write(f"duration us: median {statistics.median(dur):.2f} mean {statistics.mean(dur):.2f}\n")
            f.write(f"start-to-start us: median {statistics.median(per):.2f} mean {statistics.mean(per):.2f}\n")
    for d in sorted(os.listdir(src)):
        path = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc_") or not os.path.exists(path):
            continue
        vals = defaultdict(list)
        meta = {}
        for r in csv.DictReader(open(path)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = r
        with open(os.path.join(dst, f"{d}_{KERNEL}.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["counter", "dispatches", "mean_per_dispatch", "min", "max", "grid", "workgroup", "lds_bytes",
                        "scratch_bytes", "vgpr", "agpr", "sgpr"])
            for name, v in sorted(vals.items()):
                w.writerow([name, len(v), f"{statistics.mean(v):.2f}", f"{min(v):.2f}", f"{max(v):.2f}",
                            meta["Grid_Size"], meta["Workgroup_Size"], meta["LDS_Block_Size"], meta["Scratch_Size"],
                            meta["VGPR_Count"], meta["Accum_VGPR_Count"], meta["SGPR_Count"]])
    print("wrote", dst, sorted(os.listdir(dst)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r1")
