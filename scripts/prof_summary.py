#!/usr/bin/env python3
"""Summarise a rocprofv3 run of bench.py (scripts/gpu.sh step ``prof``) into profiles/<tag>/ and into
the tracked ``roofline_pmc.json`` that bench.py reads on the GPU box (``profiles/`` does not travel).

From <src> (a directory holding trace/ and pmc_*/ rocprofv3 CSV outputs) it writes to <dst>:
  kernel_stats.csv                      rocprofv3 --stats
  kernel_gaps.txt                       duration and start-to-start cadence of the step kernel
  pmc_<pass>_<kernel>.csv               per-dispatch mean / min / max of every counter of that pass
and, with --out, merges one entry per (kernel, grid) into the JSON file:
  traffic_bytes   2 x FETCH_SIZE + WRITE_SIZE per launch (KiB counters; the x2 read correction is this
                  kernel's calibration, DESIGN.md §5, tools/calib)
  issue_frac      SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (VALU-issuing share of a wave's resident time)
  wait_any_frac   SQ_WAIT_ANY / SQ_WAVE_CYCLES
  valu_insts_per_wave, waves, rocprof_mean_us / median_us of the kernel trace.
Usage: python scripts/prof_summary.py <src> <dst> [--out roofline_pmc.json] [--kernel zb_step_kernel]
"""
import argparse
import csv
import json
import os
import shutil
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summarise(src: str, dst: str, kernel: str) -> dict:
    os.makedirs(dst, exist_ok=True)
    info = {}
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    trace = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        rows = [r for r in csv.DictReader(open(trace)) if kernel in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        per = [(int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
        grid = int(rows[0]["Grid_Size_X"])
        with open(os.path.join(dst, "kernel_gaps.txt"), "w") as f:
            f.write(f"{kernel}: {len(rows)} dispatches, grid {grid} x wg {rows[0]['Workgroup_Size_X']}\n")
            f.write(f"duration us: median {statistics.median(dur):.2f} mean {statistics.mean(dur):.2f}\n")
            f.write(f"start-to-start us: median {statistics.median(per):.2f} mean {statistics.mean(per):.2f}\n")
        info.update(grid=grid, dispatches=len(rows), rocprof_mean_us=statistics.mean(dur),
                    rocprof_median_us=statistics.median(dur), start_to_start_median_us=statistics.median(per))
    counters = {}
    for d in sorted(os.listdir(src)):
        path = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc_") or not os.path.exists(path):
            continue
        vals = defaultdict(list)
        meta = {}
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = r
        if not meta:
            continue
        info.setdefault("grid", int(meta["Grid_Size"]))
        with open(os.path.join(dst, f"{d}_{kernel}.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["counter", "dispatches", "mean_per_dispatch", "min", "max", "grid", "workgroup", "lds_bytes",
                        "scratch_bytes", "vgpr", "agpr", "sgpr"])
            for name, v in sorted(vals.items()):
                counters[name] = statistics.mean(v)
                w.writerow([name, len(v), f"{statistics.mean(v):.2f}", f"{min(v):.2f}", f"{max(v):.2f}",
                            meta["Grid_Size"], meta["Workgroup_Size"], meta["LDS_Block_Size"], meta["Scratch_Size"],
                            meta["VGPR_Count"], meta["Accum_VGPR_Count"], meta["SGPR_Count"]])
    c = counters
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        info.update(fetch_kib=c["FETCH_SIZE"], write_kib=c["WRITE_SIZE"],
                    traffic_bytes=(2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0)
    if "SQ_WAVE_CYCLES" in c:
        if "SQ_ACTIVE_INST_VALU" in c:
            info["issue_frac"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_ANY" in c:
            info["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
        info.update(valu_insts_per_wave=c["SQ_INSTS_VALU"] / c["SQ_WAVES"], waves=c["SQ_WAVES"])
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst", nargs="?", default=None)
    ap.add_argument("--out", default=None, help="merge the roofline entry into this JSON file")
    ap.add_argument("--kernel", default=os.environ.get("KERNEL", "zb_step_kernel"))
    a = ap.parse_args()
    dst = a.dst or os.path.join(a.src, "summary")
    info = summarise(a.src, dst, a.kernel)
    info["source"] = os.path.relpath(os.path.abspath(dst), ROOT)
    print(json.dumps(info, indent=1))
    if a.out:
        db = json.load(open(a.out)) if os.path.exists(a.out) else {}
        db[f"{a.kernel}@{info['grid']}"] = info
        with open(a.out, "w") as f:
            json.dump(db, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main()
