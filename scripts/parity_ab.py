#!/usr/bin/env python3
"""Table of the full-state parity aggregates per library build (the build-flag A/B of DESIGN.md §6).

Input: the JSONL that tests/test_gpu_fullstate.py::_check appends to when ZB_PARITY_STATS is set (one
line per check and library). For every check: the device's outlier fraction and median err/tol
against the f64 oracle over the contact-active envs, next to the f32 oracle's own against f64, and the
headroom to the aggregate bound (frac <= 2 x f32 + 0.5 % for one-step checks, 3 x f32 + 0.5 % for
the multi-step ones; median <= 4 x f32 + 0.02).
Usage: python scripts/parity_ab.py <stats.jsonl> [--markdown]
"""
import json
import sys
from collections import OrderedDict


def bound(r):
    k = 3.0 if "steps from" in r["check"] else 2.0  # (tests/test_gpu_fullstate.py AGG_FRAC_K[_MULTI])
    return k * r["frac_f32"] + 0.005, 4.0 * r["med_f32"] + 0.02


def main(path, markdown=False):
    rows = [json.loads(l) for l in open(path) if l.strip()]
    libs = list(OrderedDict.fromkeys(r["lib"] for r in rows))
    checks = list(OrderedDict.fromkeys((r["task"], r["check"]) for r in rows))
    by = {(r["lib"], r["task"], r["check"]): r for r in rows}
    sep = " | " if markdown else "  "
    head = ["check", "f32 oracle frac / med"] + [f"{l}: frac / med (headroom)" for l in libs]
    print(("| " if markdown else "") + sep.join(head) + (" |" if markdown else ""))
    if markdown:
        print("|" + "---|" * len(head))
    ratio = {l: [] for l in libs}
    worst = {l: 1e9 for l in libs}
    for t, c in checks:
        base = next((by[(l, t, c)] for l in libs if (l, t, c) in by), None)
        cells = [f"{t} {c}", f"{100 * base['frac_f32']:.2f} % / {base['med_f32']:.3g}"]
        for l in libs:
            r = by.get((l, t, c))
            if r is None:
                cells.append("-")
                continue
            bf, bm = bound(r)
            head_f = 1.0 - r["frac"] / bf
            worst[l] = min(worst[l], head_f)
            if r["med_f32"] > 0:
                ratio[l].append(r["med"] / r["med_f32"])
            cells.append(f"{100 * r['frac']:.2f} % / {r['med']:.3g} ({100 * head_f:.0f} %)")
        print(("| " if markdown else "") + sep.join(cells) + (" |" if markdown else ""))
    print()
    for l in libs:
        v = sorted(ratio[l])
        if v:
            print(f"{l}: median of (device median err/tol / f32-oracle median err/tol) over {len(v)} checks "
                  f"{v[len(v) // 2]:.2f} (min {v[0]:.2f}, max {v[-1]:.2f}); smallest outlier-fraction headroom "
                  f"{100 * worst[l]:.0f} %")


if __name__ == "__main__":
    main(sys.argv[1], "--markdown" in sys.argv)
