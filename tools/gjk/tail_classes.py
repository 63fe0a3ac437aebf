"""GJK tail by contact configuration, on the CPU oracle (tooling; imports oracle/).

Rolls out random actions (walking v2 from its default pose; stand-up from folded states) with the
GJK probe on and reports the probe's GJK calls (the pairs the kernel's separating-axis test leaves
undecided, warm-started as the kernel does) by the configuration they converge to -- no contact,
face on face, a ruling lying on a face, side-by-side rulings within 5 degrees (the rim manifold's
case), side by side within 15 degrees, point-like -- with their iteration counts: which closest
features make the tail (calls of >= 8 / >= 10 iterations) that sets the step kernel's launch span.
Usage: python tools/gjk/tail_classes.py [envs] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from zbot_lab_amd import model as zm  # noqa: E402

NAMES = ["no contact", "face on face", "ruling on face (5 deg)", "side by side (5 deg)", "side by side (15 deg)",
         "point-like"]


def run(cfg, n, steps, fold, seed=1):
    sim = po.OracleSim(n, cfg, seed=seed)
    lib = sim.lib
    lib.zbo_gjk_hooks.argtypes = [C.c_int, C.c_int, C.c_void_p]
    lib.zbo_gjk_classes.argtypes = [C.c_void_p]
    nit = 18
    cls = np.zeros((6, nit), np.int64)
    lib.zbo_gjk_hooks(1, 1, None)
    lib.zbo_gjk_classes(cls.ctypes.data)  # clear
    sim.reset()
    rng = np.random.default_rng(0)
    if fold:
        st = sim.get_state()
        st[13:19] += rng.normal(0, fold, (6, n)).astype(np.float32)
        sim.set_state(st)
    for _ in range(steps):
        sim.step(rng.normal(size=(n, 6)).astype(np.float32))
    lib.zbo_gjk_classes(cls.ctypes.data)
    lib.zbo_gjk_hooks(1, 0, None)
    return cls


def report(label, cls):
    its = np.arange(cls.shape[1])
    tot = cls.sum()
    print(f"\n{label}: {tot} GJK calls, mean {float((cls.sum(0) * its).sum()) / max(tot, 1):.2f} iterations")
    for k, name in enumerate(NAMES):
        c = cls[k]
        n = c.sum()
        if n == 0:
            continue
        ge8, ge10 = c[8:].sum(), c[10:].sum()
        print(f"  {name:24s} calls {n:8d} ({n / tot:6.2%})  mean it {float((c * its).sum()) / n:5.2f}  "
              f">= 8 it {ge8:6d} ({ge8 / max(cls[:, 8:].sum(), 1):6.2%} of the tail)  >= 10 it {ge10:6d} "
              f"({ge10 / max(cls[:, 10:].sum(), 1):6.2%})")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    report("walking v2, random actions", run(zm.TaskCfg(), n, steps, 0.0))
    report("stand-up, folded starts (joint angles + N(0, 1.5)), random actions", run(zm.TaskCfg.standup(), n, steps // 3, 1.5))


if __name__ == "__main__":
    main()
