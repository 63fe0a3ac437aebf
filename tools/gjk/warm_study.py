"""How much a better GJK start can buy (tooling on the CPU oracle; test infrastructure: imports
oracle/). Rolls out random actions on walking v2, collects the link pairs the separating-axis test
leaves to GJK (zbo_undecided_pairs), and runs the oracle's hull_pair on each one three ways:
cold (hull centre difference), warm from the pair's own converged normal (the best any warm start
can do), and warm from that normal rotated by 0.01 rad (about omega * dt of a folded robot's links
in one 5 ms substep). Prints iteration means, p99, max and histograms.

    python tools/gjk/warm_study.py [envs] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from zbot_lab_amd.tasks import load_cfg  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 120
    cfg = load_cfg("zbot-6b-walking-v2")
    sim = po.OracleSim(n, cfg=cfg.task_cfg(), seed=1)
    lib = sim.lib
    lib.zbo_undecided_pairs.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.zbo_hull_pair_from.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]
    sim.reset()
    rng = np.random.default_rng(0)
    pairs = []
    for s in range(steps):
        sim.step(rng.normal(size=(n, 6)).astype(np.float32))
        if s >= 20 and s % 5 == 0:
            buf = np.zeros((4096, 38), np.float32)
            k = lib.zbo_undecided_pairs(sim.h, buf.ctypes.data, 4096)
            pairs.append(buf[:min(k, 4096)].copy())
    pairs = np.concatenate(pairs)
    out = np.zeros(8, np.float32)

    def run(a, b, v0=None):
        it = lib.zbo_hull_pair_from(a.ctypes.data, b.ctypes.data, float(cfg.task_cfg().contact_margin),
                                    None if v0 is None else v0.ctypes.data, out.ctypes.data)
        return it, out.copy()

    cold, best, off = [], [], []
    for p in pairs:
        a, b = np.ascontiguousarray(p[2:20]), np.ascontiguousarray(p[20:38])
        it, o = run(a, b)
        cold.append(it)
        nrm = o[2:5].copy()
        if o[0] > 0 and np.isfinite(nrm).all() and np.linalg.norm(nrm) > 0.5:
            best.append(run(a, b, nrm)[0])
            t = np.cross(nrm, [1.0, 0.0, 0.0])
            t /= np.linalg.norm(t) + 1e-12
            off.append(run(a, b, (nrm + 0.01 * t).astype(np.float32))[0])
    print(f"{len(pairs)} undecided pairs from {n} envs x {steps} steps (every 5th step from step 20)")
    for name, x in (("cold", cold), ("warm from its own converged normal", best), ("warm, normal off by 0.01 rad", off)):
        x = np.array(x)
        print(f"  {name:36s} {len(x):5d} calls, mean {x.mean():.2f}, p99 {np.percentile(x, 99):.0f}, max {x.max()}, "
              f"histogram {np.bincount(x).tolist()}")


if __name__ == "__main__":
    main()
