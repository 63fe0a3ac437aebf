"""GJK support-direction variants on the CPU oracle's probe (tooling; imports oracle/).

Rolls out the tail_classes.py situations (walking v2 random actions; stand-up from folded starts) with
each variant of the oracle's hull_pair (zbo_set_gjk_variant): 0 = HEAD (stop on the gap along v),
1 = stop on the best lower bound of any direction so far, 2 = Nesterov-accelerated support
directions (Montaut et al. 2022: d_k = delta d_{k-1} + (1 - delta) (delta v_k + (1 - delta) w_{k-1}),
delta = (k + 1) / (k + 3)) with the best-lower-bound stop, 3 = the same with normalised terms.
Reports the iteration histogram of the calls the kernel would make and, per contact, the error
against a tight cold GJK (tolerance 1e-10 m, 200 iterations): separation and 1 - cos(normal).
Usage: python tools/gjk/momentum_probe.py [envs] [steps] [variants...]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from zbot_lab_amd import model as zm  # noqa: E402


def run(cfg, n, steps, fold, var, double):
    sim = po.OracleSim(n, cfg, seed=1, double=double, threads=1)
    lib = sim.lib
    lib.zbo_gjk_hooks.argtypes = [C.c_int, C.c_int, C.c_void_p]
    lib.zbo_set_gjk_variant.argtypes = [C.c_int, C.c_void_p]
    hist = np.zeros(18 + 64, np.int64)
    acc = np.zeros(5, np.float64)
    lib.zbo_set_gjk_variant(var, acc.ctypes.data)
    lib.zbo_gjk_hooks(1, 2, hist.ctypes.data)  # clear
    sim.reset()
    rng = np.random.default_rng(0)
    if fold:
        st = sim.get_state()
        st[13:19] += rng.normal(0, fold, (6, n)).astype(np.float32)
        sim.set_state(st)
    for _ in range(steps):
        sim.step(rng.normal(size=(n, 6)).astype(np.float32))
    lib.zbo_gjk_hooks(1, 0, hist.ctypes.data)
    lib.zbo_set_gjk_variant(0, acc.ctypes.data)
    return hist[:18], acc


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    vars_ = [int(v) for v in sys.argv[3:]] or [0, 1, 2, 3]
    double = os.environ.get("PROBE_F64", "1") == "1"
    for label, cfg, st, fold in (("walking v2, random actions", zm.TaskCfg(), steps, 0.0),
                                 ("stand-up, folded starts", zm.TaskCfg.standup(), steps // 3, 1.5)):
        print(f"\n{label} ({'f64' if double else 'f32'} oracle, {n} envs, {st} steps)")
        for var in vars_:
            h, acc = run(cfg, n, st, fold, var, double)
            its = np.arange(h.size)
            tot = h.sum()
            print(f"  variant {var}: calls {tot:7d}  mean it {float((h * its).sum()) / max(tot, 1):5.2f}  "
                  f">=8 {h[8:].sum():6d}  >=10 {h[10:].sum():6d}  >=12 {h[12:].sum():5d}  =max {h[16:].sum():5d}  | "
                  f"contacts {int(acc[4]):6d}  sep err max {acc[0]:.2e} mean {acc[2]:.2e}  "
                  f"1-cos n max {acc[1]:.2e} mean {acc[3]:.2e}")


if __name__ == "__main__":
    main()
