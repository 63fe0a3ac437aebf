"""GJK iteration probe on the CPU oracle (tooling; test infrastructure: imports oracle/).

Rolls out random actions on the oracle with the GJK probe on (zbo_gjk_hooks): histogram of the
support iterations of the GJK calls the kernel makes (pairs its separating-axis test leaves
undecided), cold (every GJK from the hull centre difference) vs warm (from the pair's contact normal
of the previous substep of the step). Usage: [GJK_TOL=1e-4] python tools/gjk/probe.py [task] [envs] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from zbot_lab_amd.tasks import load_cfg  # noqa: E402

NH = 18  # GJK_MAX_IT + 2 (then 64 counters of undecided pairs per env-substep)


def run(task, n, steps, warm):
    cfg = load_cfg(task)
    sim = po.OracleSim(n, cfg=cfg.task_cfg(), seed=1)
    lib = sim.lib
    lib.zbo_gjk_hooks.argtypes = [C.c_int, C.c_int, C.c_void_p]
    lib.zbo_set_gjk_tol.argtypes = [C.c_double]
    lib.zbo_set_gjk_tol(float(os.environ.get("GJK_TOL", "0")))
    hist = np.zeros(NH + 64, np.int64)
    lib.zbo_gjk_hooks(warm, 1, hist.ctypes.data)  # clear
    sim.reset()
    rng = np.random.default_rng(0)
    for _ in range(steps):
        sim.step(rng.normal(size=(n, 6)).astype(np.float32))
    lib.zbo_gjk_hooks(1, 0, hist.ctypes.data)
    return hist


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "zbot-6b-walking-v2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    for warm in [int(w) for w in os.environ.get("MODES", "0,1").split(",")]:
        hh = run(task, n, steps, warm)
        h, u = hh[:NH], hh[NH:]
        tot = h.sum()
        print(f"{task} {'warm' if warm else 'cold'}: {n} envs x {steps} steps, {tot / n / steps / 4:.3f} GJK calls "
              f"per env-substep, mean {np.dot(np.arange(NH), h) / max(tot, 1):.2f} iterations; histogram "
              + " ".join(f"{i}:{int(v)}" for i, v in enumerate(h) if v))
        print("  undecided pairs per env-substep: " + " ".join(f"{i}:{int(v)}" for i, v in enumerate(u) if v))


if __name__ == "__main__":
    main()
