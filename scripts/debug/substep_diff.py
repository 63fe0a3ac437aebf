"""Parity debugging: step saved env states substep by substep on the GPU and the oracle, print the
per-substep state differences and the oracle's contact diagnostics (candidates, kept, distance of
the nearest rim point / sphere pair to the activation margin).
Usage: python scripts/debug/substep_diff.py <npz with st [dim, n] and a [n, 6]> <task> [nsub]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from fullstate import task_cfg  # noqa: E402
from oracle.pyoracle import OracleSim  # noqa: E402
from zbot_lab_amd import model as zm  # noqa: E402
from zbot_lab_amd.sim import ZbotSim  # noqa: E402

d = np.load(sys.argv[1])
task = sys.argv[2]
nsub = int(sys.argv[3]) if len(sys.argv) > 3 else 4
st, a = d["st"], d["a"]
n = st.shape[1]
cfg = task_cfg(task)
variants = {"default": {}, "no_self": dict(enable_self_collision=False), "pgs8": dict(solver_iterations=8),
            "pgs1": dict(solver_iterations=1)}
pdel = st[25:31].T.astype(np.float64)
tg = (np.clip(pdel + np.pi * np.tanh(a) * cfg.step_dt, -np.pi, np.pi) + zm.load_model().default_joint_pos).astype(np.float32)
for name, kw in variants.items():
    c = task_cfg(task)
    for k, v in kw.items():
        setattr(c, k, v)
    g = ZbotSim(n, c, device="cuda:0", seed=0)
    o = OracleSim(n, c, seed=0)
    g.set_state(torch.from_numpy(st).cuda())
    o.set_state(st)
    print(f"== {name}")
    for k in range(nsub):
        diag = o.contact_diag()
        nfg, _ = g.physics_substeps(torch.from_numpy(tg).cuda(), 1)
        nfo, _ = o.physics_substeps(tg, 1)
        sg, so = g.get_state().cpu().numpy(), o.get_state()
        dv = np.abs(sg[:25] - so[:25])
        for e in range(n):
            print(f"  sub {k} env {e}: cand {diag[e,0]:.0f} (g {diag[e,1]:.0f} s {diag[e,2]:.0f}) kept {diag[e,3]:.0f} "
                  f"margin-dist {diag[e,4]:.2e} | max|dstate| {dv[:, e].max():.3e} at row {dv[:, e].argmax()} "
                  f"| max|dF| {np.abs(nfg.cpu().numpy()[e] - nfo[e]).max():.3e}")
