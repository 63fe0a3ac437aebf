#!/usr/bin/env python3
"""Where the device's error against exact arithmetic comes from.

One physics substep (zb_physics_substeps) of walking v2 from the same states on the device (libzbot.so,
or ZBOT_LIB), the f32 oracle and the f64 oracle; per state row class, the median over envs of
|x - x_f64| for the device and for the f32 oracle, and their ratio. Three state sets isolate the
parts of the substep:
* airborne: random joint angles / velocities, root 1 m up (no contact: FK, RNEA, CRBA, Cholesky, the
  implicit PD drive and the integration only);
* ground: near-standing states (ground contacts, PGS);
* random: random full states (ground and self contacts).
Usage (GPU box): python tools/error_budget.py [n]
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(n: int = 2048) -> None:
    import torch
    from fullstate import random_states, task_cfg
    from oracle.pyoracle import OracleSim
    from zbot_lab_amd.sim import ZbotSim
    cfg = task_cfg("v2")
    rows = {"root_pos": range(0, 3), "root_quat": range(3, 7), "root_linvel": range(7, 10),
            "root_angvel": range(10, 13), "joint_pos": range(13, 19), "joint_vel": range(19, 25)}
    o = OracleSim(n, cfg, seed=3)
    sets = {}
    st = random_states("v2", o, n, seed=11)
    air = st.copy()
    air[2] += 1.0
    sets["airborne"] = air
    sets["ground"] = random_states("v2", o, n, seed=12, standing=True)
    sets["random"] = random_states("v2", o, n, seed=13)
    tgt = np.random.default_rng(5).uniform(-0.5, 0.5, (n, 6)).astype(np.float32)
    for name, s0 in sets.items():
        g = ZbotSim(n, cfg, device="cuda:0", seed=3)
        g.set_state(torch.from_numpy(s0).cuda())
        g.physics_substeps(torch.from_numpy(tgt).cuda(), 1)
        sg = g.get_state().cpu().numpy().astype(np.float64)
        out = {}
        for dbl in (False, True):
            oo = OracleSim(n, cfg, seed=3, double=dbl)
            oo.set_state(s0)
            oo.physics_substeps(tgt, 1)
            out[dbl] = oo.get_state().astype(np.float64)
        s64, s32 = out[True], out[False]
        line = []
        for k, r in rows.items():
            r = list(r)
            eg = np.abs(sg[r] - s64[r]).max(axis=0)
            eo = np.abs(s32[r] - s64[r]).max(axis=0)
            mg, mo = float(np.median(eg)), float(np.median(eo))
            line.append(f"{k} {mg:.2e}/{mo:.2e} ({mg / max(mo, 1e-30):.2f}x)")
        print(f"[{name}] device / f32 oracle median |err vs f64|: " + ", ".join(line), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2048)
