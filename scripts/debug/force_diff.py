"""Per-link net contact force after one substep, GPU vs oracle, for saved env states (parity debugging)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from fullstate import task_cfg  # noqa: E402
from oracle.pyoracle import OracleSim  # noqa: E402
from zbot_lab_amd import model as zm  # noqa: E402
from zbot_lab_amd.sim import ZbotSim  # noqa: E402

d = np.load(sys.argv[1])
task = sys.argv[2]
st, a = d["st"], d["a"]
n = st.shape[1]
cfg = task_cfg(task)
for it in (0, 1, 4):
    c = task_cfg(task)
    c.solver_iterations = it
    pdel = st[25:31].T.astype(np.float64)
    tg = (np.clip(pdel + np.pi * np.tanh(a) * cfg.step_dt, -np.pi, np.pi) + zm.load_model().default_joint_pos).astype(np.float32)
    g = ZbotSim(n, c, device="cuda:0", seed=0)
    o = OracleSim(n, c, seed=0)
    g.set_state(torch.from_numpy(st).cuda())
    o.set_state(st)
    nfg, _ = g.physics_substeps(torch.from_numpy(tg).cuda(), 1)
    nfo, _ = o.physics_substeps(tg, 1)
    nfg = nfg.cpu().numpy()
    sg, so = g.get_state().cpu().numpy(), o.get_state()
    np.set_printoptions(precision=3, suppress=True, linewidth=200)
    print(f"== PGS iterations {it}")
    for e in range(n):
        print(f" env {e} state diff rows 7..24:", (sg[7:25, e] - so[7:25, e]))
        for l in range(12):
            if np.abs(nfg[e, l]).max() + np.abs(nfo[e, l]).max() > 0:
                print(f"   link {l:2d} gpu {nfg[e, l]}  oracle {nfo[e, l]}")
