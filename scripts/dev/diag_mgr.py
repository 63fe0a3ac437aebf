"""Diagnostic: per-column GPU-vs-oracle differences of the manager env over a few steps."""
import numpy as np
import torch
from zbot_lab_amd import model as zm
from zbot_lab_amd.sim import ZbotSim
from oracle.pyoracle import OracleSim

n = 1024
cfg = zm.TaskCfg.manager_flat(feet_close_min=0.10)
g, o = ZbotSim(n, cfg, device="cuda:0", seed=21), OracleSim(n, cfg, seed=21)
rng = np.random.default_rng(4)
buckets = rng.uniform(0.3, 1.0, 64).astype(np.float32)
mu = buckets[rng.integers(0, 64, (n, 12))]
g.set_link_friction(torch.from_numpy(mu).cuda())
o.set_link_friction(mu)
rng = np.random.default_rng(8)
for k in range(4):
    a = rng.normal(size=(n, 6)).astype(np.float32)
    og, rg, tg, trg = [x.cpu().numpy() for x in g.step(torch.from_numpy(a).cuda())]
    oo, ro, to, tro = o.step(a)
    bad = np.abs(og - oo) > 5e-3 + 5e-3 * np.abs(oo)
    print(f"step {k}: flags eq {np.mean(tg == to):.4f} obs-bad envs {bad.any(1).mean():.4f} per column",
          np.round(bad.mean(0), 3).tolist())
    print("   max abs err per column", np.round(np.abs(og - oo).max(0), 4).tolist())
    rb = np.abs(rg - ro) > 5e-3 + 5e-3 * np.abs(ro)
    print(f"   reward bad {rb.mean():.4f}")
    sg, so = g.get_state().cpu().numpy(), o.get_state()
    d = np.abs(sg - so)
    print("   state rows bad>1e-3:", {r: round(float((d[r] > 1e-3).mean()), 3) for r in range(sg.shape[0]) if (d[r] > 1e-3).mean() > 0.01})
