"""Manager env step parity diagnostic: per-step mismatch fraction and worst obs columns."""
import numpy as np, torch, sys, os
sys.path.insert(0, os.getcwd())
from zbot_lab_amd import model as zm
from zbot_lab_amd.sim import ZbotSim
from oracle.pyoracle import OracleSim
n = 1024
cfg = zm.TaskCfg.manager_flat(feet_close_min=0.10)
g, o = ZbotSim(n, cfg, device="cuda:0", seed=21), OracleSim(n, cfg, seed=21)
rng = np.random.default_rng(4); b = rng.uniform(0.3, 1.0, 64).astype(np.float32); mu = b[rng.integers(0, 64, (n, 12))]
g.set_link_friction(torch.from_numpy(mu).cuda()); o.set_link_friction(mu)
rng = np.random.default_rng(8)
for k in range(3):
    a = rng.normal(size=(n, 6)).astype(np.float32)
    og, rg, tg, trg = [x.cpu().numpy() for x in g.step(torch.from_numpy(a).cuda())]
    oo, ro, to, tro = o.step(a)
    same = tg == to
    bad = ~(np.abs(og - oo) <= 5e-3 + 5e-3 * np.abs(oo))
    print(k, "flags same", same.mean(), "obs ok", (~bad.any(1))[same].mean(), "bad per col", bad[same].sum(0).tolist())
    rb = ~(np.abs(rg - ro) <= 5e-3 + 5e-3 * np.abs(ro)); print("  rew ok", (~rb)[same].mean())
