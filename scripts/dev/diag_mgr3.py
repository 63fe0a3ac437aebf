"""Manager env free-running: for envs whose obs quat diverges, print state diffs and flags."""
import numpy as np, torch, sys, os
sys.path.insert(0, os.getcwd())
from zbot_lab_amd import model as zm
from zbot_lab_amd.sim import ZbotSim
from oracle.pyoracle import OracleSim
M = zm.M
n = 1024
cfg = zm.TaskCfg.manager_flat(feet_close_min=0.10)
g, o = ZbotSim(n, cfg, device="cuda:0", seed=21), OracleSim(n, cfg, seed=21)
rng = np.random.default_rng(4); b = rng.uniform(0.3, 1.0, 64).astype(np.float32); mu = b[rng.integers(0, 64, (n, 12))]
g.set_link_friction(torch.from_numpy(mu).cuda()); o.set_link_friction(mu)
rng = np.random.default_rng(8)
print({k: v for k, v in M.items()})
for k in range(3):
    a = rng.normal(size=(n, 6)).astype(np.float32)
    og, rg, tg, trg = [x.cpu().numpy() for x in g.step(torch.from_numpy(a).cuda())]
    oo, ro, to, tro = o.step(a)
    sg, so = g.get_state().cpu().numpy(), o.get_state()
    bad = np.where(np.abs(og - oo)[:, :4].max(1) > 5e-3)[0]
    print("step", k, "bad", bad.tolist())
    for e in bad[:6]:
        print(" env", e, "term", tg[e], to[e], "trunc", trg[e], tro[e], "eplen", sg[M["EP_LEN"], e], so[M["EP_LEN"], e])
        print("   obs quat g", og[e, :4].round(4), "o", oo[e, :4].round(4))
        print("   state quat g", sg[3:7, e].round(4), "o", so[3:7, e].round(4), "pos g", sg[0:3, e].round(4), "o", so[0:3, e].round(4))
        dd = np.abs(sg[:, e] - so[:, e]); print("   worst state rows", np.argsort(-dd)[:8].tolist(), np.sort(dd)[::-1][:8].round(4).tolist())
