"""Manager env: single-step GPU vs oracle error with the GPU state re-synced to the oracle each step."""
import numpy as np, torch, sys, os
sys.path.insert(0, os.getcwd())
from zbot_lab_amd import model as zm
from zbot_lab_amd.sim import ZbotSim
from oracle.pyoracle import OracleSim
S = zm.S
n = 1024
cfg = zm.TaskCfg.manager_flat(feet_close_min=0.10)
g, o, d = ZbotSim(n, cfg, device="cuda:0", seed=21), OracleSim(n, cfg, seed=21), OracleSim(n, cfg, seed=21, double=True)
rng = np.random.default_rng(4); b = rng.uniform(0.3, 1.0, 64).astype(np.float32); mu = b[rng.integers(0, 64, (n, 12))]
g.set_link_friction(torch.from_numpy(mu).cuda()); o.set_link_friction(mu); d.set_link_friction(mu)
rng = np.random.default_rng(8)
dump = {}
for k in range(6):
    pre = o.get_state().copy()
    g.set_state(torch.from_numpy(pre).cuda()); d.set_state(pre.astype(np.float64) if False else pre)
    a = rng.normal(size=(n, 6)).astype(np.float32)
    g.step(torch.from_numpy(a).cuda()); o.step(a); d.step(a)
    sg, so, sd = g.get_state().cpu().numpy(), o.get_state(), d.get_state()
    for name, sl in (("quat", slice(3, 7)), ("angvel", slice(10, 13)), ("linvel", slice(7, 10)), ("qd", slice(19, 25))):
        eg = np.abs(sg[sl] - so[sl]).max(0); ed = np.abs(sd[sl] - so[sl]).max(0)
        print(k, name, "gpu-o32 q50/99/max", np.quantile(eg, [0.5, 0.99]).round(7).tolist(), eg.max().round(5),
              "| o64-o32 q50/99/max", np.quantile(ed, [0.5, 0.99]).round(7).tolist(), ed.max().round(5), "n>1e-2", int((eg > 1e-2).sum()), int((ed > 1e-2).sum()))
    eg = np.abs(sg[10:13] - so[10:13]).max(0)
    bad = np.argsort(-eg)[:8]
    dump[f"pre{k}"] = pre[:, bad]; dump[f"act{k}"] = a[bad]; dump[f"ids{k}"] = bad; dump[f"gpu{k}"] = sg[:, bad]; dump[f"mu{k}"] = mu[bad]
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/diag_mgr2.npz", **dump)
