"""GPU-vs-oracle diagnostic dump (run on the GPU box)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from helpers import S, perturbed_states
from zbot_lab_amd import model as zm
from zbot_lab_amd.sim import ZbotSim
from oracle.pyoracle import OracleSim
np.set_printoptions(precision=5, suppress=True, linewidth=150)
names = {v: k for k, v in S.items()}
def field_report(sg, so, tag):
    d = np.abs(sg - so)
    print(f"--- {tag}: per-field max abs diff (envs with diff>1e-3)")
    for f in range(zm.STATE_DIM):
        if d[f].max() > 1e-5:
            print(f"  field {f:2d} max {d[f].max():.3e} n>1e-3: {(d[f] > 1e-3).sum()}  worst env {d[f].argmax()}")
for nsub in (1, 4):
    for cfgname, cfg in (("full", zm.TaskCfg()), ("noself", zm.TaskCfg(enable_self_collision=False)), ("nocontact-air", None)):
        n = 512
        st = perturbed_states(n, seed=11, airborne=1.0 if cfg is None else 0.0)
        cfg = cfg or zm.TaskCfg()
        g = ZbotSim(n, cfg); o = OracleSim(n, cfg)
        g.set_state(torch.from_numpy(st).cuda()); o.set_state(st)
        tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy()
        fg, tg_ = g.physics_substeps(torch.from_numpy(tg).cuda(), nsub)
        fo, to_ = o.physics_substeps(tg, nsub)
        field_report(g.get_state().cpu().numpy(), o.get_state(), f"{cfgname} nsub={nsub}")
        df = np.abs(fg.cpu().numpy() - fo)
        print("  force diff max", df.max(), "envs >0.1N:", (df.max(axis=(1, 2)) > 0.1).sum())
# one step from default
n = 64
g = ZbotSim(n); o = OracleSim(n)
a = np.random.default_rng(0).normal(size=(n, 6)).astype(np.float32)
og, rg, tg, ug = g.step(torch.from_numpy(a).cuda()); oo, ro, to, uo = o.step(a)
og = og.cpu().numpy(); d = np.abs(og - oo)
print("step obs diff per column max:", d.max(axis=0))
print("rew diff", np.abs(rg.cpu().numpy() - ro).max())
field_report(g.get_state().cpu().numpy(), o.get_state(), "step from default")
