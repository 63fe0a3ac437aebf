import sys, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import torch
from fullstate import random_states, task_cfg, solver_mode
from oracle.pyoracle import OracleSim
from zbot_lab_amd.sim import ZbotSim
with solver_mode(1):
    n, seed = 2048, 19
    cfg = task_cfg('v2')
    g = ZbotSim(n, cfg, device="cuda:0", seed=seed); o = OracleSim(n, cfg, seed=seed)
    st = random_states('v2', o, n, seed=111)
    g.set_state(torch.from_numpy(st).cuda())
    a = np.random.default_rng(8).normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    sg = g.get_state().cpu().numpy()
    # also the one-substep net forces of env 1906's state under TGS
    g2 = ZbotSim(n, cfg, device="cuda:0", seed=seed); g2.set_state(torch.from_numpy(st).cuda())
    tg = st[13:19].T.copy()
    nf, tau = g2.physics_substeps(torch.from_numpy(np.ascontiguousarray(tg)).cuda(), 1)
    np.savez("gpurun_out/tgs_dump.npz", st=st, a=a, sg=sg, obs=obs.cpu().numpy(), rew=rew.cpu().numpy(), nf=nf.cpu().numpy(), sg1=g2.get_state().cpu().numpy())
print("ok")
