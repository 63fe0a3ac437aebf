import sys, numpy as np, torch
sys.path.insert(0, '.')
from zbot_lab_amd import model as zm
from zbot_lab_amd.sim import ZbotSim
n=256; cfg=zm.TaskCfg.standup()
bad=ZbotSim(n, cfg, device="cuda:0", seed=3)
st=bad.get_state().cpu().numpy(); st[0,5]=np.nan; st[20,77]=np.inf; st[4,200]=-np.nan
bad.set_state(torch.from_numpy(st).cuda())
a=torch.from_numpy(np.random.default_rng(0).normal(size=(n,6)).astype(np.float32)).cuda()
ob,rb,tb,ub=[x.cpu().numpy() for x in bad.step(a)]
sb=bad.get_state().cpu().numpy()
bo=np.argwhere(~np.isfinite(ob)); print("nonfinite obs", bo[:10], "terminated", tb[[5,77,200]], "rew", rb[[5,77,200]])
bs=np.argwhere(~np.isfinite(sb)); print("nonfinite state (row, env)", bs[:10])
