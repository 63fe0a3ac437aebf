"""Find the first non-finite step of a GPU random rollout and save the pre-step state (GPU box)."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np, torch
from zbot_lab_amd.sim import ZbotSim
from zbot_lab_amd import model as zm
n, steps = 1024, 400
g = ZbotSim(n, seed=7)
g.reset(None)
rng = np.random.default_rng(42)
for k in range(steps):
    st = g.get_state().cpu().numpy()
    a = rng.normal(size=(n, 6)).astype(np.float32)
    obs, r, te, tr = g.step(torch.from_numpy(a).cuda())
    post = g.get_state().cpu().numpy()
    bad = ~np.isfinite(r.cpu().numpy()) | ~np.isfinite(obs.cpu().numpy()).all(1) | ~np.isfinite(post).all(0)
    big = np.abs(post[19:25]).max(0) > 19.9
    if k % 50 == 0:
        print(k, "max |jqd|", np.abs(post[19:25]).max(), "max |root v|", np.abs(post[7:13]).max(), flush=True)
    if bad.any():
        e = np.nonzero(bad)[0]
        print("non-finite at step", k, "envs", e[:10])
        np.savez(os.path.join(R, "gpurun_out", "nan_case.npz"), state=st, actions=a, envs=e, step=k)
        # substep-level replay of the first bad env on the GPU
        g2 = ZbotSim(n, seed=7)
        g2.set_state(torch.from_numpy(st).cuda())
        pd = np.clip(st[25:31].T + np.pi * np.tanh(a) * 0.02, -np.pi, np.pi)
        tg = (pd + zm.load_model().default_joint_pos).astype(np.float32)
        for s in range(4):
            f, tau = g2.physics_substeps(torch.from_numpy(tg).cuda(), 1)
            x = g2.get_state().cpu().numpy()[:, e[0]]
            print(" substep", s, "root", x[0:13], "jq", x[13:19], "jqd", x[19:25])
        break
else:
    print("no non-finite values in", steps, "steps")
