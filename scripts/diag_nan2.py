"""Replay tests/test_gpu_parity.py::test_rollout_statistics exactly, report the first non-finite step."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np, torch
from zbot_lab_amd.sim import ZbotSim
from zbot_lab_amd import model as zm
from oracle.pyoracle import OracleSim
for trial in range(2):
    n, steps = 1024, 300
    g = ZbotSim(n, zm.TaskCfg(), device="cuda:0", seed=7)
    o = OracleSim(n, zm.TaskCfg(), seed=7)
    g.reset(None); o.reset(None)
    rng = np.random.default_rng(42)
    prev = g.get_state().cpu().numpy()
    found = False
    for k in range(steps):
        a = rng.normal(size=(n, 6)).astype(np.float32)
        _, r1, t1, _ = g.step(torch.from_numpy(a).cuda())
        _, r2, t2, _ = o.step(a)
        r1 = r1.cpu().numpy()
        if not np.isfinite(r1).all() and not found:
            e = np.nonzero(~np.isfinite(r1))[0]
            post = g.get_state().cpu().numpy()
            print(f"trial {trial}: non-finite reward at step {k}, envs {e[:8]}; post-state finite: {np.isfinite(post[:, e]).all(0)}")
            print("  reward", r1[e[:4]], "\n  prev state env", e[0], prev[:, e[0]])
            print("  post state", post[:, e[0]])
            np.savez(os.path.join(R, "gpurun_out", f"nan_case{trial}.npz"), state=prev, actions=a, envs=e, step=k)
            found = True
        prev = g.get_state().cpu().numpy()
    print(f"trial {trial}: done, found={found}")
