#!/usr/bin/env python3
"""State after K seeded steps of every task with the libzbot named by ZBOT_LIB -> gpurun_out/dump_<lib>_<K>.npz
(to compare two builds' arithmetic: scripts/bitident.py gives only digests)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zbot_lab_amd import model as zm  # noqa: E402
from zbot_lab_amd.sim import ZbotSim  # noqa: E402

N, K = 4096, int(os.environ.get("K", "1"))
out = {}
for name, cfg in (("walking", zm.TaskCfg()), ("standup", zm.TaskCfg.standup())):
    sim = ZbotSim(N, cfg, seed=7)
    sim.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    out[name + "_s0"] = sim.get_state().cpu().numpy()
    for _ in range(K):
        sim.step(torch.randn(N, zm.ACT_DIM, device="cuda", generator=g))
    out[name] = sim.get_state().cpu().numpy()
    sim.close()
lib = os.environ.get("ZBOT_LIB", "libzbot.so").replace(".so", "")
np.savez(os.path.join(R, "gpurun_out", f"dump_{lib}_{K}.npz"), **out)
print("ok", lib, K)
