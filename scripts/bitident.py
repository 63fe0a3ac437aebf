#!/usr/bin/env python3
"""Digest of a seeded rollout of every task (final state, rewards, flags, observations) with the
libzbot build named by ZBOT_LIB: two builds are bit-identical iff their digests match.
Usage (GPU box): ZBOT_LIB=libzbot_old.so python scripts/bitident.py; python scripts/bitident.py"""
import hashlib
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

from zbot_lab_amd import model as zm  # noqa: E402
from zbot_lab_amd.sim import ZbotSim  # noqa: E402

N, STEPS = int(os.environ.get("N", "4096")), int(os.environ.get("STEPS", "300"))
for name, cfg in (("walking", zm.TaskCfg()), ("standup", zm.TaskCfg.standup()),
                  ("v4", zm.TaskCfg.walking_v4()), ("manager", zm.TaskCfg.manager_flat())):
    sim = ZbotSim(N, cfg, seed=7)
    sim.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    h = hashlib.sha256()
    for _ in range(STEPS):
        obs, rew, term, trunc = sim.step(torch.randn(N, zm.ACT_DIM, device="cuda", generator=g))
        h.update(rew.cpu().numpy().tobytes())
        h.update(term.cpu().numpy().tobytes())
        h.update(trunc.cpu().numpy().tobytes())
    h.update(obs.cpu().numpy().tobytes())
    h.update(sim.get_state().cpu().numpy().tobytes())
    print(f"{os.environ.get('ZBOT_LIB', 'libzbot.so'):18s} {name:8s} {h.hexdigest()[:32]}", flush=True)
    sim.close()
