"""BASELINE.json configs[0] = C1 (zbot-6b-walking-v2, 4 envs, CPU reference articulated-body
integrator, random actions, 1000 steps): the plumbing config, run on the CPU oracle with every
DirectRLEnv bookkeeping invariant checked at every step (tests/configs_common.py)."""
from __future__ import annotations

import numpy as np

from configs_common import S, c1_step_invariants
from zbot_lab_amd import model as zm


def test_c1_four_envs_1000_random_steps(oracle_lib):
    from oracle.pyoracle import OracleSim
    o = OracleSim(4, zm.TaskCfg(), seed=42)
    o.reset()
    rng = np.random.default_rng(42)
    st = o.get_state()
    resets = 0
    for k in range(1000):
        obs, rew, te, tr = o.step(rng.standard_normal((4, 6)).astype(np.float32))
        st1 = o.get_state()
        _, counts = o.read_log()
        c1_step_invariants(k, st, st1, obs, rew, te, tr, counts)
        resets += int((te | tr).sum())
        st = st1
    assert resets > 4                      # random actions end episodes (body contact / fall)
    assert st[S["EP_LEN"]].max() < 999
