"""The solver's persistent self-contact cache at the API boundary: it is simulator-
internal (not a state row), so writes of MDP rows through the env API keep it, while writes that move
the physics invalidate it, in the kernel and in the oracle alike."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _folded_env(n=256):
    import torch
    import zbot_lab_amd
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    cfg.scene.num_envs = n
    env = zbot_lab_amd.make("zbot-6b-walking-v2", cfg=cfg)
    env.reset()
    st = env.sim.get_state()
    st[13:19] += torch.randn(6, n, device=st.device, generator=torch.Generator(device=st.device).manual_seed(3)) * 1.5
    env.sim.set_state(st)
    for _ in range(2):  # folded robots: self contacts kept in the cache
        env.step(torch.zeros(n, 6, device=env.device))
    return env


def test_episode_length_setter_keeps_the_cache(gpu):
    """rsl_rl's init_at_random_ep_len writes episode_length_buf: the counters change, the cache does not."""
    import torch
    env = _folded_env()
    wc = env.sim.get_contact_cache().clone()
    assert (wc[3::4] >= 1).any(), "no self contacts cached"
    ep = torch.randint(0, 999, (env.num_envs,), device=env.device)
    env.episode_length_buf = ep
    assert torch.equal(env.episode_length_buf, ep)
    assert torch.equal(env.sim.get_contact_cache(), wc)
    env.close()


def test_physics_substeps_invalidates_the_cache(gpu):
    """zb_physics_substeps moves the physics state: the cache is invalidated (every code -1), as the
    oracle's zbo_physics_substeps does."""
    import torch
    from oracle.pyoracle import OracleSim
    env = _folded_env()
    assert (env.sim.get_contact_cache()[3::4] >= 1).any()
    q = env.sim.get_state()[13:19].T.contiguous()
    env.sim.physics_substeps(q, 2)
    wc = env.sim.get_contact_cache().cpu().numpy()
    assert (wc[3::4] == -1).all()
    o = OracleSim(env.num_envs, env.sim.cfg, seed=0)
    o.set_state(env.sim.get_state().cpu().numpy())
    o.step(np.zeros((env.num_envs, 6), np.float32))
    assert (o.get_contact_cache()[3::4] >= 1).any()
    o.physics_substeps(np.ascontiguousarray(q.cpu().numpy()), 1)
    assert (o.get_contact_cache()[3::4] == -1).all()
    env.close()
