"""Stand-up task (zbot-6b-standup-v0): HIP kernel (libzbot.so, C ABI) vs the CPU oracle.

Same bar as tests/test_gpu_parity.py: fp32 both sides with different operation order / libm, so
continuous outputs within stated tolerances for >= 99 % of envs, flags identical for >= 99 %,
counter-based draws (episode lengths, reset poses up to sincos rounding) and integer state
bit-exact; long rollouts compared through statistics. Per-link friction (the startup material
randomisation) is set identically on both sides.
"""
from __future__ import annotations

import numpy as np
import pytest

from zbot_lab_amd import model as zm

pytestmark = pytest.mark.gpu
SU = zm.SU


def _pair(n, seed=0, **kw):
    import torch
    from oracle.pyoracle import OracleSim
    from zbot_lab_amd.sim import ZbotSim
    cfg = zm.TaskCfg.standup(**kw)
    g = ZbotSim(n, cfg, device="cuda:0", seed=seed)
    o = OracleSim(n, cfg, seed=seed)
    return g, o, torch


def _friction(n, seed):
    rng = np.random.default_rng(seed)
    buckets = rng.uniform(0.6, 1.0, 64).astype(np.float32)
    return buckets[rng.integers(0, 64, (n, 12))]


def test_create_and_observe_parity(gpu):
    g, o, torch = _pair(512, seed=11)
    sg, so = g.get_state().cpu().numpy(), o.get_state()
    assert sg.shape == (zm.SU_STATE_DIM, 512)
    np.testing.assert_allclose(sg[:7], so[:7], atol=2e-6)          # reset poses: same counter-based draws
    np.testing.assert_array_equal(sg[7:], so[7:])
    np.testing.assert_allclose(g.observe().cpu().numpy(), o.observe(), atol=1e-5)


def test_reset_parity(gpu):
    n = 1024
    g, o, torch = _pair(n, seed=5)
    ids = np.arange(1, n, 3, dtype=np.int32)
    g.reset(torch.from_numpy(ids).cuda())
    o.reset(ids)
    np.testing.assert_allclose(g.get_state().cpu().numpy(), o.get_state(), atol=2e-6)
    g.reset(None)
    o.reset(None)
    eg, eo = g.get_state().cpu().numpy(), o.get_state()
    np.testing.assert_array_equal(eg[SU["EP_LEN"]], eo[SU["EP_LEN"]])
    assert eg[SU["EP_LEN"]].max() <= 299 and len(np.unique(eg[SU["EP_LEN"]])) > 250
    np.testing.assert_allclose(eg, eo, atol=2e-6)


def test_friction_substep_parity(gpu):
    """Per-link friction reaches the solver identically (one substep from identical states)."""
    n = 512
    g, o, torch = _pair(n, seed=3)
    mu = _friction(n, 1)
    mud = _friction(n, 2)   # dynamic drawn independently (standup.py:131-132)
    g.set_link_friction(torch.from_numpy(mu).cuda(), torch.from_numpy(mud).cuda())
    o.set_link_friction(mu, mud)
    st = o.get_state()
    rng = np.random.default_rng(2)
    st[zm.S["JOINT_VEL"]:zm.S["JOINT_VEL"] + 6] = rng.normal(0, 1.0, (6, n)).astype(np.float32)
    st[zm.S["ROOT_LINVEL"]:zm.S["ROOT_LINVEL"] + 2] = rng.normal(0, 0.3, (2, n)).astype(np.float32)
    g.set_state(torch.from_numpy(st).cuda())
    o.set_state(st)
    np.testing.assert_array_equal(g.get_state().cpu().numpy()[SU["LINK_MU"]:SU["LINK_MU"] + 12], mu.T)
    np.testing.assert_array_equal(g.get_state().cpu().numpy()[SU["LINK_MU_D"]:SU["LINK_MU_D"] + 12], mud.T)
    tg = rng.normal(0, 0.5, (n, 6)).astype(np.float32)
    g.physics_substeps(torch.from_numpy(tg).cuda(), 1)
    o.physics_substeps(tg, 1)
    sg, so = g.get_state().cpu().numpy(), o.get_state()
    vel = slice(zm.S["ROOT_LINVEL"], zm.S["JOINT_VEL"] + 6)
    ok = (np.abs(sg[vel] - so[vel]) <= 2e-3 + 1e-3 * np.abs(so[vel])).all(axis=0)
    assert ok.mean() >= 0.99, ok.mean()


def test_one_step_parity(gpu):
    n = 1024
    g, o, torch = _pair(n, seed=21)
    mu = _friction(n, 4)
    g.set_link_friction(torch.from_numpy(mu).cuda())
    o.set_link_friction(mu)
    g.reset(None)
    o.reset(None)
    rng = np.random.default_rng(8)
    for k in range(3):
        a = rng.normal(size=(n, 6)).astype(np.float32)
        og, rg, tg_, trg = g.step(torch.from_numpy(a).cuda())
        oo, ro, to_, tro = o.step(a)
        og, rg, tg_, trg = og.cpu().numpy(), rg.cpu().numpy(), tg_.cpu().numpy(), trg.cpu().numpy()
        assert (trg == tro).all()
        assert (tg_ == to_).mean() >= 0.99
        same = tg_ == to_
        ok_obs = (np.abs(og - oo) <= 5e-3 + 5e-3 * np.abs(oo)).all(axis=1)
        assert ok_obs[same].mean() >= 0.98, (k, ok_obs[same].mean())
        ok_rew = np.abs(rg - ro) <= 5e-3 + 5e-3 * np.abs(ro)
        assert ok_rew[same].mean() >= 0.98, (k, ok_rew[same].mean())
    sg, so = g.get_state().cpu().numpy(), o.get_state()
    np.testing.assert_array_equal(sg[SU["EP_LEN"]], so[SU["EP_LEN"]])


def test_curriculum_parity(gpu):
    n = 256
    g, o, torch = _pair(n, seed=2, curriculum_steps=40)
    g.reset(None)
    o.reset(None)
    a = np.zeros((n, 6), np.float32)
    sg_hist, so_hist = [], []
    for k in range(60):
        g.step(torch.from_numpy(a).cuda())
        o.step(a)
        sg_hist.append(g.read_curriculum())
        so_hist.append(o.read_curriculum())
    assert sg_hist == so_hist
    assert sg_hist[-1] == (1, 60) and sg_hist[38][0] == 0


def test_rollout_statistics(gpu):
    n, steps = 1024, 200
    g, o, torch = _pair(n, seed=7)
    mu = _friction(n, 9)
    g.set_link_friction(torch.from_numpy(mu).cuda())
    o.set_link_friction(mu)
    g.reset(None)
    o.reset(None)
    rng = np.random.default_rng(42)
    rg, ro, dg, do = [], [], [], []
    for k in range(steps):
        a = rng.normal(size=(n, 6)).astype(np.float32)
        _, r1, t1, _ = g.step(torch.from_numpy(a).cuda())
        _, r2, t2, _ = o.step(a)
        assert torch.isfinite(r1).all(), k
        rg.append(r1.mean().item())
        ro.append(r2.mean())
        dg.append(t1.float().mean().item())
        do.append(t2.mean())
    rg, ro, dg, do = map(np.asarray, (rg, ro, dg, do))
    np.testing.assert_allclose(rg[:3], ro[:3], rtol=0.02, atol=0.002)
    assert abs(rg.mean() - ro.mean()) <= 0.1 * abs(ro.mean()) + 0.01, (rg.mean(), ro.mean())
    assert abs(dg.mean() - do.mean()) <= 0.25 * do.mean() + 0.002, (dg.mean(), do.mean())
    lg, cg = g.read_log()
    assert lg.shape == (4,) and torch.isfinite(lg).all()


def test_env_api(gpu):
    import torch
    import zbot_lab_amd
    from zbot_lab_amd.rl import RslRlVecEnvWrapper
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-standup-v0")
    cfg.scene.num_envs = 256
    env = zbot_lab_amd.make("zbot-6b-standup-v0", cfg=cfg)
    assert env.max_episode_length == 300 and env.num_envs == 256
    mu = env.sim.get_state()[SU["LINK_MU"]:SU["LINK_MU"] + 12]
    assert 0.6 <= mu.min().item() and mu.max().item() <= 1.0 and mu.std().item() > 0.05
    obs, extras = env.reset()
    assert obs["policy"].shape == (256, 22)
    for _ in range(20):
        obs, rew, term, trunc, extras = env.step(torch.randn(256, 6, device=env.device))
    assert rew.shape == (256,) and term.dtype == torch.bool
    assert set(extras["log"]) == {"Episode_Reward/" + k for k in zm.SU_REWARD_TERMS} | {
        "Episode_Termination/died", "Episode_Termination/time_out"}
    assert env.curriculum_stage == 0 and env.reward_scales["feet_downward_4"] == 0.0
    w = RslRlVecEnvWrapper(env)
    o = w.get_observations()
    assert o["policy"].shape == (256, 22)
    env.close()
