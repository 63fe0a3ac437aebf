"""BASELINE.json configs on the HIP path (through the C ABI):

* C1 (4 envs x 1000 random-action steps): lock-step full-state parity at every step (every state
  row incl. the per-term episode sums, obs, reward, flags, the episode log), every DirectRLEnv
  bookkeeping invariant (tests/configs_common.py), and the episode statistics against a
  free-running CPU oracle on the same actions;
* C5 (zbot-6b-standup-v0, 32 768 envs, friction DR on): full-state parity of one step from random
  states and from a 30-step rollout (tests/fullstate.py machinery, every env agrees or is an explained
  discontinuity), and bit-for-bit determinism of a 100-step rollout with DR;
* C4 (PPO at 4096 envs/GPU, PPORunnerCfgV2): a short training run at the configured size.
"""
from __future__ import annotations

import numpy as np
import pytest

import test_gpu_fullstate as F
from configs_common import c1_step_invariants
from fullstate import random_states, task_cfg
from zbot_lab_amd import model as zm

pytestmark = pytest.mark.gpu


def test_c1_four_envs_1000_steps(gpu):
    """C1 on the HIP path: 4 envs x 1000 random-action steps from a full reset. Every step, the
    oracle is set to the GPU's pre-step state and stepped with the same actions (lock-step), and
    every state row (incl. the 13 per-term episode sums), obs, reward and both flags are compared
    under the full-state rule (tests/test_gpu_fullstate.py: inside tolerance or explained by the
    oracle's own rounding-level sensitivity); the episode log of each step with resets must match.
    The DirectRLEnv bookkeeping invariants hold at every step, and the free-running oracle's episode
    statistics (4000 samples; chaotic contact lets the trajectories diverge) stay close."""
    import torch
    from fullstate import compare
    from oracle.pyoracle import OracleSim
    from zbot_lab_amd.sim import ZbotSim
    g = ZbotSim(4, zm.TaskCfg(), device="cuda:0", seed=42)
    o = OracleSim(4, zm.TaskCfg(), seed=42)       # lock-step
    f = OracleSim(4, zm.TaskCfg(), seed=42)       # free-running
    for x in (g, o, f):
        x.reset(None)
    rng = np.random.default_rng(42)
    st = g.get_state().cpu().numpy()
    np.testing.assert_allclose(st, o.get_state(), atol=1e-6)
    rg, ro, dg, do = [], [], [], []
    unexplained, outside, resets = [], 0, 0
    for k in range(1000):
        a = rng.standard_normal((4, 6)).astype(np.float32)
        wc = g.get_contact_cache().cpu().numpy()  # the solver's self-contact cache (lock-step: copied)
        obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
        obs, rew, te, tr = obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy()
        st1 = g.get_state().cpu().numpy()
        log_g = g.read_log()
        c1_step_invariants(k, st, st1, obs, rew, te, tr, log_g[1].cpu().numpy())
        o.set_state(st)
        o.set_contact_cache(wc)
        ob_o, rw_o, te_o, tr_o = o.step(a)
        ratio, ratio_rows, err, tol, flags_bad = compare("v2", st1, o.get_state(), obs, ob_o, rew, rw_o, (te, tr),
                                                         (te_o, tr_o), st, 1)
        bad = np.nonzero(ratio > 1)[0]
        if len(bad):
            outside += len(bad)
            fam = F._sensitivity("v2", 4, 42, st, [a], o.get_state(), ob_o, rw_o, (te_o, tr_o), st, 1, wc)
            F._report("v2", f"C1 lock-step, step {k}", ratio, ratio_rows, err, tol, flags_bad, fam, F._row_names("v2"))
            sens = np.max(np.stack(list(fam.values())), axis=0)
            unexplained += [(k, int(e)) for e in bad if not F._explained(ratio[e], sens[e])]
        elif (te | tr).any():  # the same envs reset: the episode log of this step agrees
            resets += 1
            mg, cg = (x.cpu().numpy() for x in log_g)
            mo, co = o.read_log()
            np.testing.assert_array_equal(cg, co)
            np.testing.assert_allclose(mg[:len(mo)], mo, rtol=1e-3, atol=1e-3)
        st = st1
        _, r2, t2, u2 = f.step(a)
        rg.append(rew.mean()); ro.append(r2.mean()); dg.append((te | tr).mean()); do.append((t2 | u2).mean())
    assert not unexplained, f"C1 lock-step: unexplained (step, env) {unexplained[:20]}"
    assert outside <= 0.02 * 4000, outside
    assert resets >= 10, resets
    rg, ro, dg, do = map(np.asarray, (rg, ro, dg, do))
    assert abs(rg.mean() - ro.mean()) <= 0.25 * abs(ro.mean()) + 0.05, (rg.mean(), ro.mean())
    assert abs(dg.mean() - do.mean()) <= 0.5 * do.mean() + 0.01, (dg.mean(), do.mean())


def _friction(n, seed):
    rng = np.random.default_rng(seed)
    buckets = rng.uniform(0.6, 1.0, 64).astype(np.float32)   # standup.py:124-136 static friction buckets
    return buckets[rng.integers(0, 64, (n, 12))]


def test_c5_standup_32768_dr_full_state(gpu):
    import torch
    from oracle.pyoracle import OracleSim
    from zbot_lab_amd.sim import ZbotSim
    n, seed = 32768, 23
    cfg = task_cfg("standup")
    g = ZbotSim(n, cfg, device="cuda:0", seed=seed)
    o = OracleSim(n, cfg, seed=seed)
    st = random_states("standup", o, n, seed=303)                     # random per-link friction rows too
    g.set_state(torch.from_numpy(st).cuda())
    a = np.random.default_rng(11).normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    assert F._check("standup", "C5 one step, 32768 envs, DR", n, seed, st, [a], out, g.get_state().cpu().numpy(),
                    torch) <= 0.02 * n
    # from a rollout state (30 random steps of the GPU path): lying / rising / fallen poses
    g2 = ZbotSim(n, cfg, device="cuda:0", seed=seed)
    g2.set_link_friction(torch.from_numpy(_friction(n, 5)).cuda())
    g2.reset(None)
    gen = torch.Generator(device="cuda:0").manual_seed(1)
    for _ in range(30):
        g2.step(torch.randn(n, 6, device="cuda:0", generator=gen))
    st2 = g2.get_state().cpu().numpy()
    g3 = ZbotSim(n, cfg, device="cuda:0", seed=seed)
    g3.set_state(torch.from_numpy(st2).cuda())
    obs, rew, te, tr = g3.step(torch.from_numpy(a).cuda())
    out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    assert F._check("standup", "C5 one step from a 30-step DR rollout", n, seed, st2, [a], out,
                    g3.get_state().cpu().numpy(), torch) <= 0.02 * n


def test_c5_standup_32768_dr_determinism(gpu):
    import torch
    from zbot_lab_amd.sim import ZbotSim
    n = 32768
    cfg = task_cfg("standup")
    mu = torch.from_numpy(_friction(n, 9)).cuda()
    outs = []
    for _ in range(2):
        g = ZbotSim(n, cfg, device="cuda:0", seed=77)
        g.set_link_friction(mu)
        g.reset(None)
        gen = torch.Generator(device="cuda:0").manual_seed(3)
        acc = torch.zeros(n, device="cuda:0")
        for _ in range(100):
            _, r, te, tr = g.step(torch.randn(n, 6, device="cuda:0", generator=gen))
            acc += r
        assert torch.isfinite(acc).all()
        outs.append((g.get_state().cpu().numpy(), acc.cpu().numpy(), g.read_curriculum()))
        g.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]


def test_c4_ppo_4096_envs(gpu, tmp_path):
    """PPORunnerCfgV2 at the configured 4096 envs/GPU: 15 iterations (rollout graph + update)."""
    import zbot_lab_amd
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2, RslRlVecEnvWrapper
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    cfg.scene.num_envs = 4096
    env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-walking-v2", cfg=cfg))
    runner = OnPolicyRunner(env, PPORunnerCfgV2().to_dict(), log_dir=str(tmp_path), device="cuda:0")
    log = runner.learn(15, init_at_random_ep_len=True)
    assert all(np.isfinite(r["loss/value_function"]) and np.isfinite(r["mean_reward"]) for r in log[1:])
    assert log[-1]["mean_episode_length"] > log[1]["mean_episode_length"]
    assert log[-1]["fps"] > 5e5, log[-1]["fps"]      # 98 304 samples per iteration
    env.close()


def test_c5_ppo_standup_32768_envs(gpu, tmp_path):
    """C5's training (zbot-6b-standup-v0 at 32 768 envs, friction DR and random reset poses on,
    Zbot6SUpEnvPPOCfg's [256, 256, 128] nets, reference rsl_rl_ppo_cfg.py:264-289): 5 iterations on
    the fused path (zbp_act rollout, zbp_minibatch / zbp_optimizer_step update): finite losses and
    rewards, the fps floor, and the curriculum counter read from the device (my_curriculum,
    standup.py:99-111: 24 steps per iteration, stage 0 until 24 000 steps)."""
    import zbot_lab_amd
    from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper
    from zbot_lab_amd.rl.cfg import Zbot6SUpEnvPPOCfg
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-standup-v0")
    cfg.scene.num_envs = 32768
    env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-standup-v0", cfg=cfg))
    runner = OnPolicyRunner(env, Zbot6SUpEnvPPOCfg().to_dict(), log_dir=str(tmp_path), device="cuda:0")
    log = runner.learn(5, init_at_random_ep_len=True)
    assert runner.alg._fused is not None          # the fused update and rollout ran
    assert all(np.isfinite(r["loss/value_function"]) and np.isfinite(r["loss/surrogate"])
               and np.isfinite(r["mean_reward"]) for r in log[1:])
    stage, counter = env.unwrapped.sim.read_curriculum()
    assert stage == 0 and counter == 5 * 24, (stage, counter)
    print(f"\nC5 PPO: fps {[round(r['fps']) for r in log]}, learn {[round(r['learn_time'], 4) for r in log]}")
    assert log[-1]["fps"] > 3e6, log[-1]["fps"]      # 786 432 samples per iteration (round 4: 7.0 M/s)
    env.close()
