"""The runner's fused rollout (zbp_act + zbp_env_post wired into OnPolicyRunner._rollout, with the
static action buffer and the pack at slot 0) against the torch rollout (PPO.act /
process_env_step / the episode bookkeeping), from one env state, policy and RNG state; and a
checkpoint load between two learn() calls with the HIP graphs on (the captured graphs hold the old
fused driver's workspace and must be re-captured).

The env is walking v2 at 4096 envs: the two rollouts feed the simulator actions that differ only by
the policy forward's summation order (MFMA vs hipBLASLt, ~1e-7), which contact switches can amplify
in a few envs over the rollout, so every field is compared per env and at most 1 % of the envs may
leave tolerance at any step (the first step: none).
"""
from __future__ import annotations

import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _runner(tmp_path, steps=8, use_graph=False):
    import zbot_lab_amd
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2, RslRlVecEnvWrapper
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    cfg.scene.num_envs = 4096
    env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-walking-v2", cfg=cfg))
    tc = PPORunnerCfgV2()
    tc.num_steps_per_env = steps
    return env, OnPolicyRunner(env, tc.to_dict(), log_dir=str(tmp_path), device="cuda:0", use_graph=use_graph)


def test_fused_rollout_matches_torch_rollout(gpu, tmp_path, monkeypatch):
    import torch
    env, runner = _runner(tmp_path)
    sim = env.unwrapped.sim
    env.unwrapped.episode_length_buf = torch.randint_like(env.unwrapped.episode_length_buf, high=1000)
    with torch.no_grad():  # a few random-action steps: feet in contact, some envs near their episode end
        for _ in range(30):
            env.step(torch.randn(4096, 6, device="cuda:0"))
    s0, wc0 = sim.get_state().clone(), sim.get_contact_cache().clone()
    obs0 = env.get_observations()
    obs0 = (obs0["policy"] if isinstance(obs0, dict) else obs0).clone()
    cur0 = (torch.randn(4096, device="cuda:0"), torch.randint(0, 50, (4096,), device="cuda:0").float())
    rec = {}
    monkeypatch.setenv("ZBOT_KERNEL_NOISE", "0")  # (torch's draw on both paths: same noise, same rollout)
    for mode in ("1", "0"):
        monkeypatch.setenv("ZBOT_ROLLOUT_FUSED", mode)
        sim.set_state(s0)
        sim.set_contact_cache(wc0)
        runner.cur_rew.copy_(cur0[0])
        runner.cur_len.copy_(cur0[1])
        st = runner.alg.storage
        st.clear()
        torch.cuda.manual_seed(1234)
        with torch.no_grad():
            last = runner._rollout(obs0.clone())
        torch.cuda.synchronize()
        assert (runner.alg.fused_rollout() is not None) == (mode == "1")
        rec[mode] = {k: getattr(st, k).clone() for k in ("observations", "actions", "rewards", "dones", "values",
                                                         "actions_log_prob", "mu", "sigma")}
        rec[mode].update(cur_rew=runner.cur_rew.clone(), cur_len=runner.cur_len.clone(), ep=runner.ep_stats.clone(),
                         last=last.clone(), step=st.step)
    f, t = rec["1"], rec["0"]
    assert f["step"] == t["step"] == 8
    assert torch.equal(f["observations"][0], t["observations"][0])
    tol = {"observations": 5e-3, "actions": 5e-3, "rewards": 2e-3, "dones": 0.0, "values": 5e-3,
           "actions_log_prob": 5e-3, "mu": 5e-3, "sigma": 0.0}
    for k, a in tol.items():
        for s in range(8):
            d = (f[k][s] - t[k][s]).abs().reshape(4096, -1).amax(dim=1)
            bad = (d > a * (1 + t[k][s].abs().reshape(4096, -1).amax(dim=1))).float().mean().item()
            assert bad <= (0.0 if s == 0 else 0.01), (k, s, bad)
    for k in ("cur_rew", "cur_len"):
        bad = ((f[k] - t[k]).abs() > 2e-3 * (1 + t[k].abs())).float().mean().item()
        assert bad <= 0.01, (k, bad)
    ep_f, ep_t = f["ep"].tolist(), t["ep"].tolist()
    print(f"\nfused vs torch rollout: ep_stats {ep_f} / {ep_t}")
    assert ep_t[2] > 0 and abs(ep_f[2] - ep_t[2]) <= 0.01 * ep_t[2] + 1
    assert abs(ep_f[1] / ep_f[2] - ep_t[1] / ep_t[2]) <= 0.02 * ep_t[1] / ep_t[2]
    env.close()


def test_checkpoint_load_between_learn_calls_with_graphs(gpu, tmp_path):
    """learn() with the rollout and update graphs, save, learn on (graphs replayed), load the
    checkpoint, learn again: the graphs are dropped and re-captured with the new fused driver, the
    loaded parameters are the ones trained on, and the optimizer's step count continues from the
    checkpoint's."""
    import torch
    env, runner = _runner(tmp_path, steps=24, use_graph=True)
    runner.learn(3, init_at_random_ep_len=True)
    assert runner._graph is not None and runner._update_graph is not None
    ck = str(tmp_path / "ck.pt")
    runner.save(ck)
    saved = copy.deepcopy(runner.alg.policy.state_dict())
    runner.learn(2)
    moved = any(not torch.equal(saved[k], v) for k, v in runner.alg.policy.state_dict().items())
    assert moved
    runner.load(ck)
    assert runner._graph is None and runner._update_graph is None
    for k, v in runner.alg.policy.state_dict().items():
        assert torch.equal(saved[k], v), k
    log = runner.learn(3)
    assert runner._graph is not None and runner._update_graph is not None
    steps = {float(runner.alg.optimizer.state[p]["step"]) for p in runner.alg.policy.parameters()}
    assert steps == {20.0 * 6}, steps          # 3 updates before the checkpoint + 3 after the load
    assert all(np.isfinite(r["loss/value_function"]) for r in log[-3:])
    after = runner.alg.policy.state_dict()
    assert any(not torch.equal(saved[k], v) for k, v in after.items())
    env.close()


@pytest.mark.parametrize("task", ["zbot-6b-walking-v2", "zbot-6b-walking-v4", "zbot-6b-walking-m-v0"])
def test_native_log_accumulator_matches_per_step_sum(gpu, task):
    """zb_set_log_accumulator: the step's finalize launch adds the log's current values
    to the caller's accumulator every step. Against the per-step torch sum of extras["log"] (the runner's
    earlier gather / index_add path) over 60 random-action steps with resets: identical (same fp32
    additions in the same order); resets do not add; None unregisters."""
    import torch
    import zbot_lab_amd
    from zbot_lab_amd import model as zm
    cfg = zbot_lab_amd.tasks.load_cfg(task)
    cfg.scene.num_envs = 1024
    env = zbot_lab_amd.make(task, cfg=cfg)
    env.reset()
    env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
    sim = env.sim
    acc = torch.zeros(zm.LOG_LEN + zm.LOG_COUNTS, device=sim.device)
    sim.set_log_accumulator(acc)
    ref = torch.zeros_like(acc)
    g = torch.Generator(device=sim.device).manual_seed(3)
    for k in range(60):
        env.step(torch.randn(1024, 6, device=sim.device, generator=g) * 2)
        ref += torch.cat([sim.log_buffer, sim.log_count_buffer.to(torch.float32)])
        if k == 30:
            sim.reset(torch.arange(8, device=sim.device))
    torch.cuda.synchronize()
    assert ref[zm.LOG_LEN:].sum() > 0  # some envs terminated
    assert torch.equal(acc, ref)
    sim.set_log_accumulator(None)
    env.step(torch.zeros(1024, 6, device=sim.device))
    torch.cuda.synchronize()
    assert torch.equal(acc, ref)
    env.close()


@pytest.mark.parametrize("task", ["zbot-6b-walking-v2", "zbot-6b-standup-v0", "zbot-6b-walking-v4",
                                  "zbot-6b-walking-m-v0"])
def test_done_buffer_matches_flags(gpu, task):
    """zb_set_done_buffer: the wrapper's dones (written by the step kernel's epilogue) equal
    (terminated | truncated).long() every step, over steps with terminations and time-outs."""
    import torch
    import zbot_lab_amd
    from zbot_lab_amd.rl.vecenv import RslRlVecEnvWrapper
    cfg = zbot_lab_amd.tasks.load_cfg(task)
    cfg.scene.num_envs = 1000  # not a multiple of the 4 envs per wave: the ragged last wave
    env = zbot_lab_amd.make(task, cfg=cfg)
    w = RslRlVecEnvWrapper(env)
    assert w._dones is not None
    env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
    g = torch.Generator(device=env.device).manual_seed(5)
    seen = torch.zeros(2, dtype=torch.long, device=env.device)
    for _ in range(50):
        _, _, dones, extras = w.step(torch.randn(1000, 6, device=env.device, generator=g) * 2)
        term, trunc = env.sim.terminated, env.sim.truncated
        assert dones.dtype == torch.long and torch.equal(dones, (term | trunc).to(torch.long))
        seen += torch.stack([term.sum(), trunc.sum()]).to(torch.long)
    assert int(seen.sum()) > 0
    env.close()


def test_runner_uses_native_log_accumulator(gpu, tmp_path):
    """The runner registers the accumulator and its per-iteration log means equal the torch path's."""
    import torch
    env, runner = _runner(tmp_path, steps=24, use_graph=False)
    torch.manual_seed(0)
    log = runner.learn(2, init_at_random_ep_len=True)
    assert runner._native_acc is not None
    keys = [k for k in log[-1] if k.startswith("Episode_")]
    assert keys and all(np.isfinite(log[-1][k]) for k in keys)
    # the same rollout's sum through the torch path, from the native accumulator's own inputs
    sim = env.unwrapped.sim
    acc = runner._native_acc.index_select(0, runner._native_idx)
    vals = torch.stack([runner._log_src[i].to(torch.float32).reshape(()) for i in range(len(runner._log_keys))])
    assert acc.shape == vals.shape and sim.log_buffer.data_ptr() == runner._log_src[0]._base.data_ptr()
    env.close()
