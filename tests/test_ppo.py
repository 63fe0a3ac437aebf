"""PPO runner: rsl_rl semantics on CPU with a small stand-in env, GAE
against a direct restatement, checkpoint round trip, and the multi-GPU gradient averaging
rehearsed with gloo (world size 2)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2
from zbot_lab_amd.rl.ppo import ActorCritic, PPO, RolloutStorage


class ToyVecEnv:
    """Target reaching with time-outs: reward = -mean (action - target)^2, the target in the obs."""

    def __init__(self, n=64, obs_dim=23, act_dim=6, max_len=20, seed=0):
        self.num_envs, self.num_actions, self.max_episode_length = n, act_dim, max_len
        self.device = "cpu"
        self.g = torch.Generator().manual_seed(seed)
        self.obs_dim = obs_dim
        self.episode_length_buf = torch.zeros(n, dtype=torch.long)
        self.target = torch.rand(n, act_dim, generator=self.g) * 2 - 1

    def _obs(self):
        o = torch.zeros(self.num_envs, self.obs_dim)
        o[:, :self.num_actions] = self.target
        return {"policy": o}

    def get_observations(self):
        return self._obs()

    def step(self, a):
        rew = -(a - self.target).square().mean(dim=1)
        self.episode_length_buf += 1
        tout = self.episode_length_buf >= self.max_episode_length
        self.episode_length_buf[tout] = 0
        self.target[tout] = torch.rand(int(tout.sum()), self.num_actions, generator=self.g) * 2 - 1
        return self._obs(), rew, tout.long(), {"time_outs": tout, "log": {}}


class LogToyEnv(ToyVecEnv):
    """extras["log"] holds one in-place tensor (like the simulator's registered log buffers) plus
    a python int, changing every step."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.k = 0
        self.buf = torch.zeros(1)

    def step(self, a):
        o, r, d, ex = super().step(a)
        self.k += 1
        self.buf[0] = float(self.k)
        ex["log"] = {"Episode_Reward/x": self.buf[0], "Episode_Termination/n": self.k % 2}
        return o, r, d, ex


def test_runner_log_is_mean_over_rollout_steps():
    """rsl_rl appends every step's extras["log"] and logs the mean over the rollout."""
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2
    cfg = PPORunnerCfgV2()
    cfg.num_steps_per_env = 4
    runner = OnPolicyRunner(LogToyEnv(n=16), cfg.to_dict(), log_dir=None, device="cpu")
    log = runner.learn(2)
    assert log[0]["Episode_Reward/x"] == pytest.approx((1 + 2 + 3 + 4) / 4)
    assert log[1]["Episode_Reward/x"] == pytest.approx((5 + 6 + 7 + 8) / 4)
    assert log[1]["Episode_Termination/n"] == pytest.approx(0.5)


def _gae_ref(rew, val, dones, last, gamma, lam):
    T = rew.shape[0]
    adv = np.zeros_like(last)
    ret = np.zeros_like(rew)
    for k in reversed(range(T)):
        nv = last if k == T - 1 else val[k + 1]
        nt = 1.0 - dones[k]
        delta = rew[k] + nt * gamma * nv - val[k]
        adv = delta + nt * gamma * lam * adv
        ret[k] = adv + val[k]
    return ret


def test_gae_matches_restatement():
    T, N = 7, 5
    rng = np.random.default_rng(0)
    st = RolloutStorage(N, T, 3, 3, 2, "cpu")
    st.rewards[:] = torch.tensor(rng.normal(size=(T, N, 1)), dtype=torch.float32)
    st.values[:] = torch.tensor(rng.normal(size=(T, N, 1)), dtype=torch.float32)
    st.dones[:] = torch.tensor(rng.random((T, N, 1)) < 0.2, dtype=torch.float32)
    last = torch.tensor(rng.normal(size=(N, 1)), dtype=torch.float32)
    st.compute_returns(last, 0.99, 0.95, normalize_advantage=False)
    ref = _gae_ref(st.rewards.numpy(), st.values.numpy(), st.dones.numpy(), last.numpy(), 0.99, 0.95)
    np.testing.assert_allclose(st.returns.numpy(), ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(st.advantages.numpy(), ref - st.values.numpy(), rtol=1e-5, atol=1e-6)


def test_actor_critic_shapes_and_log_prob():
    ac = ActorCritic(23, 23, 6)
    obs = torch.randn(8, 23)
    a = ac.act(obs)
    lp = ac.get_actions_log_prob(a)
    d = torch.distributions.Normal(ac.actor(obs), ac.std)
    torch.testing.assert_close(lp, d.log_prob(a).sum(-1))
    assert ac.evaluate(obs).shape == (8, 1)


def test_v2_network_gradient_bucket_size():
    """The flattened gradient all-reduced per minibatch (292,404 B for v2)."""
    ac = ActorCritic(23, 23, 6, actor_hidden_dims=[128, 128, 128], critic_hidden_dims=[128, 128, 128])
    assert sum(p.numel() for p in ac.parameters()) * 4 == 292_404


def test_runner_learns_toy_task_and_checkpoints(tmp_path):
    torch.manual_seed(0)
    env = ToyVecEnv()
    cfg = PPORunnerCfgV2()
    cfg.num_steps_per_env = 16
    cfg.save_interval = 5
    cfg.device = "cpu"
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=str(tmp_path), device="cpu")
    obs = env.get_observations()["policy"]
    err0 = (runner.alg.policy.act_inference(obs) - env.target).abs().mean().item()
    log = runner.learn(30, init_at_random_ep_len=True)
    obs = env.get_observations()["policy"]
    err1 = (runner.alg.policy.act_inference(obs) - env.target).abs().mean().item()
    assert err1 < 0.5 * err0, (err0, err1)
    assert log[-1]["mean_reward"] > log[1]["mean_reward"]
    files = sorted(os.listdir(tmp_path))
    assert "model_0.pt" in files and "model_30.pt" in files
    d = torch.load(tmp_path / "model_30.pt", weights_only=True)
    assert set(d) == {"model_state_dict", "optimizer_state_dict", "iter", "infos"} and d["iter"] == 30
    runner2 = OnPolicyRunner(ToyVecEnv(), cfg.to_dict(), log_dir=None, device="cpu")
    runner2.load(str(tmp_path / "model_30.pt"))
    pol = runner2.get_inference_policy()
    torch.testing.assert_close(pol(obs), runner.alg.policy.act_inference(obs))


def test_adaptive_learning_rate_rule():
    ac = ActorCritic(4, 4, 2)
    alg = PPO(ac, num_learning_epochs=1, num_mini_batches=1, learning_rate=1e-3, desired_kl=0.01)
    alg.init_storage(8, 4, 4, 4, 2)
    st = alg.storage
    with torch.no_grad():
        for k in range(4):
            obs = torch.randn(8, 4)
            a = alg.act(obs, obs)
            alg._tr["mu"] = alg._tr["mu"] + 10.0  # force a large KL between old and new policy
            alg.process_env_step(torch.randn(8), torch.zeros(8), {})
        alg.compute_returns(torch.randn(8, 4))
    alg.update()
    assert alg.learning_rate == pytest.approx(1e-3 / 1.5, rel=1e-6)
    assert st.step == 0


def _dist_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(123 + rank)  # different init per rank: broadcast must unify
    ac = ActorCritic(5, 5, 2, actor_hidden_dims=[8], critic_hidden_dims=[8])
    alg = PPO(ac, num_learning_epochs=2, num_mini_batches=2, multi_gpu_cfg={"global_rank": rank, "world_size": world})
    alg.broadcast_parameters()
    # gradient averaging: rank-specific gradients become the mean
    for p in ac.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    alg.reduce_parameters()
    grads_ok = all(torch.allclose(p.grad, torch.full_like(p, 1.5)) for p in ac.parameters())
    # one PPO update on rank-specific data keeps the replicas identical
    alg.init_storage(6, 3, 5, 5, 2)
    g = torch.Generator().manual_seed(7 + rank)
    with torch.no_grad():
        for _ in range(3):
            obs = torch.randn(6, 5, generator=g)
            alg.act(obs, obs)
            alg.process_env_step(torch.randn(6, generator=g), torch.zeros(6), {})
        alg.compute_returns(torch.randn(6, 5, generator=g))
    alg.generator = torch.Generator().manual_seed(99)  # same shuffles on both ranks
    alg.update()
    flat = torch.cat([p.detach().view(-1) for p in ac.parameters()])
    q.put((rank, grads_ok, flat.numpy(), alg.learning_rate))
    dist.destroy_process_group()


def test_multi_rank_gradient_averaging_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=120) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
    assert all(o[1] for o in out)
    np.testing.assert_allclose(out[0][2], out[1][2], rtol=0, atol=0)
    assert out[0][3] == out[1][3]


@pytest.mark.gpu
def test_gpu_training_runs_with_graphs(gpu, tmp_path):
    """A few PPO iterations on the MI355X simulator: the rollout is replayed from a HIP graph and
    training makes the robot survive longer (episode length grows)."""
    import zbot_lab_amd
    from zbot_lab_amd.rl import RslRlVecEnvWrapper
    env_cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    env_cfg.scene.num_envs = 1024
    agent = PPORunnerCfgV2()
    env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-walking-v2", cfg=env_cfg))
    runner = OnPolicyRunner(env, agent.to_dict(), log_dir=str(tmp_path), device="cuda:0")
    log = runner.learn(40, init_at_random_ep_len=True)
    assert runner._graph is not None and runner._update_graph is not None
    assert all(np.isfinite(r["loss/value_function"]) for r in log)
    assert log[-1]["mean_episode_length"] > log[3]["mean_episode_length"]
    env.close()


@pytest.mark.gpu
def test_gpu_update_graph_matches_eager(gpu):
    """The HIP-graph PPO update (captured after the first, eager update) computes the same update
    as the eager code: from one snapshot (rollout storage, parameters, Adam state, learning rate,
    batch permutation) the graph replay and an eager ``update_steps`` must agree within fp32
    tolerance, over several iterations of real rollouts."""
    import torch

    import zbot_lab_amd
    from zbot_lab_amd.rl import RslRlVecEnvWrapper

    env_cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    env_cfg.scene.num_envs = 512
    env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-walking-v2", cfg=env_cfg))
    torch.manual_seed(0)
    r = OnPolicyRunner(env, PPORunnerCfgV2().to_dict(), log_dir=None, device="cuda:0", use_graph=False,
                       graph_update=True)
    r.learn(1)  # eager update, then the capture
    assert r._update_graph is not None
    alg = r.alg
    params = list(alg.policy.parameters())

    def snapshot():
        st = [{k: v.clone() for k, v in alg.optimizer.state[p].items()} for p in params]
        return [p.detach().clone() for p in params], st, alg.lr_t.clone()

    def restore(snap):  # in place: the graph holds these tensors' addresses
        ps, st, lr = snap
        with torch.no_grad():
            for p, v, s_ in zip(params, ps, st):
                p.copy_(v)
                for k, t in s_.items():
                    alg.optimizer.state[p][k].copy_(t)
            alg.lr_t.copy_(lr)

    obs = env.get_observations()["policy"] if isinstance(env.get_observations(), dict) else env.get_observations()
    for it in range(4):
        with torch.no_grad():
            obs = r._rollout(obs)
            alg.compute_returns(obs)
        alg.draw_minibatch_indices()
        snap = snapshot()
        r._update_graph.replay()
        torch.cuda.synchronize()
        p_graph = torch.cat([p.detach().flatten() for p in params]).clone()
        lr_graph, sums_graph = float(alg.lr_t), alg.update_sums.clone()
        restore(snap)
        alg.update_steps()
        torch.cuda.synchronize()
        p_eager = torch.cat([p.detach().flatten() for p in params])
        assert torch.isfinite(p_graph).all()
        moved = (p_eager - torch.cat([v.flatten() for v in snap[0]])).abs().max()
        assert moved > 0  # the update did something
        assert (p_graph - p_eager).abs().max() <= 1e-6 + 1e-3 * moved, (it, float((p_graph - p_eager).abs().max()))
        assert abs(lr_graph - float(alg.lr_t)) <= 1e-7
        torch.testing.assert_close(sums_graph, alg.update_sums, rtol=1e-4, atol=1e-6)
    env.close()


class ViewLogToyEnv(LogToyEnv):
    """extras["log"] as fixed 0-d views into two device buffers (float means, int32 counts), like
    the walking tasks' zb_read_log buffers: the runner's one-gather-per-buffer accumulation path."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.means = torch.zeros(4)
        self.counts = torch.zeros(2, dtype=torch.int32)
        self._log = {"Episode_Reward/a": self.means[2], "Episode_Reward/b": self.means[0],
                     "Episode_Termination/c": self.counts[1]}

    def step(self, actions):
        o, r, d, ex = super().step(actions)
        self.means.copy_(torch.tensor([1.0, 0.0, 2.0, 0.0]) * self.k)
        self.counts[1] = self.k % 3
        ex["log"] = self._log
        return o, r, d, ex


def test_runner_log_views_accumulate_like_copies():
    """The gather path (_log_views) gives the mean over the rollout's steps of every key, as the
    per-key copy path does."""
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2
    cfg = PPORunnerCfgV2()
    cfg.num_steps_per_env = 4
    runner = OnPolicyRunner(ViewLogToyEnv(n=16), cfg.to_dict(), log_dir=None, device="cpu")
    log = runner.learn(2)
    assert runner._log_groups is not None and len(runner._log_groups) == 2
    assert log[0]["Episode_Reward/a"] == pytest.approx(2 * (1 + 2 + 3 + 4) / 4)
    assert log[0]["Episode_Reward/b"] == pytest.approx((1 + 2 + 3 + 4) / 4)
    assert log[1]["Episode_Termination/c"] == pytest.approx((5 % 3 + 6 % 3 + 7 % 3 + 8 % 3) / 4)


def test_fused_rollout_is_gpu_only(monkeypatch):
    """The fused rollout step (zbp_act / zbp_env_post) serves GPU storage only and can be switched
    off (ZBOT_ROLLOUT_FUSED=0); on the CPU the runner keeps the torch statements."""
    from zbot_lab_amd.rl.ppo import PPO, ActorCritic
    pol = ActorCritic(23, 23, 6)
    alg = PPO(pol, device="cpu")
    assert alg.fused_rollout() is None  # no storage yet
    alg.init_storage(64, 24, 23, 23, 6)
    assert alg.fused_rollout() is None  # CPU tensors
    monkeypatch.setenv("ZBOT_ROLLOUT_FUSED", "0")
    assert alg.fused_rollout() is None
