"""The PPO minibatch update on libzbot_ppo.so (fp32 MFMA kernels, zbot_lab_amd/rl/fused.py) against
the torch autograd statement of the same update (zbot_lab_amd/rl/ppo.py, rsl_rl semantics,
reference agents/rsl_rl_ppo_cfg.py:65-91): the gradients of one minibatch (every weight, bias and
the std) and its loss / KL statistics, and a whole update (20 minibatches with the adaptive learning
rate, clipping and Adam) from the same snapshot. Tolerances are fp32 summation-order ones."""
from __future__ import annotations

import copy
import os

import pytest

pytestmark = pytest.mark.gpu


def _alg(hidden, obs_dim=23, act=6, envs=512, steps=24, seed=0):
    import torch
    from zbot_lab_amd.rl.ppo import PPO, ActorCritic
    torch.manual_seed(seed)
    pol = ActorCritic(obs_dim, obs_dim, act, actor_hidden_dims=hidden, critic_hidden_dims=hidden)
    alg = PPO(pol, device="cuda:0")
    alg.init_storage(envs, steps, obs_dim, obs_dim, act)
    st = alg.storage
    g = torch.Generator(device="cuda:0").manual_seed(seed + 1)
    for t in (st.observations, st.critic_observations, st.actions, st.rewards, st.values, st.mu):
        t.copy_(torch.randn(t.shape, device="cuda:0", generator=g))
    st.critic_observations.copy_(st.observations + 0.1 * st.critic_observations)
    st.sigma.copy_(0.5 + torch.rand(st.sigma.shape, device="cuda:0", generator=g))
    st.dones.copy_((torch.rand(st.dones.shape, device="cuda:0", generator=g) < 0.05).float())
    with torch.no_grad():  # old log-probs near the current policy's, so ratios straddle the clip range
        pol.update_distribution(st.observations.flatten(0, 1))
        lp = pol.get_actions_log_prob(st.actions.flatten(0, 1)).view(steps, envs, 1)
        st.actions_log_prob.copy_(lp + 0.3 * torch.randn(lp.shape, device="cuda:0", generator=g))
        st.values.copy_(pol.evaluate(st.critic_observations.flatten(0, 1)).view(steps, envs, 1)
                        + 0.3 * torch.randn(st.values.shape, device="cuda:0", generator=g))
    st.step = steps
    alg.compute_returns(st.critic_observations[-1])
    st.step = steps
    alg.draw_minibatch_indices()
    return alg


def _torch_minibatch(alg, i):
    """update_steps' loss for minibatch i of the first epoch, backward into .grad (autograd)."""
    import torch
    gen = alg.storage.mini_batch_generator(alg.num_mini_batches, 1, alg.mb_indices)
    for k, mbt in enumerate(gen):
        if k == i:
            break
    obs_b, cobs_b, act_b, tv_b, adv_b, ret_b, old_lp_b, old_mu_b, old_sigma_b = mbt
    pol = alg.policy
    pol.update_distribution(obs_b)
    lp_b = pol.get_actions_log_prob(act_b)
    value_b = pol.evaluate(cobs_b)
    mu_b, sigma_b, entropy_b = pol.action_mean, pol.action_std, pol.entropy
    with torch.no_grad():
        kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1e-5)
                       + (old_sigma_b.square() + (old_mu_b - mu_b).square()) / (2.0 * sigma_b.square()) - 0.5, dim=-1)
    ratio = torch.exp(lp_b - torch.squeeze(old_lp_b))
    s1 = -torch.squeeze(adv_b) * ratio
    s2 = -torch.squeeze(adv_b) * torch.clamp(ratio, 1.0 - alg.clip_param, 1.0 + alg.clip_param)
    surr = torch.max(s1, s2).mean()
    vc = tv_b + (value_b - tv_b).clamp(-alg.clip_param, alg.clip_param)
    vl = torch.max((value_b - ret_b).pow(2), (vc - ret_b).pow(2)).mean()
    loss = surr + alg.value_loss_coef * vl - alg.entropy_coef * entropy_b.mean()
    alg.optimizer.zero_grad(set_to_none=False)
    loss.backward()
    return torch.stack([kl.mean(), vl.detach(), surr.detach(), entropy_b.mean().detach()])


@pytest.mark.parametrize("rows", ["reg", "lds"])
@pytest.mark.parametrize("hidden", [[128, 128, 128], [256, 256, 128]], ids=["v2-nets", "standup-nets"])
def test_fused_minibatch_gradients_match_autograd(gpu, hidden, rows, monkeypatch):
    """rows: the register-resident row kernel (k_rows_reg, these shapes' default) or the LDS one
    (ZBP_ROWS=lds, every other shape)."""
    import torch
    from zbot_lab_amd.rl import fused
    if rows == "lds":
        monkeypatch.setenv("ZBP_ROWS", "lds")
    alg = _alg(hidden)
    mb = alg.storage.num_envs * alg.storage.num_transitions_per_env // alg.num_mini_batches
    assert fused.supported(alg.policy, mb)
    for i in (0, 3):
        ref_stats = _torch_minibatch(alg, i)
        ref = [p.grad.detach().clone() for p in alg.policy.parameters()]
        f = fused.FusedUpdate(alg, mb)
        f.pack()
        stats = f.minibatch(alg.storage, alg.mb_indices, i * mb).clone()
        torch.cuda.synchronize()
        got = [p.grad.detach().clone() for p in alg.policy.parameters()]
        names = [n for n, _ in alg.policy.named_parameters()]
        for n, r, g in zip(names, ref, got):
            scale = r.abs().max().item()
            err = (g - r).abs().max().item()
            assert err <= 1e-5 * scale + 1e-9, (i, n, err, scale)
        torch.testing.assert_close(stats, ref_stats, rtol=1e-5, atol=1e-7)


def test_fused_minibatch_gradients_small_ragged_batch(gpu):
    """A 96-row minibatch (16 envs x 24 steps / 4): not a multiple of 64, so the LDS row kernel runs
    (k_rows_reg needs whole 64-row workgroups), and k_wgrad splits its 3 row chunks one per split."""
    from zbot_lab_amd.rl import fused
    for hidden in ([256, 256, 128], [128, 128, 128]):
        alg = _alg(hidden, envs=16)
        mb = alg.storage.num_envs * alg.storage.num_transitions_per_env // alg.num_mini_batches
        assert mb == 96 and fused.supported(alg.policy, mb)
        ref_stats = _torch_minibatch(alg, 1)
        ref = [p.grad.detach().clone() for p in alg.policy.parameters()]
        f = fused.FusedUpdate(alg, mb)
        f.pack()
        stats = f.minibatch(alg.storage, alg.mb_indices, mb).clone()
        got = [p.grad.detach().clone() for p in alg.policy.parameters()]
        for (n, _), r, g in zip(alg.policy.named_parameters(), ref, got):
            assert (g - r).abs().max().item() <= 1e-5 * r.abs().max().item() + 1e-9, (hidden, n)
        import torch
        torch.testing.assert_close(stats, ref_stats, rtol=1e-5, atol=1e-7)


def test_fused_update_matches_torch_update(gpu, monkeypatch):
    """A whole update (5 epochs x 4 minibatches: rate rule, clipping, Adam) from one snapshot, the
    fused path against the torch path: parameters, learning rate and the logged loss sums."""
    import torch
    alg_f = _alg([128, 128, 128], seed=3)
    alg_t = copy.deepcopy(alg_f)
    monkeypatch.setenv("ZBOT_PPO_FUSED", "0")
    alg_t.optimizer = torch.optim.Adam(alg_t.policy.parameters(), lr=alg_t.lr_t, fused=True, capturable=True)
    p0 = torch.cat([p.detach().flatten() for p in alg_t.policy.parameters()]).clone()
    alg_t.update_steps()
    monkeypatch.setenv("ZBOT_PPO_FUSED", "1")
    alg_f.update_steps()
    assert alg_f._fused is not None and alg_t._fused is None
    torch.cuda.synchronize()
    pf = torch.cat([p.detach().flatten() for p in alg_f.policy.parameters()])
    pt = torch.cat([p.detach().flatten() for p in alg_t.policy.parameters()])
    moved = (pt - p0).abs()
    d = (pf - pt).abs()
    print(f"\nfused vs torch update: max |dp| {d.max().item():.3g} (99.9% {d.quantile(0.999).item():.3g}), "
          f"max move {moved.max().item():.3g}, lr {float(alg_f.lr_t):.4g} / {float(alg_t.lr_t):.4g}")
    assert moved.max() > 0
    # Adam normalises each coordinate by its own gradient history: a gradient that summation order
    # moves by 1e-6 moves the step of a near-zero coordinate by up to its whole size, so the bound is
    # on the bulk and on the worst coordinate separately
    assert d.quantile(0.999) <= 1e-3 * moved.max()
    assert d.max() <= 0.05 * moved.max()
    assert abs(float(alg_f.lr_t) - float(alg_t.lr_t)) <= 1e-7 + 1e-5 * float(alg_t.lr_t)
    torch.testing.assert_close(alg_f.update_sums, alg_t.update_sums, rtol=1e-4, atol=1e-6)
    opt_f, opt_t = alg_f.optimizer, alg_t.optimizer
    for pf_, pt_ in zip(alg_f.policy.parameters(), alg_t.policy.parameters()):
        assert float(opt_f.state[pf_]["step"]) == float(opt_t.state[pt_]["step"]) == 20.0


@pytest.mark.parametrize("hidden", [[128, 128, 128], [256, 256, 128]], ids=["v2-nets", "standup-nets"])
def test_optimizer_norm_from_minibatch(gpu, hidden, monkeypatch):
    """zbp_optimizer_step's gradient norm from k_reduce's per-tile sums of squares (the one-GPU path)
    against k_norm's recomputation from .grad, with clipping active: the same parameters, rate and
    step up to the two norms' summation order."""
    import torch
    monkeypatch.setenv("ZBOT_PPO_FUSED", "1")
    a0 = _alg(hidden, seed=7)
    a1 = copy.deepcopy(a0)
    res = []
    for alg, nfm in ((a0, True), (a1, False)):
        alg.max_grad_norm = 0.05  # well below the gradients' norm: the clip coefficient scales every step
        f = alg.fused_update()
        assert f is not None
        f.pack()
        sums = torch.zeros_like(alg.update_sums)
        for i in range(3):
            f.minibatch(alg.storage, alg.mb_indices, i * f.batch)
            f.optimizer_step(sums, grads_from_minibatch=nfm)
        assert f._norm_ok
        torch.cuda.synchronize()
        res.append((torch.cat([p.detach().flatten() for p in alg.policy.parameters()]), float(alg.lr_t),
                    [float(alg.optimizer.state[p]["step"]) for p in alg.policy.parameters()], sums.clone()))
    (p0, lr0, st0, s0), (p1, lr1, st1, s1) = res
    assert st0 == st1 and set(st0) == {3.0}
    assert lr0 == lr1
    torch.testing.assert_close(p0, p1, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(s0, s1, rtol=1e-5, atol=1e-7)


def test_fused_gae_matches_torch(gpu, monkeypatch):
    """RolloutStorage.compute_returns on zbp_gae (three launches) against the torch recursion:
    returns, advantages and their normalisation."""
    import torch
    alg = _alg([128, 128, 128], envs=4096, seed=5)
    st = alg.storage
    last = torch.randn(st.num_envs, 1, device="cuda:0")
    monkeypatch.setenv("ZBOT_PPO_FUSED", "0")
    st.compute_returns(last, 0.99, 0.95, True)
    ret_t, adv_t = st.returns.clone(), st.advantages.clone()
    monkeypatch.setenv("ZBOT_PPO_FUSED", "1")
    st.returns.zero_()
    st.advantages.zero_()
    st.compute_returns(last, 0.99, 0.95, True)
    torch.cuda.synchronize()
    # the recursion rounds every op as torch's kernels do (no fma contraction): returns agree to the
    # last bit in practice; the normalisation's mean / std reduce in another order than torch's
    print(f"\nGAE fused vs torch: returns max |d| {(st.returns - ret_t).abs().max().item():.3g}, "
          f"advantages max |d| {(st.advantages - adv_t).abs().max().item():.3g}")
    torch.testing.assert_close(st.returns, ret_t, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(st.advantages, adv_t, rtol=2e-5, atol=2e-6)
    assert abs(float(st.advantages.mean())) < 1e-5 and abs(float(st.advantages.std()) - 1.0) < 1e-4


@pytest.mark.parametrize("rows", ["reg", "lds", "reg-small", "split", "split-small"])
@pytest.mark.parametrize("hidden", [[128, 128, 128], [256, 256, 128]], ids=["v2-nets", "standup-nets"])
def test_fused_act_matches_torch_policy(gpu, hidden, rows, monkeypatch):
    """zbp_act (the rollout's policy step, runner._rollout) against PPO.act's torch statement with the
    same standard-normal draw: actions, mu, sigma, log-probabilities, values and the observations in
    the storage slot (fp32 summation-order tolerances); rows not a multiple of 32 included. rows: the
    register-resident forward (k_act_reg, rollouts of >= 4096 rows; reg-small: forced at 200 rows) or
    the LDS one (ZBP_ACT=lds, and every smaller rollout)."""
    import torch
    from zbot_lab_amd.rl import fused
    if rows == "lds":
        monkeypatch.setenv("ZBP_ROWS", "lds")
        monkeypatch.setenv("ZBP_ACT", "lds")
    if rows == "reg-small":  # (the register-resident forward forced below its row threshold)
        monkeypatch.setenv("ZBP_ACT", "reg")
    if rows == "reg":  # (k_act_reg itself; the 128-wide nets take k_act_split by default, round 6)
        monkeypatch.setenv("ZBP_ACT", "reg")
    if rows.startswith("split"):  # k_act_split: the 128-wide nets' default from 4096 rows; forced below
        if hidden[0] != 128:
            pytest.skip("k_act_split serves the 128-wide nets")
        if rows == "split-small":
            monkeypatch.setenv("ZBP_ACT", "split")
    # (k_act_reg takes rollouts of >= 4096 rows; 16 400 is not a multiple of its 64-row workgroups)
    for envs in {"reg": (16400, 4096), "lds": (4096, 200), "reg-small": (200,), "split": (16400, 4096),
                 "split-small": (200, 40)}[rows]:
        alg = _alg(hidden, envs=envs)
        fu = fused.FusedUpdate(alg, 256)  # (the minibatch size shapes only the update's row buffers)
        st = alg.storage
        st.clear()
        obs = torch.randn(envs, 23, device="cuda:0")
        st.step = 3
        fu.pack()
        a = fu.act(obs, obs, st)
        noise = fu._noise.clone()
        pol = alg.policy
        with torch.no_grad():
            pol.update_distribution(obs)
            mu, sd = pol.action_mean, pol.action_std
            ref_a = mu + sd * noise
            ref_lp = pol.get_actions_log_prob(ref_a)
            ref_v = pol.evaluate(obs)
        torch.cuda.synchronize()
        tol = lambda r: 1e-5 * max(1.0, float(r.abs().max()))  # noqa: E731
        assert (a - ref_a).abs().max() <= tol(ref_a)
        assert (st.actions[3] - ref_a).abs().max() <= tol(ref_a)
        assert (st.mu[3] - mu).abs().max() <= tol(mu)
        assert torch.equal(st.sigma[3], sd.expand_as(st.sigma[3]))
        assert (st.actions_log_prob[3].view(-1) - ref_lp).abs().max() <= tol(ref_lp)
        assert (st.values[3] - ref_v).abs().max() <= tol(ref_v)
        assert torch.equal(st.observations[3], obs) and torch.equal(st.critic_observations[3], obs)


def test_fused_act_kernel_noise(gpu):
    """zbp_act with the in-kernel draw (io->noise NULL, the runner's default): the noise implied by the
    actions, (a - mu) / sigma, is standard normal (moments, tails, no correlation across actions),
    differs between rollout steps and after a re-pack, and repeats for the same counter and step; the
    log-probability and the storage slot are those of the actions drawn."""
    import torch
    from zbot_lab_amd.rl import fused
    envs = 16384
    alg = _alg([128, 128, 128], envs=envs)
    fu = fused.FusedUpdate(alg, 256)
    st = alg.storage
    st.clear()
    obs = torch.randn(envs, 23, device="cuda:0")
    fu.pack()
    draws = {}
    for key, k, repack in (("a", 3, False), ("b", 4, False), ("c", 3, True)):
        if repack:
            fu.pack()
        st.step = k
        a = fu.act(obs, obs, st, kernel_noise=True).clone()
        draws[key] = ((a - st.mu[k]) / st.sigma[k], a, k)
    torch.cuda.synchronize()
    z = draws["a"][0]
    n = z.numel()
    assert abs(float(z.mean())) < 5.0 / n ** 0.5
    assert abs(float(z.std()) - 1.0) < 0.02
    assert abs(float((z.abs() > 1.96).float().mean()) - 0.05) < 0.005
    c = torch.corrcoef(z.T)
    assert float((c - torch.eye(c.shape[0], device=c.device)).abs().max()) < 0.05
    for other in ("b", "c"):
        r = torch.corrcoef(torch.stack([z.flatten(), draws[other][0].flatten()]))[0, 1]
        assert abs(float(r)) < 0.05, other
    # the log-probability stored is the drawn actions' under (mu, sigma)
    pol = alg.policy
    with torch.no_grad():
        pol.update_distribution(obs)
        ref_lp = pol.get_actions_log_prob(draws["c"][1])
    assert (st.actions_log_prob[3].view(-1) - ref_lp).abs().max() <= 1e-4 * max(1.0, float(ref_lp.abs().max()))
    assert torch.equal(st.actions[3], draws["c"][1])


def test_fused_env_post_matches_torch(gpu):
    """zbp_env_post against PPO.process_env_step + the runner's episode bookkeeping: storage reward
    with the time-out bootstrap and done exactly, cur_rew / cur_len exactly, ep_stats to fp32
    summation order."""
    import torch
    from zbot_lab_amd.rl import fused
    alg = _alg([128, 128, 128], envs=4096)
    mb = alg.storage.num_envs * alg.storage.num_transitions_per_env // alg.num_mini_batches
    fu = fused.FusedUpdate(alg, mb)
    st = alg.storage
    n = st.num_envs
    g = torch.Generator(device="cuda:0").manual_seed(5)
    rew = torch.randn(n, device="cuda:0", generator=g)
    dones = (torch.rand(n, device="cuda:0", generator=g) < 0.2).long()
    tout = (torch.rand(n, device="cuda:0", generator=g) < 0.5) & (dones > 0)
    cur_rew = torch.randn(n, device="cuda:0", generator=g)
    cur_len = torch.randint(0, 100, (n,), device="cuda:0", generator=g).float()
    ep = torch.tensor([1.0, 2.0, 3.0], device="cuda:0")
    r_cur, r_len, r_ep = cur_rew.clone(), cur_len.clone(), ep.clone()
    st.step = 5
    val = st.values[5].clone()
    fu.env_post(st, rew, dones, tout, alg.gamma, cur_rew, cur_len, ep)
    torch.cuda.synchronize()
    ref_r = rew + alg.gamma * torch.squeeze(val * tout.unsqueeze(1).float(), 1)
    assert torch.equal(st.rewards[5].view(-1), ref_r) and torch.equal(st.dones[5].view(-1), dones.float())
    assert st.step == 6
    r_cur += rew
    r_len += 1
    d = dones > 0
    r_ep += torch.stack([torch.where(d, r_cur, 0.0).sum(), torch.where(d, r_len, 0.0).sum(), d.sum().float()])
    r_cur.masked_fill_(d, 0.0)
    r_len.masked_fill_(d, 0.0)
    assert torch.equal(cur_rew, r_cur) and torch.equal(cur_len, r_len)
    assert torch.allclose(ep, r_ep, rtol=1e-5, atol=1e-3)
