"""PPO as rsl-rl-lib runs it for ``PPORunnerCfgV2`` (reference ``scripts/rsl_rl/train.py:158-205``,
``agents/rsl_rl_ppo_cfg.py:65-91``; algorithm walk-through in the reference's
``ppo_learning_notes.md:99-181,417-421,521-548``). rsl_rl itself is not installed in this image, so
this is a compatible restatement: same module names and tensor semantics, same checkpoint keys.

* ``ActorCritic``: ELU MLPs (actor 23 -> 128x3 -> 6, critic 23 -> 128x3 -> 1), state-independent
  Gaussian std initialised to ``init_noise_std``.
* ``RolloutStorage``: [T, N] transitions; GAE(gamma, lam) with time-out bootstrapping done in
  ``PPO.process_env_step`` (rewards += gamma * V(s) * time_out), advantages normalised over the
  whole batch.
* ``PPO.update``: ``num_learning_epochs`` x ``num_mini_batches`` shuffled minibatches; adaptive LR
  from the Gaussian KL (desired_kl, x/÷1.5, bounded [1e-5, 1e-2]); clipped surrogate + clipped
  value loss - entropy bonus; global-norm gradient clipping; Adam.
* On a GPU the minibatches run on ``libzbot_ppo.so`` (``zbot_lab_amd/rl/fused.py``, hand-written fp32
  MFMA kernels: forward, loss, backward in four launches per minibatch; on one GPU the adaptive
  learning rate, clipping and Adam fused too) whenever the nets fit its limits; the torch autograd path
  below is the same statement and serves CPU tensors (``ZBOT_PPO_FUSED=0`` selects it on a GPU).
* Multi-GPU: one process per GPU; per minibatch ONE all-reduce averages the
  flattened gradient with the minibatch's KL mean appended (one bucket, 292 KB for v2) before the
  learning-rate rule and clipping — RCCL over xGMI when the process group is ``nccl`` (torch's
  name for RCCL on ROCm), gloo on CPU. Every rank applies the rule to the same averaged KL.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn

_ACT = {"elu": nn.ELU, "relu": nn.ReLU, "tanh": nn.Tanh, "selu": nn.SELU, "lrelu": nn.LeakyReLU}


def _split(batch: int) -> int:
    """Chunks for the split-K weight gradient: the largest s <= 64 dividing the batch with >= 256
    rows per chunk (1 = plain GEMM)."""
    for s in (64, 48, 32, 24, 16, 8, 4, 2):
        if batch % s == 0 and batch // s >= 256:
            return s
    return 1


class _LinearSplitK(torch.autograd.Function):
    """y = x W^T + b with the weight gradient dW = dY^T X computed as a batched GEMM over row chunks
    plus a sum. The PPO minibatches are 24 576 rows x 128 features: as one GEMM, dW is a 128 x 128
    output with a 24 576-long reduction that the BLAS library tiles into a handful of workgroups
    (81 us per call, 22 % of a training iteration's GPU time); split 64 ways it fills the chip."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, go):
        x, w = ctx.saved_tensors
        gx = go @ w if ctx.needs_input_grad[0] else None
        rows = x.shape[0]
        s = _split(rows)
        if s > 1:
            gw = torch.bmm(go.view(s, rows // s, -1).transpose(1, 2), x.view(s, rows // s, -1)).sum(0)
        else:
            gw = go.t() @ x
        return gx, gw, go.sum(0)


class PPOLinear(nn.Linear):
    """``nn.Linear`` (same parameters and state-dict keys) whose training-time backward uses the
    split-K weight gradient on the GPU; inference and TorchScript export see a plain linear layer."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if torch.is_grad_enabled() and x.is_cuda and x.dim() == 2:
            return _LinearSplitK.apply(x, self.weight, self.bias)
        return nn.functional.linear(x, self.weight, self.bias)


def _mlp(n_in: int, hidden: list, n_out: int, activation: str) -> nn.Sequential:
    layers, d = [], n_in
    for h in hidden:
        layers += [PPOLinear(d, h), _ACT[activation]()]
        d = h
    layers.append(PPOLinear(d, n_out))
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    is_recurrent = False

    def __init__(self, num_actor_obs: int, num_critic_obs: int, num_actions: int,
                 actor_hidden_dims=(128, 128, 128), critic_hidden_dims=(128, 128, 128),
                 activation: str = "elu", init_noise_std: float = 1.0, **_):
        super().__init__()
        self.actor = _mlp(num_actor_obs, list(actor_hidden_dims), num_actions, activation)
        self.critic = _mlp(num_critic_obs, list(critic_hidden_dims), 1, activation)
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution: torch.distributions.Normal | None = None
        torch.distributions.Normal.set_default_validate_args(False)

    # -- rsl_rl interface
    def update_distribution(self, obs: torch.Tensor) -> None:
        mean = self.actor(obs)
        self.distribution = torch.distributions.Normal(mean, mean * 0.0 + self.std)

    def act(self, obs: torch.Tensor) -> torch.Tensor:
        self.update_distribution(obs)
        # = Normal.sample(); written as mean + std * N(0, 1) because torch.normal(tensor, tensor)
        # is not capturable in a HIP graph on this ROCm build (randn_like is)
        d = self.distribution
        return d.mean + d.stddev * torch.randn_like(d.mean)

    def act_inference(self, obs: torch.Tensor) -> torch.Tensor:
        return self.actor(obs)

    def evaluate(self, obs: torch.Tensor) -> torch.Tensor:
        return self.critic(obs)

    def get_actions_log_prob(self, actions: torch.Tensor) -> torch.Tensor:
        return self.distribution.log_prob(actions).sum(dim=-1)

    @property
    def action_mean(self) -> torch.Tensor:
        return self.distribution.mean

    @property
    def action_std(self) -> torch.Tensor:
        return self.distribution.stddev

    @property
    def entropy(self) -> torch.Tensor:
        return self.distribution.entropy().sum(dim=-1)

    def reset(self, dones=None):
        return None


class RolloutStorage:
    """[T, N] buffers of one rollout (rsl_rl ``RolloutStorage``, non-recurrent)."""

    def __init__(self, num_envs: int, num_transitions_per_env: int, obs_dim: int, critic_obs_dim: int,
                 action_dim: int, device):
        T, N = num_transitions_per_env, num_envs
        f = dict(device=device, dtype=torch.float32)
        self.observations = torch.zeros(T, N, obs_dim, **f)
        self.critic_observations = torch.zeros(T, N, critic_obs_dim, **f)
        self.actions = torch.zeros(T, N, action_dim, **f)
        self.rewards = torch.zeros(T, N, 1, **f)
        self.dones = torch.zeros(T, N, 1, **f)
        self.values = torch.zeros(T, N, 1, **f)
        self.actions_log_prob = torch.zeros(T, N, 1, **f)
        self.mu = torch.zeros(T, N, action_dim, **f)
        self.sigma = torch.zeros(T, N, action_dim, **f)
        self.returns = torch.zeros(T, N, 1, **f)
        self.advantages = torch.zeros(T, N, 1, **f)
        self.num_envs, self.num_transitions_per_env = N, T
        self.step = 0

    def add(self, obs, critic_obs, actions, rewards, dones, values, log_prob, mu, sigma) -> None:
        if self.step >= self.num_transitions_per_env:
            raise OverflowError("rollout buffer overflow")
        k = self.step
        self.observations[k].copy_(obs)
        self.critic_observations[k].copy_(critic_obs)
        self.actions[k].copy_(actions)
        self.rewards[k].copy_(rewards.view(-1, 1))
        self.dones[k].copy_(dones.view(-1, 1))
        self.values[k].copy_(values)
        self.actions_log_prob[k].copy_(log_prob.view(-1, 1))
        self.mu[k].copy_(mu)
        self.sigma[k].copy_(sigma)
        self.step += 1

    def clear(self) -> None:
        self.step = 0

    def compute_returns(self, last_values: torch.Tensor, gamma: float, lam: float,
                        normalize_advantage: bool = True) -> None:
        if self.values.is_cuda and os.environ.get("ZBOT_PPO_FUSED", "1") != "0":
            from . import fused  # the same recursion in three launches (zbp_gae)
            if fused.available():
                fused.gae(self, last_values, gamma, lam, normalize_advantage)
                return
        adv = torch.zeros_like(last_values)
        for k in reversed(range(self.num_transitions_per_env)):
            next_values = last_values if k == self.num_transitions_per_env - 1 else self.values[k + 1]
            not_terminal = 1.0 - self.dones[k]
            delta = self.rewards[k] + not_terminal * gamma * next_values - self.values[k]
            adv = delta + not_terminal * gamma * lam * adv
            self.returns[k] = adv + self.values[k]
        # in place: the buffers stay ordinary tensors even when this runs under inference_mode
        self.advantages.copy_(self.returns - self.values)
        if normalize_advantage:
            self.advantages.copy_((self.advantages - self.advantages.mean()) / (self.advantages.std() + 1e-8))

    def mini_batch_generator(self, num_mini_batches: int, num_epochs: int, indices: torch.Tensor):
        """rsl_rl's generator: ONE permutation of the batch (``indices``, drawn by the caller) serves
        every epoch; minibatch i of each epoch is its i-th slice. The permutation comes in as a
        tensor so that a graph-captured update reads whatever the last draw wrote."""
        batch = self.num_envs * self.num_transitions_per_env
        mb = batch // num_mini_batches
        flat = lambda t: t.flatten(0, 1)  # noqa: E731
        obs, cobs, act = flat(self.observations), flat(self.critic_observations), flat(self.actions)
        val, ret, lp = flat(self.values), flat(self.returns), flat(self.actions_log_prob)
        adv, mu, sig = flat(self.advantages), flat(self.mu), flat(self.sigma)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                b = indices[i * mb:(i + 1) * mb]
                yield obs[b], cobs[b], act[b], val[b], adv[b], ret[b], lp[b], mu[b], sig[b]


class PPO:
    def __init__(self, policy: ActorCritic, num_learning_epochs: int = 5, num_mini_batches: int = 4,
                 clip_param: float = 0.2, gamma: float = 0.99, lam: float = 0.95, value_loss_coef: float = 1.0,
                 entropy_coef: float = 0.005, learning_rate: float = 1e-3, max_grad_norm: float = 1.0,
                 use_clipped_value_loss: bool = True, schedule: str = "adaptive", desired_kl: float = 0.01,
                 device="cpu", multi_gpu_cfg: dict | None = None, **_):
        self.device = device
        self.policy = policy.to(device)
        # the learning rate lives on the device: the adaptive-KL rule updates it without a host
        # sync per minibatch; on GPUs Adam is the fused kernel reading it
        self.lr_t = torch.tensor(float(learning_rate), device=device)
        on_gpu = torch.device(device).type == "cuda"
        self.optimizer = torch.optim.Adam(self.policy.parameters(), lr=self.lr_t if on_gpu else learning_rate,
                                          fused=on_gpu or None, capturable=on_gpu)
        self.update_sums = torch.zeros(3, device=device)  # value, surrogate, entropy of the last update
        self.storage: RolloutStorage | None = None
        self.clip_param, self.gamma, self.lam = clip_param, gamma, lam
        self.num_learning_epochs, self.num_mini_batches = num_learning_epochs, num_mini_batches
        self.value_loss_coef, self.entropy_coef = value_loss_coef, entropy_coef
        self.max_grad_norm, self.use_clipped_value_loss = max_grad_norm, use_clipped_value_loss
        self.schedule, self.desired_kl = schedule, desired_kl
        self.is_multi_gpu = multi_gpu_cfg is not None
        self.gpu_global_rank = multi_gpu_cfg["global_rank"] if multi_gpu_cfg else 0
        self.gpu_world_size = multi_gpu_cfg["world_size"] if multi_gpu_cfg else 1
        self._tr: dict = {}
        self.generator: torch.Generator | None = None
        self._fused = None  # rl/fused.FusedUpdate, built at the first GPU update
        # world > 1 on the fused path: each minibatch is [graph: kernels, flatten] -> all-reduce ->
        # [graph: average, unflatten, rate rule, clip, Adam, re-pack] (capture_update_segments)
        self._flat = None
        self._seg_pre, self._seg_post = None, None

    def init_storage(self, num_envs: int, num_transitions_per_env: int, obs_dim: int, critic_obs_dim: int,
                     action_dim: int) -> None:
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, obs_dim, critic_obs_dim, action_dim,
                                      self.device)
        mb = num_envs * num_transitions_per_env // self.num_mini_batches
        self.mb_indices = torch.arange(mb * self.num_mini_batches, device=self.device)

    def draw_minibatch_indices(self) -> None:
        """The update's batch permutation (rsl_rl ``mini_batch_generator``: one ``randperm`` per
        update), drawn eagerly into a fixed buffer: a captured update replays with the new draw."""
        torch.randperm(self.mb_indices.numel(), out=self.mb_indices, generator=self.generator)

    # -- rollout
    def act(self, obs: torch.Tensor, critic_obs: torch.Tensor) -> torch.Tensor:
        actions = self.policy.act(obs).detach()
        self._tr = dict(obs=obs, critic_obs=critic_obs, actions=actions,
                        values=self.policy.evaluate(critic_obs).detach(),
                        log_prob=self.policy.get_actions_log_prob(actions).detach(),
                        mu=self.policy.action_mean.detach(), sigma=self.policy.action_std.detach())
        return actions

    def process_env_step(self, rewards: torch.Tensor, dones: torch.Tensor, extras: dict) -> None:
        r = rewards.clone()
        if "time_outs" in extras:  # bootstrap on time-outs
            r += self.gamma * torch.squeeze(self._tr["values"] * extras["time_outs"].unsqueeze(1).to(self.device), 1)
        t = self._tr
        self.storage.add(t["obs"], t["critic_obs"], t["actions"], r, dones, t["values"], t["log_prob"], t["mu"],
                         t["sigma"])
        self.policy.reset(dones)

    def compute_returns(self, last_critic_obs: torch.Tensor) -> None:
        last_values = self.policy.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam, normalize_advantage=True)

    # -- multi-GPU
    def broadcast_parameters(self) -> None:
        if not self.is_multi_gpu:
            return
        for p in self.policy.state_dict().values():
            dist.broadcast(p.data, src=0)

    def reduce_parameters(self, kl_mean: torch.Tensor | None = None) -> torch.Tensor | None:
        """Average the gradients over ranks: one flattened bucket, one all-reduce. The minibatch's
        KL mean rides in the same bucket (no separate scalar collective); it is
        consumed only by the learning-rate rule right before ``optimizer.step``, so averaging it
        after the backward pass is the same as rsl_rl's all-reduce before it."""
        if not self.is_multi_gpu:
            return kl_mean
        grads = [p.grad.view(-1) for p in self.policy.parameters() if p.grad is not None]
        if kl_mean is not None:
            grads.append(kl_mean.reshape(1))
        flat = torch.cat(grads)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat /= self.gpu_world_size
        off = 0
        for p in self.policy.parameters():
            if p.grad is not None:
                n = p.numel()
                p.grad.data.copy_(flat[off:off + n].view_as(p.grad.data))
                off += n
        return flat[off] if kl_mean is not None else None

    def _adapt_learning_rate(self, kl_mean: torch.Tensor) -> None:
        """rsl_rl's adaptive schedule on the device: lr / 1.5 above 2 desired_kl, x 1.5 below half of
        it, within [1e-5, 1e-2]; every rank applies it to the same averaged KL, so the rates stay
        identical without rsl_rl's broadcast from rank 0."""
        with torch.no_grad():
            lr = self.lr_t
            up = (kl_mean > 0.0) & (kl_mean < self.desired_kl / 2.0)
            new_lr = torch.where(kl_mean > self.desired_kl * 2.0, torch.clamp(lr / 1.5, min=1e-5),
                                 torch.where(up, torch.clamp(lr * 1.5, max=1e-2), lr))
            self.lr_t.copy_(new_lr)
        if not isinstance(self.optimizer.param_groups[0]["lr"], torch.Tensor):
            lr_f = float(self.lr_t)  # CPU: plain float learning rate
            for g in self.optimizer.param_groups:
                g["lr"] = lr_f

    # -- update
    def update(self) -> dict:
        self.draw_minibatch_indices()
        self.update_steps()
        return self.update_stats()

    def update_stats(self) -> dict:
        n = self.num_learning_epochs * self.num_mini_batches
        m = (self.update_sums / n).tolist()
        return {"value_function": m[0], "surrogate": m[1], "entropy": m[2]}

    def fused_update(self):
        """The libzbot_ppo driver for this policy and minibatch size, or None (CPU tensors, nets
        outside the kernels' limits, or ZBOT_PPO_FUSED=0)."""
        if self._fused is None and os.environ.get("ZBOT_PPO_FUSED", "1") != "0" and self.storage is not None:
            from . import fused
            mb = self.storage.num_envs * self.storage.num_transitions_per_env // self.num_mini_batches
            if fused.supported(self.policy, mb):
                self._fused = fused.FusedUpdate(self, mb)
        return self._fused

    def fused_rollout(self):
        """The libzbot_ppo driver for the rollout's policy steps (zbp_act / zbp_env_post), or None
        (CPU, nets outside the kernels' limits, ZBOT_PPO_FUSED=0 or ZBOT_ROLLOUT_FUSED=0)."""
        if os.environ.get("ZBOT_ROLLOUT_FUSED", "1") == "0" or self.storage is None or not self.storage.values.is_cuda:
            return None
        return self.fused_update()

    def invalidate_fused(self) -> None:
        """Parameters / optimizer state replaced (checkpoint load): rebuild the fused driver."""
        self._fused = None
        self._flat, self._seg_pre, self._seg_post = None, None, None

    def update_steps(self) -> None:
        """All minibatch updates with no host synchronisation (graph-capturable on a GPU), over the
        permutation in ``mb_indices`` (``draw_minibatch_indices`` first)."""
        sums = self.update_sums
        sums.zero_()
        adaptive = self.desired_kl is not None and self.schedule == "adaptive"
        f = self.fused_update()
        if f is not None:
            self._update_steps_fused(f, sums, adaptive)
            return
        for (obs_b, cobs_b, act_b, target_values_b, adv_b, returns_b, old_lp_b, old_mu_b,
             old_sigma_b) in self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs,
                                                               self.mb_indices):
            # rsl_rl calls policy.act() here; the sampled actions are unused, so only the
            # distribution is rebuilt (no random draw inside the update)
            self.policy.update_distribution(obs_b)
            lp_b = self.policy.get_actions_log_prob(act_b)
            value_b = self.policy.evaluate(cobs_b)
            mu_b, sigma_b, entropy_b = self.policy.action_mean, self.policy.action_std, self.policy.entropy

            kl_mean = None
            if adaptive:
                with torch.no_grad():
                    kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1e-5)
                                   + (old_sigma_b.square() + (old_mu_b - mu_b).square()) / (2.0 * sigma_b.square())
                                   - 0.5, dim=-1)
                    kl_mean = torch.mean(kl)

            ratio = torch.exp(lp_b - torch.squeeze(old_lp_b))
            surrogate = -torch.squeeze(adv_b) * ratio
            surrogate_clipped = -torch.squeeze(adv_b) * torch.clamp(ratio, 1.0 - self.clip_param,
                                                                    1.0 + self.clip_param)
            surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
            if self.use_clipped_value_loss:
                value_clipped = target_values_b + (value_b - target_values_b).clamp(-self.clip_param,
                                                                                    self.clip_param)
                value_loss = torch.max((value_b - returns_b).pow(2), (value_clipped - returns_b).pow(2)).mean()
            else:
                value_loss = (returns_b - value_b).pow(2).mean()
            loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_b.mean()

            self.optimizer.zero_grad(set_to_none=False)
            loss.backward()
            kl_mean = self.reduce_parameters(kl_mean)
            if adaptive:
                self._adapt_learning_rate(kl_mean)
            nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
            self.optimizer.step()

            sums += torch.stack([value_loss.detach(), surrogate_loss.detach(), entropy_b.mean().detach()])
        # release the last minibatch's autograd graph: a live graph keeps its AccumulateGrad nodes,
        # which remember the stream they were created on, and a later HIP-graph capture of this
        # update would then synchronise with that (default) stream and break the capture
        self.policy.distribution = None
        self.storage.clear()

    def _update_steps_fused(self, f, sums: torch.Tensor, adaptive: bool) -> None:
        """update_steps on libzbot_ppo: the same minibatches (rsl_rl's generator order), each one
        zbp_minibatch (forward, loss, backward into every .grad), then zbp_optimizer_step (the adaptive
        rate on the minibatch KL, global-norm clipping, Adam, the re-pack). With world > 1 the gradients
        and the KL are averaged over the ranks in between: one flat bucket, one all-reduce per minibatch
        (reference train.py:125-132; rsl_rl's reduce_parameters), the steps on either side of it HIP
        graphs once ``capture_update_segments`` ran."""
        f.pack()
        mb = f.batch
        if self.is_multi_gpu:
            if self._flat is None:
                ps = self._grad_params()
                self._flat = torch.zeros(sum(p.numel() for p in ps) + 1, device=self.lr_t.device)
            for _ in range(self.num_learning_epochs):
                for i in range(self.num_mini_batches):
                    if self._seg_pre is not None:
                        self._seg_pre[i].replay()
                    else:
                        self._mgpu_pre(f, i * mb)
                    dist.all_reduce(self._flat, op=dist.ReduceOp.SUM)
                    if self._seg_post is not None:
                        self._seg_post.replay()
                    else:
                        self._mgpu_post(f, sums)
        else:
            for _ in range(self.num_learning_epochs):
                for i in range(self.num_mini_batches):
                    f.minibatch(self.storage, self.mb_indices, i * mb)
                    f.optimizer_step(sums, grads_from_minibatch=True)
        self.storage.clear()

    def _grad_params(self) -> list:
        """The optimizer's parameters in bucket order (every one has a .grad on the fused path)."""
        return [p for g in self.optimizer.param_groups for p in g["params"]]

    def _mgpu_pre(self, f, offset: int) -> None:
        """One rank's minibatch: gradients into .grad, then [every .grad, the minibatch KL] into the
        flat all-reduce bucket."""
        stats = f.minibatch(self.storage, self.mb_indices, offset)
        torch.cat([p.grad.reshape(-1) for p in self._grad_params()] + [stats[0:1]], out=self._flat)

    def _mgpu_post(self, f, sums: torch.Tensor) -> None:
        """The ranks' average back into .grad and the KL slot, then the fused optimizer step."""
        self._flat.div_(self.gpu_world_size)
        ps = self._grad_params()
        off = 0
        views = []
        for p in ps:
            views.append(self._flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        torch._foreach_copy_([p.grad for p in ps], views)
        f.stats[0:1].copy_(self._flat[off:off + 1])
        f.optimizer_step(sums)

    def capture_update_segments(self) -> bool:
        """world > 1, fused path, after one eager update (the driver, its Adam state and the bucket
        exist): capture the minibatch segments on either side of the all-reduce as HIP graphs -- one
        per minibatch slot before it (its row offset; reused by every epoch) and one after it. The
        all-reduce stays outside the graphs (a collective is never captured). Returns
        whether the segments are in use."""
        f = self._fused
        if not self.is_multi_gpu or f is None or self._flat is None or not hasattr(f, "_params"):
            return False
        mb = f.batch
        pre = []
        for i in range(self.num_mini_batches):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._mgpu_pre(f, i * mb)
            pre.append(g)
        post = torch.cuda.CUDAGraph()
        with torch.cuda.graph(post):
            self._mgpu_post(f, self.update_sums)
        self._seg_pre, self._seg_post = pre, post
        return True

    def restore_learning_rate(self) -> None:
        """After ``optimizer.load_state_dict``: the checkpoint's rate becomes ``lr_t`` (the adaptive
        rule's state) and every param group reads ``lr_t`` again. ``load_state_dict`` replaces a
        tensor ``lr`` with a new tensor, which the adaptive rule would no longer update."""
        lr = self.optimizer.param_groups[0]["lr"]
        self.lr_t.copy_(lr.detach().reshape(()) if torch.is_tensor(lr) else torch.tensor(float(lr)))
        for g in self.optimizer.param_groups:
            g["lr"] = self.lr_t if torch.is_tensor(g["lr"]) else float(self.lr_t)

    @property
    def learning_rate(self) -> float:
        return float(self.lr_t)
