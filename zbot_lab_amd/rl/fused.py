"""ctypes binding of ``libzbot_ppo.so`` (``include/zbot_ppo.h``): the PPO minibatch update of the
rsl_rl ActorCritic as hand-written fp32 MFMA kernels (``csrc/ppo_mlp.hip``).

``FusedUpdate`` drives ``PPO.update_steps`` on a GPU: per minibatch one ``zbp_minibatch`` call
(actor / critic forward, the clipped-surrogate + clipped-value + entropy loss, the backward pass into
every ``.grad``) and, on one GPU, one ``zbp_optimizer_step`` (adaptive learning rate, global-norm
clipping, Adam on torch's own optimizer state, workspace re-pack). With a process group the gradient
all-reduce, the rate rule, clipping and ``torch.optim.Adam`` stay torch's (``PPO.update_steps``). The
semantics are PPO.update_steps' (``zbot_lab_amd/rl/ppo.py``; rsl_rl, reference
``agents/rsl_rl_ppo_cfg.py:65-91``); the GPU test ``tests/test_gpu_ppo_fused.py`` holds the two
paths together. Nothing here runs on the CPU: the torch path serves CPU tensors.
"""
from __future__ import annotations

import ctypes as C
import os

import torch
import torch.nn as nn

from .._native import ZbotError

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(HERE, "libzbot_ppo.so")
MAXL = 4
MAXP = 24


class Net(C.Structure):
    _fields_ = [("n_layers", C.c_int32), ("dim", C.c_int32 * (MAXL + 1)), ("w", C.c_void_p * MAXL),
                ("b", C.c_void_p * MAXL), ("gw", C.c_void_p * MAXL), ("gb", C.c_void_p * MAXL)]


class Batch(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("critic_obs", C.c_void_p), ("actions", C.c_void_p), ("values", C.c_void_p),
                ("advantages", C.c_void_p), ("returns", C.c_void_p), ("log_prob", C.c_void_p), ("mu", C.c_void_p),
                ("sigma", C.c_void_p), ("idx", C.c_void_p), ("idx_offset", C.c_int64), ("batch", C.c_int32),
                ("obs_dim", C.c_int32), ("critic_obs_dim", C.c_int32), ("num_actions", C.c_int32)]


class LossCfg(C.Structure):
    _fields_ = [("clip_param", C.c_float), ("value_loss_coef", C.c_float), ("entropy_coef", C.c_float),
                ("use_clipped_value_loss", C.c_int32)]


class ActIO(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("critic_obs", C.c_void_p), ("noise", C.c_void_p), ("actions", C.c_void_p),
                ("st_obs", C.c_void_p), ("st_critic_obs", C.c_void_p), ("st_actions", C.c_void_p),
                ("st_values", C.c_void_p), ("st_log_prob", C.c_void_p), ("st_mu", C.c_void_p), ("st_sigma", C.c_void_p),
                ("rows", C.c_int32), ("obs_dim", C.c_int32), ("critic_obs_dim", C.c_int32), ("num_actions", C.c_int32),
                ("noise_step", C.c_int32), ("noise_seed", C.c_int32)]


class Params(C.Structure):
    _fields_ = [("n_params", C.c_int32), ("numel", C.c_int64 * MAXP), ("param", C.c_void_p * MAXP),
                ("grad", C.c_void_p * MAXP), ("exp_avg", C.c_void_p * MAXP), ("exp_avg_sq", C.c_void_p * MAXP),
                ("step", C.c_void_p * MAXP)]


EXPORTED = ["zbp_workspace_floats", "zbp_pack", "zbp_minibatch", "zbp_optimizer_step", "zbp_gae", "zbp_act",
            "zbp_env_post", "zbp_last_error"]
_lib = None


_warned = False


def available() -> bool:
    """Whether libzbot_ppo.so is built. When it is not, the PPO update, GAE and rollout run on the
    torch statement (the reference's rsl_rl path) after a one-time warning; the simulator itself has
    no such fallback (libzbot.so is required)."""
    global _warned
    if os.path.exists(LIB_PATH):
        return True
    if not _warned:
        import warnings
        warnings.warn(f"{LIB_PATH} not built (python -m zbot_lab_amd.build): PPO runs on the torch path")
        _warned = True
    return False


def lib():
    """Load libzbot_ppo.so (raises ZbotError when it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ZbotError(f"{LIB_PATH} not built: run `python -m zbot_lab_amd.build` (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.zbp_last_error.restype = C.c_char_p
    L.zbp_workspace_floats.restype = C.c_int64
    L.zbp_workspace_floats.argtypes = [C.POINTER(Net), C.POINTER(Net), C.c_int32]
    L.zbp_pack.argtypes = [C.POINTER(Net), C.POINTER(Net), P, C.c_int32, P]
    L.zbp_minibatch.argtypes = [C.POINTER(Net), C.POINTER(Net), P, P, C.POINTER(Batch), C.POINTER(LossCfg), P, P, P]
    L.zbp_optimizer_step.argtypes = [C.POINTER(Params), P, P, P, C.c_float, C.c_float, C.c_float, C.c_float,
                                     C.c_float, C.POINTER(Net), C.POINTER(Net), P, C.c_int32, C.c_int32, P]
    L.zbp_gae.argtypes = [P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_int32, P, P]
    L.zbp_act.argtypes = [C.POINTER(Net), C.POINTER(Net), P, C.POINTER(ActIO), P, C.c_int32, P]
    L.zbp_env_post.argtypes = [P, P, P, P, C.c_float, P, P, P, P, P, C.c_int32, P]
    for n in ("zbp_pack", "zbp_minibatch", "zbp_optimizer_step", "zbp_gae", "zbp_act", "zbp_env_post"):
        getattr(L, n).restype = C.c_int
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().zbp_last_error()
        raise ZbotError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def _p(t: torch.Tensor | None):
    if t is None:
        return None
    if not t.is_contiguous():
        raise ZbotError("tensor passed to libzbot_ppo must be contiguous")
    return C.c_void_p(t.data_ptr())


def gae(storage, last_values: torch.Tensor, gamma: float, lam: float, normalize: bool) -> None:
    """RolloutStorage.compute_returns in three launches (zbp_gae): returns, advantages and their
    normalisation, in place in the storage."""
    sc = getattr(storage, "_gae_scratch", None)
    if sc is None:
        sc = storage._gae_scratch = torch.zeros(512, device=storage.values.device)
    lv = last_values.reshape(-1).contiguous()
    _check(lib().zbp_gae(_p(storage.rewards), _p(storage.dones), _p(storage.values), _p(lv), _p(storage.returns),
                         _p(storage.advantages), storage.num_transitions_per_env, storage.num_envs, float(gamma),
                         float(lam), int(normalize), _p(sc), C.c_void_p(torch.cuda.current_stream(sc.device).cuda_stream)),
           "zbp_gae")


def mlp_layers(seq: nn.Sequential):
    """The Linear layers of an rsl_rl MLP, or None when it is not Linear / ELU alternating."""
    lin = [m for m in seq if isinstance(m, nn.Linear)]
    acts = [m for m in seq if not isinstance(m, nn.Linear)]
    if len(lin) < 1 or len(lin) > MAXL or len(acts) != len(lin) - 1 or not all(isinstance(a, nn.ELU) and a.alpha == 1.0
                                                                                 for a in acts):
        return None
    return lin


def supported(policy, batch: int) -> bool:
    """Whether the fused kernels cover this ActorCritic and minibatch size (ELU MLPs, <= 4 layers,
    inputs <= 32, hidden multiples of 32 up to 256, critic output 1, batch a multiple of 32, fp32 on a
    GPU)."""
    try:
        la, lc = mlp_layers(policy.actor), mlp_layers(policy.critic)
    except TypeError:
        return False
    if la is None or lc is None or batch % 32 or batch < 32 or not available():
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 for p in policy.parameters()):
        return False
    for lin, out in ((la, None), (lc, 1)):
        if lin[0].in_features > 32 or lin[-1].out_features > 32 or (out and lin[-1].out_features != out):
            return False
        if any(m.out_features % 32 or m.out_features > 256 for m in lin[:-1]):
            return False
    return la[-1].out_features <= 13


def _net(layers) -> Net:
    n = Net()
    n.n_layers = len(layers)
    dims = [layers[0].in_features] + [m.out_features for m in layers]
    for i, d in enumerate(dims):
        n.dim[i] = d
    for i, m in enumerate(layers):
        for t in (m.weight, m.bias):
            if t.grad is None:
                t.grad = torch.zeros_like(t)
        n.w[i], n.b[i] = m.weight.data_ptr(), m.bias.data_ptr()
        n.gw[i], n.gb[i] = m.weight.grad.data_ptr(), m.bias.grad.data_ptr()
    return n


class FusedUpdate:
    """The PPO update's minibatches on libzbot_ppo (one GPU: the optimizer too)."""

    def __init__(self, alg, batch: int):
        self.alg = alg
        self.batch = batch
        pol = alg.policy
        self.la, self.lc = mlp_layers(pol.actor), mlp_layers(pol.critic)
        if pol.std.grad is None:
            pol.std.grad = torch.zeros_like(pol.std)
        self.stats = torch.zeros(4, device=pol.std.device)  # kl mean, value loss, surrogate, entropy
        self.loss = LossCfg(alg.clip_param, alg.value_loss_coef, alg.entropy_coef, int(alg.use_clipped_value_loss))
        self._bind()

    def _bind(self) -> None:
        """(Re)read every pointer: parameters, .grad buffers, workspace (after a checkpoint load)."""
        self.na, self.nc = _net(self.la), _net(self.lc)
        n = lib().zbp_workspace_floats(C.byref(self.na), C.byref(self.nc), self.batch)
        if n < 0:
            raise ZbotError("zbp_workspace_floats: unsupported shapes")
        if getattr(self, "ws", None) is None or self.ws.numel() != n:
            self.ws = torch.zeros(int(n), device=self.alg.policy.std.device)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.ws.device).cuda_stream)

    def pack(self) -> None:
        _check(lib().zbp_pack(C.byref(self.na), C.byref(self.nc), _p(self.ws), self.batch, self._stream()), "zbp_pack")

    def minibatch(self, storage, indices: torch.Tensor, offset: int) -> torch.Tensor:
        """Gradients of minibatch rows indices[offset:offset + batch] into every .grad; returns the
        stats tensor (kl mean, value loss, surrogate loss, entropy)."""
        flat = lambda t: t.flatten(0, 1)  # noqa: E731
        obs, cobs = flat(storage.observations), flat(storage.critic_observations)
        b = Batch()
        b.obs, b.critic_obs, b.actions = obs.data_ptr(), cobs.data_ptr(), flat(storage.actions).data_ptr()
        b.values, b.advantages = storage.values.data_ptr(), storage.advantages.data_ptr()
        b.returns, b.log_prob = storage.returns.data_ptr(), storage.actions_log_prob.data_ptr()
        b.mu, b.sigma = storage.mu.data_ptr(), storage.sigma.data_ptr()
        b.idx, b.idx_offset, b.batch = indices.data_ptr(), int(offset), self.batch
        b.obs_dim, b.critic_obs_dim, b.num_actions = obs.shape[-1], cobs.shape[-1], storage.actions.shape[-1]
        pol = self.alg.policy
        _check(lib().zbp_minibatch(C.byref(self.na), C.byref(self.nc), _p(pol.std), _p(pol.std.grad), C.byref(b),
                                   C.byref(self.loss), _p(self.ws), _p(self.stats), self._stream()), "zbp_minibatch")
        return self.stats

    def _adam_state(self) -> Params:
        """torch.optim.Adam's own state (created here in torch's layout if the optimizer has not
        stepped yet), in the optimizer's param order."""
        opt = self.alg.optimizer
        ps = [p for g in opt.param_groups for p in g["params"]]
        if len(ps) > MAXP:
            raise ZbotError("too many parameter tensors for zbp_optimizer_step")
        g = opt.param_groups[0]
        if g.get("weight_decay", 0) or g.get("amsgrad") or g.get("maximize"):
            raise ZbotError("zbp_optimizer_step implements plain Adam")
        # one step counter drives every parameter's bias correction in the kernels (they read step[0]
        # and write it back to all): refuse states whose counters differ (a partially loaded state)
        steps = {float(opt.state[p]["step"]) if opt.state[p] else 0.0 for p in ps}
        if len(steps) > 1:
            raise ZbotError(f"zbp_optimizer_step needs one Adam step count for every parameter, got {sorted(steps)}")
        P = Params()
        P.n_params = len(ps)
        for i, p in enumerate(ps):
            st = opt.state[p]
            if not st:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            P.numel[i] = p.numel()
            P.param[i], P.grad[i] = p.data_ptr(), p.grad.data_ptr()
            P.exp_avg[i], P.exp_avg_sq[i] = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            P.step[i] = st["step"].data_ptr()
        self._steps = [opt.state[p]["step"] for p in ps]  # (keep the tensors alive)
        return P

    def _grads_all_from_minibatch(self) -> bool:
        """The optimizer's parameters are exactly what zbp_minibatch writes gradients for (both nets'
        weights and biases, the std): then the norm can come from its per-tile sums."""
        ps = [p for g in self.alg.optimizer.param_groups for p in g["params"]]
        want = sum(n.dim[l] * n.dim[l + 1] + n.dim[l + 1] for n in (self.na, self.nc) for l in range(n.n_layers))
        return sum(p.numel() for p in ps) == want + int(self.na.dim[self.na.n_layers])

    def optimizer_step(self, acc: torch.Tensor, grads_from_minibatch: bool = False) -> None:
        """Adaptive learning rate (on the minibatch KL), global-norm clipping and Adam on one GPU,
        then the re-pack; acc[0:3] += value loss, surrogate, entropy. grads_from_minibatch: the .grad
        buffers are untouched since the last minibatch() (one GPU), so the gradient norm is taken from
        that call's per-tile sums of squares instead of a launch of its own."""
        alg = self.alg
        g = alg.optimizer.param_groups[0]
        b1, b2 = g["betas"]
        dk = alg.desired_kl if (alg.desired_kl is not None and alg.schedule == "adaptive") else 0.0
        if not hasattr(self, "_params"):
            self._params = self._adam_state()
            self._norm_ok = self._grads_all_from_minibatch()
        nfm = 1 if (grads_from_minibatch and self._norm_ok) else 0
        _check(lib().zbp_optimizer_step(C.byref(self._params), _p(alg.lr_t), _p(self.stats), _p(acc), float(dk),
                                        float(alg.max_grad_norm), float(b1), float(b2), float(g["eps"]),
                                        C.byref(self.na), C.byref(self.nc), _p(self.ws), self.batch, nfm,
                                        self._stream()),
               "zbp_optimizer_step")

    # -- rollout (runner._rollout's policy step and post-step bookkeeping, one launch each)
    def act(self, obs: torch.Tensor, critic_obs: torch.Tensor, storage, kernel_noise: bool = False) -> torch.Tensor:
        """PPO.act on zbp_act: the actions (a static buffer) and the transition fields written
        straight into the storage slot ``storage.step``; the noise is torch.randn_like's draw, as in
        the torch path, or with ``kernel_noise`` the kernel's own counter-based standard normal (no
        torch launch; another stream of the same distribution). The weight images are re-packed at a
        rollout's first step (parameters may have changed outside zbp_optimizer_step: a torch
        optimizer, a checkpoint load)."""
        k = storage.step
        if k >= storage.num_transitions_per_env:
            raise OverflowError("rollout buffer overflow")
        if k == 0:
            self.pack()
        n, na = obs.shape[0], storage.actions.shape[-1]
        if getattr(self, "_act_out", None) is None or self._act_out.shape != (n, na):
            self._act_out = torch.zeros(n, na, device=obs.device)
            self._noise = torch.zeros(n, na, device=obs.device)
        if not kernel_noise:
            torch.randn(n, na, out=self._noise, device=obs.device)
        obs, critic_obs = obs.contiguous(), critic_obs.contiguous()
        io = ActIO()
        io.obs, io.critic_obs, io.actions = obs.data_ptr(), critic_obs.data_ptr(), self._act_out.data_ptr()
        io.noise = None if kernel_noise else self._noise.data_ptr()
        io.noise_step = k
        if getattr(self, "_noise_seed", None) is None:  # from torch's generator: per-rank seeds carry over
            self._noise_seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        io.noise_seed = self._noise_seed
        io.st_obs, io.st_critic_obs = storage.observations[k].data_ptr(), storage.critic_observations[k].data_ptr()
        io.st_actions, io.st_values = storage.actions[k].data_ptr(), storage.values[k].data_ptr()
        io.st_log_prob, io.st_mu = storage.actions_log_prob[k].data_ptr(), storage.mu[k].data_ptr()
        io.st_sigma = storage.sigma[k].data_ptr()
        io.rows, io.obs_dim, io.critic_obs_dim, io.num_actions = n, obs.shape[-1], critic_obs.shape[-1], na
        _check(lib().zbp_act(C.byref(self.na), C.byref(self.nc), _p(self.alg.policy.std), C.byref(io), _p(self.ws),
                             self.batch, self._stream()), "zbp_act")
        return self._act_out

    def env_post(self, storage, rewards: torch.Tensor, dones: torch.Tensor, time_outs, gamma: float,
                 cur_rew: torch.Tensor, cur_len: torch.Tensor, ep_stats: torch.Tensor) -> None:
        """PPO.process_env_step + the runner's episode statistics (zbp_env_post); advances the slot."""
        k = storage.step
        tout = time_outs
        if tout is not None and tout.dtype not in (torch.bool, torch.uint8):  # (bool: one byte, 0 / 1)
            tout = tout.to(torch.uint8)
        if dones.dtype != torch.int64:
            dones = dones.to(torch.int64)
        _check(lib().zbp_env_post(_p(rewards.contiguous()), _p(dones.contiguous()),
                                  None if tout is None else _p(tout.contiguous()), _p(storage.values[k]),
                                  float(gamma), _p(storage.rewards[k]), _p(storage.dones[k]), _p(cur_rew), _p(cur_len),
                                  _p(ep_stats), rewards.shape[0], self._stream()), "zbp_env_post")
        self._tout = tout  # (alive until the stream has consumed it)
        storage.step += 1

    def rebind(self) -> None:
        """After parameters or optimizer state were replaced (checkpoint load)."""
        self._bind()
        if hasattr(self, "_params"):
            del self._params
