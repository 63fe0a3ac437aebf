"""``OnPolicyRunner`` with rsl-rl-lib's interface, as the reference's training script drives it
(``scripts/rsl_rl/train.py:158-205``: ``OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=...,
device=...)``, ``runner.learn(num_learning_iterations=max_iterations, init_at_random_ep_len=True)``;
``play.py:150-175``: ``runner.load(path)``, ``runner.get_inference_policy(device=...)``).

Checkpoints keep rsl_rl's keys (``model_state_dict``, ``optimizer_state_dict``, ``iter``,
``infos``) as ``model_{it}.pt``. Multi-GPU follows rsl_rl: when ``WORLD_SIZE > 1`` the process
group must already be initialised (torchrun, one process per GPU; ``nccl`` = RCCL on ROCm), rank 0
logs and saves, parameters are broadcast from rank 0 at start and PPO averages gradients per
minibatch (``PPO.reduce_parameters``).

Speed: the rollout keeps obs/actions on the GPU, the env step is one fused kernel, and episode
statistics are accumulated on the device (one host sync per iteration for the log line). On a GPU
the whole 24-step rollout (policy sampling, the env kernels through the C ABI, storage writes,
statistics) is captured once as a HIP graph and replayed every iteration, and so is the PPO update
(20 minibatches of forward, backward, gradient all-reduce, clipping and fused Adam; the batch
permutation is drawn eagerly into a fixed buffer before each replay); the first iteration runs
both eagerly and serves as the capture warm-up.
"""
from __future__ import annotations

import contextlib
import os
import statistics
import time
from collections import deque

import torch
import torch.distributed as dist

from .ppo import PPO, ActorCritic


@contextlib.contextmanager
def _blas_workspace_fence(device):
    """Drop the BLAS library's cached per-stream workspaces before and after a graph capture. The
    GEMMs of a captured graph keep the workspace address they ran with; a workspace cached from
    eager work (or from another capture) is later reused or freed by code outside the graph, and
    the replay then computes with -- and writes into -- memory that belongs to someone else (seen
    here as a captured PPO update that matched the eager one only until the next capture / eager
    GEMM). Cleared around the capture, the graph allocates its own workspace in its private pool."""
    torch.cuda.synchronize(device)
    torch._C._cuda_clearCublasWorkspaces()
    try:
        yield
    finally:
        torch.cuda.synchronize(device)
        torch._C._cuda_clearCublasWorkspaces()


def _policy_obs(obs):
    return obs["policy"] if isinstance(obs, dict) or hasattr(obs, "keys") else obs


class OnPolicyRunner:
    def __init__(self, env, train_cfg: dict, log_dir: str | None = None, device: str = "cpu",
                 use_graph: bool | None = None, graph_update: bool | None = None):
        self.cfg = train_cfg
        self.alg_cfg = dict(train_cfg["algorithm"])
        self.policy_cfg = dict(train_cfg["policy"])
        self.device = device
        self._dev_is_cuda = torch.device(device).type == "cuda"
        self.env = env
        self._configure_multi_gpu()
        obs = _policy_obs(self.env.get_observations())
        num_obs = obs.shape[1]
        self.alg_cfg.pop("class_name", None)
        self.policy_cfg.pop("class_name", None)
        for k in ("actor_obs_normalization", "critic_obs_normalization"):
            if self.policy_cfg.pop(k, False):
                raise NotImplementedError(f"{k}=True (rsl_rl EmpiricalNormalization) is not implemented")
        policy = ActorCritic(num_obs, num_obs, self.env.num_actions, **self.policy_cfg).to(self.device)
        self.alg = PPO(policy, device=self.device, multi_gpu_cfg=self.multi_gpu_cfg, **self.alg_cfg)
        self.num_steps_per_env = int(train_cfg["num_steps_per_env"])
        self.save_interval = int(train_cfg["save_interval"])
        self.alg.init_storage(self.env.num_envs, self.num_steps_per_env, num_obs, num_obs, self.env.num_actions)
        self.log_dir = log_dir
        self.current_learning_iteration = 0
        self.tot_timesteps = 0
        self.tot_time = 0.0
        self.log: list[dict] = []
        # episode statistics persist across learn() calls (device accumulators, rsl_rl's deques)
        self.rewbuffer, self.lenbuffer = deque(maxlen=100), deque(maxlen=100)
        self.cur_rew = torch.zeros(self.env.num_envs, device=self.device)
        self.cur_len = torch.zeros(self.env.num_envs, device=self.device)
        self.ep_stats = torch.zeros(3, device=self.device)  # reward sum, length sum, count
        self._log_keys, self._log_acc = None, None
        self._native_acc, self._native_idx = None, None  # the step's finalize launch sums the log (zb_set_log_accumulator)
        from .. import GRAPHS_SAFE
        self.use_graph = (torch.device(device).type == "cuda" and GRAPHS_SAFE) if use_graph is None else use_graph
        self._graph = None
        self._g_obs = None
        self._update_graph = None
        # the 20 minibatch updates are captured as a second graph after the first (eager) update;
        # PPO.update_steps releases its autograd graph so the capture sees fresh AccumulateGrad
        # nodes on the capture stream (a live one from the eager update pinned the default stream
        # and broke the capture)
        # Multi-GPU: a collective is never captured. On the fused path each minibatch's kernels before
        # and after its gradient all-reduce are two graphs and the all-reduce runs between them
        # (PPO.capture_update_segments); without the fused driver the update stays eager there
        self.graph_update = self.use_graph if graph_update is None else graph_update

    def _configure_multi_gpu(self) -> None:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        self.is_distributed = world > 1
        if not self.is_distributed:
            self.gpu_global_rank, self.gpu_world_size, self.multi_gpu_cfg = 0, 1, None
            return
        if not dist.is_initialized():
            raise RuntimeError("WORLD_SIZE > 1 but torch.distributed is not initialised (launch with torchrun)")
        self.gpu_global_rank = dist.get_rank()
        self.gpu_world_size = dist.get_world_size()
        self.multi_gpu_cfg = {"global_rank": self.gpu_global_rank, "world_size": self.gpu_world_size}

    # ------------------------------------------------------------------ training
    def learn(self, num_learning_iterations: int, init_at_random_ep_len: bool = False,
              callback=None) -> list[dict]:
        """``callback(record)`` (optional) runs after every iteration with its log record, so a caller
        can print progress from one ``learn(max_iterations)`` call (checkpoints follow
        ``save_interval`` plus one at the end, as rsl_rl)."""
        env = self.env
        if init_at_random_ep_len:
            env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
        obs = _policy_obs(env.get_observations()).to(self.device)
        self.alg.policy.train()
        if self.is_distributed:
            self.alg.broadcast_parameters()
        rewbuffer, lenbuffer = self.rewbuffer, self.lenbuffer
        start_iter = self.current_learning_iteration
        for it in range(start_iter, start_iter + num_learning_iterations):
            t0 = time.perf_counter()
            with torch.no_grad():  # not inference_mode: graph capture updates the RNG state tensors
                if self.use_graph and self._graph is not None:
                    self._graph.replay()
                    obs = self._g_obs
                else:
                    obs = self._rollout(obs)
                    if self.use_graph:
                        self._capture(obs)
                        obs = self._g_obs
                if self._dev_is_cuda:  # the rollout's GPU time counts as collection, not learning
                    torch.cuda.synchronize(self.device)
                collect_time = time.perf_counter() - t0
                t1 = time.perf_counter()
                self.alg.compute_returns(obs)
            self.alg.draw_minibatch_indices()
            if self._update_graph is not None:
                self._update_graph.replay()
                self.alg.storage.clear()  # host-side step counter (the replay runs no Python)
            else:
                self.alg.update_steps()
                if self.graph_update and not self.is_distributed:
                    self._capture_update()
                elif self.graph_update and self.alg._seg_pre is None and not self.alg.capture_update_segments():
                    self.graph_update = False  # (no fused driver: eager multi-GPU update)
            losses = self.alg.update_stats()
            learn_time = time.perf_counter() - t1
            stats = self.ep_stats.tolist()
            if stats[2] > 0:
                rewbuffer.append(stats[0] / stats[2])
                lenbuffer.append(stats[1] / stats[2])
            self.current_learning_iteration = it
            self.tot_timesteps += self.num_steps_per_env * env.num_envs * self.gpu_world_size
            self.tot_time += collect_time + learn_time
            rec = {"iteration": it, "collection_time": collect_time, "learn_time": learn_time,
                   "fps": self.num_steps_per_env * env.num_envs * self.gpu_world_size / (collect_time + learn_time),
                   "mean_reward": statistics.mean(rewbuffer) if rewbuffer else float("nan"),
                   "mean_episode_length": statistics.mean(lenbuffer) if lenbuffer else float("nan"),
                   "learning_rate": self.alg.learning_rate, "mean_noise_std": self.alg.policy.std.mean().item(),
                   **{f"loss/{k}": v for k, v in losses.items()}}
            if self._log_keys:  # rsl_rl: mean over the rollout's per-step extras["log"] values
                acc = self._log_acc if self._native_acc is None else self._native_acc.index_select(0, self._native_idx)
                for k, v in zip(self._log_keys, (acc / self.num_steps_per_env).tolist()):
                    rec[k] = v
            self.log.append(rec)
            if callback is not None:
                callback(rec)
            if self.gpu_global_rank == 0 and self.log_dir and (it % self.save_interval == 0):
                self.save(os.path.join(self.log_dir, f"model_{it}.pt"))
        self.current_learning_iteration = start_iter + num_learning_iterations
        if self.gpu_global_rank == 0 and self.log_dir:
            self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))
        return self.log

    def _rollout(self, obs: torch.Tensor) -> torch.Tensor:
        """num_steps_per_env env steps into the storage; episode statistics into ep_stats."""
        env = self.env
        self.ep_stats.zero_()
        if self._log_acc is not None:
            self._log_acc.zero_()
        if self._native_acc is not None:
            self._native_acc.zero_()
        # on a GPU the policy step and the post-step bookkeeping are one launch each (libzbot_ppo:
        # zbp_act, zbp_env_post) instead of ~40 torch kernels; same statements as the loop below
        fr = self.alg.fused_rollout()
        if fr is not None:
            st = self.alg.storage
            # the action noise drawn inside zbp_act (ZBOT_KERNEL_NOISE=0: torch.randn, as the torch path)
            kn = os.environ.get("ZBOT_KERNEL_NOISE", "1") != "0"
            for _ in range(self.num_steps_per_env):
                actions = fr.act(obs, obs, st, kernel_noise=kn)
                obs_d, rewards, dones, extras = env.step(actions.to(env.device))
                obs = _policy_obs(obs_d).to(self.device)
                tout = extras.get("time_outs") if isinstance(extras, dict) else None
                fr.env_post(st, rewards.to(self.device), dones.to(self.device),
                            None if tout is None else tout.to(self.device), self.alg.gamma, self.cur_rew, self.cur_len,
                            self.ep_stats)
                self._accumulate_log(extras)
            self._extras = extras
            return obs
        for _ in range(self.num_steps_per_env):
            actions = self.alg.act(obs, obs)
            obs_d, rewards, dones, extras = env.step(actions.to(env.device))
            obs = _policy_obs(obs_d).to(self.device)
            rewards, dones = rewards.to(self.device), dones.to(self.device)
            self.alg.process_env_step(rewards, dones, extras)
            self.cur_rew += rewards
            self.cur_len += 1
            d = dones > 0
            self.ep_stats += torch.stack([torch.where(d, self.cur_rew, 0.0).sum(),
                                          torch.where(d, self.cur_len, 0.0).sum(), d.sum().float()])
            self.cur_rew.masked_fill_(d, 0.0)
            self.cur_len.masked_fill_(d, 0.0)
            self._accumulate_log(extras)
        self._extras = extras
        return obs

    def _accumulate_log(self, extras) -> None:
        """Sum this step's extras["log"] values on the device (rsl_rl appends every step's log and
        averages at log time; here the sum is captured in the rollout graph)."""
        log = extras.get("log") if isinstance(extras, dict) else None
        if not log:
            return
        if self._log_keys is None:
            self._log_keys = list(log.keys())
            self._log_acc = torch.zeros(len(self._log_keys), device=self.device)
            self._log_groups = self._log_views(log)
            if self._native_log_setup():
                return
        if self._native_acc is not None:
            if all(log[k] is self._log_src[i] for i, k in enumerate(self._log_keys)):
                return  # summed by the env's own finalize launch
            raise RuntimeError("extras['log'] changed its buffers after the native log accumulator was registered")
        if self._log_groups is not None and all(log[k] is self._log_src[i] for i, k in enumerate(self._log_keys)):
            # the env's log values are fixed 0-d views into a few device buffers: one gather + one
            # index_add per buffer instead of a copy per key
            for base, src, dst in self._log_groups:
                self._log_acc.index_add_(0, dst, base.index_select(0, src).to(torch.float32))
            return
        vals = [log[k] if torch.is_tensor(log[k]) else torch.tensor(float(log[k])) for k in self._log_keys]
        self._log_acc += torch.stack([v.to(self.device, torch.float32).reshape(()) for v in vals])

    def _native_log_setup(self) -> bool:
        """When every log value is a view of the simulator's own log buffers (zb_set_log_buffers), register
        an accumulator that the step's finalize launch adds them to (zb_set_log_accumulator): no torch
        launch per step for the log. This step, which ran before the registration, is
        added here once."""
        sim = getattr(getattr(self.env, "unwrapped", self.env), "sim", None)
        if (self._log_groups is None or sim is None or not hasattr(sim, "set_log_accumulator")
                or getattr(sim, "device", None) != self._log_acc.device):
            return False
        from .. import model as zm
        means, counts = sim.log_buffer, sim.log_count_buffer
        idx = []
        for v in self._log_src:
            if v._base is means:
                idx.append(v.storage_offset() - means.storage_offset())
            elif v._base is counts:
                idx.append(zm.LOG_LEN + v.storage_offset() - counts.storage_offset())
            else:
                return False
        self._native_idx = torch.tensor(idx, device=self._log_acc.device)
        self._native_acc = torch.zeros(zm.LOG_LEN + zm.LOG_COUNTS, device=self._log_acc.device)
        now = torch.cat([means.to(torch.float32), counts.to(torch.float32)])
        self._native_acc.copy_(now)  # this step's values (the accumulator starts from zero each rollout)
        sim.set_log_accumulator(self._native_acc)
        return True

    def _log_views(self, log):
        """[(flat base buffer, source indices, accumulator indices)] when every log value is a 0-d
        view of a 1-d device buffer (walking v2 / v4 / manager: zb_read_log's buffers), else None."""
        self._log_src = [log[k] for k in self._log_keys]
        groups = {}
        for i, v in enumerate(self._log_src):
            b = v._base if torch.is_tensor(v) else None
            if b is None or v.dim() != 0 or b.dim() != 1 or not b.is_contiguous() or b.device != self._log_acc.device:
                return None
            e = groups.setdefault(id(b), (b, [], []))
            e[1].append(v.storage_offset() - b.storage_offset())
            e[2].append(i)
        dev = self._log_acc.device
        return [(b, torch.tensor(src, device=dev), torch.tensor(dst, device=dev)) for b, src, dst in groups.values()]

    def _capture(self, obs: torch.Tensor) -> None:
        """Record one rollout (reading obs from a static buffer) as a graph; nothing executes."""
        self._g_obs = obs.clone()
        storage_step = self.alg.storage.step
        self.alg.storage.step = 0
        g = torch.cuda.CUDAGraph()
        with _blas_workspace_fence(self.device), torch.cuda.graph(g):
            last = self._rollout(self._g_obs)
            self._g_obs.copy_(last)
        self.alg.storage.step = storage_step
        self._graph = g

    def _capture_update(self) -> None:
        """Record the 20 minibatch updates (forward, backward, gradient all-reduce, clip, fused Adam
        with a device learning rate) as a graph; the eager first update was the warm-up."""
        g = torch.cuda.CUDAGraph()
        with _blas_workspace_fence(self.device), torch.cuda.graph(g):
            self.alg.update_steps()
        self._update_graph = g

    # ------------------------------------------------------------------ checkpoints / inference
    def save(self, path: str, infos: dict | None = None) -> None:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        torch.save({"model_state_dict": self.alg.policy.state_dict(),
                    "optimizer_state_dict": self.alg.optimizer.state_dict(),
                    "iter": self.current_learning_iteration, "infos": infos}, path)

    def load(self, path: str, load_optimizer: bool = True) -> dict | None:
        d = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.policy.load_state_dict(d["model_state_dict"])
        if load_optimizer:
            self.alg.optimizer.load_state_dict(d["optimizer_state_dict"])
            self.alg.restore_learning_rate()
            self.alg.invalidate_fused()  # the fused update re-reads the new optimizer state
        # captured graphs hold the old fused driver's workspace: re-capture on the next iteration
        self._graph, self._update_graph = None, None
        self.current_learning_iteration = d["iter"]
        return d.get("infos")

    def get_inference_policy(self, device=None):
        self.alg.policy.eval()
        if device is not None:
            self.alg.policy.to(device)
        return self.alg.policy.act_inference
