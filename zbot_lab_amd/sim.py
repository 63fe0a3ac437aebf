"""Torch-facing handle on the HIP simulator (``libzbot.so``): one handle = N envs on one GPU.

All calls are stream-ordered on the current torch CUDA stream and never synchronise the host.
Persistent state lives in HBM, owned by the library (SoA ``[ZB_STATE_DIM][N]`` fp32).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as nat
from . import model as zm


def _stream(device: torch.device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class ZbotSim:
    def __init__(self, num_envs: int, cfg: zm.TaskCfg | None = None, device: str | torch.device = "cuda:0",
                 seed: int = 0, robot: zm.RobotModel | None = None):
        if num_envs < 1:
            raise ValueError("num_envs must be >= 1")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise nat.ZbotError("ZbotSim runs on a ROCm GPU only (device must be cuda:<i>); there is no CPU path")
        if not torch.cuda.is_available():
            raise nat.ZbotError("no ROCm GPU visible: the HIP simulator cannot run here")
        self.lib = nat.lib()
        self.num_envs = int(num_envs)
        self.cfg = cfg or zm.TaskCfg()
        self.task = self.cfg.task
        self.obs_dim, self.state_dim = self.cfg.obs_dim, self.cfg.state_dim
        self.num_terms = len(self.cfg.reward_terms)
        if robot is None:
            robot = (zm.standup_model() if self.task == zm.TASK_STANDUP_V0
                     else zm.load_v09_model() if self.task == zm.TASK_MANAGER_V0 else zm.load_model())
        self.robot = robot
        self._m = zm.pack_model(self.robot)
        self._c = self.cfg.pack()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(self.lib.zb_create(C.byref(self._m), C.byref(self._c), self.num_envs, idx, int(seed) & (2**64 - 1),
                                         C.byref(h)), "zb_create")
        self._h = h
        if self.lib.zb_state_dim(h) != self.state_dim:
            raise nat.ZbotError("libzbot state layout does not match zbot_lab_amd.model")
        # persistent outputs (reference: terminated/truncated buffers are mutated in place)
        self.terminated = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
        self.truncated = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
        self._log_means = torch.zeros(zm.LOG_LEN, dtype=torch.float32, device=self.device)  # include/zbot.h ZB_LOG_LEN
        self._log_counts = torch.zeros(zm.LOG_COUNTS, dtype=torch.int32, device=self.device)  # ZB_LOG_COUNTS
        # the library fills these in stream order at every step/reset with resets (no copies)
        nat.check(self.lib.zb_set_log_buffers(self._h, nat.ptr(self._log_means), nat.ptr(self._log_counts)),
                  "zb_set_log_buffers")

    # ------------------------------------------------------------------ lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.zb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ ops
    def reset(self, env_ids: torch.Tensor | None = None) -> None:
        if env_ids is None:
            nat.check(self.lib.zb_reset(self._h, None, self.num_envs, _stream(self.device)), "zb_reset")
            return
        ids = env_ids.to(device=self.device, dtype=torch.int32).contiguous()
        if ids.numel() == 0:
            return
        nat.check(self.lib.zb_reset(self._h, nat.ptr(ids), ids.numel(), _stream(self.device)), "zb_reset")

    def step(self, actions: torch.Tensor):
        a = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if a.shape != (self.num_envs, zm.ACT_DIM):
            raise ValueError(f"actions must be [{self.num_envs}, {zm.ACT_DIM}], got {tuple(a.shape)}")
        obs = torch.empty(self.num_envs, self.obs_dim, dtype=torch.float32, device=self.device)
        rew = torch.empty(self.num_envs, dtype=torch.float32, device=self.device)
        nat.check(self.lib.zb_step(self._h, nat.ptr(a), nat.ptr(obs), nat.ptr(rew), nat.ptr(self.terminated),
                                   nat.ptr(self.truncated), _stream(self.device)), "zb_step")
        return obs, rew, self.terminated, self.truncated

    def step_into(self, actions: torch.Tensor, obs: torch.Tensor, rew: torch.Tensor) -> None:
        """Allocation-free variant for benchmarking / graph capture (caller-owned outputs)."""
        nat.check(self.lib.zb_step(self._h, nat.ptr(actions), nat.ptr(obs), nat.ptr(rew), nat.ptr(self.terminated),
                                   nat.ptr(self.truncated), _stream(self.device)), "zb_step")

    def observe(self) -> torch.Tensor:
        obs = torch.empty(self.num_envs, self.obs_dim, dtype=torch.float32, device=self.device)
        nat.check(self.lib.zb_observe(self._h, nat.ptr(obs), _stream(self.device)), "zb_observe")
        return obs

    def read_log(self):
        """(term_means[num_terms], counts[ZB_LOG_COUNTS]) device tensors of the most recent step that had resets
        (registered with zb_set_log_buffers, so no per-step copy)."""
        return self._log_means[:self.num_terms], self._log_counts

    @property
    def log_buffer(self) -> torch.Tensor:
        """The whole float[ZB_LOG_LEN] log buffer (term means, then the curriculum entries)."""
        return self._log_means

    @property
    def log_count_buffer(self) -> torch.Tensor:
        """The int32[ZB_LOG_COUNTS] termination-count buffer."""
        return self._log_counts

    def done_buffer(self) -> torch.Tensor:
        """A persistent int64 [N] tensor that every later step fills with terminated | truncated from the step
        kernel's own flag stores (zb_set_done_buffer): rsl_rl's dones without the wrapper's two torch
        launches per step. Registered on first use; the same tensor afterwards."""
        if getattr(self, "_dones", None) is None:
            self._dones = torch.zeros(self.num_envs, dtype=torch.long, device=self.device)
            nat.check(self.lib.zb_set_done_buffer(self._h, nat.ptr(self._dones)), "zb_set_done_buffer")
        return self._dones

    def set_log_accumulator(self, acc: torch.Tensor | None) -> None:
        """Register a device float[ZB_LOG_LEN + ZB_LOG_COUNTS] accumulator that every later step adds the
        log's current values to inside its finalize launch (zb_set_log_accumulator; the PPO runner's
        per-rollout sum of extras["log"]); None unregisters. The tensor must stay alive while registered."""
        if acc is not None and (acc.dtype != torch.float32 or acc.device != self.device or not acc.is_contiguous()
                                or acc.numel() != zm.LOG_LEN + zm.LOG_COUNTS):
            raise ValueError(f"accumulator must be a contiguous float32 [{zm.LOG_LEN + zm.LOG_COUNTS}] tensor on {self.device}")
        self._log_acc_ref = acc
        nat.check(self.lib.zb_set_log_accumulator(self._h, nat.ptr(acc)), "zb_set_log_accumulator")

    def set_link_friction(self, mu: torch.Tensor, mu_dynamic: torch.Tensor | None = None) -> None:
        """Standup / manager: per-link static (and dynamic; default = static) friction [N, 12]
        (randomize_rigid_body_material)."""
        m = mu.to(device=self.device, dtype=torch.float32).contiguous()
        md = m if mu_dynamic is None else mu_dynamic.to(device=self.device, dtype=torch.float32).contiguous()
        for t in (m, md):
            if t.shape != (self.num_envs, zm.NUM_LINKS):
                raise ValueError(f"friction must be [{self.num_envs}, {zm.NUM_LINKS}]")
        nat.check(self.lib.zb_set_link_friction_sd(self._h, nat.ptr(m), nat.ptr(md), _stream(self.device)),
                  "zb_set_link_friction_sd")
        torch.cuda.current_stream(self.device).synchronize()  # `m` may be a temporary

    def read_curriculum(self):
        """(curriculum stage, common_step_counter) from the device (synchronises)."""
        st, n = C.c_int32(), C.c_int64()
        nat.check(self.lib.zb_read_curriculum(self._h, C.byref(st), C.byref(n)), "zb_read_curriculum")
        return int(st.value), int(n.value)

    def get_state(self) -> torch.Tensor:
        st = torch.empty(self.state_dim, self.num_envs, dtype=torch.float32, device=self.device)
        nat.check(self.lib.zb_get_state(self._h, nat.ptr(st), _stream(self.device)), "zb_get_state")
        return st

    def set_state(self, st: torch.Tensor) -> None:
        s = st.to(device=self.device, dtype=torch.float32).contiguous()
        if s.shape != (self.state_dim, self.num_envs):
            raise ValueError(f"state must be [{self.state_dim}, {self.num_envs}]")
        nat.check(self.lib.zb_set_state(self._h, nat.ptr(s), _stream(self.device)), "zb_set_state")
        torch.cuda.current_stream(self.device).synchronize()  # `s` may be a temporary

    def get_contact_cache(self) -> torch.Tensor:
        """the solver's persistent self-contact cache [ZB_WARM_ROWS, N] (include/zbot.h)"""
        wc = torch.empty(16, self.num_envs, dtype=torch.float32, device=self.device)
        nat.check(self.lib.zb_get_contact_cache(self._h, nat.ptr(wc), _stream(self.device)), "zb_get_contact_cache")
        return wc

    def set_contact_cache(self, wc: torch.Tensor) -> None:
        w = wc.to(device=self.device, dtype=torch.float32).contiguous()
        if w.shape != (16, self.num_envs):
            raise ValueError(f"contact cache must be [16, {self.num_envs}]")
        nat.check(self.lib.zb_set_contact_cache(self._h, nat.ptr(w), _stream(self.device)), "zb_set_contact_cache")
        torch.cuda.current_stream(self.device).synchronize()

    def profile_begin(self, max_launches: int, stride: int = 1) -> None:
        """Time the next zb_step_kernel launches with HIP events: every ``stride``-th one, at most
        ``max_launches`` of them (the event dispatch adds ~5.7 us to a step it brackets)."""
        nat.check(self.lib.zb_profile_stride(self._h, int(stride)), "zb_profile_stride")
        nat.check(self.lib.zb_profile_begin(self._h, int(max_launches)), "zb_profile_begin")

    def profile_end(self):
        """(summed zb_step_kernel milliseconds, launches timed)."""
        ms, n = C.c_float(), C.c_int()
        nat.check(self.lib.zb_profile_end(self._h, C.byref(ms), C.byref(n)), "zb_profile_end")
        return float(ms.value), int(n.value)

    def physics_substeps(self, targets: torch.Tensor, nsub: int):
        t = targets.to(device=self.device, dtype=torch.float32).contiguous()
        nf = torch.zeros(self.num_envs, zm.NUM_LINKS, 3, dtype=torch.float32, device=self.device)
        tau = torch.zeros(self.num_envs, zm.NUM_DOF, dtype=torch.float32, device=self.device)
        nat.check(self.lib.zb_physics_substeps(self._h, nat.ptr(t), int(nsub), nat.ptr(nf), nat.ptr(tau),
                                               _stream(self.device)), "zb_physics_substeps")
        return nf, tau
