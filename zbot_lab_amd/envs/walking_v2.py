"""``zbot-6b-walking-v2`` with the reference's DirectRLEnv interface, stepped by the HIP simulator.

Reference: ``source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v2.py`` (``v2.py``):
``ZbotDirectEnvCfgV2`` (v2.py:26-206) and ``ZbotDirectEnvV2`` (v2.py:208-605), driven by Isaac Lab's
``DirectRLEnv.step`` / ``reset``. Callers see the same 5-tuple ``step`` contract
(``obs {"policy": [N,23]}, reward [N], terminated [N] bool, truncated [N] bool, extras``), the
same ``reset() -> (obs, extras)`` and the attributes rsl_rl and the reference scripts use
(``num_envs``, ``device``, ``step_dt``, ``max_episode_length``, settable ``episode_length_buf``,
``cfg``, ``single_action_space``, ``single_observation_space``, ``unwrapped``, ...).

Everything per step runs in one fused HIP kernel (``libzbot.so``); this class only moves
pointers. Differences from the reference are listed in DESIGN.md §4 (no rendering, env-local
coordinates internally, `episode_length_buf` returned as a copy).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import model as zm
from .. import spaces
from ..sim import ZbotSim


@dataclass
class SimulationCfg:
    dt: float = 1.0 / 200.0          # v2.py:48
    render_interval: int = 4          # v2.py:49
    device: str = "cuda:0"
    gravity: tuple = (0.0, 0.0, -9.81)
    static_friction: float = 1.0      # v2.py:49-56 (multiply combine with the ground's 1.0)
    dynamic_friction: float = 1.0
    restitution: float = 0.0


@dataclass
class InteractiveSceneCfg:
    num_envs: int = 4096              # v2.py:73-75
    env_spacing: float = 4.0
    replicate_physics: bool = True


@dataclass
class SolverCfg:
    """Parameters of this simulator's contact/drive solver."""
    iterations: int = 4               # PGS sweeps/substep = solver_position_iteration_count=4 (zbot_cfg.py:637)
    contact_margin: float = 0.004
    baumgarte: float = 0.2
    self_collision: bool = True       # enabled_self_collisions=True (zbot_cfg.py:636)
    # zb_task_cfg.solver_mode. 1 (default, round 6): PhysX TGS with solver_position_iteration_count 4 /
    # velocity 0 (zbot_cfg.py:637-638) -- 4 sub-iterations of dt / 4 on the step's constraint rows, each
    # contact's separation advanced by the accumulated relative motion along its normal;
    # 0: 4 projected Gauss-Seidel sweeps on one linearisation (rounds 1-5 default); 2: 1 + the ground
    # contacts re-evaluated at every sub-iteration's pose; 3: 2 + the self contacts too
    mode: int = 1
    # zb_task_cfg.self_manifold. 3 (default, round 6; walking v2 and stand-up): cap-on-cap (up to 4
    # points), a link lying on another's cap (up to 3), side-by-side rims (up to 3) -- PhysX PCM keeps up
    # to 4 points per convex pair (zbot_cfg.py:636); 2: without the ruling-on-face case (v4 / manager
    # default); 1: caps only; 0: one point per pair
    self_manifold: int = 3


def _scales(**kw) -> dict:
    return {"reward_scales": dict(kw)}


# The staged training recipe of v2.py:78-206: the reference trains 2000 iterations per stage and
# chains the stages with ``--resume`` (README.md:69), editing the active ``reward_cfg`` between
# runs; ``step4`` is the active one (v2.py:190-206). scripts/train.py --reward_cfg selects a stage.
# step0 ("just stepping walk base") adds the feet-force terms (v2.py:563-571); step1 has three
# variants, v0 marked "use this" (v2.py:94-148).
REWARD_CFGS = {
    "step0": _scales(base_vel_forward=1.0, feet_downward=-1.0, feet_forward=-1.0, base_heading_x=-1.0,  # v2.py:78-92
                     feet_force_diff=0.5, feet_force_sum=-0.1, base_pos_y_err=-1.0),
    "step1": _scales(base_vel_forward=1.0, feet_downward=-1.0, feet_forward=-1.0, base_heading_x=-1.0,  # v2.py:94-110
                     base_heading_x_sum=-3.0, step_length=5.0, airtime_balance=-15.0, action_rate=-0.1,
                     torques=-0.002, feet_slide=-10.0, base_pos_y_err=-1.0),
    "step1_v1": _scales(base_vel_forward=1.0, feet_downward=-1.5, feet_forward=-0.5, base_heading_x=-1.0,  # v2.py:112-129
                        base_heading_x_sum=-3.0, step_length=5.0, airtime_balance=-15.0, action_rate=-0.1,
                        torques=-0.002, feet_slide=-10.0, base_pos_y_err=-1.5, base_pos_y_err_sum=-1.5),
    "step1_v2": _scales(base_vel_forward=1.0, feet_downward=-2.0, feet_forward=-0.2, base_heading_x=-1.0,  # v2.py:131-148
                        base_heading_x_sum=-5.0, step_length=5.0, airtime_balance=-15.0, action_rate=-0.1,
                        torques=-0.002, feet_slide=-10.0, base_pos_y_err=-2.0, base_pos_y_err_sum=-2.0),
    "step2": _scales(base_vel_forward=1.0, feet_downward=-2.0, feet_forward=-1.0, base_heading_x=-1.0,  # v2.py:150-167
                     base_heading_x_sum=-3.0, step_length=5.0, airtime_balance=-15.0, action_rate=-0.1,
                     torques=-0.002, feet_slide=-10.0, base_pos_y_err=-1.0, base_pos_y_err_sum=-2.0),
    "step3": _scales(base_vel_forward=1.0, feet_downward=-2.0, feet_forward=-1.0, base_heading_x=-1.0,  # v2.py:169-186
                     base_heading_x_sum=-5.0, step_length=5.0, airtime_balance=-15.0, action_rate=-0.1,
                     torques=-0.002, feet_slide=-10.0, base_pos_y_err=-2.0, base_pos_y_err_sum=-2.0),
    "step4": {"reward_scales": dict(zm.REWARD_WEIGHTS)},                                              # v2.py:190-206
}


@dataclass
class ZbotDirectEnvCfgV2:
    """Mirror of ``ZbotDirectEnvCfgV2`` (v2.py:26-206)."""
    episode_length_s: float = 20.0
    decimation: int = 4
    action_space: int = 6
    observation_space: int = 23
    state_space: int = 0
    termination_height: float = 0.22
    sim: SimulationCfg = field(default_factory=SimulationCfg)
    scene: InteractiveSceneCfg = field(default_factory=InteractiveSceneCfg)
    solver: SolverCfg = field(default_factory=SolverCfg)
    seed: int | None = None
    reward_cfg: dict = field(default_factory=lambda: {"reward_scales": dict(zm.REWARD_WEIGHTS)})

    def task_cfg(self) -> zm.TaskCfg:
        unknown = set(self.reward_cfg["reward_scales"]) - set(zm.REWARD_TERMS)
        if unknown:  # ZbotDirectEnvV2.__init__ would fail the same way (getattr "_reward_" + name, v2.py:252)
            raise NotImplementedError(f"reward terms not compiled into zb_step_kernel: {sorted(unknown)}")
        return zm.TaskCfg(
            sim_dt=self.sim.dt, decimation=self.decimation, episode_length_s=self.episode_length_s,
            termination_height=self.termination_height,
            reward_weights=dict(self.reward_cfg["reward_scales"]), gravity=-self.sim.gravity[2],
            friction=self.sim.static_friction, friction_dynamic=self.sim.dynamic_friction, contact_margin=self.solver.contact_margin,
            baumgarte=self.solver.baumgarte, solver_iterations=self.solver.iterations,
            enable_self_collision=self.solver.self_collision, solver_mode=self.solver.mode, self_manifold=self.solver.self_manifold,
        )


def grid_env_origins(num_envs: int, spacing: float) -> torch.Tensor:
    """Isaac Lab's TerrainImporter grid of env origins (plane terrain, ``env_spacing``)."""
    num_rows = int(np.ceil(num_envs / np.sqrt(num_envs)))
    num_cols = int(np.ceil(num_envs / num_rows))
    ii, jj = torch.meshgrid(torch.arange(num_rows), torch.arange(num_cols), indexing="ij")
    origins = torch.zeros(num_envs, 3)
    origins[:, 0] = -(ii.flatten()[:num_envs] - (num_rows - 1) / 2) * spacing
    origins[:, 1] = (jj.flatten()[:num_envs] - (num_cols - 1) / 2) * spacing
    return origins


class ZbotDirectEnvV2:
    """DirectRLEnv-compatible ``zbot-6b-walking-v2`` (v2.py:208-605) on the MI355X simulator."""

    is_vector_env = True
    metadata = {"render_modes": [None], "isaac_sim_version": None}
    _termination_keys = ("Episode_Termination/body_contact", "Episode_Termination/time_out")  # v2.py:449-457
    _ep_len_row = zm.S["EP_LEN"]

    def __init__(self, cfg: ZbotDirectEnvCfgV2 | None = None, render_mode: str | None = None, **kwargs):
        self.cfg = cfg or ZbotDirectEnvCfgV2()
        if render_mode not in (None, "rgb_array"):
            raise ValueError("rendering is out of scope for this simulator")
        self.render_mode = render_mode
        self.device = torch.device(kwargs.get("device", self.cfg.sim.device))
        self.num_envs = int(kwargs.get("num_envs", self.cfg.scene.num_envs))
        self.physics_dt = self.cfg.sim.dt
        self.step_dt = self.cfg.sim.dt * self.cfg.decimation
        self.max_episode_length_s = self.cfg.episode_length_s
        self.max_episode_length = math.ceil(self.max_episode_length_s / self.step_dt)
        seed = self.cfg.seed if self.cfg.seed is not None else 0
        self._task = self.cfg.task_cfg()
        self.sim = ZbotSim(self.num_envs, self._task, device=self.device, seed=seed)
        self.device = self.sim.device
        self.env_origins = grid_env_origins(self.num_envs, self.cfg.scene.env_spacing).to(self.device)
        # v2.py:250-252 — weights scaled by step_dt (kept as a new dict; the reference mutates cfg)
        self.reward_scales = {k: v * self.step_dt for k, v in self.cfg.reward_cfg["reward_scales"].items()}
        self.single_observation_space = spaces.Dict(policy=spaces.Box(-np.inf, np.inf, (self.cfg.observation_space,)))
        self.single_action_space = spaces.Box(-np.inf, np.inf, (self.cfg.action_space,))
        self.observation_space = spaces.Dict(
            policy=spaces.Box(-np.inf, np.inf, (self.num_envs, self.cfg.observation_space)))
        self.action_space = spaces.Box(-np.inf, np.inf, (self.num_envs, self.cfg.action_space))
        self.common_step_counter = 0
        self.extras: dict = {}
        self._log_keys = [f"Episode_Reward/{k}" for k in self._task.reward_terms]
        self.obs_buf = None
        self._startup()

    def _startup(self) -> None:
        """Startup events (none for v2)."""

    # ------------------------------------------------------------------ gym API
    @property
    def unwrapped(self):
        return self

    @property
    def reset_terminated(self) -> torch.Tensor:
        return self.sim.terminated

    @property
    def reset_time_outs(self) -> torch.Tensor:
        return self.sim.truncated

    @property
    def reset_buf(self) -> torch.Tensor:
        return self.sim.terminated | self.sim.truncated

    @property
    def episode_length_buf(self) -> torch.Tensor:
        """Copy of the in-HBM episode counters (int64, like Isaac Lab's buffer)."""
        return self.sim.get_state()[self._ep_len_row].round().to(torch.long)

    @episode_length_buf.setter
    def episode_length_buf(self, value: torch.Tensor) -> None:
        """Writes only the counter row: the solver's self-contact cache (simulator-internal, not a
        state row) survives, so rsl_rl's init_at_random_ep_len does not cold-start GJK."""
        st = self.sim.get_state()
        wc = self.sim.get_contact_cache()
        st[self._ep_len_row] = value.to(device=self.device, dtype=torch.float32)
        self.sim.set_state(st)
        self.sim.set_contact_cache(wc)

    def seed(self, seed: int = -1) -> int:
        return seed

    def reset(self, seed: int | None = None, options: dict | None = None):
        """DirectRLEnv.reset: reset all envs (v2.py:413-459, full-reset episode-length draw)."""
        self.sim.reset(None)
        self.obs_buf = {"policy": self.sim.observe()}
        self._update_log()
        return self.obs_buf, self.extras

    def step(self, action: torch.Tensor):
        """DirectRLEnv.step: one fused kernel (physics x decimation, sensor, dones, rewards, resets, obs)."""
        obs, rew, term, trunc = self.sim.step(action)
        self.common_step_counter += 1
        self.obs_buf = {"policy": obs}
        self.reward_buf = rew
        self._update_log()
        return self.obs_buf, rew, term, trunc, self.extras

    def _update_log(self) -> None:
        # the library refreshes the registered log buffers in stream order; the dict of views into
        # them is built once (no per-step tensor work)
        if getattr(self, "_log", None) is None:
            means, counts = self.sim.read_log()
            # _episode_sums holds the active reward_cfg's keys only (v2.py:254-256)
            rc = getattr(self.cfg, "reward_cfg", None)
            active = rc["reward_scales"] if isinstance(rc, dict) and "reward_scales" in rc else None
            self._log = {k: means[i] for i, k in enumerate(self._log_keys)
                         if active is None or k.split("/", 1)[1] in active}
            self._log[self._termination_keys[0]] = counts[0]
            self._log[self._termination_keys[1]] = counts[1]
        self.extras["log"] = self._log

    def get_observations(self):
        if self.obs_buf is None:
            self.obs_buf = {"policy": self.sim.observe()}
        return self.obs_buf

    def render(self, recompute: bool = False):
        return None

    def close(self) -> None:
        if getattr(self, "sim", None) is not None:
            self.sim.close()
            self.sim = None
