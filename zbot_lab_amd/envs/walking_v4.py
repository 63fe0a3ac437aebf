"""``zbot-6b-walking-v4`` (commands, events, curricula) with the reference's DirectRLEnv interface.

Reference: ``source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v4.py`` (``v4.py``):
``EventCfg`` (268-439), ``Zbot6SEnvV4Cfg`` (443-686) and ``Zbot6SEnvV4`` (688-1239) on ``ZBOT_6S_CFG``.
v2's robot and physics; one fused kernel per step (``zb_v4_step_kernel``) also runs the events:

* ``reset_base`` (reset_root_state_uniform, body-frame yaw ~ U(-3.14, 3.14), x / y ~ U(-0.5, 0.5))
  and ``reset_command_resample`` (resample_commands) for every env that resets;
* ``interval_command_resample`` every 3-6 s per env (Isaac Lab's interval event timers);
* ``my_curric`` (my_curriculum, three stages at 12 / 24 / 144 x max_episode_length steps: reward
  weights and the command sign probability) and ``vel_range`` (range_curriculum: the command
  ranges widen while the buffered tracking rewards exceed 85 % of their weights) — both kept in
  device counters and applied by the per-call epilogue.

Observations [N, 24]: base quat, joint_pos - default, joint_vel, actions, commanded velocity,
heading error. ``extras["log"]`` adds ``Curriculum/curriculum_stage``, ``vel_lower_bound``,
``vel_upper_bound``, ``yaw_bound`` (v4.py:952-957).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .. import model as zm
from .standup_v0 import EventTermCfg
from .walking_v2 import InteractiveSceneCfg, SimulationCfg, SolverCfg, ZbotDirectEnvV2


def _cmd_params():
    return {"velocity_range": (0.3, 0.3), "yaw_range": (-0.1, 0.1), "dual_sign": True, "offset": 0.0, "prob_pos": 1.0}


@dataclass
class EventCfgV4:
    """v4.py:268-439 (reset pose, curricula, reset / interval command resampling)."""
    reset_base: EventTermCfg = field(default_factory=lambda: EventTermCfg(
        "reset_root_state_uniform", "reset",
        {"pose_range": {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "yaw": (-3.14, 3.14)},
         "velocity_range": {k: (0.0, 0.0) for k in ("x", "y", "z", "roll", "pitch", "yaw")}}))
    my_curric: EventTermCfg | None = field(default_factory=lambda: EventTermCfg("my_curriculum", "reset"))
    vel_range: EventTermCfg | None = field(default_factory=lambda: EventTermCfg(
        "range_curriculum", "reset", {"limit_ranges": (0.0, 0.3), "limit_yaw_ranges": (-0.5, 0.5)}))  # v4.py:686
    reset_command_resample: EventTermCfg = field(default_factory=lambda: EventTermCfg(
        "resample_commands", "reset", _cmd_params()))
    interval_command_resample: EventTermCfg = field(default_factory=lambda: EventTermCfg(
        "resample_commands", "interval", dict(_cmd_params(), interval_range_s=(3.0, 6.0))))


@dataclass
class Zbot6SEnvV4Cfg:
    """Mirror of ``Zbot6SEnvV4Cfg`` (v4.py:443-686)."""
    episode_length_s: float = 20.0
    decimation: int = 4
    action_space: int = 6
    observation_space: int = 24
    state_space: int = 0
    termination_height: float = 0.20
    contact_history_length: int = 3
    sim: SimulationCfg = field(default_factory=SimulationCfg)
    scene: InteractiveSceneCfg = field(default_factory=InteractiveSceneCfg)
    # (the ruling-on-face manifold is compiled into the walking v2 / stand-up kernels only)
    solver: SolverCfg = field(default_factory=lambda: SolverCfg(self_manifold=2))
    events: EventCfgV4 = field(default_factory=EventCfgV4)
    seed: int | None = None
    reward_cfg: dict = field(default_factory=lambda: {"reward_scales": dict(zm.V4_REWARD_WEIGHTS)})

    def task_cfg(self) -> zm.TaskCfg:
        pr = self.events.reset_base.params["pose_range"]
        cp = self.events.reset_command_resample.params
        ip = self.events.interval_command_resample.params
        vr = self.events.vel_range
        kw = dict(
            sim_dt=self.sim.dt, decimation=self.decimation, episode_length_s=self.episode_length_s,
            termination_height=self.termination_height, reward_weights=dict(self.reward_cfg["reward_scales"]),
            gravity=-self.sim.gravity[2], friction=self.sim.static_friction, friction_dynamic=self.sim.dynamic_friction,
            contact_margin=self.solver.contact_margin, baumgarte=self.solver.baumgarte,
            solver_iterations=self.solver.iterations, enable_self_collision=self.solver.self_collision,
            solver_mode=self.solver.mode, self_manifold=self.solver.self_manifold,
            reset_pose_range=tuple(tuple(pr.get(k, (0.0, 0.0))) for k in ("x", "y", "roll", "yaw")),
            cmd_vel_range=tuple(cp["velocity_range"]), cmd_yaw_range=tuple(cp["yaw_range"]),
            cmd_dual_sign=bool(cp["dual_sign"]), cmd_offset=float(cp["offset"]), cmd_prob_pos=float(cp["prob_pos"]),
            cmd_interval_s=tuple(ip.get("interval_range_s", (3.0, 6.0))),
        )
        if vr is not None:
            kw.update(range_limit_vel=tuple(vr.params["limit_ranges"]), range_limit_yaw=tuple(vr.params["limit_yaw_ranges"]))
        else:
            kw.update(range_period_episodes=0)
        return zm.TaskCfg.walking_v4(curriculum=self.events.my_curric is not None, **kw)


class Zbot6SEnvV4(ZbotDirectEnvV2):
    """DirectRLEnv-compatible ``zbot-6b-walking-v4`` (v4.py:688-1239) on the MI355X simulator."""

    _termination_keys = ("Episode_Termination/died", "Episode_Termination/time_out")  # v4.py:945-950
    _ep_len_row = zm.V4["EP_LEN"]
    _curriculum_keys = ("Curriculum/curriculum_stage", "Curriculum/vel_lower_bound", "Curriculum/vel_upper_bound",
                        "Curriculum/yaw_bound")

    def __init__(self, cfg: Zbot6SEnvV4Cfg | None = None, render_mode: str | None = None, **kwargs):
        super().__init__(cfg or Zbot6SEnvV4Cfg(), render_mode=render_mode, **kwargs)

    def _update_log(self) -> None:
        if getattr(self, "_log", None) is None:
            super()._update_log()
            buf = self.sim.log_buffer
            for k, key in enumerate(self._curriculum_keys):
                self._log[key] = buf[16 + k]
        self.extras["log"] = self._log

    @property
    def commands(self) -> torch.Tensor:
        """[N, 2] (forward velocity, relative yaw) — a copy of the in-HBM command rows."""
        st = self.sim.get_state()
        return st[zm.V4["COMMANDS"]:zm.V4["COMMANDS"] + 2].T.contiguous()

    @property
    def target_heading_yaw(self) -> torch.Tensor:
        return self.sim.get_state()[zm.V4["TARGET_YAW"]].clone()

    @property
    def current_yaw(self) -> torch.Tensor:
        return self.sim.get_state()[zm.V4["CURRENT_YAW"]].clone()

    @property
    def curriculum_stage(self) -> int:
        return self.sim.read_curriculum()[0]

    @property
    def reward_scales(self) -> dict:
        """Reward weights of the current curriculum stage (the reference mutates this dict)."""
        return dict(self._task.stage_weights()[self.curriculum_stage])

    @reward_scales.setter
    def reward_scales(self, value) -> None:  # set by the base __init__; the weights live in _task
        pass
