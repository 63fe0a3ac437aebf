"""``zbot-6b-standup-v0`` (snake -> biped stand-up) with the reference's DirectRLEnv interface.

Reference: ``source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6_standup_env_v0.py`` (``standup.py``):
``EventCfg`` (120-188), ``Zbot6SUpEnvCfg`` (191-447) and ``Zbot6SUpEnv`` (450-856) on ``ZBOT_6S_CFG_2``
(``assets/zbot_cfg.py:721-763``, the robot lying on its side). Same robot, actuators and physics as
the walking task; per step everything (4 substeps, dones, rewards, the reset events, observations)
runs in the fused stand-up kernel of ``libzbot.so``:

* startup event ``physics_material`` (randomize_rigid_body_material, 124-136): 64 material buckets
  (static, dynamic friction ~ U[0.6, 1.0], restitution 0) drawn once, one bucket per link shape per
  env; the per-link static and dynamic friction go to the kernel (``zb_set_link_friction_sd``), which combines
  it with the terrain's 1.0 (ground contacts) or the other link's (self contacts) by multiplying;
* reset event ``reset_base`` (reset_root_state_uniform, 33-97, 159-175): x, y ~ U(-0.5, 0.5),
  roll ~ U(-pi/4, pi/4), yaw ~ U(-3.14, 3.14) applied in the kernel at every reset;
* reset event ``my_curric`` (my_curriculum, 99-111): stage 0 -> 1 once common_step_counter >=
  max_episode_length * 80 (tracked on the device), weights {feet_downward_4: 2, shape_symmetry: -2}.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .. import model as zm
from .walking_v2 import InteractiveSceneCfg, SimulationCfg, SolverCfg, ZbotDirectEnvV2


@dataclass
class EventTermCfg:
    func: str
    mode: str
    params: dict = field(default_factory=dict)


@dataclass
class EventCfg:
    """standup.py:120-188 (startup material randomisation, reset pose, curriculum)."""
    physics_material: EventTermCfg = field(default_factory=lambda: EventTermCfg(
        "randomize_rigid_body_material", "startup",
        {"static_friction_range": (0.6, 1.0), "dynamic_friction_range": (0.6, 1.0), "restitution_range": (0.0, 0.0),
         "num_buckets": 64}))
    reset_base: EventTermCfg = field(default_factory=lambda: EventTermCfg(
        "reset_root_state_uniform", "reset",
        {"pose_range": {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "roll": (-0.7854, 0.7854), "yaw": (-3.14, 3.14)},
         "velocity_range": {k: (0.0, 0.0) for k in ("x", "y", "z", "roll", "pitch", "yaw")}}))
    my_curric: EventTermCfg | None = field(default_factory=lambda: EventTermCfg("my_curriculum", "reset"))


@dataclass
class Zbot6SUpEnvCfg:
    """Mirror of ``Zbot6SUpEnvCfg`` (standup.py:191-447)."""
    episode_length_s: float = 6.0
    decimation: int = 4
    action_space: int = 6
    observation_space: int = 22
    state_space: int = 0
    termination_height: float = 0.20   # declared by the reference, unused by its dones
    sim: SimulationCfg = field(default_factory=SimulationCfg)
    scene: InteractiveSceneCfg = field(default_factory=InteractiveSceneCfg)
    solver: SolverCfg = field(default_factory=SolverCfg)
    events: EventCfg = field(default_factory=EventCfg)
    seed: int | None = None
    reward_cfg: dict = field(default_factory=lambda: {"reward_scales": dict(zm.SU_REWARD_WEIGHTS)})
    curriculum_weights: dict = field(default_factory=lambda: dict(zm.SU_CURRICULUM_WEIGHTS))

    def task_cfg(self) -> zm.TaskCfg:
        pr = self.events.reset_base.params["pose_range"]
        return zm.TaskCfg.standup(
            sim_dt=self.sim.dt, decimation=self.decimation, episode_length_s=self.episode_length_s,
            termination_height=self.termination_height, reward_weights=dict(self.reward_cfg["reward_scales"]),
            gravity=-self.sim.gravity[2], friction=self.sim.static_friction,
            friction_dynamic=self.sim.dynamic_friction,
            contact_margin=self.solver.contact_margin, baumgarte=self.solver.baumgarte,
            solver_iterations=self.solver.iterations, enable_self_collision=self.solver.self_collision,
            solver_mode=self.solver.mode, self_manifold=self.solver.self_manifold,
            reset_pose_range=tuple(tuple(pr.get(k, (0.0, 0.0))) for k in ("x", "y", "roll", "yaw")),
            curriculum=self.events.my_curric is not None, curriculum_weights=dict(self.curriculum_weights),
        )


class Zbot6SUpEnv(ZbotDirectEnvV2):
    """DirectRLEnv-compatible ``zbot-6b-standup-v0`` (standup.py:450-856) on the MI355X simulator."""

    _termination_keys = ("Episode_Termination/died", "Episode_Termination/time_out")  # standup.py:665-670
    _ep_len_row = zm.SU["EP_LEN"]

    def __init__(self, cfg: Zbot6SUpEnvCfg | None = None, render_mode: str | None = None, **kwargs):
        super().__init__(cfg or Zbot6SUpEnvCfg(), render_mode=render_mode, **kwargs)

    def _startup(self) -> None:
        """randomize_rigid_body_material (mode "startup"): buckets drawn once on the CPU, then a
        random bucket per (env, link shape); static and dynamic coefficients go to the solver."""
        p = self.cfg.events.physics_material.params
        g = torch.Generator().manual_seed(self.cfg.seed if self.cfg.seed is not None else 0)
        ranges = torch.tensor([p["static_friction_range"], p["dynamic_friction_range"], p["restitution_range"]])
        nb = int(p["num_buckets"])
        self.material_buckets = torch.rand(nb, 3, generator=g) * (ranges[:, 1] - ranges[:, 0]) + ranges[:, 0]
        bucket_ids = torch.randint(0, nb, (self.num_envs, zm.NUM_LINKS), generator=g)
        self.link_materials = self.material_buckets[bucket_ids]  # [N, 12, (static, dynamic, restitution)]
        self.sim.set_link_friction(self.link_materials[..., 0], self.link_materials[..., 1])

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
