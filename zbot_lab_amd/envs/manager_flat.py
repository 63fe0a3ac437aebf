"""``zbot-6b-walking-m-v0``: the reference's manager-based flat env with the ManagerBasedRLEnv API.

Reference: ``source/zbot/zbot/tasks/zbotlab_manager`` — ``zbotlab_env_cfg.py`` (scene, commands,
actions, observations, events, rewards, terminations, curriculum: ``ZbotLabRoughEnvCfg``),
``config/zbot6b_manager/rough_env_cfg.py`` (``ZBOT_6S_V2_CFG``, events / terminations removed) and
``flat_env_cfg.py`` (``Zbot6BFlatEnvCfg``: plane, reward overrides), registered as
``isaaclab.envs:ManagerBasedRLEnv`` (``config/zbot6b_manager/__init__.py:18-26``).

Isaac Lab's managers evaluate python term functions one by one; here the term *configuration* is
kept (same cfg classes, names, weights and params, so user code that edits ``cfg.rewards.x.weight``
or ``cfg.commands.base_velocity.ranges`` keeps working) and compiled into the fused HIP step kernel
(``zb_m_step_kernel``): action processing, 4 physics substeps with the per-step contact sensor,
terminations, rewards, the reset events, the command manager and the observation group run in one
launch per step. ``task_cfg()`` validates the cfg: a term the kernel does not implement (e.g. one the
flat cfg sets to ``None``, or a different ``func``) raises instead of being ignored.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, fields

import numpy as np
import torch

from .. import model as zm
from .. import spaces
from .standup_v0 import EventTermCfg
from .walking_v2 import SimulationCfg, SolverCfg, ZbotDirectEnvV2


# ----------------------------------------------------------------------------- manager term cfgs
@dataclass
class ObsTerm:
    func: str
    noise: tuple | None = None           # AdditiveUniformNoiseCfg(n_min, n_max)
    params: dict = field(default_factory=dict)


@dataclass
class RewTerm:
    func: str
    weight: float
    params: dict = field(default_factory=dict)


@dataclass
class DoneTerm:
    func: str
    params: dict = field(default_factory=dict)
    time_out: bool = False


@dataclass
class CurrTerm:
    func: str
    params: dict = field(default_factory=dict)


EventTerm = EventTermCfg


@dataclass
class Ranges:
    lin_vel_x: tuple = (0.0, 0.0)
    lin_vel_y: tuple = (0.0, 0.0)
    ang_vel_z: tuple = (0.0, 0.0)
    heading: tuple | None = None


@dataclass
class UniformLevelVelocityCommandCfg:
    """mdp/commands/velocity_command.py (UniformVelocityCommandCfg + limit_ranges); mgr.py:99-117."""
    asset_name: str = "robot"
    resampling_time_range: tuple = (10.0, 10.0)
    rel_standing_envs: float = 0.02
    rel_heading_envs: float = 1.0
    heading_command: bool = False
    debug_vis: bool = True
    ranges: Ranges = field(default_factory=lambda: Ranges(lin_vel_x=(-0.1, 0.1)))
    limit_ranges: Ranges = field(default_factory=lambda: Ranges(lin_vel_x=(-0.3, 0.3)))


@dataclass
class CommandsCfg:
    base_velocity: UniformLevelVelocityCommandCfg = field(default_factory=UniformLevelVelocityCommandCfg)


@dataclass
class RelativeJointPositionActionCfg:
    """mgr.py:125-131."""
    asset_name: str = "robot"
    joint_names: list = field(default_factory=lambda: ["joint.*"])
    scale: float = 0.04 * math.pi
    clip: dict = field(default_factory=lambda: {"joint.*": [-0.04 * math.pi, 0.04 * math.pi]})
    use_zero_offset: bool = True


@dataclass
class ActionsCfg:
    joint_pos: RelativeJointPositionActionCfg = field(default_factory=RelativeJointPositionActionCfg)


@dataclass
class PolicyCfg:
    """mgr.py:139-158 (terms in order, corruption on, concatenated)."""
    base_quat: ObsTerm = field(default_factory=lambda: ObsTerm("root_quat_w", (-0.01, 0.01)))
    velocity_commands: ObsTerm = field(default_factory=lambda: ObsTerm(
        "generated_commands", None, {"command_name": "base_velocity"}))
    joint_pos: ObsTerm = field(default_factory=lambda: ObsTerm("joint_pos_rel", (-0.01, 0.01)))
    joint_vel: ObsTerm = field(default_factory=lambda: ObsTerm("joint_vel_rel", (-1.5, 1.5)))
    actions: ObsTerm = field(default_factory=lambda: ObsTerm("last_action"))
    enable_corruption: bool = True
    concatenate_terms: bool = True


@dataclass
class ObservationsCfg:
    policy: PolicyCfg = field(default_factory=PolicyCfg)


def _feet(p=None):
    return dict({"asset_cfg": "robot:foot.*"}, **(p or {}))


@dataclass
class RewardsCfg:
    """mgr.py:261-377 after flat_env_cfg.py:169-182 (weights 5.0 / -6.5 / -15.0, six terms None)."""
    track_lin_vel_xy_exp: RewTerm | None = field(default_factory=lambda: RewTerm(
        "track_lin_vel_xy_yaw_frame_exp", 1.0, {"command_name": "base_velocity", "std": math.sqrt(0.25)}))
    track_ang_vel_z_exp: RewTerm | None = field(default_factory=lambda: RewTerm(
        "track_ang_vel_z_world_exp", 0.5, {"command_name": "base_velocity", "std": math.sqrt(0.25)}))
    termination_penalty: RewTerm | None = field(default_factory=lambda: RewTerm("is_terminated", -200.0))
    dof_torques_l2: RewTerm | None = field(default_factory=lambda: RewTerm("joint_torques_l2", -1.0e-5))
    dof_acc_l2: RewTerm | None = field(default_factory=lambda: RewTerm("joint_acc_l2", -2.5e-7))
    action_rate_l2: RewTerm | None = field(default_factory=lambda: RewTerm("action_rate_l2", -0.01))
    foot_step_length: RewTerm | None = field(default_factory=lambda: RewTerm(
        "foot_step_length", 5.0, _feet({"sensor_cfg": "contact_forces:foot.*", "command_name": None})))
    foot_downward: RewTerm | None = field(default_factory=lambda: RewTerm("foot_downward", -1.0, _feet()))
    foot_forward: RewTerm | None = field(default_factory=lambda: RewTerm("foot_forward", -0.5, _feet()))
    gait: RewTerm | None = None
    feet_slide: RewTerm | None = field(default_factory=lambda: RewTerm(
        "feet_slide", -6.5, _feet({"sensor_cfg": "contact_forces:foot.*"})))
    feet_clearance: RewTerm | None = None
    feet_air_time: RewTerm | None = None
    air_time_variance: RewTerm | None = field(default_factory=lambda: RewTerm(
        "air_time_balance_penalty", -15.0, {"sensor_cfg": "contact_forces:foot.*"}))
    base_vel_forward: RewTerm | None = None
    feet_force_pattern: RewTerm | None = None
    undesired_contacts: RewTerm | None = None


@dataclass
class TerminationsCfg:
    """mgr.py:379-398; rough_env_cfg.py:45 removes base_contact."""
    time_out: DoneTerm | None = field(default_factory=lambda: DoneTerm("time_out", time_out=True))
    base_contact: DoneTerm | None = None
    base_height: DoneTerm | None = field(default_factory=lambda: DoneTerm(
        "root_height_below_minimum", {"minimum_height": 0.2}))
    feet_close: DoneTerm | None = field(default_factory=lambda: DoneTerm(
        "feet_close", {"minimum_distance": 0.12, "asset_cfg": "robot:foot.*"}))


@dataclass
class EventCfg:
    """mgr.py:164-258; rough_env_cfg.py:37-41 removes add_base_mass, base_com, push_robot."""
    init_my_data: EventTerm | None = field(default_factory=lambda: EventTerm("init_my_data", "startup"))
    physics_material: EventTerm | None = field(default_factory=lambda: EventTerm(
        "randomize_rigid_body_material", "startup",
        {"static_friction_range": (0.3, 1.0), "dynamic_friction_range": (0.3, 1.0), "restitution_range": (0.0, 0.0),
         "num_buckets": 64}))
    add_base_mass: EventTerm | None = None
    base_com: EventTerm | None = None
    reset_base: EventTerm | None = field(default_factory=lambda: EventTerm(
        "reset_root_state_uniform", "reset",
        {"pose_range": {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "yaw": (-3.14, 3.14)},
         "velocity_range": {k: (0.0, 0.0) for k in ("x", "y", "z", "roll", "pitch", "yaw")}}))
    reset_robot_joints: EventTerm | None = field(default_factory=lambda: EventTerm(
        "reset_joints_by_scale", "reset", {"position_range": (1.0, 1.0), "velocity_range": (1.0, 1.0)}))
    reset_my_data: EventTerm | None = field(default_factory=lambda: EventTerm("reset_my_data", "reset"))
    push_robot: EventTerm | None = None


@dataclass
class CurriculumCfg:
    terrain_levels: CurrTerm | None = None      # flat_env_cfg.py:189
    lin_vel_cmd_levels: CurrTerm | None = field(default_factory=lambda: CurrTerm("lin_vel_cmd_levels"))


@dataclass
class SceneCfg:
    num_envs: int = 4096                         # mgr.py:419
    env_spacing: float = 2.5
    replicate_physics: bool = True
    terrain_type: str = "plane"                  # flat_env_cfg.py:186


@dataclass
class Zbot6BFlatEnvCfg:
    """Mirror of ``Zbot6BFlatEnvCfg`` (flat_env_cfg.py:89-189 over rough_env_cfg.py / mgr.py:414-452)."""
    scene: SceneCfg = field(default_factory=SceneCfg)
    observations: ObservationsCfg = field(default_factory=ObservationsCfg)
    actions: ActionsCfg = field(default_factory=ActionsCfg)
    commands: CommandsCfg = field(default_factory=CommandsCfg)
    rewards: RewardsCfg = field(default_factory=RewardsCfg)
    terminations: TerminationsCfg = field(default_factory=TerminationsCfg)
    events: EventCfg = field(default_factory=EventCfg)
    curriculum: CurriculumCfg = field(default_factory=CurriculumCfg)
    decimation: int = 4
    episode_length_s: float = 20.0
    sim: SimulationCfg = field(default_factory=SimulationCfg)
    # (the ruling-on-face manifold is compiled into the walking v2 / stand-up kernels only)
    solver: SolverCfg = field(default_factory=lambda: SolverCfg(self_manifold=2))
    seed: int | None = None

    # the DirectRLEnv-style fields the shared env base reads
    action_space = 6
    observation_space = zm.M_OBS_DIM

    @property
    def reward_cfg(self) -> dict:
        return {"reward_scales": {k: t.weight for k, t in _active(self.rewards)}}

    def task_cfg(self) -> zm.TaskCfg:
        """Compile the manager cfg into the kernel's task parameters (raises on unsupported terms)."""
        rew = _active(self.rewards)
        names = [k for k, _ in rew]
        if names != zm.M_REWARD_TERMS:
            raise NotImplementedError(f"reward terms {names} != the compiled set {zm.M_REWARD_TERMS}")
        expect = RewardsCfg()
        for k, t in rew:
            ref = getattr(expect, k)
            if t.func != ref.func or t.params != ref.params:
                raise NotImplementedError(f"reward term {k}: func / params {t.func} {t.params} not compiled")
        term = _active(self.terminations)
        if [k for k, _ in term] != zm.M_TERMINATION_TERMS:
            raise NotImplementedError(f"termination terms {[k for k, _ in term]} != {zm.M_TERMINATION_TERMS}")
        cmd = self.commands.base_velocity
        if cmd.heading_command or tuple(cmd.ranges.ang_vel_z) != (0.0, 0.0) or \
                tuple(cmd.limit_ranges.ang_vel_z) != (0.0, 0.0):
            raise NotImplementedError("heading / angular-velocity commands are not compiled (flat cfg: 0)")
        lo, hi = cmd.resampling_time_range
        if lo != hi:
            raise NotImplementedError("resampling_time_range must be a single value (flat cfg: (10, 10))")
        act = self.actions.joint_pos
        (clo, chi), = act.clip.values()
        if not act.use_zero_offset or clo != -chi:
            raise NotImplementedError("RelativeJointPositionAction: zero offset and a symmetric clip are compiled")
        pol = self.observations.policy
        noise = [getattr(pol, k).noise for k in ("base_quat", "joint_pos", "joint_vel")]
        if [f.name for f in fields(pol)][:5] != ["base_quat", "velocity_commands", "joint_pos", "joint_vel", "actions"] \
                or any(n is not None and n[0] != -n[1] for n in noise):
            raise NotImplementedError("policy observation group: the compiled terms / symmetric noise only")
        ev = self.events
        for k in ("add_base_mass", "base_com", "push_robot"):
            if getattr(ev, k) is not None:
                raise NotImplementedError(f"event {k} is not compiled (the flat cfg removes it)")
        pr = ev.reset_base.params["pose_range"]
        if any(pr.get(k, (0.0, 0.0)) != (0.0, 0.0) for k in ("z", "pitch")) or \
                any(tuple(v) != (0.0, 0.0) for v in ev.reset_base.params["velocity_range"].values()):
            raise NotImplementedError("reset_base: z / pitch offsets and velocities are not compiled")
        if tuple(ev.reset_robot_joints.params["position_range"]) != (1.0, 1.0):
            raise NotImplementedError("reset_joints_by_scale: only the default (1, 1) scale is compiled")
        if self.curriculum.terrain_levels is not None:
            raise NotImplementedError("terrain_levels needs the rough terrain generator (out of scope)")
        return zm.TaskCfg.manager_flat(
            sim_dt=self.sim.dt, decimation=self.decimation, episode_length_s=self.episode_length_s,
            reward_weights={k: t.weight for k, t in rew},
            termination_height=float(self.terminations.base_height.params["minimum_height"]),
            feet_close_min=float(self.terminations.feet_close.params["minimum_distance"]),
            gravity=-self.sim.gravity[2], friction=self.sim.static_friction,
            friction_dynamic=self.sim.dynamic_friction,
            contact_margin=self.solver.contact_margin, baumgarte=self.solver.baumgarte,
            solver_iterations=self.solver.iterations, enable_self_collision=self.solver.self_collision,
            solver_mode=self.solver.mode, self_manifold=self.solver.self_manifold,
            reset_pose_range=tuple(tuple(pr.get(k, (0.0, 0.0))) for k in ("x", "y", "roll", "yaw")),
            cmd_vel_range=tuple(cmd.ranges.lin_vel_x), cmd_yaw_range=tuple(cmd.ranges.lin_vel_y),
            range_limit_vel=tuple(cmd.limit_ranges.lin_vel_x), range_limit_yaw=tuple(cmd.limit_ranges.lin_vel_y),
            cmd_resample_s=float(lo), cmd_rel_standing=float(cmd.rel_standing_envs),
            action_scale=float(act.scale), action_clip=float(chi),
            obs_corruption=bool(pol.enable_corruption),
            obs_noise=tuple(0.0 if n is None else float(n[1]) for n in noise),
            range_period_steps=None if self.curriculum.lin_vel_cmd_levels is not None else -1,
        )


@dataclass
class Zbot6BFlatEnvCfg_PLAY(Zbot6BFlatEnvCfg):
    """flat_env_cfg.py:193-204: 64 envs, no corruption, commands over the limit ranges."""

    def __post_init__(self):
        self.scene.num_envs = 64
        self.scene.env_spacing = 2.5
        self.observations.policy.enable_corruption = False
        self.commands.base_velocity.ranges = self.commands.base_velocity.limit_ranges


def _active(group) -> list:
    return [(f.name, getattr(group, f.name)) for f in fields(group) if getattr(group, f.name) is not None]


# ----------------------------------------------------------------------------- manager views
class _CommandManager:
    """The CommandManager accessors the reference's mdp / scripts use (get_command, get_term)."""

    def __init__(self, env: "ZbotManagerBasedRLEnv"):
        self._env = env

    # command_manager
    def get_command(self, name: str) -> torch.Tensor:
        if name != "base_velocity":
            raise KeyError(name)
        st = self._env.sim.get_state()
        return st[zm.M["COMMANDS"]:zm.M["COMMANDS"] + 3].T.contiguous()

    def get_term(self, name: str):
        if name != "base_velocity":
            raise KeyError(name)
        return self._env.cfg.commands.base_velocity


class ZbotManagerBasedRLEnv(ZbotDirectEnvV2):
    """``ManagerBasedRLEnv`` over ``Zbot6BFlatEnvCfg`` on the MI355X simulator."""

    _ep_len_row = zm.M["EP_LEN"]

    def __init__(self, cfg: Zbot6BFlatEnvCfg | None = None, render_mode: str | None = None, **kwargs):
        cfg = cfg or Zbot6BFlatEnvCfg()
        super().__init__(cfg, render_mode=render_mode, **kwargs)
        self.command_manager = _CommandManager(self)
        self.single_observation_space = spaces.Dict(policy=spaces.Box(-np.inf, np.inf, (zm.M_OBS_DIM,)))
        self.observation_space = spaces.Dict(policy=spaces.Box(-np.inf, np.inf, (self.num_envs, zm.M_OBS_DIM)))

    def _startup(self) -> None:
        """Startup events: init_my_data (the feet buffers live in the state rows) and
        randomize_rigid_body_material over every body shape (64 buckets of static / dynamic
        friction ~ U[0.3, 1.0]; static and dynamic coefficients go to the solver)."""
        ev = self.cfg.events.physics_material
        if ev is None:
            return
        p = ev.params
        g = torch.Generator().manual_seed(self.cfg.seed if self.cfg.seed is not None else 0)
        ranges = torch.tensor([p["static_friction_range"], p["dynamic_friction_range"], p["restitution_range"]])
        nb = int(p["num_buckets"])
        self.material_buckets = torch.rand(nb, 3, generator=g) * (ranges[:, 1] - ranges[:, 0]) + ranges[:, 0]
        bucket_ids = torch.randint(0, nb, (self.num_envs, zm.NUM_LINKS), generator=g)
        self.link_materials = self.material_buckets[bucket_ids]
        self.sim.set_link_friction(self.link_materials[..., 0], self.link_materials[..., 1])

    def _update_log(self) -> None:
        """extras["log"] in ManagerBasedRLEnv._reset_idx order: Episode_Reward/<term> (reward
        manager: mean episodic sum / 20 s), Curriculum/lin_vel_cmd_levels, Metrics/base_velocity/*,
        Episode_Termination/<term> counts (device 0-dim tensors: no per-step host sync)."""
        if getattr(self, "_log", None) is None:
            means, counts = self.sim.read_log()
            buf = self.sim.log_buffer
            log = {f"Episode_Reward/{k}": means[i] for i, k in enumerate(zm.M_REWARD_TERMS)}
            if self.cfg.curriculum.lin_vel_cmd_levels is not None:
                log["Curriculum/lin_vel_cmd_levels"] = buf[16]
            log["Metrics/base_velocity/error_vel_xy"] = buf[17]
            log["Metrics/base_velocity/error_vel_yaw"] = buf[18]
            log["Episode_Termination/time_out"] = counts[1]
            log["Episode_Termination/base_height"] = counts[0]
            log["Episode_Termination/feet_close"] = counts[2]
            self._log = log
        self.extras["log"] = self._log

    @property
    def max_episode_length_s(self) -> float:
        return self.cfg.episode_length_s

    @max_episode_length_s.setter
    def max_episode_length_s(self, value) -> None:
        pass

    @property
    def reward_scales(self) -> dict:
        return {k: t.weight for k, t in _active(self.cfg.rewards)}

    @reward_scales.setter
    def reward_scales(self, value) -> None:  # set by the base __init__; the weights live in the cfg
        pass
