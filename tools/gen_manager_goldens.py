"""Generate manager-env golden vectors from the reference's OWN code (build container only).

Target: ``zbot-6b-walking-m-v0`` = ``ManagerBasedRLEnv`` over ``Zbot6BFlatEnvCfg``
(``source/zbot/zbot/tasks/zbotlab_manager``). The reference modules are imported from
/root/reference with stub ``isaaclab`` / ``isaaclab_rl`` / ``zbot.assets`` packages (Isaac Lab is not
in the reference tree):

* the config classes ``zbotlab_env_cfg.py`` -> ``rough_env_cfg.py`` -> ``flat_env_cfg.py`` and
  ``agents/rsl_rl_ppo_cfg.py`` are instantiated (``__post_init__`` chains run), and every value the
  simulator consumes is recorded: reward terms (order, weight, params), terminations, command
  ranges / limits / resampling / standing fraction, action scale / clip / offset, observation terms
  and noise, events, curriculum terms, dt / decimation / episode length, PPO runner settings;
* the MDP term functions of ``mdp/rewards.py``, ``mdp/terminations.py`` and ``mdp/curriculums.py``
  are called through the cfg's own ``func`` / ``params`` / ``weight`` on seeded synthetic
  articulation / contact-sensor frames (32 envs x 16 calls, the RewardManager's
  ``value = func(env, **params) * weight * dt`` accumulation), plus ``init_my_data`` /
  ``reset_my_data`` and ``lin_vel_cmd_levels`` around its trigger.

Isaac Lab functions the cfg names that are not in the reference tree (``is_terminated``,
``joint_torques_l2``, ``joint_acc_l2``, ``action_rate_l2``, ``time_out``,
``root_height_below_minimum``, ``yaw_quat``, ``quat_apply``, ``quat_apply_inverse``) are restated here
from their published definitions; those four reward terms are therefore pinned to the restatement,
not to reference code. Output: ``tests/golden/mdp_manager.npz`` (data only).
"""
from __future__ import annotations

import importlib
import json
import os
import sys
import types

import numpy as np
import torch

REF_TASKS = "/root/reference/source/zbot/zbot/tasks"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "mdp_manager.npz")
N, T = 32, 16
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_standup_goldens import _Cfg, quat_apply, random_quat, upright_ish  # noqa: E402


# --- Isaac Lab math / mdp functions the cfg uses (isaaclab.utils.math, isaaclab.envs.mdp), restated --
def quat_conjugate(q):
    return torch.cat((q[..., 0:1], -q[..., 1:]), dim=-1)


def quat_apply_inverse(quat, vec):
    return quat_apply(quat_conjugate(quat), vec)


def yaw_quat(quat):
    shape = quat.shape
    q = quat.view(-1, 4)
    qw, qx, qy, qz = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    yaw = torch.atan2(2 * (qw * qz + qx * qy), 1 - 2 * (qy * qy + qz * qz))
    out = torch.zeros_like(q)
    out[:, 3] = torch.sin(yaw / 2)
    out[:, 0] = torch.cos(yaw / 2)
    out = out / out.norm(dim=-1, keepdim=True)
    return out.view(shape)


def is_terminated(env):
    return env.termination_manager.terminated.float()


def joint_torques_l2(env, asset_cfg=None):
    return torch.sum(torch.square(env.scene["robot"].data.applied_torque), dim=1)


def joint_acc_l2(env, asset_cfg=None):
    return torch.sum(torch.square(env.scene["robot"].data.joint_acc), dim=1)


def action_rate_l2(env):
    return torch.sum(torch.square(env.action_manager.action - env.action_manager.prev_action), dim=1)


def time_out(env):
    return env.episode_length_buf >= env.max_episode_length


def root_height_below_minimum(env, minimum_height, asset_cfg=None):
    return env.scene["robot"].data.root_pos_w[:, 2] < minimum_height


class _Named:
    """Placeholder for an Isaac Lab function the simulator implements natively (names only)."""

    def __init__(self, name):
        self.__name__ = name

    def __call__(self, *a, **k):
        raise RuntimeError(f"{self.__name__} is not restated by the golden generator")


class SceneEntityCfg(_Cfg):
    def __init__(self, name, body_names=None, joint_names=None, **kw):
        super().__init__(name=name, body_names=body_names, joint_names=joint_names, **kw)
        self.body_ids = [0, 11] if body_names == "foot.*" else slice(None)


class UniformVelocityCommandCfg(_Cfg):
    class Ranges(_Cfg):
        pass


class _Group(_Cfg):
    """ObservationGroupCfg stand-in (a configclass: __post_init__ runs on construction)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        if hasattr(self, "__post_init__"):
            self.__post_init__()


class _CfgBase:
    """ManagerBasedRLEnvCfg / RslRlOnPolicyRunnerCfg stand-in: class-level configclass fields."""

    def __init__(self):
        self.sim = _Cfg(dt=None, render_interval=None, physics_material=None, physx=_Cfg())
        self.__post_init__()

    def __post_init__(self):
        pass


def install_stubs():
    def mod(name, path=None, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        if path is not None:
            m.__path__ = [path]
        sys.modules[name] = m
        return m

    names = {}

    def named(attr):
        if attr.startswith("__"):
            raise AttributeError(attr)
        return names.setdefault(attr, _Named(attr))

    envs_mdp = mod("isaaclab.envs.mdp", UniformVelocityCommandCfg=UniformVelocityCommandCfg,
                   is_terminated=is_terminated, joint_torques_l2=joint_torques_l2, joint_acc_l2=joint_acc_l2,
                   action_rate_l2=action_rate_l2, time_out=time_out,
                   root_height_below_minimum=root_height_below_minimum,
                   RelativeJointPositionActionCfg=_Cfg, JointPositionActionCfg=_Cfg)
    envs_mdp.__getattr__ = named
    mod("isaaclab.envs", ManagerBasedRLEnvCfg=_CfgBase, ManagerBasedRLEnv=object, mdp=envs_mdp)
    mod("isaaclab.managers", CurriculumTermCfg=_Cfg, EventTermCfg=_Cfg, ObservationGroupCfg=_Group,
        ObservationTermCfg=_Cfg, RewardTermCfg=_Cfg, SceneEntityCfg=SceneEntityCfg, TerminationTermCfg=_Cfg)
    sim = mod("isaaclab.sim", RigidBodyMaterialCfg=_Cfg, MdlFileCfg=_Cfg, DomeLightCfg=_Cfg, UsdFileCfg=_Cfg)
    umath = mod("isaaclab.utils.math", quat_apply=quat_apply, quat_apply_inverse=quat_apply_inverse,
                yaw_quat=yaw_quat)
    mod("isaaclab.utils.noise", AdditiveUniformNoiseCfg=_Cfg)
    mod("isaaclab.utils.assets", ISAAC_NUCLEUS_DIR="nucleus", ISAACLAB_NUCLEUS_DIR="nucleus")
    mod("isaaclab.utils", configclass=lambda c: c, math=umath)
    mod("isaaclab.assets", ArticulationCfg=_Cfg, AssetBaseCfg=_Cfg, Articulation=object, RigidObject=object)
    mod("isaaclab.scene", InteractiveSceneCfg=_Cfg)
    mod("isaaclab.sensors", ContactSensorCfg=_Cfg, ContactSensor=object)
    mod("isaaclab.terrains", TerrainImporterCfg=_Cfg, TerrainImporter=object)
    mod("isaaclab.terrains.config")
    mod("isaaclab.terrains.config.rough", ROUGH_TERRAINS_CFG=_Cfg(curriculum=None))
    marker = _Cfg()
    mod("isaaclab.markers")
    mod("isaaclab.markers.config", RED_ARROW_X_MARKER_CFG=marker)
    mod("isaaclab", sim=sim)
    mod("isaaclab_rl")
    mod("isaaclab_rl.rsl_rl", RslRlOnPolicyRunnerCfg=_CfgBase, RslRlPpoActorCriticCfg=_Cfg,
        RslRlPpoAlgorithmCfg=_Cfg)
    robot_cfg = _Cfg()
    mod("zbot.assets", ZBOT_6S_2_CFG=robot_cfg, ZBOT_6S_V1_CFG=robot_cfg, ZBOT_6S_V2_CFG=robot_cfg)
    # reference packages resolved from /root/reference without running their __init__ (gym.register)
    mod("zbot", path=os.path.dirname(REF_TASKS))
    mod("zbot.tasks", path=REF_TASKS)
    mgr = os.path.join(REF_TASKS, "zbotlab_manager")
    mod("zbot.tasks.zbotlab_manager", path=mgr)
    mod("zbot.tasks.zbotlab_manager.config", path=os.path.join(mgr, "config"))
    mod("zbot.tasks.zbotlab_manager.config.zbot6b_manager", path=os.path.join(mgr, "config", "zbot6b_manager"))
    mod("zbot.tasks.zbotlab_manager.config.zbot6b_manager.agents",
        path=os.path.join(mgr, "config", "zbot6b_manager", "agents"))
    mdp = importlib.import_module("zbot.tasks.zbotlab_manager.mdp")
    mdp.__getattr__ = named
    return mdp


def fields(obj):
    """configclass fields in declaration order (class attributes, then instance overrides)."""
    out = {}
    for klass in reversed(type(obj).__mro__):
        for k, v in vars(klass).items():
            if not k.startswith("_") and not callable(v) and not isinstance(v, (property, classmethod, staticmethod)):
                out[k] = None
    for k in list(out):
        out[k] = getattr(obj, k)
    for k, v in vars(obj).items():
        if not k.startswith("_") and k not in out:
            out[k] = v
    return out


def fname(f):
    return getattr(f, "__name__", str(f))


def cfg_record(cfg, ppo):
    rew = [(k, fname(t.func), float(t.weight), {p: v for p, v in getattr(t, 'params', {}).items() if not isinstance(v, SceneEntityCfg)})
           for k, t in fields(cfg.rewards).items() if t is not None]
    term = [(k, fname(t.func), bool(getattr(t, "time_out", False)),
             {p: v for p, v in getattr(t, "params", {}).items() if not isinstance(v, SceneEntityCfg)})
            for k, t in fields(cfg.terminations).items() if t is not None]
    cmd = cfg.commands.base_velocity
    act = cfg.actions.joint_pos
    pol = cfg.observations.policy
    obs = [(k, fname(t.func), None if getattr(t, "noise", None) is None else [t.noise.n_min, t.noise.n_max])
           for k, t in fields(pol).items() if isinstance(t, _Cfg) and hasattr(t, "func")]
    ev = [(k, fname(t.func), t.mode, {p: v for p, v in getattr(t, "params", {}).items()
                                      if not isinstance(v, SceneEntityCfg)})
          for k, t in fields(cfg.events).items() if t is not None]
    cur = [(k, fname(t.func)) for k, t in fields(cfg.curriculum).items() if t is not None]
    rec = dict(
        decimation=cfg.decimation, episode_length_s=cfg.episode_length_s, sim_dt=cfg.sim.dt,
        rewards=rew, terminations=term, observations=obs, enable_corruption=bool(pol.enable_corruption),
        events=ev, curriculum=cur,
        command=dict(resampling_time_range=list(cmd.resampling_time_range), rel_standing_envs=cmd.rel_standing_envs,
                     heading_command=cmd.heading_command,
                     ranges=dict(lin_vel_x=list(cmd.ranges.lin_vel_x), lin_vel_y=list(cmd.ranges.lin_vel_y),
                                 ang_vel_z=list(cmd.ranges.ang_vel_z)),
                     limit_ranges=dict(lin_vel_x=list(cmd.limit_ranges.lin_vel_x),
                                       lin_vel_y=list(cmd.limit_ranges.lin_vel_y),
                                       ang_vel_z=list(cmd.limit_ranges.ang_vel_z))),
        action=dict(scale=act.scale, clip=act.clip, use_zero_offset=act.use_zero_offset, joint_names=act.joint_names),
        contact_sensor=dict(history_length=cfg.scene.contact_forces.history_length,
                            track_air_time=cfg.scene.contact_forces.track_air_time,
                            update_period=cfg.scene.contact_forces.update_period),
        terrain_type=cfg.scene.terrain.terrain_type, num_envs=cfg.scene.num_envs,
        env_spacing=cfg.scene.env_spacing,
        ppo=dict(num_steps_per_env=ppo.num_steps_per_env, max_iterations=ppo.max_iterations,
                 save_interval=ppo.save_interval, experiment_name=ppo.experiment_name,
                 policy=vars(ppo.policy), algorithm=vars(ppo.algorithm)),
    )
    return rec


# ------------------------------------------------------------------------ fake env for the terms
class _Data:
    pass


class _Robot:
    def __init__(self):
        self.data = _Data()


class _Sensor:
    def __init__(self):
        self.data = _Data()
        self.cfg = _Cfg(track_air_time=True)


class _Scene(dict):
    def __init__(self, robot, sensor):
        super().__init__(robot=robot, contact_forces=sensor)
        self.sensors = {"contact_forces": sensor}


def make_frame(rng):
    f = {}
    f["root_pos_w"] = np.stack([rng.normal(0, 0.3, N), rng.normal(0, 0.3, N), rng.uniform(0.16, 0.30, N)], 1)
    f["root_quat_w"] = random_quat(rng, N)
    f["root_link_lin_vel_w"] = rng.normal(0, 0.3, (N, 3))
    f["root_link_ang_vel_w"] = rng.normal(0, 0.8, (N, 3))
    pos = rng.normal(0, 0.08, (N, 12, 3))
    pos[:, :, 2] = rng.uniform(0.0, 0.3, (N, 12))
    pos[:, 0, :2] = f["root_pos_w"][:, :2] + rng.normal(0, 0.07, (N, 2))
    pos[:, 11, :2] = pos[:, 0, :2] + rng.normal(0, 0.09, (N, 2))     # feet distance around 0.12
    f["body_link_pos_w"] = pos
    quat = np.stack([random_quat(rng, N) for _ in range(12)], axis=1)
    quat[:, 0] = upright_ish(rng, N, +1)
    quat[:, 11] = upright_ish(rng, N, -1)
    f["body_link_quat_w"] = quat
    f["body_lin_vel_w"] = rng.normal(0, 0.4, (N, 12, 3))
    f["applied_torque"] = rng.uniform(-20, 20, (N, 6))
    f["joint_acc"] = rng.normal(0, 300.0, (N, 6))
    hist = rng.normal(0, 0.6, (N, 3, 12, 3))
    big = rng.random((N, 3, 12)) < 0.35
    hist[..., 2] += np.where(big, rng.uniform(0, 30, (N, 3, 12)), 0)
    f["net_forces_w_history"] = hist
    f["last_air_time"] = rng.uniform(0, 1.0, (N, 12))
    return {k: v.astype(np.float32) for k, v in f.items()}


def main():
    mdp = install_stubs()
    flat = importlib.import_module("zbot.tasks.zbotlab_manager.config.zbot6b_manager.flat_env_cfg")
    agents = importlib.import_module("zbot.tasks.zbotlab_manager.config.zbot6b_manager.agents.rsl_rl_ppo_cfg")
    cfg = flat.Zbot6BFlatEnvCfg()
    ppo = agents.Zbot6BFlatPPORunnerCfg()
    rec = cfg_record(cfg, ppo)

    rng = np.random.default_rng(20260214)
    robot, sensor = _Robot(), _Sensor()
    robot.data.GRAVITY_VEC_W = torch.tensor([0.0, 0.0, -1.0]).repeat(N, 1)
    cmd = np.stack([rng.uniform(-0.3, 0.3, N), rng.choice([0.0, 0.1, -0.2], N), rng.choice([0.0, 0.3], N)],
                   1).astype(np.float32)
    step_dt = cfg.sim.dt * cfg.decimation
    max_len = int(np.ceil(cfg.episode_length_s / step_dt))
    env = types.SimpleNamespace(
        num_envs=N, device="cpu", sim=_Cfg(device="cpu"), scene=_Scene(robot, sensor),
        command_manager=_Cfg(get_command=lambda name: torch.from_numpy(cmd)),
        action_manager=_Cfg(action=None, prev_action=None), termination_manager=_Cfg(terminated=None),
        episode_length_buf=torch.zeros(N, dtype=torch.long), max_episode_length=max_len,
        max_episode_length_s=cfg.episode_length_s, step_dt=step_dt)
    mdp.init_my_data(env, None)
    init = {"feet_down_pos_last": rng.normal(0, 0.2, (N, 2, 3)).astype(np.float32),
            "feet_contact_forces_last": rng.uniform(0, 20, (N, 2)).astype(np.float32),
            "feet_step_length": rng.uniform(0, 0.08, (N, 2)).astype(np.float32)}
    env.feet_down_pos_last[:] = torch.from_numpy(init["feet_down_pos_last"])
    env.feet_contact_forces_last[:] = torch.from_numpy(init["feet_contact_forces_last"])
    env.feet_step_length[:] = torch.from_numpy(init["feet_step_length"])
    ep0 = rng.choice([10, 500, 997, 998, 999], N).astype(np.int64)
    env.episode_length_buf[:] = torch.from_numpy(ep0)

    rew_terms = [(k, t) for k, t in fields(cfg.rewards).items() if t is not None]
    term_terms = [(k, t) for k, t in fields(cfg.terminations).items() if t is not None]
    out = {k: [] for k in ("frames", "actions", "prev_actions", "terms", "reward", "episode_sums", "dones",
                           "feet_down_pos_last", "feet_contact_forces_last", "feet_step_length", "ep_len")}
    frames = []
    sums = torch.zeros(N, len(rew_terms))
    prev = np.zeros((N, 6), np.float32)
    for t in range(T):
        f = make_frame(rng)
        frames.append(f)
        for k in ("root_pos_w", "root_quat_w", "root_link_lin_vel_w", "root_link_ang_vel_w", "body_link_pos_w",
                  "body_link_quat_w", "body_lin_vel_w", "applied_torque", "joint_acc"):
            setattr(robot.data, k, torch.from_numpy(f[k].copy()))
        for k in ("net_forces_w_history", "last_air_time"):
            setattr(sensor.data, k, torch.from_numpy(f[k].copy()))
        act = rng.normal(0, 1.0, (N, 6)).astype(np.float32)
        env.action_manager.action = torch.from_numpy(act)
        env.action_manager.prev_action = torch.from_numpy(prev)
        env.episode_length_buf += 1   # ManagerBasedRLEnv.step, before the managers
        dones = []
        for k, tc in term_terms:      # TerminationManager.compute
            dones.append(tc.func(env, **getattr(tc, 'params', {})).bool())
        dones = torch.stack(dones, 1)
        tout_cols = [i for i, (k, tc) in enumerate(term_terms) if getattr(tc, "time_out", False)]
        term_cols = [i for i in range(len(term_terms)) if i not in tout_cols]
        env.termination_manager.terminated = dones[:, term_cols].any(1)
        vals = []
        reward = torch.zeros(N)
        for i, (k, tc) in enumerate(rew_terms):   # RewardManager.compute
            raw = tc.func(env, **getattr(tc, 'params', {}))
            v = raw * tc.weight * step_dt
            reward += v
            sums[:, i] += v
            vals.append(raw.float())
        out["frames"].append(f)
        out["actions"].append(act)
        out["prev_actions"].append(prev.copy())
        out["terms"].append(torch.stack(vals, 1).numpy())
        out["reward"].append(reward.numpy())
        out["episode_sums"].append(sums.numpy().copy())
        out["dones"].append(dones.numpy())
        out["feet_down_pos_last"].append(env.feet_down_pos_last.numpy().copy())
        out["feet_contact_forces_last"].append(env.feet_contact_forces_last.numpy().copy())
        out["feet_step_length"].append(env.feet_step_length.numpy().copy())
        out["ep_len"].append(env.episode_length_buf.numpy().astype(np.int32).copy())
        prev = act

    gold = {"config_json": np.array(json.dumps(rec, default=float)),
            "reward_names": np.array([k for k, _ in rew_terms]),
            "termination_names": np.array([k for k, _ in term_terms]),
            "commands": cmd, "step_dt": np.float32(step_dt), "max_episode_length": np.int32(max_len),
            "init_ep_len": ep0.astype(np.int32)}
    for k, v in init.items():
        gold["init_" + k] = v
    for k in out:
        if k == "frames":
            for fk in frames[0]:
                gold["frame_" + fk] = np.stack([fr[fk] for fr in frames])
        else:
            gold[k] = np.stack(out[k])

    # reset_my_data: feet_down_pos_last <- the feet body_link_pos_w of the reset envs; the other
    # per-env buffers zeroed
    ids = torch.tensor([1, 4, 9])
    mdp.reset_my_data(env, ids, SceneEntityCfg("robot", body_names="foot.*"))
    gold["reset_ids"] = ids.numpy().astype(np.int32)
    gold["reset_feet_down_pos_last"] = env.feet_down_pos_last.numpy().copy()
    gold["reset_feet_step_length"] = env.feet_step_length.numpy().copy()
    gold["reset_feet_contact_forces_last"] = env.feet_contact_forces_last.numpy().copy()

    # lin_vel_cmd_levels: (common_step_counter, mean episodic tracking sum) -> ranges after
    cterm = cfg.commands.base_velocity
    ranges0 = (list(cterm.ranges.lin_vel_x), list(cterm.ranges.lin_vel_y))
    rm_sums = {"track_lin_vel_xy_exp": torch.zeros(4)}
    wterm = cfg.rewards.track_lin_vel_xy_exp
    cenv = types.SimpleNamespace(
        device="cpu", command_manager=_Cfg(get_term=lambda name: _Cfg(cfg=cterm)),
        reward_manager=_Cfg(_episode_sums=rm_sums, get_term_cfg=lambda name: wterm),
        max_episode_length=max_len, max_episode_length_s=cfg.episode_length_s, common_step_counter=0)
    cases = [(0, 16.5), (1000, 15.9), (1000, 16.1), (1500, 19.0), (2000, 17.0), (3000, 18.0), (4000, 19.5),
             (4001, 20.0), (5000, 12.0), (6000, 16.2)]
    rows = []
    for counter, total in cases:
        cenv.common_step_counter = counter
        rm_sums["track_lin_vel_xy_exp"][:] = torch.tensor([total - 0.3, total + 0.3, total - 0.1, total + 0.1])
        val = mdp.lin_vel_cmd_levels(cenv, torch.arange(4))
        rows.append([counter, total / cfg.episode_length_s, *cterm.ranges.lin_vel_x, *cterm.ranges.lin_vel_y,
                     float(val)])
    gold["curriculum_rows"] = np.array(rows, np.float64)
    gold["curriculum_ranges0"] = np.array(ranges0, np.float64)
    np.savez_compressed(OUT, **gold)
    print("wrote", os.path.abspath(OUT), {k: np.asarray(v).shape for k, v in gold.items()})


if __name__ == "__main__":
    main()
