"""Generate MDP golden vectors from the reference's OWN v2 code (build container only).

SURVEY.md Appendix B recipe: the reference module
``source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v2.py`` is imported from
/root/reference with stub ``isaaclab`` / ``gymnasium`` / ``zbot.assets`` packages (Isaac Lab, Isaac
Sim and gymnasium are not installed). The stubs only supply what v2 touches: config classes that
accept kwargs, ``configclass`` = identity, ``quat_apply`` (standard wxyz rotation), and a
``DirectRLEnv`` base that wires fake robot / contact-sensor / terrain data objects. The env is then
driven exactly like ``DirectRLEnv.step`` calls it (minus physics and resets):

    _pre_physics_step(a) ; episode_length_buf += 1 ; reset_terminated, reset_time_outs = _get_dones()
    reward = _get_rewards() ; obs = _get_observations()

on seeded synthetic body / contact states. Inputs and outputs are written to
``tests/golden/mdp_v2.npz`` (data only — no reference code leaves this container). Per-term
rewards are captured by wrapping each ``_reward_<name>``.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v2.py"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "mdp_v2.npz")
N, T = 16, 12


def quat_apply(quat, vec):
    shape = vec.shape
    quat = quat.reshape(-1, 4)
    vec = vec.reshape(-1, 3)
    xyz = quat[:, 1:]
    t = xyz.cross(vec, dim=-1) * 2
    return (vec + quat[:, 0:1] * t + xyz.cross(t, dim=-1)).view(shape)


class _Cfg:
    def __init__(self, *args, **kwargs):
        self.__dict__.update(kwargs)

    def replace(self, **kwargs):
        c = _Cfg(**self.__dict__)
        c.__dict__.update(kwargs)
        return c

    def func(self, *args, **kwargs):
        return None


class _Data:
    pass


class _Robot:
    def __init__(self):
        self.data = _Data()

    def find_bodies(self, expr):
        return {"base": ([6], ["base"]), "foot.*": ([0, 11], ["foot_0", "foot_1"])}[expr]


class _Sensor:
    def __init__(self):
        self.data = _Data()

    def find_bodies(self, expr):
        names = ["foot_0", "b1", "a2", "b2", "a3", "b3", "base", "b4", "a5", "b5", "a6", "foot_1"]
        if expr == "foot.*":
            return [0, 11], ["foot_0", "foot_1"]
        if expr == "base|a.*|b.*":
            ids = [i for i, n in enumerate(names) if n == "base" or n[0] in "ab"]
            return ids, [names[i] for i in ids]
        raise KeyError(expr)


FAKES = {}


class DirectRLEnv:
    def __init__(self, cfg, render_mode=None, **kwargs):
        self.cfg = cfg
        self.num_envs = N
        self.device = "cpu"
        self.sim = _Cfg(device="cpu")
        self.step_dt = cfg.sim.dt * cfg.decimation
        self.max_episode_length_s = cfg.episode_length_s
        self.max_episode_length = int(np.ceil(cfg.episode_length_s / self.step_dt))
        self.single_action_space = _Cfg(shape=(cfg.action_space,))
        self._robot = FAKES["robot"]
        self._contact_sensor = FAKES["sensor"]
        self._terrain = FAKES["terrain"]
        self.episode_length_buf = torch.zeros(N, dtype=torch.long)
        self.reset_terminated = torch.zeros(N, dtype=torch.bool)
        self.reset_time_outs = torch.zeros(N, dtype=torch.bool)
        self.extras = {}


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    spaces = mod("gymnasium.spaces", flatdim=lambda s: int(np.prod(s.shape)))
    mod("gymnasium", spaces=spaces)
    sim = mod("isaaclab.sim", SimulationCfg=_Cfg, RigidBodyMaterialCfg=_Cfg, DomeLightCfg=_Cfg)
    umath = mod("isaaclab.utils.math", quat_apply=quat_apply)
    utils = mod("isaaclab.utils", configclass=lambda c: c, math=umath)
    mod("isaaclab.assets", Articulation=object, ArticulationCfg=_Cfg)
    mod("isaaclab.envs", DirectRLEnv=DirectRLEnv, DirectRLEnvCfg=object)
    mod("isaaclab.scene", InteractiveSceneCfg=_Cfg)
    mod("isaaclab.sensors", ContactSensor=object, ContactSensorCfg=_Cfg)
    mod("isaaclab.terrains", TerrainImporterCfg=_Cfg)
    mod("isaaclab", sim=sim, utils=utils)
    mod("zbot.assets", ZBOT_6S_CFG=_Cfg())
    mod("zbot")


def random_quat(rng, n):
    q = rng.normal(size=(n, 4))
    return (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)


def make_frame(rng, origins):
    """One synthetic post-physics snapshot of everything v2 reads from the robot / sensor."""
    f = {}
    f["joint_pos"] = (rng.normal(0, 0.5, (N, 6))).astype(np.float32)
    f["joint_vel"] = rng.normal(0, 2.0, (N, 6)).astype(np.float32)
    pos = rng.normal(0, 0.1, (N, 12, 3)).astype(np.float32)
    pos[:, :, 2] = rng.uniform(0.0, 0.35, (N, 12))
    pos[:, 6, 2] = rng.uniform(0.2, 0.32, N)          # base height around the 0.22 threshold
    pos[:, 6, 1] = rng.normal(0, 0.3, N)             # base y around the +-0.5 band
    pos[:, :, :2] += origins[:, None, :2]             # world frame = env origin + local
    f["body_link_pos_w"] = pos
    quat = np.stack([random_quat(rng, N) for _ in range(12)], axis=1)
    f["body_link_quat_w"] = quat
    f["body_com_lin_vel_w"] = rng.normal(0, 0.5, (N, 12, 3)).astype(np.float32)
    f["applied_torque"] = rng.uniform(-20, 20, (N, 6)).astype(np.float32)
    hist = rng.normal(0, 0.15, (N, 5, 12, 3)).astype(np.float32)
    big = rng.random((N, 5, 12)) < 0.2
    hist[..., 2] += np.where(big, rng.uniform(0, 30, (N, 5, 12)), 0)
    quiet = rng.random(N) < 0.6                       # some envs with no undesired contact at all
    undesired = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
    for e in np.nonzero(quiet)[0]:
        hist[e][:, undesired, :] *= 0.01
    f["net_forces_w_history"] = hist
    f["last_air_time"] = rng.uniform(0, 1.0, (N, 12)).astype(np.float32)
    f["current_contact_time"] = rng.uniform(0, 1.0, (N, 12)).astype(np.float32)
    return f


def apply_frame(robot, sensor, f):
    for k in ("joint_pos", "joint_vel", "body_link_pos_w", "body_link_quat_w", "body_com_lin_vel_w", "applied_torque"):
        setattr(robot.data, k, torch.from_numpy(f[k].copy()))
    for k in ("net_forces_w_history", "last_air_time", "current_contact_time"):
        setattr(sensor.data, k, torch.from_numpy(f[k].copy()))


def main():
    install_stubs()
    rng = np.random.default_rng(20260213)
    robot, sensor = _Robot(), _Sensor()
    q0 = np.array([0.312, 0.837, -2.02, 2.02, -0.837, -0.312], np.float32)
    robot.data.default_joint_pos = torch.from_numpy(np.tile(q0, (N, 1)))
    robot.data.GRAVITY_VEC_W = torch.tensor([0.0, 0.0, -1.0]).repeat(N, 1)
    origins = rng.normal(0, 4.0, (N, 3)).astype(np.float32)
    origins[:, 2] = 0
    terrain = _Cfg(env_origins=torch.from_numpy(origins))
    FAKES.update(robot=robot, sensor=sensor, terrain=terrain)

    spec = importlib.util.spec_from_file_location("ref_zbot_v2", REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    cfg = ref.ZbotDirectEnvCfgV2()
    cfg.reward_cfg = {"reward_scales": dict(ref.ZbotDirectEnvCfgV2.reward_cfg["reward_scales"])}
    env = ref.ZbotDirectEnvV2(cfg)
    term_names = list(env.reward_scales.keys())
    scaled = [float(env.reward_scales[k]) for k in term_names]

    captured = {}
    for name in term_names:
        fn = env.reward_functions[name]

        def wrap(fn=fn, name=name):
            def g():
                v = fn()
                captured[name] = v.detach().clone()
                return v
            return g
        env.reward_functions[name] = wrap()

    frames = [make_frame(rng, origins) for _ in range(T + 1)]
    apply_frame(robot, sensor, frames[0])
    env.episode_length_buf[:] = torch.from_numpy(rng.integers(975, 999, N))
    # non-trivial persistent state at t=0
    env.feet_down_pos_last[:] = torch.from_numpy(rng.normal(0, 0.2, (N, 2, 3)).astype(np.float32))
    env.feet_contact_forces_last[:] = torch.from_numpy(rng.uniform(0, 20, (N, 2)).astype(np.float32))
    env.feet_step_length[:] = torch.from_numpy(rng.normal(0, 0.05, (N, 2)).astype(np.float32))
    init_state = {
        "feet_down_pos_last": env.feet_down_pos_last.numpy().copy(),
        "feet_contact_forces_last": env.feet_contact_forces_last.numpy().copy(),
        "feet_step_length": env.feet_step_length.numpy().copy(),
        "episode_length_buf": env.episode_length_buf.numpy().astype(np.int32).copy(),
    }
    obs0 = env._get_observations()["policy"].numpy().copy()

    rec = {k: [] for k in ("actions", "tanh_actions", "prev_actions", "p_delta", "processed_actions", "died",
                           "time_out", "reward", "terms", "obs", "heading_sum", "y_err_sum", "feet_step_length",
                           "feet_down_pos_last", "feet_contact_forces_last", "episode_sums", "episode_length_buf")}
    for t in range(T):
        a = rng.normal(0, 1.5, (N, 6)).astype(np.float32)
        env._pre_physics_step(torch.from_numpy(a))
        apply_frame(robot, sensor, frames[t + 1])
        env.episode_length_buf += 1
        died, tout = env._get_dones()
        env.reset_terminated[:] = died
        env.reset_time_outs[:] = tout
        rec["prev_actions"].append(env._previous_actions.numpy().copy())
        r = env._get_rewards()
        obs = env._get_observations()["policy"]
        rec["actions"].append(a)
        rec["tanh_actions"].append(env._actions.numpy().copy())
        rec["p_delta"].append(env.p_delta.numpy().copy())
        rec["processed_actions"].append(env._processed_actions.numpy().copy())
        rec["died"].append(died.numpy().copy())
        rec["time_out"].append(tout.numpy().copy())
        rec["reward"].append(r.numpy().copy())
        rec["terms"].append(np.stack([captured[k].numpy() * s for k, s in zip(term_names, scaled)], axis=1))
        rec["obs"].append(obs.numpy().copy())
        rec["heading_sum"].append(env.base_heading_x_sum.numpy().copy())
        rec["y_err_sum"].append(env.base_pos_y_err_sum.numpy().copy())
        rec["feet_step_length"].append(env.feet_step_length.numpy().copy())
        rec["feet_down_pos_last"].append(env.feet_down_pos_last.numpy().copy())
        rec["feet_contact_forces_last"].append(env.feet_contact_forces_last.numpy().copy())
        rec["episode_sums"].append(np.stack([env._episode_sums[k].numpy() for k in term_names], axis=1))
        rec["episode_length_buf"].append(env.episode_length_buf.numpy().astype(np.int32).copy())

    out = {f"frame_{k}": np.stack([fr[k] for fr in frames]) for k in frames[0]}
    out.update({k: np.stack(v) for k, v in rec.items()})
    out.update({f"init_{k}": v for k, v in init_state.items()})
    out["obs0"] = obs0
    out["env_origins"] = origins
    out["default_joint_pos"] = q0
    out["term_names"] = np.array(term_names)
    out["scales_x_step_dt"] = np.array(scaled, np.float64)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print("wrote", os.path.normpath(OUT), {k: v.shape for k, v in out.items() if hasattr(v, "shape")})
    print("died rate", np.mean(out["died"]), "timeouts", np.mean(out["time_out"]))


if __name__ == "__main__":
    main()
