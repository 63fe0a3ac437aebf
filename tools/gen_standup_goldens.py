"""Generate stand-up MDP golden vectors from the reference's OWN standup code (build container only).

Same recipe as ``tools/gen_mdp_goldens.py``: the reference module
``source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6_standup_env_v0.py`` is imported from
/root/reference with stub ``isaaclab`` / ``gymnasium`` / ``zbot.assets`` packages (Isaac Lab, Isaac
Sim and gymnasium are not installed). The stubs supply config classes that accept kwargs,
``configclass`` = identity, the Isaac Lab math the module calls (``quat_apply``, ``quat_mul``,
``quat_from_euler_xyz``, ``sample_uniform`` — restated here from their published definitions,
Isaac Lab being absent) and a ``DirectRLEnv`` base wiring a fake robot. The env is driven the way
``DirectRLEnv.step`` calls it (minus physics and resets):

    _pre_physics_step(a) ; episode_length_buf += 1 ; common_step_counter += 1
    reset_terminated, reset_time_outs = _get_dones() ; reward = _get_rewards() ; obs = _get_observations()

on seeded synthetic body states, then ``_reset_idx`` on a subset (episode log), the module's own
``reset_root_state_uniform`` on chosen samples (reset pose composition) and ``my_curriculum`` around
its threshold. Inputs and outputs go to ``tests/golden/mdp_standup.npz`` (data only — no reference
code leaves this container).
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6_standup_env_v0.py"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "mdp_standup.npz")
N, T = 32, 16


# --- Isaac Lab math (isaaclab.utils.math), restated -------------------------------------------
def quat_apply(quat, vec):
    shape = vec.shape
    quat = quat.reshape(-1, 4)
    vec = vec.reshape(-1, 3)
    xyz = quat[:, 1:]
    t = xyz.cross(vec, dim=-1) * 2
    return (vec + quat[:, 0:1] * t + xyz.cross(t, dim=-1)).view(shape)


def quat_mul(q1, q2):
    w1, x1, y1, z1 = q1.unbind(-1)
    w2, x2, y2, z2 = q2.unbind(-1)
    return torch.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], dim=-1)


def quat_from_euler_xyz(roll, pitch, yaw):
    cy, sy = torch.cos(yaw * 0.5), torch.sin(yaw * 0.5)
    cr, sr = torch.cos(roll * 0.5), torch.sin(roll * 0.5)
    cp, sp = torch.cos(pitch * 0.5), torch.sin(pitch * 0.5)
    return torch.stack([cy * cr * cp + sy * sr * sp, cy * sr * cp - sy * cr * sp,
                        cy * cr * sp + sy * sr * cp, sy * cr * cp - cy * sr * sp], dim=-1)


SAMPLES = {}


def sample_uniform(lower, upper, size, device):
    if "next" in SAMPLES:  # the reset-pose test feeds chosen samples through the module
        return SAMPLES.pop("next")
    return torch.rand(*size, device=device) * (upper - lower) + lower


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


NAMES = ["foot_0", "b1", "a2", "b2", "a3", "b3", "base", "b4", "a5", "b5", "a6", "foot_1"]


class _Robot:
    def __init__(self):
        self.data = _Data()
        self._ALL_INDICES = torch.arange(N)
        self.written = {}

    def find_bodies(self, expr):
        return {"base": ([6], ["base"]), "foot.*": ([0, 11], ["foot_0", "foot_1"])}[expr]

    def reset(self, env_ids):
        pass

    def write_joint_state_to_sim(self, pos, vel, joint_ids, env_ids):
        self.written["joint"] = (pos.clone(), vel.clone(), env_ids.clone())

    def write_root_pose_to_sim(self, pose, env_ids):
        self.written["root_pose"] = pose.clone()

    def write_root_velocity_to_sim(self, vel, env_ids):
        self.written["root_vel"] = vel.clone()


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
        self._terrain = FAKES["terrain"]
        self.scene = _Cfg(env_origins=FAKES["terrain"].env_origins)
        self.episode_length_buf = torch.zeros(N, dtype=torch.long)
        self.reset_terminated = torch.zeros(N, dtype=torch.bool)
        self.reset_time_outs = torch.zeros(N, dtype=torch.bool)
        self.common_step_counter = 0
        self.extras = {}

    def _reset_idx(self, env_ids):  # Isaac Lab: events + episode_length_buf[env_ids] = 0
        self.episode_length_buf[env_ids] = 0


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    spaces = mod("gymnasium.spaces", flatdim=lambda s: int(np.prod(s.shape)))
    mod("gymnasium", spaces=spaces)
    sim = mod("isaaclab.sim", SimulationCfg=_Cfg, RigidBodyMaterialCfg=_Cfg, DomeLightCfg=_Cfg)
    umath = mod("isaaclab.utils.math", quat_apply=quat_apply, quat_mul=quat_mul,
                quat_from_euler_xyz=quat_from_euler_xyz, sample_uniform=sample_uniform)
    utils = mod("isaaclab.utils", configclass=lambda c: c, math=umath)
    mdp = mod("isaaclab.envs.mdp", randomize_rigid_body_material=None)
    mod("isaaclab.envs", DirectRLEnv=DirectRLEnv, DirectRLEnvCfg=object, mdp=mdp)
    mod("isaaclab.managers", EventTermCfg=_Cfg, SceneEntityCfg=_Cfg)
    mod("isaaclab.markers", VisualizationMarkers=object, VisualizationMarkersCfg=_Cfg)
    mod("isaaclab.markers.config", RED_ARROW_X_MARKER_CFG=_Cfg(), GREEN_ARROW_X_MARKER_CFG=_Cfg())
    mod("isaaclab.assets", Articulation=object, ArticulationCfg=_Cfg)
    mod("isaaclab.scene", InteractiveSceneCfg=_Cfg)
    mod("isaaclab.sensors", ContactSensor=object, ContactSensorCfg=_Cfg)
    mod("isaaclab.terrains", TerrainImporterCfg=_Cfg)
    mod("isaaclab", sim=sim, utils=utils)
    mod("zbot.assets", ZBOT_6S_CFG_2=_Cfg())
    mod("zbot")


def random_quat(rng, n):
    q = rng.normal(size=(n, 4))
    return (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)


def upright_ish(rng, n, sign):
    """Quaternions whose z axis (times sign) has z-component spread around the 0.5 threshold."""
    out = []
    for _ in range(n):
        tilt = rng.uniform(0.0, 2.2)
        ax = rng.normal(size=3)
        ax[2] = 0
        ax /= np.linalg.norm(ax)
        q = np.r_[np.cos(tilt / 2), np.sin(tilt / 2) * ax]
        yaw = rng.uniform(-np.pi, np.pi)
        qz = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
        w1, x1, y1, z1 = q
        w2, x2, y2, z2 = qz
        q = np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                      w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])
        if sign < 0:  # flip so that R (0,0,-1) tilts like R (0,0,1) above
            q = np.array([q[1], -q[0], q[3], -q[2]])  # q * (0, 1, 0, 0)
        out.append(q)
    return np.array(out, np.float32)


def make_frame(rng, origins):
    f = {}
    f["joint_pos"] = rng.normal(0, 0.8, (N, 6)).astype(np.float32)
    f["joint_vel"] = rng.normal(0, 2.0, (N, 6)).astype(np.float32)
    pos = rng.normal(0, 0.1, (N, 12, 3)).astype(np.float32)
    pos[:, :, 2] = rng.uniform(0.02, 0.32, (N, 12))
    pos[:, 6, 2] = rng.uniform(0.03, 0.30, N)           # base height across 0.1 / 0.15 / 0.22
    pos[:, :, :2] += origins[:, None, :2]
    quat = np.stack([random_quat(rng, N) for _ in range(12)], axis=1)
    quat[:, 0] = upright_ish(rng, N, +1)
    quat[:, 11] = upright_ish(rng, N, -1)
    linvel = rng.normal(0, 0.4, (N, 12, 3)).astype(np.float32)
    angvel = rng.normal(0, 2.0, (N, 12, 3)).astype(np.float32)
    f["body_link_pos_w"] = pos
    f["body_link_quat_w"] = quat
    f["body_link_lin_vel_w"] = linvel
    f["body_link_state_w"] = np.concatenate([pos, quat, linvel, angvel], axis=-1).astype(np.float32)
    return f


def apply_frame(robot, f):
    for k in ("joint_pos", "joint_vel", "body_link_pos_w", "body_link_quat_w", "body_link_lin_vel_w",
              "body_link_state_w"):
        setattr(robot.data, k, torch.from_numpy(f[k].copy()))


def main():
    install_stubs()
    rng = np.random.default_rng(20260115)
    robot = _Robot()
    robot.data.default_joint_pos = torch.zeros(N, 6)
    robot.data.default_joint_vel = torch.zeros(N, 6)
    robot.data.GRAVITY_VEC_W = torch.tensor([0.0, 0.0, -1.0]).repeat(N, 1)
    root0 = np.array([0.0, 0.0, 0.05, 0.707, 0.0, -0.707, 0.0] + [0.0] * 6, np.float32)  # ZBOT_6S_CFG_2
    robot.data.default_root_state = torch.from_numpy(np.tile(root0, (N, 1)))
    origins = rng.normal(0, 4.0, (N, 3)).astype(np.float32)
    origins[:, 2] = 0
    terrain = _Cfg(env_origins=torch.from_numpy(origins))
    FAKES.update(robot=robot, terrain=terrain)

    spec = importlib.util.spec_from_file_location("ref_zbot_standup", REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    cfg = ref.Zbot6SUpEnvCfg()
    cfg.reward_cfg = {"reward_scales": dict(ref.Zbot6SUpEnvCfg.reward_cfg["reward_scales"])}
    env = ref.Zbot6SUpEnv(cfg)
    term_names = list(env.reward_scales.keys())

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
    apply_frame(robot, frames[0])
    # episode lengths around the 50-step refresh and the 300-step time-out
    env.episode_length_buf[:] = torch.from_numpy(rng.choice([45, 46, 47, 48, 95, 96, 97, 140, 285, 290, 292],
                                                            N).astype(np.int64))
    env.center_z_last[:] = torch.from_numpy(rng.uniform(0.05, 0.30, N).astype(np.float32))
    env.p_delta[:] = torch.from_numpy(rng.uniform(-2.5, 2.5, (N, 6)).astype(np.float32))
    init = {"episode_length_buf": env.episode_length_buf.numpy().astype(np.int32).copy(),
            "center_z_last": env.center_z_last.numpy().copy(), "p_delta": env.p_delta.numpy().copy()}

    rec = {k: [] for k in ("actions", "tanh_actions", "p_delta", "processed_actions", "died", "time_out", "reward",
                           "terms", "obs", "center_z_last", "episode_sums", "episode_length_buf", "stage")}
    stage_at = T // 2  # switch to the curriculum weights half way (my_curriculum's effect)
    for t in range(T):
        if t == stage_at:
            env.common_step_counter = env.max_episode_length * 80
            ref.my_curriculum(env, torch.arange(N))
        a = rng.normal(0, 1.5, (N, 6)).astype(np.float32)
        env._pre_physics_step(torch.from_numpy(a))
        apply_frame(robot, frames[t + 1])
        env.episode_length_buf += 1
        env.common_step_counter += 1
        died, tout = env._get_dones()
        env.reset_terminated[:] = died
        env.reset_time_outs[:] = tout
        r = env._get_rewards()
        obs = env._get_observations()["policy"]
        rec["actions"].append(a)
        rec["tanh_actions"].append(env._actions.numpy().copy())
        rec["p_delta"].append(env.p_delta.numpy().copy())
        rec["processed_actions"].append(env._processed_actions.numpy().copy())
        rec["died"].append(died.numpy().copy())
        rec["time_out"].append(tout.numpy().copy())
        rec["reward"].append(r.numpy().copy())
        rec["terms"].append(np.stack([captured[k].numpy() * env.reward_scales[k] * env.step_dt for k in term_names], 1))
        rec["obs"].append(obs.numpy().copy())
        rec["center_z_last"].append(env.center_z_last.numpy().copy())
        rec["episode_sums"].append(np.stack([env._episode_sums[k].numpy() for k in term_names], axis=1))
        rec["episode_length_buf"].append(env.episode_length_buf.numpy().astype(np.int32).copy())
        rec["stage"].append(env.curriculum_stage)

    out = {f"frame_{k}": np.stack([fr[k] for fr in frames]) for k in frames[0]}
    out.update({k: np.stack(v) for k, v in rec.items()})
    out.update({f"init_{k}": v for k, v in init.items()})
    out["term_names"] = np.array(term_names)
    out["weights_stage0"] = np.array([ref.Zbot6SUpEnvCfg.reward_cfg["reward_scales"][k] for k in term_names])
    out["weights_stage1"] = np.array([env.reward_scales[k] for k in term_names])
    out["step_dt"] = np.array(env.step_dt)
    out["max_episode_length"] = np.array(env.max_episode_length)

    # _reset_idx episode log on a subset (after the last step)
    ids = torch.tensor(sorted(rng.choice(N, 9, replace=False)))
    out["log_env_ids"] = ids.numpy().astype(np.int32)
    out["log_ep_len"] = env.episode_length_buf[ids].numpy().astype(np.int32)
    out["log_sums"] = np.stack([env._episode_sums[k][ids].numpy().copy() for k in term_names], 1)
    env.reset_terminated[:] = torch.from_numpy(rng.random(N) < 0.5)
    env.reset_time_outs[:] = ~env.reset_terminated
    out["log_terminated"] = env.reset_terminated[ids].numpy().copy()
    env.episode_length_buf[ids[0]] = 0  # the clamp(min=step_dt) branch
    out["log_ep_len"][0] = 0
    env._reset_idx(ids)
    out["log_means"] = np.array([float(env.extras["log"]["Episode_Reward/" + k]) for k in term_names])
    out["log_died"] = np.array(env.extras["log"]["Episode_Termination/died"])
    out["log_time_out"] = np.array(env.extras["log"]["Episode_Termination/time_out"])
    out["reset_p_delta"] = env.p_delta[ids].numpy().copy()
    out["reset_center_z_last"] = env.center_z_last[ids].numpy().copy()

    # reset_root_state_uniform on chosen samples (x, y, z, roll, pitch, yaw) — the module's own code
    smp = np.zeros((N, 6), np.float32)
    smp[:, 0] = rng.uniform(-0.5, 0.5, N)
    smp[:, 1] = rng.uniform(-0.5, 0.5, N)
    smp[:, 3] = rng.uniform(-0.7854, 0.7854, N)
    smp[:, 5] = rng.uniform(-3.14, 3.14, N)
    SAMPLES["next"] = torch.from_numpy(smp)
    params = cfg.events.reset_base.params
    ref.reset_root_state_uniform(env, torch.arange(N), params["pose_range"], params["velocity_range"])
    out["pose_samples"] = smp
    out["pose_out"] = robot.written["root_pose"].numpy()
    out["pose_vel_out"] = robot.written["root_vel"].numpy()
    out["pose_current_yaw"] = env.current_yaw.numpy().copy()
    out["pose_range"] = np.array([params["pose_range"][k] for k in ("x", "y", "roll", "yaw")], np.float64)

    # my_curriculum threshold: stage after a reset event at common_step_counter = c
    thr = []
    for c in (env.max_episode_length * 80 - 1, env.max_episode_length * 80, env.max_episode_length * 80 + 1):
        env.curriculum_stage = 0
        env.reward_scales = dict(ref.Zbot6SUpEnvCfg.reward_cfg["reward_scales"])
        env.common_step_counter = c
        ref.my_curriculum(env, torch.arange(N))
        thr.append((c, env.curriculum_stage))
    out["curriculum_threshold"] = np.array(thr, np.int64)

    # EventCfg.physics_material params (startup friction randomisation)
    pm = cfg.events.physics_material.params
    out["material_static_range"] = np.array(pm["static_friction_range"])
    out["material_dynamic_range"] = np.array(pm["dynamic_friction_range"])
    out["material_num_buckets"] = np.array(pm["num_buckets"])
    out["episode_length_s"] = np.array(cfg.episode_length_s)
    out["observation_space"] = np.array(cfg.observation_space)

    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print("wrote", os.path.normpath(OUT), {k: v.shape for k, v in out.items() if hasattr(v, "shape")})
    print("died rate", np.mean(out["died"]), "timeouts", np.mean(out["time_out"]), "stages", out["stage"])


if __name__ == "__main__":
    main()
