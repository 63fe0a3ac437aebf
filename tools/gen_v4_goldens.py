"""Generate walking-v4 golden vectors from the reference's OWN v4 code (build container only).

Same recipe as ``tools/gen_mdp_goldens.py`` / ``gen_standup_goldens.py``: the reference module
``source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v4.py`` is imported from
/root/reference with stub ``isaaclab`` / ``gymnasium`` / ``zbot.assets`` packages. Isaac Lab's
math helpers used by the module are restated here from their published definitions
(``quat_apply``, ``quat_mul``, ``quat_from_euler_xyz``, ``sample_uniform``, ``wrap_to_pi``).

Recorded (data only, ``tests/golden/mdp_v4.npz``):
* the MDP: ``_pre_physics_step -> episode_length_buf += 1 -> _get_dones -> _get_rewards ->
  _get_observations`` over 16 calls on seeded synthetic robot / contact-sensor states (32 envs,
  fixed commands / target headings, curriculum stage 0 for 6 calls, then 1, then 3);
* ``resample_commands`` on chosen uniform / Bernoulli draws (the module's ``torch`` replaced by a
  proxy that serves them);
* ``my_curriculum`` transitions at chosen common_step_counter values;
* ``range_curriculum`` on chosen reward buffers and step counts;
* ``_reset_idx`` episode log incl. the Curriculum entries.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types
from collections import deque

import numpy as np
import torch

REF = "/root/reference/source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v4.py"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "mdp_v4.npz")
N, T = 32, 16
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_standup_goldens import (_Cfg, _Data, quat_apply, quat_from_euler_xyz, quat_mul,  # noqa: E402
                                 random_quat, sample_uniform, upright_ish)


def wrap_to_pi(angles):
    angles = angles.clone()
    angles %= 2 * np.pi
    angles -= 2 * np.pi * (angles > np.pi)
    return angles


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
        self.written["joint"] = (pos.clone(), vel.clone())

    def write_root_pose_to_sim(self, pose, env_ids):
        self.written["root_pose"] = pose.clone()

    def write_root_velocity_to_sim(self, vel, env_ids):
        self.written["root_vel"] = vel.clone()


NAMES = ["foot_0", "b1", "a2", "b2", "a3", "b3", "base", "b4", "a5", "b5", "a6", "foot_1"]


class _Sensor:
    def __init__(self):
        self.data = _Data()

    def find_bodies(self, expr):
        if expr == "foot.*":
            return [0, 11], ["foot_0", "foot_1"]
        if expr == "base|a.*|b.*":
            ids = [i for i, n in enumerate(NAMES) if n == "base" or n[0] in "ab"]
            return ids, [NAMES[i] for i in ids]
        raise KeyError(expr)


class _EventManager:
    def __init__(self, cfg):
        self.terms = {"reset_command_resample": cfg.events.reset_command_resample,
                      "interval_command_resample": cfg.events.interval_command_resample}

    def get_term_cfg(self, name):
        return self.terms[name]


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
        self.scene = _Cfg(env_origins=FAKES["terrain"].env_origins)
        self.episode_length_buf = torch.zeros(N, dtype=torch.long)
        self.reset_terminated = torch.zeros(N, dtype=torch.bool)
        self.reset_time_outs = torch.zeros(N, dtype=torch.bool)
        self.common_step_counter = 0
        self.extras = {}
        self.event_manager = _EventManager(cfg)

    def set_debug_vis(self, v):
        pass

    def _reset_idx(self, env_ids):
        self.episode_length_buf[env_ids] = 0


class _TorchProxy(types.ModuleType):
    """The module's ``torch`` with rand / bernoulli served from queues (resample_commands draws)."""

    def __init__(self):
        super().__init__("torch_proxy")
        self.queue = {"rand": [], "bernoulli": []}

    def __getattr__(self, name):
        return getattr(torch, name)

    def rand(self, *a, **k):
        return self.queue["rand"].pop(0) if self.queue["rand"] else torch.rand(*a, **k)

    def bernoulli(self, p, *a, **k):
        return self.queue["bernoulli"].pop(0) if self.queue["bernoulli"] else torch.bernoulli(p, *a, **k)


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
                quat_from_euler_xyz=quat_from_euler_xyz, sample_uniform=sample_uniform, wrap_to_pi=wrap_to_pi)
    utils = mod("isaaclab.utils", configclass=lambda c: c, math=umath)
    mdp = mod("isaaclab.envs.mdp", randomize_rigid_body_material=None)
    mod("isaaclab.envs", DirectRLEnv=DirectRLEnv, DirectRLEnvCfg=object, mdp=mdp)
    mod("isaaclab.managers", EventTermCfg=_Cfg, SceneEntityCfg=_Cfg)
    marker = _Cfg(markers={"arrow": _Cfg(scale=None)})
    mod("isaaclab.markers", VisualizationMarkers=object, VisualizationMarkersCfg=_Cfg)
    mod("isaaclab.markers.config", RED_ARROW_X_MARKER_CFG=marker, GREEN_ARROW_X_MARKER_CFG=marker)
    mod("isaaclab.assets", Articulation=object, ArticulationCfg=_Cfg)
    mod("isaaclab.scene", InteractiveSceneCfg=_Cfg)
    mod("isaaclab.sensors", ContactSensor=object, ContactSensorCfg=_Cfg)
    mod("isaaclab.terrains", TerrainImporterCfg=_Cfg)
    mod("isaaclab", sim=sim, utils=utils)
    mod("zbot.assets", ZBOT_6S_CFG=_Cfg())
    mod("zbot")


def make_frame(rng, origins):
    f = {}
    f["joint_pos"] = rng.normal(0, 0.5, (N, 6)).astype(np.float32)
    f["joint_vel"] = rng.normal(0, 2.0, (N, 6)).astype(np.float32)
    f["joint_acc"] = rng.normal(0, 300.0, (N, 6)).astype(np.float32)
    f["applied_torque"] = rng.uniform(-20, 20, (N, 6)).astype(np.float32)
    pos = rng.normal(0, 0.08, (N, 12, 3)).astype(np.float32)
    pos[:, :, 2] = rng.uniform(0.0, 0.35, (N, 12))
    pos[:, 6, 2] = rng.uniform(0.16, 0.32, N)            # base height around the 0.20 threshold
    pos[:, :, :2] += origins[:, None, :2]
    f["body_link_pos_w"] = pos
    quat = np.stack([random_quat(rng, N) for _ in range(12)], axis=1)
    quat[:, 0] = upright_ish(rng, N, +1)
    quat[:, 11] = upright_ish(rng, N, -1)
    f["body_link_quat_w"] = quat
    f["body_link_lin_vel_w"] = rng.normal(0, 0.4, (N, 12, 3)).astype(np.float32)
    f["body_com_lin_vel_w"] = rng.normal(0, 0.4, (N, 12, 3)).astype(np.float32)
    hist = rng.normal(0, 0.1, (N, 3, 12, 3)).astype(np.float32)
    big = rng.random((N, 3, 12)) < 0.25
    hist[..., 2] += np.where(big, rng.uniform(0, 30, (N, 3, 12)), 0)
    quiet = rng.random(N) < 0.6
    undesired = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
    for e in np.nonzero(quiet)[0]:
        hist[e][:, undesired, :] *= 0.01
    f["net_forces_w_history"] = hist
    for k in ("current_air_time", "current_contact_time", "last_air_time", "last_contact_time"):
        v = rng.uniform(0, 1.0, (N, 12)).astype(np.float32)
        if k.startswith("current"):
            v[rng.random((N, 12)) < 0.5] = 0.0
        f[k] = v
    return f


def apply_frame(robot, sensor, f):
    for k in ("joint_pos", "joint_vel", "joint_acc", "applied_torque", "body_link_pos_w", "body_link_quat_w",
              "body_link_lin_vel_w", "body_com_lin_vel_w"):
        setattr(robot.data, k, torch.from_numpy(f[k].copy()))
    for k in ("net_forces_w_history", "current_air_time", "current_contact_time", "last_air_time",
              "last_contact_time"):
        setattr(sensor.data, k, torch.from_numpy(f[k].copy()))


def main():
    install_stubs()
    rng = np.random.default_rng(20260121)
    robot, sensor = _Robot(), _Sensor()
    robot.data.default_joint_pos = torch.from_numpy(np.tile(np.array([0.312, 0.837, -2.02, 2.02, -0.837, -0.312],
                                                                     np.float32), (N, 1)))
    robot.data.default_joint_vel = torch.zeros(N, 6)
    robot.data.GRAVITY_VEC_W = torch.tensor([0.0, 0.0, -1.0]).repeat(N, 1)
    root0 = np.array([0.0, -0.06, 0.0, 1.0, 0.0, 0.0, 0.0] + [0.0] * 6, np.float32)  # ZBOT_6S_CFG init_state
    robot.data.default_root_state = torch.from_numpy(np.tile(root0, (N, 1)))
    origins = rng.normal(0, 4.0, (N, 3)).astype(np.float32)
    origins[:, 2] = 0
    terrain = _Cfg(env_origins=torch.from_numpy(origins))
    FAKES.update(robot=robot, sensor=sensor, terrain=terrain)

    spec = importlib.util.spec_from_file_location("ref_zbot_v4", REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    proxy = _TorchProxy()
    ref.torch = proxy
    cfg = ref.Zbot6SEnvV4Cfg()
    base_w = dict(ref.Zbot6SEnvV4Cfg.reward_cfg["reward_scales"])
    cfg.reward_cfg = {"reward_scales": dict(base_w)}
    env = ref.Zbot6SEnvV4(cfg)
    term_names = list(env.reward_scales.keys())
    L = env.max_episode_length

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
    env.episode_length_buf[:] = torch.from_numpy(rng.choice([100, 500, 985, 990, 995], N).astype(np.int64))
    cmd = np.stack([rng.choice([-0.3, -0.1, 0.0, 0.2, 0.3], N), rng.uniform(-0.5, 0.5, N)], 1).astype(np.float32)
    env.commands[:] = torch.from_numpy(cmd)
    env.target_heading_yaw[:] = torch.from_numpy(rng.uniform(-np.pi, np.pi, N).astype(np.float32))
    env.feet_contact_forces_last[:] = torch.from_numpy(rng.uniform(0, 20, (N, 2)).astype(np.float32))
    env.feet_down_pos_last[:] = torch.from_numpy(rng.normal(0, 0.2, (N, 2, 3)).astype(np.float32))
    env.feet_step_length[:] = torch.from_numpy(rng.normal(0, 0.05, (N, 2)).astype(np.float32))
    init = {"episode_length_buf": env.episode_length_buf.numpy().astype(np.int32).copy(),
            "commands": cmd, "target_heading_yaw": env.target_heading_yaw.numpy().copy(),
            "feet_contact_forces_last": env.feet_contact_forces_last.numpy().copy(),
            "feet_down_pos_last": env.feet_down_pos_last.numpy().copy(),
            "feet_step_length": env.feet_step_length.numpy().copy()}

    rec = {k: [] for k in ("actions", "tanh_actions", "prev_actions", "p_delta", "died", "time_out", "reward",
                           "terms", "obs", "current_yaw", "heading_err", "feet_step_length", "feet_down_pos_last",
                           "feet_contact_forces_last", "episode_sums", "episode_length_buf", "stage")}
    stage_plan = {6: 1, 11: 3}
    for t in range(T):
        if t in stage_plan:  # the reference's stage weights (applied via my_curriculum's own code)
            while env.curriculum_stage < stage_plan[t]:
                env.common_step_counter = L * {0: 12, 1: 24, 2: 144}[env.curriculum_stage]
                ref.my_curriculum(env, torch.arange(N))
        a = rng.normal(0, 1.5, (N, 6)).astype(np.float32)
        env._pre_physics_step(torch.from_numpy(a))
        apply_frame(robot, sensor, frames[t + 1])
        env.episode_length_buf += 1
        env.common_step_counter += 1
        died, tout = env._get_dones()
        env.reset_terminated[:] = died
        env.reset_time_outs[:] = tout
        rec["prev_actions"].append(env._previous_actions.numpy().copy())
        r = env._get_rewards()
        obs = env._get_observations()["policy"]
        rec["actions"].append(a)
        rec["tanh_actions"].append(env._actions.numpy().copy())
        rec["p_delta"].append(env.p_delta.numpy().copy())
        rec["died"].append(died.numpy().copy())
        rec["time_out"].append(tout.numpy().copy())
        rec["reward"].append(r.numpy().copy())
        rec["terms"].append(np.stack([captured[k].numpy() * env.reward_scales[k] * env.step_dt for k in term_names], 1))
        rec["obs"].append(obs.numpy().copy())
        rec["current_yaw"].append(env.current_yaw.numpy().copy())
        rec["heading_err"].append(env.heading_err.numpy().copy())
        rec["feet_step_length"].append(env.feet_step_length.numpy().copy())
        rec["feet_down_pos_last"].append(env.feet_down_pos_last.numpy().copy())
        rec["feet_contact_forces_last"].append(env.feet_contact_forces_last.numpy().copy())
        rec["episode_sums"].append(np.stack([env._episode_sums[k].numpy() for k in term_names], axis=1))
        rec["episode_length_buf"].append(env.episode_length_buf.numpy().astype(np.int32).copy())
        rec["stage"].append(env.curriculum_stage)

    out = {f"frame_{k}": np.stack([fr[k] for fr in frames]) for k in frames[0]}
    out.update({k: np.stack(v) for k, v in rec.items()})
    out.update({f"init_{k}": v for k, v in init.items()})
    out["term_names"] = np.array(term_names)
    out["weights_stage0"] = np.array([base_w[k] for k in term_names])
    out["weights_stage3"] = np.array([env.reward_scales[k] for k in term_names])
    out["step_dt"] = np.array(env.step_dt)
    out["max_episode_length"] = np.array(L)

    # resample_commands on chosen draws: (prob_pos, velocity_range, yaw_range, offset) cases
    cases = []
    for prob, vr, yr, off in ((1.0, (0.3, 0.3), (-0.1, 0.1), 0.0), (0.8, (0.1, 0.3), (-0.5, 0.5), 0.0),
                              (0.6, (0.0, 0.3), (-0.3, 0.3), 0.1)):
        sign_u = rng.random(N).astype(np.float32)
        u_vel = rng.random(N).astype(np.float32)
        u_yaw = rng.random(N).astype(np.float32)
        cur = rng.uniform(-np.pi, np.pi, N).astype(np.float32)
        env.current_yaw[:] = torch.from_numpy(cur)
        proxy.queue["bernoulli"] = [torch.from_numpy((sign_u < prob).astype(np.float32))]
        proxy.queue["rand"] = [torch.from_numpy(u_vel), torch.from_numpy(u_yaw)]
        ref.resample_commands(env, torch.arange(N), vr, yr, True, off, prob)
        cases.append(dict(prob=prob, vr=vr, yr=yr, off=off, sign_u=sign_u, u_vel=u_vel, u_yaw=u_yaw, cur=cur,
                          cmd=env.commands.numpy().copy(), target=env.target_heading_yaw.numpy().copy()))
    for k in ("sign_u", "u_vel", "u_yaw", "cur", "cmd", "target"):
        out["resample_" + k] = np.stack([c[k] for c in cases])
    out["resample_params"] = np.array([[c["prob"], *c["vr"], *c["yr"], c["off"]] for c in cases], np.float32)

    # my_curriculum: (common_step_counter, stage before) -> stage after, prob_pos after
    mc = []
    for steps, st0 in ((12 * L - 1, 0), (12 * L, 0), (24 * L, 0), (24 * L, 1), (100 * L, 2), (144 * L, 2),
                       (144 * L + 7, 2), (200 * L, 3)):
        env.curriculum_stage = st0
        env.common_step_counter = steps
        for tc in env.event_manager.terms.values():
            tc.params["prob_pos"] = 1.0
        ref.my_curriculum(env, torch.arange(N))
        mc.append((steps, st0, env.curriculum_stage, env.event_manager.terms["reset_command_resample"].params["prob_pos"]))
    out["my_curriculum_cases"] = np.array(mc, np.float64)

    # range_curriculum: buffers / step counts -> new ranges
    env.reward_scales = dict(base_w)
    rc = []
    for steps, nbuf, vmean, ymean in ((48 * L, 24, 0.9, 0.9), (48 * L, 19, 0.9, 0.9), (48 * L + 1, 24, 0.9, 0.9),
                                      (60 * L, 24, 0.8, 0.9), (60 * L, 24, 0.9, 0.8), (36 * L, 24, 0.9, 0.9)):
        for tc in env.event_manager.terms.values():
            tc.params["velocity_range"] = (0.3, 0.3)
            tc.params["yaw_range"] = (-0.45, 0.45)
        env.curriculum_vel_reward_buffer = deque([vmean] * nbuf, maxlen=24)
        env.curriculum_yaw_reward_buffer = deque([ymean] * nbuf, maxlen=24)
        env.common_step_counter = steps
        ref.range_curriculum(env, torch.arange(N), limit_ranges=(0.0, 0.3), limit_yaw_ranges=(-0.5, 0.5))
        p = env.event_manager.terms["reset_command_resample"].params
        rc.append((steps, nbuf, vmean, ymean, *p["velocity_range"], *p["yaw_range"]))
    out["range_curriculum_cases"] = np.array(rc, np.float64)

    # _reset_idx episode log + Curriculum entries
    ids = torch.tensor(sorted(rng.choice(N, 9, replace=False)))
    env.curriculum_stage = 1
    env.event_manager.terms["reset_command_resample"].params["velocity_range"] = (0.25, 0.3)
    env.event_manager.terms["reset_command_resample"].params["yaw_range"] = (-0.15, 0.15)
    out["log_ep_len"] = env.episode_length_buf[ids].numpy().astype(np.int32)
    out["log_sums"] = np.stack([env._episode_sums[k][ids].numpy().copy() for k in term_names], 1)
    env.reset_terminated[:] = torch.from_numpy(rng.random(N) < 0.5)
    env.reset_time_outs[:] = ~env.reset_terminated
    out["log_terminated"] = env.reset_terminated[ids].numpy().copy()
    env._reset_idx(ids)
    log = env.extras["log"]
    out["log_means"] = np.array([float(log["Episode_Reward/" + k]) for k in term_names])
    out["log_counts"] = np.array([log["Episode_Termination/died"], log["Episode_Termination/time_out"]])
    out["log_curriculum"] = np.array([log["Curriculum/curriculum_stage"], log["Curriculum/vel_lower_bound"],
                                      log["Curriculum/vel_upper_bound"], log["Curriculum/yaw_bound"]], np.float64)
    out["reset_feet_contact_forces_last"] = env.feet_contact_forces_last[ids].numpy().copy()
    out["reset_feet_step_length"] = env.feet_step_length[ids].numpy().copy()

    # reset_root_state_uniform (v4 variant: body-frame yaw) on chosen samples
    smp = np.zeros((N, 6), np.float32)
    smp[:, 0] = rng.uniform(-0.5, 0.5, N)
    smp[:, 1] = rng.uniform(-0.5, 0.5, N)
    smp[:, 5] = rng.uniform(-3.14, 3.14, N)
    from gen_standup_goldens import SAMPLES  # the restated sample_uniform serves these once
    SAMPLES["next"] = torch.from_numpy(smp)
    params = cfg.events.reset_base.params
    ref.reset_root_state_uniform(env, torch.arange(N), params["pose_range"], params["velocity_range"])
    out["pose_samples"] = smp
    out["pose_out"] = robot.written["root_pose"].numpy()
    out["pose_current_yaw"] = env.current_yaw.numpy().copy()
    out["env_origins"] = origins
    out["episode_length_s"] = np.array(cfg.episode_length_s)
    out["observation_space"] = np.array(cfg.observation_space)
    out["interval_range_s"] = np.array(cfg.events.interval_command_resample.interval_range_s)
    out["limit_yaw_ranges"] = np.array(cfg.events.vel_range.params["limit_yaw_ranges"])
    out["limit_ranges"] = np.array(cfg.events.vel_range.params["limit_ranges"])

    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print("wrote", os.path.normpath(OUT), {k: v.shape for k, v in out.items() if hasattr(v, "shape")})
    print("died rate", np.mean(out["died"]), "timeouts", np.mean(out["time_out"]), "stages", out["stage"])
    print("my_curriculum", out["my_curriculum_cases"])
    print("range", out["range_curriculum_cases"])


if __name__ == "__main__":
    main()
