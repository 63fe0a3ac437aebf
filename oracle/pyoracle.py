"""ctypes binding of the CPU oracle (oracle/zbot_oracle.c). TEST INFRASTRUCTURE ONLY.

Importable only from tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg, as the
checker / CPU baseline. The product path never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from zbot_lab_amd import model as zm

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")

_f = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u8 = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load(double: bool = False):
    name = "libzbot_oracle_f64.so" if double else "libzbot_oracle.so"
    path = os.path.join(BUILD, name)
    if not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    P = C.c_void_p
    lib.zbo_create.restype = P
    lib.zbo_create.argtypes = [C.POINTER(zm.ZbModel), C.POINTER(zm.ZbTaskCfg), C.c_int, C.c_uint64]
    lib.zbo_destroy.argtypes = [P]
    lib.zbo_set_threads.argtypes = [C.c_int]
    lib.zbo_reset.argtypes = [P, C.c_void_p, C.c_int]
    lib.zbo_step.argtypes = [P, _f, _f, _f, _u8, _u8]
    lib.zbo_observe.argtypes = [P, _f]
    lib.zbo_read_log.argtypes = [P, _f, _i]
    lib.zbo_get_state.argtypes = [P, _f]
    lib.zbo_set_state.argtypes = [P, _f]
    lib.zbo_get_contact_cache.argtypes = [P, _f]
    lib.zbo_set_contact_cache.argtypes = [P, _f]
    lib.zbo_physics_substeps.argtypes = [P, _f, C.c_int, C.c_void_p, C.c_void_p]
    lib.zbo_link_poses.argtypes = [P, _f, _f]
    lib.zbo_contact_diag.argtypes = [P, _f]
    lib.zbo_hull_pair.argtypes = [_f, _f, C.c_float, _f]
    lib.zbo_hull_pair_from.argtypes = [_f, _f, C.c_float, C.c_void_p, _f]
    lib.zbo_pair_manifold.argtypes = [_f, _f, C.c_float, _f]
    lib.zbo_gjk_pairs.argtypes = [_f, C.c_void_p, C.c_int, C.c_float, _f, C.c_void_p]
    lib.zbo_set_gjk_tol.argtypes = [C.c_double]
    lib.zbo_set_face_cos.argtypes = [C.c_double]
    lib.zbo_set_sensor_force_scale.argtypes = [C.c_double]
    lib.zbo_set_plant.argtypes = [C.c_int]
    lib.zbo_contact_activity.argtypes = [P, _i, C.c_int]
    lib.zbo_self_min_sep.argtypes = [P, _f]
    lib.zbo_pair_classes.argtypes = [P, _f]
    lib.zbo_link_com_vel.argtypes = [P, _f]
    lib.zbo_energy_momentum.argtypes = [P, _f]
    lib.zbo_pre_physics.argtypes = [C.c_int, C.POINTER(zm.ZbTaskCfg), _f, _f, _f, _f, _f]
    lib.zbo_obs_cache.argtypes = [C.c_int, _f, _f, _f, _f, _f, _f]
    lib.zbo_mdp_eval.argtypes = [C.c_int, C.POINTER(zm.ZbTaskCfg), _f, _f, _f, _f, _f, _f, _i, _f, _f, _f,
                                 _f, _f, _f, _f, _u8, _u8]
    lib.zbo_state_dim.argtypes = [P]
    lib.zbo_set_link_friction.argtypes = [P, _f, C.c_void_p]
    lib.zbo_read_curriculum.argtypes = [P, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    lib.zbo_su_mdp_eval.argtypes = [C.c_int, C.POINTER(zm.ZbTaskCfg), C.c_int, _f, _f, _i, _f, _f, _f, _f, _u8, _u8]
    lib.zbo_su_reset_pose.argtypes = [C.POINTER(zm.ZbModel), C.POINTER(zm.ZbTaskCfg), C.c_uint64, C.c_uint64, C.c_int,
                                      _f, _f]
    lib.zbo_su_pose_from_samples.argtypes = [C.POINTER(zm.ZbModel), C.c_int, _f, C.c_int, _f, _f]
    lib.zbo_v4_mdp_eval.argtypes = [C.c_int, C.POINTER(zm.ZbTaskCfg), C.c_int, C.POINTER(zm.ZbModel)] + [_f] * 12 + \
        [_i, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _u8, _u8, _f, _f]
    lib.zbo_v4_commands_from_draws.argtypes = [C.c_int, _f, _f, _f, _f, _f, _f, _f]
    lib.zbo_curriculum_probe.argtypes = [C.POINTER(zm.ZbTaskCfg), C.c_int64, C.c_int, C.c_int, C.c_int, C.c_float,
                                         C.c_float, _f]
    lib.zbo_m_mdp_eval.argtypes = [C.c_int, C.POINTER(zm.ZbTaskCfg)] + [_f] * 11 + [_i, _f, _f, _f, _f, _f, _f, _f,
                                                                                _f, _f, _u8, _u8, _u8]
    lib.zbo_m_curriculum_probe.argtypes = [C.POINTER(zm.ZbTaskCfg), C.c_int64, C.c_float, _f]
    lib.zbo_m_process_actions.argtypes = [C.c_int, C.POINTER(zm.ZbTaskCfg), C.POINTER(zm.ZbModel), _f, _f, _f, _f]
    return lib


_LIBS: dict = {}


def lib(double: bool = False):
    if double not in _LIBS:
        _LIBS[double] = _load(double)
    return _LIBS[double]


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class OracleSim:
    """Mirror of the libzbot C ABI on the CPU (same state layout, same semantics)."""

    def __init__(self, num_envs: int, cfg: zm.TaskCfg | None = None, seed: int = 0, double: bool = False,
                 threads: int = 0):
        self.lib = lib(double)
        self.cfg = cfg or zm.TaskCfg()
        self.n = num_envs
        self.obs_dim, self.state_dim = self.cfg.obs_dim, self.cfg.state_dim
        self.num_terms = len(self.cfg.reward_terms)
        task = self.cfg.task
        self._m = zm.pack_model(zm.standup_model() if task == zm.TASK_STANDUP_V0
                                else zm.load_v09_model() if task == zm.TASK_MANAGER_V0 else None)
        self._c = self.cfg.pack()
        if threads:
            self.lib.zbo_set_threads(threads)
        self.h = self.lib.zbo_create(C.byref(self._m), C.byref(self._c), num_envs, seed)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.zbo_destroy(h)
            self.h = None

    def reset(self, env_ids=None):
        if env_ids is None:
            self.lib.zbo_reset(self.h, None, self.n)
        else:
            ids = np.ascontiguousarray(env_ids, dtype=np.int32)
            self.lib.zbo_reset(self.h, ids.ctypes.data_as(C.c_void_p), len(ids))

    def step(self, actions):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        rew = np.zeros(self.n, np.float32)
        term = np.zeros(self.n, np.uint8)
        trunc = np.zeros(self.n, np.uint8)
        self.lib.zbo_step(self.h, f32(actions), obs, rew, term, trunc)
        return obs, rew, term.astype(bool), trunc.astype(bool)

    def observe(self):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        self.lib.zbo_observe(self.h, obs)
        return obs

    def read_log(self, full: bool = False):
        m = np.zeros(zm.LOG_LEN, np.float32)
        c = np.zeros(zm.LOG_COUNTS, np.int32)
        self.lib.zbo_read_log(self.h, m, c)
        return (m if full else m[:self.num_terms]), c

    def set_link_friction(self, mu, mu_dynamic=None):
        md = None if mu_dynamic is None else f32(mu_dynamic)
        if self.lib.zbo_set_link_friction(self.h, f32(mu), None if md is None else md.ctypes.data_as(C.c_void_p)) != 0:
            raise ValueError("per-link friction is a standup / manager task state")

    def read_curriculum(self):
        st, n = C.c_int32(), C.c_int64()
        self.lib.zbo_read_curriculum(self.h, C.byref(st), C.byref(n))
        return int(st.value), int(n.value)

    def get_state(self):
        st = np.zeros((self.state_dim, self.n), np.float32)
        self.lib.zbo_get_state(self.h, st)
        return st

    def set_state(self, st):
        self.lib.zbo_set_state(self.h, f32(st))

    def get_contact_cache(self):
        wc = np.zeros((16, self.n), np.float32)
        self.lib.zbo_get_contact_cache(self.h, wc)
        return wc

    def set_contact_cache(self, wc):
        self.lib.zbo_set_contact_cache(self.h, f32(wc))

    def physics_substeps(self, targets, nsub):
        nf = np.zeros((self.n, zm.NUM_LINKS, 3), np.float32)
        at = np.zeros((self.n, zm.NUM_DOF), np.float32)
        self.lib.zbo_physics_substeps(self.h, f32(targets), nsub, nf.ctypes.data_as(C.c_void_p),
                                      at.ctypes.data_as(C.c_void_p))
        return nf, at

    def link_poses(self):
        p = np.zeros((self.n, zm.NUM_LINKS, 3), np.float32)
        q = np.zeros((self.n, zm.NUM_LINKS, 4), np.float32)
        self.lib.zbo_link_poses(self.h, p, q)
        return p, q

    def contact_diag(self):
        """[n, 6]: candidates, ground, self pairs in contact, kept, min |sep - margin|, kept self points
        (a face manifold counts each point) of the current state."""
        d = np.zeros((self.n, 6), np.float32)
        self.lib.zbo_contact_diag(self.h, d)
        return d

    def contact_activity(self, clear: bool = True):
        """[n, 2]: loaded ground / self contacts (lambda_n > 0 after the solve) summed over the
        substeps of the steps since the last clear (test hook)."""
        out = np.zeros((self.n, 2), np.int32)
        self.lib.zbo_contact_activity(self.h, out, int(clear))
        return out

    def pair_classes(self):
        """[n, 10] self-contact classes per env (oracle zbo_pair_classes): pairs in contact, face-manifold
        pairs, side-by-side rim-manifold pairs, overlapping-core pairs, min separation, self points,
        first face / rim pair index (-1: none), ruling-on-face pairs, first ruling-on-face pair index."""
        d = np.zeros((self.n, 10), np.float32)
        self.lib.zbo_pair_classes(self.h, d)
        return d

    def self_min_sep(self):
        """[n]: the smallest self-collision separation of the current state (-2 CORE_M: overlapping
        cores, deeper than the shape model)."""
        d = np.zeros(self.n, np.float32)
        self.lib.zbo_self_min_sep(self.h, d)
        return d

    def link_com_vel(self):
        v = np.zeros((self.n, zm.NUM_LINKS, 3), np.float32)
        self.lib.zbo_link_com_vel(self.h, v)
        return v

    def energy_momentum(self):
        o = np.zeros((self.n, 7), np.float32)
        self.lib.zbo_energy_momentum(self.h, o)
        return o


class planted_bug:
    """Context manager: the oracle library (f32 or f64) runs with a planted contact bug
    (zbo_set_plant: 1 ground mu x 1.1 on one contact, 2 one self normal flipped, 3 no push-out cap)."""

    def __init__(self, mode: int, double: bool = True):
        self.mode, self.double = mode, double

    def __enter__(self):
        lib(self.double).zbo_set_plant(self.mode)
        return self

    def __exit__(self, *exc):
        lib(self.double).zbo_set_plant(0)


def su_mdp_eval(cfg: zm.TaskCfg, stage: int, link_state, p_delta, ep_len, center_z_last, ep_sums):
    """Stand-up _get_dones + _get_rewards on raw body_link_state_w inputs (zbo_su_mdp_eval)."""
    n = len(ep_len)
    c = cfg.pack()
    czl = f32(center_z_last).copy()
    sums = f32(ep_sums).copy()
    rew = np.zeros(n, np.float32)
    terms = np.zeros((n, zm.SU_NUM_TERMS), np.float32)
    died = np.zeros(n, np.uint8)
    tout = np.zeros(n, np.uint8)
    lib().zbo_su_mdp_eval(n, C.byref(c), int(stage), f32(link_state), f32(p_delta),
                          np.ascontiguousarray(ep_len, np.int32), czl, sums, rew, terms, died, tout)
    return dict(reward=rew, terms=terms, died=died.astype(bool), time_out=tout.astype(bool), center_z_last=czl,
                episode_sums=sums)


def su_reset_pose(cfg: zm.TaskCfg, seed: int, ctr: int, n: int):
    """Root (pos [n,3], quat [n,4]) of reset_root_state_uniform at RNG position ctr."""
    m = zm.pack_model(zm.standup_model())
    c = cfg.pack()
    pos = np.zeros((n, 3), np.float32)
    quat = np.zeros((n, 4), np.float32)
    lib().zbo_su_reset_pose(C.byref(m), C.byref(c), seed, ctr, n, pos, quat)
    return pos, quat


def su_pose_from_samples(samples, body_frame: bool = False, robot=None):
    """Root (pos [n,3], quat [n,4]) from reset_root_state_uniform samples [n,4] = x, y, roll, yaw
    (standup: world-frame delta on ZBOT_6S_CFG_2; v4: body-frame delta on ZBOT_6S_CFG)."""
    m = zm.pack_model(robot if robot is not None else zm.standup_model())
    smp = f32(samples)
    n = len(smp)
    pos = np.zeros((n, 3), np.float32)
    quat = np.zeros((n, 4), np.float32)
    lib().zbo_su_pose_from_samples(C.byref(m), n, smp, int(body_frame), pos, quat)
    return pos, quat


def v4_mdp_eval(cfg: zm.TaskCfg, stage: int, frame: dict, ep_len, act, prev_act, state: dict):
    """v4 _get_dones + _get_rewards on Isaac-Lab-shaped frame data (zbo_v4_mdp_eval). ``state`` holds
    commands, target_yaw, feet_down_pos, feet_step_len, feet_f_last, ep_sums (updated copies returned)."""
    n = len(ep_len)
    c = cfg.pack()
    m = zm.pack_model()
    st = {k: f32(v).copy() for k, v in state.items()}
    out = dict(reward=np.zeros(n, np.float32), terms=np.zeros((n, zm.V4_NUM_TERMS), np.float32),
               died=np.zeros(n, np.uint8), time_out=np.zeros(n, np.uint8), cur_yaw=np.zeros(n, np.float32),
               heading_err=np.zeros(n, np.float32))
    lib().zbo_v4_mdp_eval(n, C.byref(c), int(stage), C.byref(m), f32(frame["body_link_pos_w"]),
                          f32(frame["body_link_quat_w"]), f32(frame["body_link_lin_vel_w"]),
                          f32(frame["body_com_lin_vel_w"]), f32(frame["joint_vel"]), f32(frame["joint_acc"]),
                          f32(frame["applied_torque"]), f32(frame["net_forces_w_history"]),
                          f32(frame["current_air_time"]), f32(frame["current_contact_time"]),
                          f32(frame["last_air_time"]), f32(frame["last_contact_time"]),
                          np.ascontiguousarray(ep_len, np.int32), f32(act), f32(prev_act), st["commands"],
                          st["target_yaw"], st["feet_down_pos"], st["feet_step_len"], st["feet_f_last"], st["ep_sums"],
                          out["reward"], out["terms"], out["died"], out["time_out"], out["cur_yaw"], out["heading_err"])
    out["died"] = out["died"].astype(bool)
    out["time_out"] = out["time_out"].astype(bool)
    out.update(st)
    return out


def v4_commands_from_draws(params, u_sign, u_vel, u_yaw, cur_yaw):
    n = len(u_sign)
    cmd = np.zeros((n, 2), np.float32)
    tgt = np.zeros(n, np.float32)
    lib().zbo_v4_commands_from_draws(n, f32(params), f32(u_sign), f32(u_vel), f32(u_yaw), f32(cur_yaw), cmd, tgt)
    return cmd, tgt


def curriculum_probe(cfg: zm.TaskCfg, steps: int, io, run_my=True, run_range=True, ring_n=0, ring_vel=0.0,
                     ring_yaw=0.0):
    """The reset-event curricula on a counter state io = [stage, prob_pos, vel lo, vel hi, yaw lo, yaw hi]."""
    c = cfg.pack()
    v = f32(io).copy()
    lib().zbo_curriculum_probe(C.byref(c), int(steps), int(run_my), int(run_range), int(ring_n), float(ring_vel),
                               float(ring_yaw), v)
    return v


FEET = [0, 11]  # feet rows of the golden frames' 12-body layout (tools/gen_manager_goldens.py)


def m_mdp_eval(cfg: zm.TaskCfg, frame: dict, ep_len, act, prev_act, commands, state: dict):
    """Manager flat terminations + rewards on Isaac-Lab-shaped frame data (zbo_m_mdp_eval). ``state``
    holds feet_down_pos [n,2,3], feet_step_len [n,2], feet_f_last [n,2], ep_sums [n,11] (updated
    copies returned)."""
    n = len(ep_len)
    c = cfg.pack()
    st = {k: f32(v).copy() for k, v in state.items()}
    out = dict(reward=np.zeros(n, np.float32), terms=np.zeros((n, zm.M_NUM_TERMS), np.float32),
               low=np.zeros(n, np.uint8), close=np.zeros(n, np.uint8), time_out=np.zeros(n, np.uint8))
    lib().zbo_m_mdp_eval(n, C.byref(c), f32(frame["root_pos_w"]), f32(frame["root_quat_w"]),
                         f32(frame["root_link_lin_vel_w"]), f32(frame["root_link_ang_vel_w"]),
                         f32(frame["body_link_pos_w"][:, FEET]), f32(frame["body_link_quat_w"][:, FEET]),
                         f32(frame["body_lin_vel_w"][:, FEET]), f32(frame["net_forces_w_history"][:, :, FEET]),
                         f32(frame["last_air_time"][:, FEET]), f32(frame["applied_torque"]), f32(frame["joint_acc"]),
                         np.ascontiguousarray(ep_len, np.int32), f32(act), f32(prev_act), f32(commands),
                         st["feet_down_pos"], st["feet_step_len"], st["feet_f_last"], st["ep_sums"],
                         out["reward"], out["terms"], out["low"], out["close"], out["time_out"])
    for k in ("low", "close", "time_out"):
        out[k] = out[k].astype(bool)
    out.update(st)
    return out


def m_curriculum_probe(cfg: zm.TaskCfg, steps: int, reward: float, ranges):
    """lin_vel_cmd_levels on ranges [x lo, x hi, y lo, y hi]; returns (fired, new ranges)."""
    c = cfg.pack()
    io = f32(ranges).copy()
    fired = lib().zbo_m_curriculum_probe(C.byref(c), int(steps), float(reward), io)
    return bool(fired), io


def m_process_actions(cfg: zm.TaskCfg, actions, jq):
    """RelativeJointPositionAction: (processed actions [n,6] Isaac Lab order, chain targets q + delta)."""
    c = cfg.pack()
    m = zm.pack_model(zm.load_v09_model())
    a = f32(actions)
    proc = np.zeros_like(a)
    tg = np.zeros_like(a)
    lib().zbo_m_process_actions(len(a), C.byref(c), C.byref(m), a, f32(jq), proc, tg)
    return proc, tg
