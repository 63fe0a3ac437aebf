"""Robot model + task constants -> the ``zb_model`` / ``zb_task_cfg`` structs of ``include/zbot.h``.

The robot is ``ZBOT_6S_CFG`` (reference ``source/zbot/zbot/assets/zbot_cfg.py:621-669``) built on
``zbot_6s_new.usd``; the decoded asset lives in ``assets/zbot6s_model.json`` (written by
``tools/extract_model.py``). Here the 12 links / 6 revolute + 5 fixed joints are merged into the 7
rigid composites the simulator integrates (fixed joints have no DoF), and every per-link quantity
(link frame, authored COM, collision circles, round-1 self-collision spheres) is expressed in its
composite's frame. PhysX uses the authored mass properties verbatim, so do we.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

ASSET = os.path.join(os.path.dirname(__file__), "assets", "zbot6s_model.json")

NUM_LINKS, NUM_BODIES, NUM_DOF = 12, 7, 6
OBS_DIM, ACT_DIM, NUM_TERMS, HIST = 23, 6, 15, 5
MAX_SELF_PAIRS = 64
STATE_DIM = 87

LINK_NAMES = ["foot_0", "b1", "a2", "b2", "a3", "b3", "base", "b4", "a5", "b5", "a6", "foot_1"]
JOINT_NAMES = ["joint1", "joint2", "joint3", "joint4", "joint5", "joint6"]
REWARD_TERMS = [  # dict order of ZbotDirectEnvCfgV2.reward_cfg (v2.py:190-206), then step0's feet-force terms
    "base_vel_forward", "feet_downward", "feet_forward", "base_heading_x", "base_heading_x_sum",
    "step_length", "airtime_balance", "action_rate", "torques", "feet_slide", "base_pos_y_err",
    "base_pos_y_err_sum", "airtime_sum", "feet_force_diff", "feet_force_sum",   # v2.py:78-91, 563-571
]
REWARD_WEIGHTS = {  # v2.py:190-206 ("train reward 2000 step4")
    "base_vel_forward": 1.0, "feet_downward": -2.0, "feet_forward": -1.0, "base_heading_x": -1.0,
    "base_heading_x_sum": -5.0, "step_length": 5.0, "airtime_balance": -15.0, "action_rate": -0.1,
    "torques": -0.002, "feet_slide": -10.0, "base_pos_y_err": -2.0, "base_pos_y_err_sum": -2.0,
    "airtime_sum": 3.0,
}

# zbot-6b-standup-v0 (include/zbot.h enum zb_standup_state_field / zb_standup_reward_term)
TASK_WALKING_V2, TASK_STANDUP_V0, TASK_WALKING_V4, TASK_MANAGER_V0 = 0, 1, 2, 3
MAX_REWARD_TERMS, MAX_STAGES, LOG_LEN, LOG_COUNTS = 16, 4, 20, 4
SU_OBS_DIM, SU_NUM_TERMS, SU_STATE_DIM = 22, 4, 67
SU_REWARD_TERMS = ["upward_2", "shape_symmetry", "feet_downward", "feet_downward_4"]  # standup.py:418-427
SU_REWARD_WEIGHTS = {"upward_2": 10.0, "shape_symmetry": -1.0, "feet_downward": -1.0, "feet_downward_4": 0.0}
SU_CURRICULUM_WEIGHTS = {"upward_2": 10.0, "shape_symmetry": -2.0, "feet_downward": -1.0,
                         "feet_downward_4": 2.0}  # my_curriculum stage 1 (standup.py:103-107)
SU = dict(P_DELTA=25, ACTIONS=31, CENTER_Z_LAST=37, EP_LEN=38, EP_SUMS=39, LINK_MU=43, LINK_MU_D=55)
# ZBOT_6S_CFG_2 init_state (zbot_cfg.py:744-753): lying on its side, joints straight
SU_ROOT_POS = (0.0, 0.0, 0.05)
SU_ROOT_ROT = (0.707, 0.0, -0.707, 0.0)

# zbot-6b-walking-v4 (include/zbot.h enum zb_v4_state_field / zb_v4_reward_term)
V4_OBS_DIM, V4_NUM_TERMS, V4_STATE_DIM, V4_HIST, V4_RING = 24, 15, 85, 3, 24
V4_REWARD_TERMS = [  # dict order of Zbot6SEnvV4Cfg.reward_cfg (v4.py:620-641)
    "track_lin_vel_x", "track_heading_yaw", "lin_vel_y", "action_rate", "torques", "joint_vel", "joint_acc",
    "feet_downward", "feet_forward", "step_length", "feet_air_time_biped", "airtime_variance", "feet_slide",
    "feet_harmony", "feet_close",
]
V4_REWARD_WEIGHTS = {
    "track_lin_vel_x": 1.0, "track_heading_yaw": 1.0, "lin_vel_y": -1.0, "action_rate": -0.1, "torques": -2e-4,
    "joint_vel": -0.001, "joint_acc": -2.5e-7, "feet_downward": -1.0, "feet_forward": -0.5, "step_length": 5.0,
    "feet_air_time_biped": 1.0, "airtime_variance": -5.0, "feet_slide": -1.0, "feet_harmony": 0.0, "feet_close": -10.0,
}
# my_curriculum (v4.py:137-199): (common_step_counter threshold in episodes, weight updates, prob_pos)
V4_STAGES = [
    (12, {"airtime_variance": -10.0, "feet_forward": -1.0, "feet_slide": -2.0}, None),
    (24, {"airtime_variance": -40.0, "feet_downward": -5.0}, 0.8),
    (144, {"feet_harmony": 1.0, "feet_downward": -10.0, "step_length": 7.0, "track_heading_yaw": 2.0,
           "feet_close": -120.0}, 0.6),
]
V4 = dict(P_DELTA=25, ACTIONS=31, COMMANDS=37, TARGET_YAW=39, INTERVAL_LEFT=40, FEET_DOWN_POS=41,
          FEET_STEP_LEN=47, FEET_F_LAST=49, FEET_FZ_HIST=51, UNDES_FMAX_HIST=57, FEET_AIR_CUR=60,
          FEET_CONTACT_CUR=62, FEET_AIR_LAST=64, FEET_CONTACT_LAST=66, EP_LEN=68, EP_SUMS=69, CURRENT_YAW=84)

# zbot-6b-walking-m-v0, the manager-based flat env (include/zbot.h enum zb_manager_state_field /
# zb_manager_reward_term); RewardsCfg order after flat_env_cfg.py's overrides (mgr.py:262-357)
M_OBS_DIM, M_NUM_TERMS, M_STATE_DIM = 25, 11, 100
M_REWARD_TERMS = [
    "track_lin_vel_xy_exp", "track_ang_vel_z_exp", "termination_penalty", "dof_torques_l2", "dof_acc_l2",
    "action_rate_l2", "foot_step_length", "foot_downward", "foot_forward", "feet_slide", "air_time_variance",
]
M_REWARD_WEIGHTS = {
    "track_lin_vel_xy_exp": 1.0, "track_ang_vel_z_exp": 0.5, "termination_penalty": -200.0,
    "dof_torques_l2": -1.0e-5, "dof_acc_l2": -2.5e-7, "action_rate_l2": -0.01, "foot_step_length": 5.0,
    "foot_downward": -1.0, "foot_forward": -0.5, "feet_slide": -6.5, "air_time_variance": -15.0,
}
M_TERMINATION_TERMS = ["time_out", "base_height", "feet_close"]  # mgr.py:379-398 minus base_contact (flat)
M = dict(ACTIONS=25, COMMANDS=31, CMD_TIME_LEFT=34, CMD_STANDING=35, FEET_DOWN_POS=36, FEET_STEP_LEN=42,
         FEET_F_LAST=44, FEET_FZ_HIST=46, FEET_FN_HIST=52, FEET_AIR_CUR=58, FEET_AIR_LAST=60, METRICS=62,
         EP_LEN=64, EP_SUMS=65, LINK_MU=76, LINK_MU_D=88)

# state field offsets (include/zbot.h enum zb_state_field)
S = dict(ROOT_POS=0, ROOT_QUAT=3, ROOT_LINVEL=7, ROOT_ANGVEL=10, JOINT_POS=13, JOINT_VEL=19,
         P_DELTA=25, ACTIONS=31, FEET_DOWN_POS=37, FEET_STEP_LEN=43, FEET_F_LAST=45, HEADING_SUM=47,
         Y_ERR_SUM=48, FEET_FZ_HIST=49, UNDES_FMAX_HIST=59, FEET_AIR_CUR=64, FEET_AIR_LAST=66,
         FEET_CONTACT_CUR=68, EP_LEN=70, EP_SUMS=71, FEET_FORCE_SUM=86)


# ----------------------------------------------------------------------------- ctypes mirrors
class ZbModel(C.Structure):
    _fields_ = [
        ("body_mass", C.c_float * NUM_BODIES),
        ("body_com", (C.c_float * 3) * NUM_BODIES),
        ("body_inertia", (C.c_float * 6) * NUM_BODIES),
        ("joint_parent_pos", (C.c_float * 3) * NUM_DOF),
        ("joint_parent_rot", (C.c_float * 4) * NUM_DOF),
        ("joint_child_pos", (C.c_float * 3) * NUM_DOF),
        ("joint_child_rot", (C.c_float * 4) * NUM_DOF),
        ("link_body", C.c_int32 * NUM_LINKS),
        ("link_pos", (C.c_float * 3) * NUM_LINKS),
        ("link_rot", (C.c_float * 4) * NUM_LINKS),
        ("link_com", (C.c_float * 3) * NUM_LINKS),
        ("link_circle", ((C.c_float * 9) * 2) * NUM_LINKS),
        ("link_sphere", ((C.c_float * 4) * 2) * NUM_LINKS),
        ("link_bound", (C.c_float * 4) * NUM_LINKS),
        ("num_self_pairs", C.c_int32),
        ("self_pairs", (C.c_int32 * 2) * MAX_SELF_PAIRS),
        ("default_root_pos", C.c_float * 3),
        ("default_root_quat", C.c_float * 4),
        ("default_joint_pos", C.c_float * NUM_DOF),
        ("kp", C.c_float), ("kd", C.c_float), ("effort_limit", C.c_float),
        ("velocity_limit", C.c_float), ("max_depenetration_velocity", C.c_float),
        ("max_angular_velocity", C.c_float),
        ("base_link", C.c_int32), ("foot_links", C.c_int32 * 2), ("undesired_links", C.c_int32 * 10),
        ("api_root_link", C.c_int32), ("api_root_in_root", C.c_float * 7),
        ("api_joint_index", C.c_int32 * NUM_DOF), ("api_joint_sign", C.c_float * NUM_DOF),
        ("link_circle_dup", C.c_int32 * NUM_LINKS),
    ]


class ZbTaskCfg(C.Structure):
    _fields_ = [
        ("sim_dt", C.c_float), ("decimation", C.c_int32), ("max_episode_length", C.c_int32),
        ("termination_height", C.c_float), ("reward_scales", C.c_float * NUM_TERMS),
        ("terminal_penalty", C.c_float), ("joint_speed_limit", C.c_float), ("gravity", C.c_float),
        ("friction", C.c_float), ("contact_force_threshold", C.c_float),
        ("contact_margin", C.c_float), ("baumgarte", C.c_float),
        ("solver_iterations", C.c_int32), ("enable_self_collision", C.c_int32),
        ("task", C.c_int32), ("reset_pose_range", (C.c_float * 2) * 4), ("reset_pose_body_frame", C.c_int32),
        ("center_z_init", C.c_float), ("center_z_drop", C.c_float), ("center_z_period", C.c_int32),
        ("num_stages", C.c_int32), ("stage_steps", C.c_int32 * MAX_STAGES),
        ("stage_scales", (C.c_float * MAX_REWARD_TERMS) * MAX_STAGES), ("stage_prob_pos", C.c_float * MAX_STAGES),
        ("cmd_vel_range", C.c_float * 2), ("cmd_yaw_range", C.c_float * 2), ("cmd_dual_sign", C.c_int32),
        ("cmd_offset", C.c_float), ("cmd_interval_s", C.c_float * 2),
        ("range_limit_vel", C.c_float * 2), ("range_limit_yaw", C.c_float * 2), ("range_start_steps", C.c_int32),
        ("range_period_steps", C.c_int32), ("range_min_buffer", C.c_int32), ("range_threshold", C.c_float),
        ("range_delta", C.c_float), ("undesired_force_threshold", C.c_float), ("feet_f_last_init", C.c_float),
        ("action_scale", C.c_float), ("action_clip", C.c_float), ("obs_corruption", C.c_int32),
        ("obs_noise", C.c_float * 3), ("cmd_resample_s", C.c_float), ("cmd_rel_standing", C.c_float),
        ("feet_close_min", C.c_float),
        ("reset_feet_refresh", C.c_int32),
        ("friction_dynamic", C.c_float),
        ("solver_mode", C.c_int32), ("self_manifold", C.c_int32),
        ("reward_active", C.c_uint32),
    ]


# ----------------------------------------------------------------------------- math helpers
def qmul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz,
                     aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw])


def qconj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def qmat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def qrot(q, v):
    return qmat(q) @ np.asarray(v, dtype=np.float64)


def qnorm(q):
    q = np.asarray(q, dtype=np.float64)
    return q / np.linalg.norm(q)


@dataclass
class Xf:
    """Rigid transform (p, q): x_parent = R(q) x_child + p."""
    p: np.ndarray = field(default_factory=lambda: np.zeros(3))
    q: np.ndarray = field(default_factory=lambda: np.array([1.0, 0, 0, 0]))

    def __mul__(self, o: "Xf") -> "Xf":
        return Xf(self.p + qrot(self.q, o.p), qnorm(qmul(self.q, o.q)))

    def inv(self) -> "Xf":
        qi = qconj(self.q)
        return Xf(-qrot(qi, self.p), qi)

    def apply(self, x):
        return self.p + qrot(self.q, x)


def rz(theta: float) -> Xf:
    return Xf(np.zeros(3), np.array([math.cos(theta / 2), 0.0, 0.0, math.sin(theta / 2)]))


# ----------------------------------------------------------------------------- model build
@dataclass
class RobotModel:
    raw: dict
    link_body: list
    link_xf: list          # link frame in body frame
    joints: list           # revolute joints in chain order: dict(parent_xf, child_xf, name)
    body_mass: np.ndarray
    body_com: np.ndarray
    body_inertia: np.ndarray  # (7,3,3) about COM, body frame
    link_com: np.ndarray
    circles: np.ndarray    # (12,2,9) C, E1, E2 in body frame
    spheres: np.ndarray    # (12,2,4)
    bounds: np.ndarray     # (12,4)
    self_pairs: list
    default_joint_pos: np.ndarray
    default_root_pos: np.ndarray
    default_root_quat: np.ndarray
    cfg: dict
    # Isaac Lab view of the articulation (differs from the internal chain when the USD's
    # articulation root is not the first chain link, e.g. zbot_6s_v09.usd rooted at the base):
    link_names: list = field(default_factory=lambda: list(LINK_NAMES))
    joint_names: list = field(default_factory=lambda: list(JOINT_NAMES))  # USD name of internal joint k
    joint_sign: np.ndarray = field(default_factory=lambda: np.ones(NUM_DOF))  # q_usd = sign * q_internal
    api_joint_index: list = field(default_factory=lambda: list(range(NUM_DOF)))  # Isaac Lab index of joint k
    api_root_link: int = 0            # chain index of the Isaac Lab root link
    api_root_in_root: tuple = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))  # its pose in the chain root frame
    base_link: int = 6

    def fk(self, root_pos, root_quat, q):
        """World transforms of the 7 bodies and 12 links (float64, composition order of PhysX)."""
        bodies = [Xf(np.asarray(root_pos, float), qnorm(root_quat))]
        for k, j in enumerate(self.joints):
            bodies.append(bodies[k] * j["parent_xf"] * rz(q[k]) * j["child_xf"])
        links = [bodies[self.link_body[i]] * self.link_xf[i] for i in range(NUM_LINKS)]
        return bodies, links


def _perp_basis(n):
    n = n / np.linalg.norm(n)
    e1 = np.cross(n, [0.0, 1.0, 0.0])
    if np.linalg.norm(e1) < 1e-6:
        e1 = np.cross(n, [1.0, 0.0, 0.0])
    e1 /= np.linalg.norm(e1)
    return e1, np.cross(n, e1)


_AXIS_TO_Z = {  # rotation taking the local z axis onto the joint axis
    "Z": np.array([1.0, 0.0, 0.0, 0.0]),
    "Y": np.array([math.cos(-math.pi / 4), math.sin(-math.pi / 4), 0.0, 0.0]),   # Rx(-90 deg): z -> y
    "X": np.array([math.cos(math.pi / 4), 0.0, math.sin(math.pi / 4), 0.0]),     # Ry(+90 deg): z -> x
}


def load_model(path: str = ASSET) -> RobotModel:
    """Build the serial-chain model from a decoded asset whose ``links`` are listed in chain order
    (first link = the simulator's root). Joints may point either way along the chain (a USD whose
    articulation root is mid-chain); a joint traversed against its body0 -> body1 direction is
    inverted and its angle negated. Revolute axes other than Z get a constant frame rotation."""
    raw = json.load(open(path))
    names = [l["name"] for l in raw["links"]]
    assert len(names) == NUM_LINKS
    links = {l["name"]: l for l in raw["links"]}
    pair = {frozenset((j["body0"], j["body1"])): j for j in raw["joints"]}

    link_body = [0] * NUM_LINKS
    link_xf = [Xf() for _ in range(NUM_LINKS)]
    joints = []
    joint_names, joint_sign = [], []
    body = 0
    for k in range(1, NUM_LINKS):
        prev, cur = names[k - 1], names[k]
        j = pair[frozenset((prev, cur))]
        fwd = j["body0"] == prev
        T0 = Xf(np.array(j["local_pos0"], float), qnorm(j["local_rot0_wxyz"]))
        T1 = Xf(np.array(j["local_pos1"], float), qnorm(j["local_rot1_wxyz"]))
        Tp, Tc = (T0, T1) if fwd else (T1, T0)  # parent-side / child-side joint frames
        if j["type"] == "fixed":
            link_body[k] = body
            link_xf[k] = link_xf[k - 1] * Tp * Tc.inv()
        else:
            A = Xf(np.zeros(3), _AXIS_TO_Z[j["axis"]])
            body += 1
            link_body[k] = body
            link_xf[k] = Xf()
            joints.append({"name": j["name"], "parent_xf": link_xf[k - 1] * Tp * A, "child_xf": (Tc * A).inv()})
            joint_names.append(j["name"])
            joint_sign.append(1.0 if fwd else -1.0)
    assert body == NUM_BODIES - 1 and len(joints) == NUM_DOF

    # composite mass properties (authored link values, used verbatim)
    body_mass = np.zeros(NUM_BODIES)
    body_mc = np.zeros((NUM_BODIES, 3))
    link_com = np.zeros((NUM_LINKS, 3))
    link_I = []
    for i, name in enumerate(names):
        l = links[name]
        xf = link_xf[i]
        com_b = xf.apply(l["com"])
        link_com[i] = com_b
        Rpa = qmat(qnorm(l["principal_axes_wxyz"]))
        I_link = Rpa @ np.diag(l["diag_inertia"]) @ Rpa.T
        Rl = qmat(xf.q)
        link_I.append(Rl @ I_link @ Rl.T)
        body_mass[link_body[i]] += l["mass"]
        body_mc[link_body[i]] += l["mass"] * com_b
    body_com = body_mc / body_mass[:, None]
    body_inertia = np.zeros((NUM_BODIES, 3, 3))
    for i, name in enumerate(names):
        b = link_body[i]
        d = link_com[i] - body_com[b]
        m = links[name]["mass"]
        body_inertia[b] += link_I[i] + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))

    circles = np.zeros((NUM_LINKS, 2, 9))
    spheres = np.zeros((NUM_LINKS, 2, 4))
    bounds = np.zeros((NUM_LINKS, 4))
    for i, name in enumerate(names):
        l = links[name]
        xf = link_xf[i]
        pts = []
        for k, cdef in enumerate(l["circles"]):
            Cb = xf.apply(cdef["center"])
            nb = qrot(xf.q, cdef["normal"])
            e1, e2 = _perp_basis(nb)
            r = cdef["radius"]
            circles[i, k] = np.r_[Cb, r * e1, r * e2]
            th = np.linspace(0, 2 * np.pi, 256, endpoint=False)
            pts.append(Cb + r * (np.outer(np.cos(th), e1) + np.outer(np.sin(th), e2)))
        for k, s in enumerate(l["spheres"]):
            spheres[i, k] = np.r_[xf.apply(s["center"]), s["radius"]]
        pts = np.vstack(pts)
        ctr = 0.5 * (circles[i, 0, :3] + circles[i, 1, :3])
        bounds[i] = np.r_[ctr, np.linalg.norm(pts - ctr, axis=1).max() + 1e-4]

    # PhysX filters self-collision between joint-connected links (incl. fixed joints)
    connected = {frozenset((names.index(j["body0"]), names.index(j["body1"]))) for j in raw["joints"]}
    self_pairs = [(a, b) for a in range(NUM_LINKS) for b in range(a + 1, NUM_LINKS)
                  if frozenset((a, b)) not in connected]

    cfg = raw["cfg"]
    sign = np.array(joint_sign)
    q0 = sign * np.array([cfg["joint_pos"][n] for n in joint_names], float)
    # Isaac Lab orders joints breadth-first from the articulation root (PhysX tensor API)
    root_name = cfg.get("root_link", names[0])
    root_idx = names.index(root_name)
    order, seen, queue = [], {root_name}, [root_name]
    while queue:
        cur = queue.pop(0)
        nbr = sorted((j for j in raw["joints"] if cur in (j["body0"], j["body1"])),
                     key=lambda j: min(names.index(j["body0"]), names.index(j["body1"])))
        for j in nbr:
            other = j["body1"] if j["body0"] == cur else j["body0"]
            if other in seen:
                continue
            seen.add(other)
            queue.append(other)
            if j["type"] != "fixed":
                order.append(j["name"])
    api_index = [order.index(n) for n in joint_names]
    rm = RobotModel(raw=raw, link_body=link_body, link_xf=link_xf, joints=joints,
                    body_mass=body_mass, body_com=body_com, body_inertia=body_inertia,
                    link_com=link_com, circles=circles, spheres=spheres, bounds=bounds,
                    self_pairs=self_pairs, default_joint_pos=q0,
                    default_root_pos=np.array(cfg["root_pos"], float),
                    default_root_quat=np.array(cfg["root_rot_wxyz"], float), cfg=cfg,
                    link_names=names, joint_names=joint_names, joint_sign=sign, api_joint_index=api_index,
                    api_root_link=root_idx, base_link=names.index("base"))
    if root_idx != 0:
        # the cfg's root pose is the Isaac Lab root's; the chain root's follows from the default pose
        _, lk = rm.fk(np.zeros(3), np.array([1.0, 0, 0, 0]), q0)
        T = lk[root_idx]
        rm.api_root_in_root = (tuple(T.p), tuple(T.q))
        Xroot = Xf(rm.default_root_pos, qnorm(rm.default_root_quat)) * T.inv()
        rm.default_root_pos, rm.default_root_quat = Xroot.p, Xroot.q
    return rm


V09_ASSET = os.path.join(os.path.dirname(__file__), "assets", "zbot6s_v09_model.json")


def load_v09_model() -> RobotModel:
    """ZBOT_6S_V2_CFG on zbot_6s_v09.usd (zbot_cfg.py:959-1005): the manager-based env's robot."""
    return load_model(V09_ASSET)


def standup_model(rm: RobotModel | None = None) -> RobotModel:
    """``ZBOT_6S_CFG_2`` (zbot_cfg.py:721-763): the same robot / actuators as ``ZBOT_6S_CFG`` with
    the lying initial state (root (0, 0, 0.05), rot (0.707, 0, -0.707, 0), joints 0)."""
    import dataclasses
    rm = rm or load_model()
    return dataclasses.replace(rm, default_joint_pos=np.zeros(NUM_DOF),
                               default_root_pos=np.array(SU_ROOT_POS, float),
                               default_root_quat=np.array(SU_ROOT_ROT, float))


def pack_model(rm: RobotModel | None = None) -> ZbModel:
    rm = rm or load_model()
    m = ZbModel()
    for b in range(NUM_BODIES):
        m.body_mass[b] = rm.body_mass[b]
        for a in range(3):
            m.body_com[b][a] = rm.body_com[b][a]
        I = rm.body_inertia[b]
        for a, v in enumerate((I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2])):
            m.body_inertia[b][a] = v
    for k, j in enumerate(rm.joints):
        for a in range(3):
            m.joint_parent_pos[k][a] = j["parent_xf"].p[a]
            m.joint_child_pos[k][a] = j["child_xf"].p[a]
        for a in range(4):
            m.joint_parent_rot[k][a] = j["parent_xf"].q[a]
            m.joint_child_rot[k][a] = j["child_xf"].q[a]
    for i in range(NUM_LINKS):
        m.link_body[i] = rm.link_body[i]
        for a in range(3):
            m.link_pos[i][a] = rm.link_xf[i].p[a]
            m.link_com[i][a] = rm.link_com[i][a]
        for a in range(4):
            m.link_rot[i][a] = rm.link_xf[i].q[a]
            m.link_bound[i][a] = rm.bounds[i][a]
        for k in range(2):
            for a in range(9):
                m.link_circle[i][k][a] = rm.circles[i, k, a]
            for a in range(4):
                m.link_sphere[i][k][a] = rm.spheres[i, k, a]
    m.num_self_pairs = len(rm.self_pairs)
    for p, (a, b) in enumerate(rm.self_pairs):
        m.self_pairs[p][0], m.self_pairs[p][1] = a, b
    for a in range(3):
        m.default_root_pos[a] = rm.default_root_pos[a]
    for a in range(4):
        m.default_root_quat[a] = rm.default_root_quat[a]
    for k in range(NUM_DOF):
        m.default_joint_pos[k] = rm.default_joint_pos[k]
    c = rm.cfg
    m.kp, m.kd = c["stiffness"], c["damping"]
    m.effort_limit, m.velocity_limit = c["effort_limit"], c["velocity_limit"]
    m.max_depenetration_velocity = c["max_depenetration_velocity"]
    # RigidBodyPropertiesCfg(max_angular_velocity=1000.0) in every ZBOT cfg (zbot_cfg.py:632, 683, 732,
    # 775); Isaac Lab's unit is deg/s, the simulator's rad/s
    m.max_angular_velocity = math.radians(c.get("max_angular_velocity_deg", 1000.0))
    m.base_link = rm.base_link
    feet = [i for i, n in enumerate(rm.link_names) if n.startswith("foot")]  # "foot.*"
    m.foot_links[0], m.foot_links[1] = feet
    undesired = [i for i, n in enumerate(rm.link_names) if n == "base" or n[0] in "ab"]  # "base|a.*|b.*"
    assert len(undesired) == 10
    for k, i in enumerate(undesired):
        m.undesired_links[k] = i
    m.api_root_link = rm.api_root_link
    (px, py, pz), q = rm.api_root_in_root
    for a, v in enumerate((px, py, pz, *q)):
        m.api_root_in_root[a] = v
    for k in range(NUM_DOF):
        m.api_joint_index[k] = rm.api_joint_index[k]
        m.api_joint_sign[k] = rm.joint_sign[k]
    for i, bits in enumerate(duplicate_circles(rm)):
        m.link_circle_dup[i] = bits
    return m


def duplicate_circles(rm: RobotModel, tol: float = 1e-5) -> list:
    """Per link, bit ci set when circle ci coincides with a circle of a lower-indexed link of the same
    rigid composite (the mated faces of b_i and a_{i+1} across each fixed joint: same centre, plane and
    radius). Ground detection skips those, so a mated face yields one contact set (owned by the
    lower link) instead of two near-identical sets whose order in the 12-slot selection would be
    decided by rounding."""
    out = [0] * NUM_LINKS
    body = lambda l: (l + 1) >> 1  # noqa: E731  (the serial-chain topology, include/zbot.h)
    for l in range(NUM_LINKS):
        for ci in range(2):
            A = np.asarray(rm.circles[l, ci], np.float64)
            nA = np.cross(A[3:6], A[6:9])
            for k in range(l):
                if body(k) != body(l):
                    continue
                for cj in range(2):
                    B = np.asarray(rm.circles[k, cj], np.float64)
                    nB = np.cross(B[3:6], B[6:9])
                    same_plane = np.linalg.norm(np.cross(nA / np.linalg.norm(nA), nB / np.linalg.norm(nB))) < tol
                    same_r = abs(np.linalg.norm(A[3:6]) - np.linalg.norm(B[3:6])) < tol
                    if np.abs(A[:3] - B[:3]).max() < tol and same_plane and same_r:
                        out[l] |= 1 << ci
    return out


@dataclass
class TaskCfg:
    """ZbotDirectEnvCfgV2 (v2.py:26-206) plus the simulator's solver parameters."""
    sim_dt: float = 1.0 / 200.0
    decimation: int = 4
    episode_length_s: float = 20.0
    termination_height: float = 0.22
    reward_weights: dict = field(default_factory=lambda: dict(REWARD_WEIGHTS))
    terminal_penalty: float = 20.0
    joint_speed_limit: float = 1.0
    gravity: float = 9.81
    friction: float = 1.0
    friction_dynamic: float = 1.0
    contact_force_threshold: float = 1.0
    contact_margin: float = 0.004
    baumgarte: float = 0.2
    solver_iterations: int = 4   # = solver_position_iteration_count (zbot_cfg.py:637)
    solver_mode: int = 0         # 0: PGS sweeps on one linearisation; 1: TGS-style; 2: TGS + per-iteration ground refresh; 3: + self-contact refresh (zb_task_cfg.solver_mode)
    self_manifold: int = 2       # 2: cap-on-cap (up to 4 points) + side-by-side rims (up to 3); 1: caps only; 0: one point per pair
    enable_self_collision: bool = True
    task: int = TASK_WALKING_V2
    # stand-up / v4 reset pose (reset_root_state_uniform): x, y, roll, yaw ranges
    reset_pose_range: tuple = ((-0.5, 0.5), (-0.5, 0.5), (-0.7854, 0.7854), (-3.14, 3.14))
    reset_pose_body_frame: bool = False
    center_z_init: float = 0.05
    center_z_drop: float = 0.05
    center_z_period: int = 50
    # curriculum: [(common_step_counter threshold, {term: weight updates}, prob_pos or None)], cumulative
    stages: list = field(default_factory=list)
    # v4 commands / range curriculum
    cmd_vel_range: tuple = (0.3, 0.3)
    cmd_yaw_range: tuple = (-0.1, 0.1)
    cmd_dual_sign: bool = True
    cmd_offset: float = 0.0
    cmd_prob_pos: float = 1.0
    cmd_interval_s: tuple = (3.0, 6.0)
    range_limit_vel: tuple = (0.0, 0.3)
    range_limit_yaw: tuple = (-0.5, 0.5)
    range_start_episodes: int = 48
    range_period_episodes: int = 12
    range_min_buffer: int = 20
    range_threshold: float = 0.85
    range_delta: float = 0.05
    undesired_force_threshold: float = 1.0
    feet_f_last_init: float = 0.0
    # manager env: RelativeJointPositionAction, observation noise, UniformLevelVelocityCommand
    action_scale: float = 0.04 * math.pi
    action_clip: float = 0.04 * math.pi
    obs_corruption: bool = True
    obs_noise: tuple = (0.01, 0.01, 1.5)
    cmd_resample_s: float = 10.0
    cmd_rel_standing: float = 0.02
    feet_close_min: float = 0.12
    # feet_down_pos_last on reset: False = pre-reset feet (the reference's call order, v2.py:436),
    # True = post-reset feet
    reset_feet_refresh: bool = False
    range_period_steps: int | None = None   # manager: lin_vel_cmd_levels fires on counter % this == 0

    @classmethod
    def standup(cls, curriculum_steps: int | None = None, curriculum: bool = True,
                curriculum_weights: dict | None = None, **kw) -> "TaskCfg":
        """Zbot6SUpEnvCfg (standup.py:191-447): 6 s episodes, terminal penalty 2, 4 reward terms,
        my_curriculum at max_episode_length * 80 steps (or ``curriculum_steps``)."""
        d = dict(task=TASK_STANDUP_V0, episode_length_s=6.0, terminal_penalty=2.0, termination_height=0.20,
                 reward_weights=dict(SU_REWARD_WEIGHTS))
        d.update(kw)
        c = cls(**d)
        if curriculum:
            thr = c.max_episode_length * 80 if curriculum_steps is None else curriculum_steps
            c.stages = [(thr, dict(curriculum_weights or SU_CURRICULUM_WEIGHTS), None)]
        return c

    @classmethod
    def walking_v4(cls, curriculum: bool = True, stage_scale: float | None = None, **kw) -> "TaskCfg":
        """Zbot6SEnvV4Cfg (v4.py:443-686): 20 s episodes, history-3 contact sensor, died on an
        undesired body force > 0.5 N or base below 0.20 m, 15 reward terms, commands, curricula.
        ``stage_scale`` rescales the curriculum thresholds (tests)."""
        d = dict(task=TASK_WALKING_V4, episode_length_s=20.0, terminal_penalty=20.0, termination_height=0.20,
                 reward_weights=dict(V4_REWARD_WEIGHTS), reset_pose_range=((-0.5, 0.5), (-0.5, 0.5), (0.0, 0.0),
                                                                           (-3.14, 3.14)),
                 reset_pose_body_frame=True, undesired_force_threshold=0.5, feet_f_last_init=15.0)
        d.update(kw)
        c = cls(**d)
        if curriculum:
            L = c.max_episode_length if stage_scale is None else stage_scale
            c.stages = [(int(ep * L), dict(w), p) for ep, w, p in V4_STAGES]
        return c

    @classmethod
    def manager_flat(cls, **kw) -> "TaskCfg":
        """Zbot6BFlatEnvCfg (flat_env_cfg.py:10-111 over rough_env_cfg.py / mgr.py): ZBOT_6S_V2_CFG,
        20 s episodes, relative joint-position actions, 11 reward terms, terminations time_out /
        base_height < 0.2 / feet_close < 0.12, x-velocity command ~ U(-0.1, 0.1) widened by
        lin_vel_cmd_levels up to (-0.3, 0.3), observation noise on."""
        d = dict(task=TASK_MANAGER_V0, episode_length_s=20.0, termination_height=0.2, terminal_penalty=0.0,
                 reward_weights=dict(M_REWARD_WEIGHTS),
                 reset_pose_range=((-0.5, 0.5), (-0.5, 0.5), (0.0, 0.0), (-3.14, 3.14)), reset_pose_body_frame=True,
                 cmd_vel_range=(-0.1, 0.1), cmd_yaw_range=(0.0, 0.0), range_limit_vel=(-0.3, 0.3),
                 range_limit_yaw=(0.0, 0.0), range_threshold=0.8, range_delta=0.1)
        d.update(kw)
        return cls(**d)

    @property
    def obs_dim(self) -> int:
        return {TASK_STANDUP_V0: SU_OBS_DIM, TASK_WALKING_V4: V4_OBS_DIM,
                TASK_MANAGER_V0: M_OBS_DIM}.get(self.task, OBS_DIM)

    @property
    def state_dim(self) -> int:
        return {TASK_STANDUP_V0: SU_STATE_DIM, TASK_WALKING_V4: V4_STATE_DIM,
                TASK_MANAGER_V0: M_STATE_DIM}.get(self.task, STATE_DIM)

    @property
    def reward_terms(self) -> list:
        return {TASK_STANDUP_V0: SU_REWARD_TERMS, TASK_WALKING_V4: V4_REWARD_TERMS,
                TASK_MANAGER_V0: M_REWARD_TERMS}.get(self.task, REWARD_TERMS)

    @property
    def step_dt(self) -> float:
        return self.sim_dt * self.decimation

    @property
    def max_episode_length(self) -> int:
        return math.ceil(self.episode_length_s / self.step_dt)

    def stage_weights(self) -> list:
        """Reward weights of every curriculum stage (stage 0 = reward_weights), cumulative updates."""
        out = [dict(self.reward_weights)]
        for _, upd, _ in self.stages:
            w = dict(out[-1])
            w.update(upd)
            out.append(w)
        return out

    def pack(self) -> ZbTaskCfg:
        c = ZbTaskCfg()
        c.sim_dt = self.sim_dt
        c.decimation = self.decimation
        c.max_episode_length = self.max_episode_length
        c.termination_height = self.termination_height
        if self.task == TASK_WALKING_V2:
            unknown = set(self.reward_weights) - set(REWARD_TERMS)
            if unknown:
                raise NotImplementedError(f"reward terms not compiled into zb_step_kernel: {sorted(unknown)}")
            for k, name in enumerate(REWARD_TERMS):
                # v2.py:250-252 multiplies every weight by step_dt at env construction
                c.reward_scales[k] = self.reward_weights.get(name, 0.0) * self.step_dt
                # the terms of the active reward_cfg (a stateful term's buffers advance only then)
                if name in self.reward_weights:
                    c.reward_active |= 1 << k
        else:
            c.reward_active = 0xFFFFFFFF
        # standup.py:624 / v4.py:886 multiply by step_dt per term in _get_rewards (the kernel does)
        ws = self.stage_weights()
        if len(ws) > MAX_STAGES:
            raise ValueError(f"at most {MAX_STAGES - 1} curriculum stages")
        c.num_stages = len(ws)
        prob = self.cmd_prob_pos
        for sidx, w in enumerate(ws):
            for k, name in enumerate(self.reward_terms if self.task != TASK_WALKING_V2 else []):
                c.stage_scales[sidx][k] = w.get(name, 0.0)
            if sidx > 0:
                c.stage_steps[sidx] = int(self.stages[sidx - 1][0])
                if self.stages[sidx - 1][2] is not None:
                    prob = self.stages[sidx - 1][2]
            c.stage_prob_pos[sidx] = prob
        c.cmd_vel_range[0], c.cmd_vel_range[1] = self.cmd_vel_range
        c.cmd_yaw_range[0], c.cmd_yaw_range[1] = self.cmd_yaw_range
        c.cmd_dual_sign = int(self.cmd_dual_sign)
        c.cmd_offset = self.cmd_offset
        c.cmd_interval_s[0], c.cmd_interval_s[1] = self.cmd_interval_s
        c.range_limit_vel[0], c.range_limit_vel[1] = self.range_limit_vel
        c.range_limit_yaw[0], c.range_limit_yaw[1] = self.range_limit_yaw
        c.range_start_steps = self.max_episode_length * self.range_start_episodes
        c.range_period_steps = self.max_episode_length * self.range_period_episodes
        if self.task == TASK_MANAGER_V0:  # lin_vel_cmd_levels: common_step_counter % max_episode_length
            c.range_period_steps = self.range_period_steps or self.max_episode_length
        c.range_min_buffer = self.range_min_buffer
        c.range_threshold = self.range_threshold
        c.range_delta = self.range_delta
        c.undesired_force_threshold = self.undesired_force_threshold
        c.feet_f_last_init = self.feet_f_last_init
        c.action_scale = self.action_scale
        c.action_clip = self.action_clip
        c.obs_corruption = int(self.obs_corruption)
        for k in range(3):
            c.obs_noise[k] = self.obs_noise[k]
        c.cmd_resample_s = self.cmd_resample_s
        c.cmd_rel_standing = self.cmd_rel_standing
        c.feet_close_min = self.feet_close_min
        c.reset_feet_refresh = int(self.reset_feet_refresh)
        c.friction_dynamic = self.friction_dynamic
        c.solver_mode = int(self.solver_mode)
        c.self_manifold = int(self.self_manifold)
        c.reset_pose_body_frame = int(self.reset_pose_body_frame)
        c.task = self.task
        for k in range(4):
            c.reset_pose_range[k][0], c.reset_pose_range[k][1] = self.reset_pose_range[k]
        c.center_z_init = self.center_z_init
        c.center_z_drop = self.center_z_drop
        c.center_z_period = self.center_z_period
        c.terminal_penalty = self.terminal_penalty
        c.joint_speed_limit = self.joint_speed_limit
        c.gravity = self.gravity
        c.friction = self.friction
        c.contact_force_threshold = self.contact_force_threshold
        c.contact_margin = self.contact_margin
        c.baumgarte = self.baumgarte
        c.solver_iterations = self.solver_iterations
        c.enable_self_collision = int(self.enable_self_collision)
        return c


def default_state(num_envs: int, rm: RobotModel | None = None) -> np.ndarray:
    """SoA state [STATE_DIM][N] at the default pose (ep_len 0, everything else zero)."""
    rm = rm or load_model()
    st = np.zeros((STATE_DIM, num_envs), np.float32)
    st[S["ROOT_POS"]:S["ROOT_POS"] + 3] = rm.default_root_pos[:, None]
    st[S["ROOT_QUAT"]:S["ROOT_QUAT"] + 4] = rm.default_root_quat[:, None]
    st[S["JOINT_POS"]:S["JOINT_POS"] + 6] = rm.default_joint_pos[:, None]
    _, links = rm.fk(rm.default_root_pos, rm.default_root_quat, rm.default_joint_pos)
    for f, li in enumerate((0, 11)):
        st[S["FEET_DOWN_POS"] + 3 * f:S["FEET_DOWN_POS"] + 3 * f + 3] = links[li].p[:, None]
    return st
