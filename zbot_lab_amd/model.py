"""Robot model + task constants -> the ``zb_model`` / ``zb_task_cfg`` structs of ``include/zbot.h``.

The robot is ``ZBOT_6S_CFG`` (reference ``source/zbot/zbot/assets/zbot_cfg.py:621-669``) built on
``zbot_6s_new.usd``; the decoded asset lives in ``assets/zbot6s_model.json`` (written by
``tools/extract_model.py``). Here the 12 links / 6 revolute + 5 fixed joints are merged into the 7
rigid composites the simulator integrates (fixed joints have no DoF), and every per-link quantity
(link frame, authored COM, collision circles, self-collision spheres) is expressed in its
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
OBS_DIM, ACT_DIM, NUM_TERMS, HIST = 23, 6, 13, 5
MAX_SELF_PAIRS = 64
STATE_DIM = 84

LINK_NAMES = ["foot_0", "b1", "a2", "b2", "a3", "b3", "base", "b4", "a5", "b5", "a6", "foot_1"]
JOINT_NAMES = ["joint1", "joint2", "joint3", "joint4", "joint5", "joint6"]
REWARD_TERMS = [  # dict order of ZbotDirectEnvCfgV2.reward_cfg (v2.py:190-206)
    "base_vel_forward", "feet_downward", "feet_forward", "base_heading_x", "base_heading_x_sum",
    "step_length", "airtime_balance", "action_rate", "torques", "feet_slide", "base_pos_y_err",
    "base_pos_y_err_sum", "airtime_sum",
]
REWARD_WEIGHTS = {  # v2.py:190-206 ("train reward 2000 step4")
    "base_vel_forward": 1.0, "feet_downward": -2.0, "feet_forward": -1.0, "base_heading_x": -1.0,
    "base_heading_x_sum": -5.0, "step_length": 5.0, "airtime_balance": -15.0, "action_rate": -0.1,
    "torques": -0.002, "feet_slide": -10.0, "base_pos_y_err": -2.0, "base_pos_y_err_sum": -2.0,
    "airtime_sum": 3.0,
}

# zbot-6b-standup-v0 (include/zbot.h enum zb_standup_state_field / zb_standup_reward_term)
TASK_WALKING_V2, TASK_STANDUP_V0 = 0, 1
SU_OBS_DIM, SU_NUM_TERMS, SU_STATE_DIM = 22, 4, 55
SU_REWARD_TERMS = ["upward_2", "shape_symmetry", "feet_downward", "feet_downward_4"]  # standup.py:418-427
SU_REWARD_WEIGHTS = {"upward_2": 10.0, "shape_symmetry": -1.0, "feet_downward": -1.0, "feet_downward_4": 0.0}
SU_CURRICULUM_WEIGHTS = {"upward_2": 10.0, "shape_symmetry": -2.0, "feet_downward": -1.0,
                         "feet_downward_4": 2.0}  # my_curriculum stage 1 (standup.py:103-107)
SU = dict(P_DELTA=25, ACTIONS=31, CENTER_Z_LAST=37, EP_LEN=38, EP_SUMS=39, LINK_MU=43)
# ZBOT_6S_CFG_2 init_state (zbot_cfg.py:744-753): lying on its side, joints straight
SU_ROOT_POS = (0.0, 0.0, 0.05)
SU_ROOT_ROT = (0.707, 0.0, -0.707, 0.0)

# state field offsets (include/zbot.h enum zb_state_field)
S = dict(ROOT_POS=0, ROOT_QUAT=3, ROOT_LINVEL=7, ROOT_ANGVEL=10, JOINT_POS=13, JOINT_VEL=19,
         P_DELTA=25, ACTIONS=31, FEET_DOWN_POS=37, FEET_STEP_LEN=43, FEET_F_LAST=45, HEADING_SUM=47,
         Y_ERR_SUM=48, FEET_FZ_HIST=49, UNDES_FMAX_HIST=59, FEET_AIR_CUR=64, FEET_AIR_LAST=66,
         FEET_CONTACT_CUR=68, EP_LEN=70, EP_SUMS=71)


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
        ("base_link", C.c_int32), ("foot_links", C.c_int32 * 2), ("undesired_links", C.c_int32 * 10),
    ]


class ZbTaskCfg(C.Structure):
    _fields_ = [
        ("sim_dt", C.c_float), ("decimation", C.c_int32), ("max_episode_length", C.c_int32),
        ("termination_height", C.c_float), ("reward_scales", C.c_float * NUM_TERMS),
        ("terminal_penalty", C.c_float), ("joint_speed_limit", C.c_float), ("gravity", C.c_float),
        ("friction", C.c_float), ("contact_force_threshold", C.c_float),
        ("contact_margin", C.c_float), ("baumgarte", C.c_float),
        ("solver_iterations", C.c_int32), ("enable_self_collision", C.c_int32),
        ("task", C.c_int32), ("reset_pose_range", (C.c_float * 2) * 4),
        ("center_z_init", C.c_float), ("center_z_drop", C.c_float), ("center_z_period", C.c_int32),
        ("curriculum_steps", C.c_int32), ("curriculum_scales", C.c_float * NUM_TERMS),
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


def load_model(path: str = ASSET) -> RobotModel:
    raw = json.load(open(path))
    links = {l["name"]: l for l in raw["links"]}
    assert [l["name"] for l in raw["links"]] == LINK_NAMES
    by_parent = {j["body0"]: j for j in raw["joints"]}
    root = [l["name"] for l in raw["links"] if l["articulation_root"]]
    assert root == ["foot_0"], root

    link_body = [0] * NUM_LINKS
    link_xf = [Xf() for _ in range(NUM_LINKS)]
    joints = []
    body = 0
    cur = "foot_0"
    while cur in by_parent:
        j = by_parent[cur]
        lp0 = np.array(j["local_pos0"], float)
        lr0 = qnorm(j["local_rot0_wxyz"])
        lp1 = np.array(j["local_pos1"], float)
        lr1 = qnorm(j["local_rot1_wxyz"])
        child = j["body1"]
        ci, pi = LINK_NAMES.index(child), LINK_NAMES.index(cur)
        j0 = Xf(lp0, lr0)
        j1inv = Xf(lp1, lr1).inv()
        if j["type"] == "fixed":
            link_body[ci] = body
            link_xf[ci] = link_xf[pi] * j0 * j1inv
        else:
            assert j["axis"] == "Z"
            body += 1
            link_body[ci] = body
            link_xf[ci] = Xf()
            joints.append({"name": j["name"], "parent_xf": link_xf[pi] * j0, "child_xf": j1inv})
        cur = child
    assert body == NUM_BODIES - 1 and [j["name"] for j in joints] == JOINT_NAMES

    # composite mass properties (authored link values, used verbatim)
    body_mass = np.zeros(NUM_BODIES)
    body_mc = np.zeros((NUM_BODIES, 3))
    link_com = np.zeros((NUM_LINKS, 3))
    link_I = []
    for i, name in enumerate(LINK_NAMES):
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
    for i, name in enumerate(LINK_NAMES):
        b = link_body[i]
        d = link_com[i] - body_com[b]
        m = links[name]["mass"]
        body_inertia[b] += link_I[i] + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))

    circles = np.zeros((NUM_LINKS, 2, 9))
    spheres = np.zeros((NUM_LINKS, 2, 4))
    bounds = np.zeros((NUM_LINKS, 4))
    for i, name in enumerate(LINK_NAMES):
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
    connected = {frozenset((LINK_NAMES.index(j["body0"]), LINK_NAMES.index(j["body1"])))
                 for j in raw["joints"]}
    self_pairs = [(a, b) for a in range(NUM_LINKS) for b in range(a + 1, NUM_LINKS)
                  if frozenset((a, b)) not in connected]

    cfg = raw["cfg"]
    q0 = np.array([cfg["joint_pos"][n] for n in JOINT_NAMES], float)
    return RobotModel(raw=raw, link_body=link_body, link_xf=link_xf, joints=joints,
                      body_mass=body_mass, body_com=body_com, body_inertia=body_inertia,
                      link_com=link_com, circles=circles, spheres=spheres, bounds=bounds,
                      self_pairs=self_pairs, default_joint_pos=q0,
                      default_root_pos=np.array(cfg["root_pos"], float),
                      default_root_quat=np.array(cfg["root_rot_wxyz"], float), cfg=cfg)


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
    m.base_link = LINK_NAMES.index("base")
    m.foot_links[0], m.foot_links[1] = LINK_NAMES.index("foot_0"), LINK_NAMES.index("foot_1")
    undesired = [i for i, n in enumerate(LINK_NAMES) if n == "base" or n[0] in "ab"]
    assert len(undesired) == 10
    for k, i in enumerate(undesired):
        m.undesired_links[k] = i
    return m


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
    contact_force_threshold: float = 1.0
    contact_margin: float = 0.004
    baumgarte: float = 0.2
    solver_iterations: int = 4   # = solver_position_iteration_count (zbot_cfg.py:637)
    enable_self_collision: bool = True
    task: int = TASK_WALKING_V2
    # stand-up task only (standup.py)
    reset_pose_range: tuple = ((-0.5, 0.5), (-0.5, 0.5), (-0.7854, 0.7854), (-3.14, 3.14))  # x, y, roll, yaw
    center_z_init: float = 0.05
    center_z_drop: float = 0.05
    center_z_period: int = 50
    curriculum_steps: int | None = None  # my_curriculum threshold; None = max_episode_length * 80 (standup.py:102)
    curriculum_weights: dict | None = None

    @classmethod
    def standup(cls, **kw) -> "TaskCfg":
        """Zbot6SUpEnvCfg (standup.py:191-447): 6 s episodes, terminal penalty 2, 4 reward terms."""
        d = dict(task=TASK_STANDUP_V0, episode_length_s=6.0, terminal_penalty=2.0, termination_height=0.20,
                 reward_weights=dict(SU_REWARD_WEIGHTS), curriculum_weights=dict(SU_CURRICULUM_WEIGHTS))
        d.update(kw)
        return cls(**d)

    @property
    def obs_dim(self) -> int:
        return SU_OBS_DIM if self.task == TASK_STANDUP_V0 else OBS_DIM

    @property
    def state_dim(self) -> int:
        return SU_STATE_DIM if self.task == TASK_STANDUP_V0 else STATE_DIM

    @property
    def reward_terms(self) -> list:
        return SU_REWARD_TERMS if self.task == TASK_STANDUP_V0 else REWARD_TERMS

    @property
    def step_dt(self) -> float:
        return self.sim_dt * self.decimation

    @property
    def max_episode_length(self) -> int:
        return math.ceil(self.episode_length_s / self.step_dt)

    def pack(self) -> ZbTaskCfg:
        c = ZbTaskCfg()
        c.sim_dt = self.sim_dt
        c.decimation = self.decimation
        c.max_episode_length = self.max_episode_length
        c.termination_height = self.termination_height
        if self.task == TASK_STANDUP_V0:
            # standup.py:624 multiplies by step_dt per term in _get_rewards (the kernel does)
            for k, name in enumerate(SU_REWARD_TERMS):
                c.reward_scales[k] = self.reward_weights.get(name, 0.0)
                cw = self.curriculum_weights if self.curriculum_weights is not None else self.reward_weights
                c.curriculum_scales[k] = cw.get(name, 0.0)
            thr = self.max_episode_length * 80 if self.curriculum_steps is None else self.curriculum_steps
            c.curriculum_steps = thr if self.curriculum_weights else 0
        else:
            for k, name in enumerate(REWARD_TERMS):
                # v2.py:250-252 multiplies every weight by step_dt at env construction
                c.reward_scales[k] = self.reward_weights.get(name, 0.0) * self.step_dt
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
