"""Shared test helpers: seeded perturbed simulator states (numpy, SoA [87][N] for walking v2, include/zbot.h)."""
from __future__ import annotations

import numpy as np

from zbot_lab_amd import model as zm

S = zm.S


def quat_from_axis_angle(axis, angle):
    axis = np.asarray(axis, float)
    axis = axis / np.linalg.norm(axis, axis=-1, keepdims=True)
    h = 0.5 * np.asarray(angle, float)
    return np.concatenate([np.cos(h)[..., None], axis * np.sin(h)[..., None]], axis=-1)


def perturbed_states(n: int, seed: int = 0, jq_sigma: float = 0.25, jqd_sigma: float = 1.0, tilt: float = 0.05,
                     lift: float = 0.01, vel: float = 0.1, airborne: float = 0.0) -> np.ndarray:
    """Default pose + seeded perturbations. ``airborne`` lifts that fraction of envs by 0.3 m."""
    rng = np.random.default_rng(seed)
    rm = zm.load_model()
    st = zm.default_state(n, rm)
    st[S["JOINT_POS"]:S["JOINT_POS"] + 6] += rng.normal(0, jq_sigma, (6, n)).astype(np.float32)
    st[S["JOINT_VEL"]:S["JOINT_VEL"] + 6] = rng.normal(0, jqd_sigma, (6, n)).astype(np.float32)
    ax = rng.normal(size=(n, 3))
    ang = rng.uniform(0, tilt, n)
    q = quat_from_axis_angle(ax, ang)
    st[S["ROOT_QUAT"]:S["ROOT_QUAT"] + 4] = q.T.astype(np.float32)
    st[S["ROOT_POS"] + 2] += rng.uniform(0, lift, n).astype(np.float32)
    up = rng.random(n) < airborne
    st[S["ROOT_POS"] + 2, up] += 0.3
    st[S["ROOT_LINVEL"]:S["ROOT_LINVEL"] + 3] = rng.normal(0, vel, (3, n)).astype(np.float32)
    st[S["ROOT_ANGVEL"]:S["ROOT_ANGVEL"] + 3] = rng.normal(0, vel, (3, n)).astype(np.float32)
    st[S["EP_LEN"]] = rng.integers(0, 990, n).astype(np.float32)
    st[S["P_DELTA"]:S["P_DELTA"] + 6] = rng.normal(0, 0.3, (6, n)).astype(np.float32)
    st[S["ACTIONS"]:S["ACTIONS"] + 6] = np.tanh(rng.normal(0, 1, (6, n))).astype(np.float32)
    return st


def rel_err(a, b, floor):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), floor)
