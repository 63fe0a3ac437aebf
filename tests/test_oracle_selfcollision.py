"""Self collision on the exact link shape.

Each link's collider is the convex hull of two 5 cm circles. The oracle's ``hull_pair`` (GJK on
the support function of the rounded core, oracle/zbot_oracle.c) is checked here against an
independent brute-force distance: the largest separating gap over directions (the support
functions of the circles give each hull's extent along a direction exactly; for disjoint convex
sets the maximum over directions is the distance), found on a dense direction grid and refined
by Nelder-Mead. The
robot's own link shapes (from zbot6s_model.json) are used at random relative poses, plus the
known answers of two parallel coaxial disks (gap = distance between the planes) and of
penetrating pairs (separation -overlap while the overlap is below 2 CORE_M).
"""
from __future__ import annotations


import numpy as np
import pytest

from oracle import pyoracle
from zbot_lab_amd import model as zm

CORE_M = 0.004  # = oracle CORE_M / kernel kCoreM (GJK_TOL 1e-5 m)


def _quat(rng):
    q = rng.normal(size=4)
    return q / np.linalg.norm(q)


def _rot(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def core_circles(circles):
    """[2][9] body-frame circles (C, E1, E2) -> core circles (same rule as the oracle's load_mdl)."""
    out = np.zeros((2, 9))
    for c in range(2):
        C0, E1, E2 = circles[c, :3], circles[c, 3:6], circles[c, 6:9]
        n = np.cross(E1, E2)
        n /= np.linalg.norm(n)
        r = np.linalg.norm(E1)
        sg = -1.0 if n @ (circles[1 - c, :3] - C0) < 0 else 1.0
        out[c, :3] = C0 + sg * CORE_M * n
        out[c, 3:6] = E1 * (r - CORE_M) / r
        out[c, 6:9] = E2 * (r - CORE_M) / r
    return out


def world(core, R, p):
    w = np.zeros_like(core)
    for c in range(2):
        w[c, :3] = R @ core[c, :3] + p
        w[c, 3:6] = R @ core[c, 3:6]
        w[c, 6:9] = R @ core[c, 6:9]
    return w


def rim_points(h, k=256):
    th = np.linspace(0, 2 * np.pi, k, endpoint=False)
    pts = [h[c, :3] + np.cos(th)[:, None] * h[c, 3:6] + np.sin(th)[:, None] * h[c, 6:9] for c in range(2)]
    return np.concatenate(pts)


def sat_gap(ha, hb, n):
    """Separation of the two core hulls along unit n (A above B): min over A - max over B of the
    projections, from the exact circle supports. A lower bound of the distance for every n, equal
    to it for the closest points' normal."""
    def lo(h):
        return min(h[c, :3] @ n - np.hypot(h[c, 3:6] @ n, h[c, 6:9] @ n) for c in range(2))

    def hi(h):
        return max(h[c, :3] @ n + np.hypot(h[c, 3:6] @ n, h[c, 6:9] @ n) for c in range(2))
    return lo(ha) - hi(hb)


def brute_distance(ha, hb):
    """Hull distance by brute force: the largest separating gap over a dense sphere of directions
    refined by Nelder-Mead (max_n sat_gap = the distance for disjoint convex sets)."""
    from scipy.optimize import minimize
    rng = np.random.default_rng(0)
    dirs = rng.normal(size=(4000, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    best = max(dirs, key=lambda n: sat_gap(ha, hb, n))

    def f(x):
        n = x / np.linalg.norm(x)
        return -sat_gap(ha, hb, n)
    res = minimize(f, best, method="Nelder-Mead", options={"xatol": 1e-10, "fatol": 1e-12, "maxiter": 4000})
    return -res.fun


def hull_pair(ha, hb, margin):
    lib = pyoracle.lib()
    out = np.zeros(8, np.float32)
    lib.zbo_hull_pair(np.ascontiguousarray(ha, np.float32).ravel(), np.ascontiguousarray(hb, np.float32).ravel(),
                      margin, out)
    return out


@pytest.fixture(scope="module")
def link_cores():
    rm = zm.load_model()
    return [core_circles(np.asarray(rm.circles[l], np.float64)) for l in range(zm.NUM_LINKS)]


def test_gjk_matches_brute_force_on_robot_links(link_cores):
    rng = np.random.default_rng(3)
    checked = 0
    for _ in range(40):
        la, lb = rng.integers(0, zm.NUM_LINKS, size=2)
        ha = world(link_cores[la], _rot(_quat(rng)), np.zeros(3))
        hb = world(link_cores[lb], _rot(_quat(rng)), rng.normal(size=3) * 0.06 + np.array([0, 0, 0.11]))
        d_ref = brute_distance(ha, hb)
        if d_ref < 1e-4:
            continue  # cores overlap: the fallback path, checked below
        out = hull_pair(ha, hb, 1e3)  # no early exit
        assert out[0] == 1.0
        d = out[1] + 2 * CORE_M
        assert abs(d - d_ref) < 1e-5 + 1e-3 * d_ref, (la, lb, d, d_ref)
        n = out[2:5]
        assert abs(np.linalg.norm(n) - 1) < 1e-5
        # the contact normal separates the cores by d (GJK's distance is an upper bound, the gap
        # along any direction a lower bound), and x lies midway between the core surfaces along n
        assert abs(sat_gap(ha, hb, n) - d) < 1e-5 + 1e-3 * d
        xa, xb = out[5:8] + n * d / 2, out[5:8] - n * d / 2
        assert abs(min(rim_points(ha, 4096) @ n) - xa @ n) < 5e-5
        assert abs(max(rim_points(hb, 4096) @ n) - xb @ n) < 5e-5
        checked += 1
    assert checked >= 25


def test_parallel_disks_gap_and_penetration():
    """Two coaxial flat links (circles in parallel planes): the caps are exact, so the separation
    is the plane gap, including penetrations below 2 CORE_M."""
    r = 0.05
    circ = np.zeros((2, 9))
    circ[0, :3] = [0, 0, 0]; circ[0, 3:6] = [r, 0, 0]; circ[0, 6:9] = [0, r, 0]
    circ[1, :3] = [0, 0, 0.053]; circ[1, 3:6] = [r, 0, 0]; circ[1, 6:9] = [0, r, 0]
    core = core_circles(circ)
    for gap in (0.02, 0.003, 0.0005, -0.002, -0.006):
        ha = world(core, np.eye(3), np.array([0, 0, 0.053 + gap]))
        hb = world(core, np.eye(3), np.zeros(3))
        out = hull_pair(ha, hb, 0.004)
        assert (out[0] == 1.0) == (gap < 0.004)
        if out[0]:
            assert abs(out[1] - gap) < 2e-6, (gap, out[1])
            assert np.allclose(out[2:5], [0, 0, 1], atol=1e-5)


def test_far_pairs_exit_early_without_contact(link_cores):
    rng = np.random.default_rng(5)
    for _ in range(20):
        ha = world(link_cores[0], _rot(_quat(rng)), np.zeros(3))
        hb = world(link_cores[3], _rot(_quat(rng)), np.array([0.0, 0.0, 0.4]))
        assert hull_pair(ha, hb, 0.004)[0] == 0.0


def test_self_contacts_in_random_rollouts():
    """The exact shape finds self contacts the inscribed spheres missed: random-action rollouts
    from the default pose report self candidates, all finite."""
    sim = pyoracle.OracleSim(64, seed=1)
    sim.reset()
    rng = np.random.default_rng(0)
    n_self = 0
    for _ in range(60):
        obs, rew, term, trunc = sim.step(rng.normal(size=(64, 6)).astype(np.float32) * 2)
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
        n_self += int(sim.contact_diag()[:, 2].sum())
    assert n_self > 0


def test_overlapping_cores_penetration_estimate(link_cores):
    """Overlapping cores (deeper than 2 CORE_M, beyond GJK's distance): the separating-axis estimate
    over the centre difference and the four circle normals gives the core separation, never
    shallower than the true penetration (the largest gap over all directions, brute force) and
    usually equal to it; the normal separates along that axis."""
    rng = np.random.default_rng(5)
    res = []
    while len(res) < 40:
        la, lb = rng.integers(0, zm.NUM_LINKS, size=2)
        ha = world(link_cores[la], _rot(_quat(rng)), np.zeros(3))
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        hb = world(link_cores[lb], _rot(_quat(rng)), d * rng.uniform(0.02, 0.06))
        out = hull_pair(ha, hb, 1e3)
        if out[1] > -2 * CORE_M + 1e-6:
            continue  # the cores do not overlap
        d_sat = out[1] + 2 * CORE_M
        d_ref = brute_distance(ha, hb)
        assert d_sat <= d_ref + 1e-6, (d_sat, d_ref)          # a bound: never shallower
        n = out[2:5]
        assert abs(np.linalg.norm(n) - 1) < 1e-5
        assert abs(sat_gap(ha, hb, n) - min(d_sat, 0.0)) < 1e-5  # the gap along the reported normal
        res.append(d_sat / d_ref)
    r = np.asarray(res)
    assert np.median(r) < 1.2 and (r < 1.5).mean() > 0.75, r
