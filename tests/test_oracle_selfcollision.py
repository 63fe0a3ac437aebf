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


import ctypes as C
import os

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


def pair_manifold(ha, hb, margin):
    out = np.zeros((4, 7), np.float32)
    k = pyoracle.lib().zbo_pair_manifold(np.ascontiguousarray(ha, np.float32).ravel(),
                                          np.ascontiguousarray(hb, np.float32).ravel(), margin, out.ravel())
    return out[:k]


def _flat_link(r0, r1=None):
    """Two parallel circles 5.3 cm apart (a flat stack), radii r0 (face at z = 0) and r1 (top)."""
    r1 = r0 if r1 is None else r1
    circ = np.zeros((2, 9))
    circ[0, 3:6] = [r0, 0, 0]; circ[0, 6:9] = [0, r0, 0]
    circ[1, :3] = [0, 0, 0.053]; circ[1, 3:6] = [r1, 0, 0]; circ[1, 6:9] = [0, r1, 0]
    return core_circles(circ)


def _check_manifold_geometry(ha, hb, pts, margin):
    """Every manifold point: normal = the pair normal, x the midpoint of a core-rim point of one face
    and its foot on the other face's plane along n, the foot inside that face's core disk, sep the
    core gap along n minus 2 CORE_M, within the margin."""
    for p in pts:
        sep, n, x = p[0], p[1:4], p[4:7]
        assert abs(np.linalg.norm(n) - 1) < 1e-5 and sep < margin
        xa, xb = x + n * (sep / 2 + CORE_M), x - n * (sep / 2 + CORE_M)  # the two core points
        # one of them on a face plane of its hull, the other on a core rim (brute force over circles)
        def on_plane(h, y):
            return min(abs(np.cross(h[c, 3:6], h[c, 6:9]) @ (y - h[c, :3])) / np.linalg.norm(np.cross(h[c, 3:6], h[c, 6:9]))
                       for c in range(2))

        def on_rim(h, y):
            return min(abs(np.linalg.norm(y - h[c, :3]) - np.linalg.norm(h[c, 3:6])) + on_plane(h[c:c + 1].repeat(2, 0), y)
                       for c in range(2))
        assert on_plane(ha, xa) < 2e-5 and on_plane(hb, xb) < 2e-5
        assert min(on_rim(ha, xa), on_rim(hb, xb)) < 5e-5


def test_face_manifold_parallel_caps():
    """Cap on cap (cfg self_manifold): a smaller disk face below a larger one gives the 4 rim points
    of the smaller face, each at the plane gap; offset equal disks give the two tips of the lens
    (one rim point of each face); the GJK contact alone when the faces do not face each other."""
    big, small = _flat_link(0.05), _flat_link(0.04)
    for gap in (0.003, 0.0005, -0.002):
        ha = world(big, np.eye(3), np.array([0, 0, 0.053 + gap]))
        hb = world(small, np.eye(3), np.array([0.004, -0.003, 0.0]))
        pts = pair_manifold(ha, hb, 0.004)
        assert len(pts) == 4, (gap, pts)
        assert np.allclose(pts[:, 0], gap, atol=2e-6), pts[:, 0]
        assert np.allclose(pts[:, 1:4], [0, 0, 1], atol=1e-5)
        _check_manifold_geometry(ha, hb, pts, 0.004)
    ha = world(big, np.eye(3), np.array([0, 0, 0.053 + 0.001]))
    hb = world(big, np.eye(3), np.array([0.03, 0.0, 0.0]))
    pts = pair_manifold(ha, hb, 0.004)
    assert len(pts) == 4, pts
    # the lens corners: B's rim point toward A's centre (x = 0.03 - r_core), B's two rim crossings
    # (0.03 rad inside the lens), A's rim point toward B's centre (x = r_core)
    rc = 0.05 - CORE_M
    np.testing.assert_allclose(pts[[0, 3], 4], [0.03 - rc, rc], atol=1e-6)
    assert abs(pts[1, 4] - 0.015) < 2e-3 and abs(pts[2, 4] - 0.015) < 2e-3 and pts[1, 5] * pts[2, 5] < 0
    _check_manifold_geometry(ha, hb, pts, 0.004)
    _check_manifold_geometry(ha, hb, pts, 0.004)
    # side by side (rim on rim): one point, the GJK contact
    R = _rot(np.array([np.cos(np.pi / 4), np.sin(np.pi / 4), 0, 0]))
    ha = world(big, R, np.array([0, 0.0, 0.11]))
    hb = world(big, R, np.zeros(3))
    pts = pair_manifold(ha, hb, 0.004)
    if len(pts):
        assert len(pts) == 1
        np.testing.assert_allclose(pts[0, :4], hull_pair(ha, hb, 0.004)[1:5], atol=1e-6)


def test_face_manifold_tilted_caps_keep_points_within_margin(link_cores):
    """Tilted faces (up to 12 degrees): the rim points whose gap exceeds the margin drop out, the
    rest satisfy the geometry; robot link shapes at random face-to-face poses."""
    rng = np.random.default_rng(11)
    counts = []
    for _ in range(60):
        tilt = rng.uniform(0, np.radians(12))
        ax = rng.normal(size=3)
        ax[2] = 0
        ax /= np.linalg.norm(ax)
        q = np.concatenate([[np.cos(tilt / 2)], np.sin(tilt / 2) * ax])
        ha = world(_flat_link(0.05), _rot(q), np.array([rng.uniform(-0.02, 0.02), rng.uniform(-0.02, 0.02),
                                                        0.053 + rng.uniform(-0.003, 0.004)]))
        hb = world(_flat_link(0.05), np.eye(3), np.zeros(3))
        pts = pair_manifold(ha, hb, 0.004)
        if len(pts) == 0:
            continue
        counts.append(len(pts))
        if len(pts) > 1:
            _check_manifold_geometry(ha, hb, pts, 0.004)
            d_ref = brute_distance(ha, hb)
            assert pts[:, 0].min() >= d_ref - 2 * CORE_M - 1e-5  # no point deeper than the true distance
    assert len(counts) > 30 and max(counts) == 4 and min(counts) >= 1


def test_manifold_in_folded_rollouts():
    """Folded stand-up robots keep more self-contact points with the manifold on (face-to-face pairs
    contribute up to 4) than with one point per pair from the same states; rollouts stay finite."""
    tot = {}
    for mf in (0, 1):
        cfg = zm.TaskCfg.standup()
        cfg.self_manifold = mf
        sim = pyoracle.OracleSim(256, cfg, seed=3)
        sim.reset()
        st = sim.get_state()
        st[13:19] += np.random.default_rng(4).normal(0, 1.5, (6, 256)).astype(np.float32)
        sim.set_state(st)
        rng = np.random.default_rng(0)
        n = 0
        for _ in range(20):
            obs, rew, te, tr = sim.step(rng.normal(size=(256, 6)).astype(np.float32))
            assert np.isfinite(obs).all() and np.isfinite(rew).all()
            n += int(sim.contact_diag()[:, 5].sum())
        tot[mf] = n
    assert tot[1] > tot[0] > 0, tot


def _rot_axis(axis, ang):
    axis = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def _ruling_line_gap(ha, hb, n, t_pts):
    """Gap along n between the two hulls' support rulings (the segments between their circles'
    support points along -n / +n) at the points t_pts (brute force: nearest points on the lines)."""
    def sup(h, d):
        p = []
        for c in range(2):
            a, b = d @ h[c, 3:6], d @ h[c, 6:9]
            p.append(h[c, :3] + (a * h[c, 3:6] + b * h[c, 6:9]) / np.hypot(a, b))
        return np.array(p)
    pa, pb = sup(ha, -n), sup(hb, n)
    return pa, pb


def test_rim_manifold_side_by_side():
    """Side by side (cfg self_manifold 2): two links lying with parallel axes touch along a line;
    the pair gives the GJK point plus the two ends of the rulings' overlap, every point at the line
    gap (constant along parallel rulings), normals perpendicular to the rulings; with the second link
    shifted along the axis the overlap shrinks to the common part; rulings crossing at 20 degrees
    give the GJK point alone; a tilt within 5 degrees keeps the ends at the rulings' gap there."""
    link = _flat_link(0.05)
    axis_x = _rot_axis([0, 1, 0], np.pi / 2)  # the link's axis (z) along x: lying on its side
    for gap in (0.002, 0.0004):
        ha = world(link, axis_x, np.array([0.0, 0.0, 2 * 0.05 + gap]))
        hb = world(link, axis_x, np.array([0.0, 0.0, 0.0]))
        pts = pair_manifold(ha, hb, 0.004)
        assert len(pts) in (2, 3), (gap, pts)  # (an end within 1 mm of the GJK point is not repeated)
        np.testing.assert_allclose(pts[:, 0], gap, atol=5e-6)
        np.testing.assert_allclose(pts[1:, 1:4], np.tile([0, 0, 1], (len(pts) - 1, 1)), atol=1e-5)  # the ends
        np.testing.assert_allclose(pts[0, 1:4], [0, 0, 1], atol=3e-3)  # the GJK point keeps GJK's normal
        # the points span the core rulings (the link lies along x in [0, 0.053], its cores inset by CORE_M)
        assert abs(pts[:, 4].min() - CORE_M) < 1e-3 + 1e-5 and abs(pts[:, 4].max() - (0.053 - CORE_M)) < 1e-3 + 1e-5
    ha = world(link, axis_x, np.array([0.02, 0.0, 2 * 0.05 + 0.001]))
    hb = world(link, axis_x, np.array([0.0, 0.0, 0.0]))
    pts = pair_manifold(ha, hb, 0.004)
    assert len(pts) in (2, 3)
    assert abs(pts[:, 4].min() - (0.02 + CORE_M)) < 1e-3 + 1e-5 and abs(pts[:, 4].max() - (0.053 - CORE_M)) < 1e-3 + 1e-5
    # crossing rulings: one point
    ha = world(link, _rot_axis([0, 0, 1], np.radians(20)) @ axis_x, np.array([0.0, 0.0, 0.101]))
    hb = world(link, axis_x, np.array([0.0, 0.0, 0.0]))
    pts = pair_manifold(ha, hb, 0.004)
    assert len(pts) == 1
    # a small tilt (3 degrees about y): the ends' separations are the gaps of the two core rulings
    # along the reported normal at those ends (direct evaluation on the support lines)
    ha = world(link, _rot_axis([0, 1, 0], np.radians(3)) @ axis_x, np.array([0.0, 0.0, 0.1005]))
    hb = world(link, axis_x, np.array([0.0, 0.0, 0.0]))
    pts = pair_manifold(ha, hb, 0.004)
    assert len(pts) >= 2, pts
    n = pts[-1, 1:4].astype(float)  # (an end's normal: perpendicular to A's ruling)
    pa, pb = _ruling_line_gap(ha, hb, n, None)
    for p in pts[1:]:
        x = p[4:7].astype(float)
        ta = (x - pa[0]) @ (pa[1] - pa[0]) / np.sum((pa[1] - pa[0]) ** 2)
        tb = (x - pb[0]) @ (pb[1] - pb[0]) / np.sum((pb[1] - pb[0]) ** 2)
        xa, xb = pa[0] + ta * (pa[1] - pa[0]), pb[0] + tb * (pb[1] - pb[0])
        assert abs((xa - xb) @ n - 2 * CORE_M - p[0]) < 2e-5, (p, (xa - xb) @ n - 2 * CORE_M)
    assert pts[:, 0].max() - pts[:, 0].min() > 1e-3  # the tilt shows in the gaps along the line
    assert abs(n @ (pa[1] - pa[0])) < 1e-6  # perpendicular to A's ruling


def test_rim_manifold_mode_switch():
    """self_manifold 1 keeps the face manifold only: the side-by-side pair is the GJK point alone."""
    link = _flat_link(0.05)
    axis_x = _rot_axis([0, 1, 0], np.pi / 2)
    ha = world(link, axis_x, np.array([0.0, 0.0, 0.101]))
    hb = world(link, axis_x, np.array([0.0, 0.0, 0.0]))
    lib = pyoracle.lib()
    lib.zbo_set_pair_manifold_mode.argtypes = [C.c_int]
    try:
        lib.zbo_set_pair_manifold_mode(1)
        assert len(pair_manifold(ha, hb, 0.004)) == 1
    finally:
        lib.zbo_set_pair_manifold_mode(2)
    assert len(pair_manifold(ha, hb, 0.004)) >= 2


def test_ruling_on_face_manifold():
    """A link lying on another's cap (cfg self_manifold 3, round 5): the GJK point
    plus the two ends of the lying link's core ruling clipped to the cap's core disk, each with the
    cap's normal and the end's height above the cap plane minus 2 CORE_M (direct evaluation); a ruling
    reaching past the cap is cut at the disk's rim; a 3-degree tilt shows in the ends' gaps; a
    10-degree tilt (outside RIM_DEG) and self_manifold 2 give the GJK point alone."""
    link = _flat_link(0.05)
    axis_x = _rot_axis([0, 1, 0], np.pi / 2)  # the link's axis along x: lying on its side
    rc = 0.05 - CORE_M
    lib = pyoracle.lib()
    lib.zbo_set_pair_manifold_mode.argtypes = [C.c_int]
    try:
        lib.zbo_set_pair_manifold_mode(3)
        hb = world(link, np.eye(3), np.zeros(3))                    # upright: its top cap at z = 0.053
        for px, gap in ((-0.02, 0.002), (-0.02, 0.0004), (0.02, 0.001)):
            ha = world(link, axis_x, np.array([px, 0.0, 0.053 + 0.05 + gap]))
            pts = pair_manifold(ha, hb, 0.004)
            assert len(pts) in (2, 3), (px, gap, pts)
            np.testing.assert_allclose(pts[:, 0], gap, atol=5e-6)
            np.testing.assert_allclose(pts[1:, 1:4], np.tile([0, 0, 1], (len(pts) - 1, 1)), atol=1e-6)
            np.testing.assert_allclose(pts[1:, 6], 0.053 - CORE_M + (gap + 2 * CORE_M) / 2, atol=1e-6)  # midpoints
            lo, hi = px + CORE_M, min(px + 0.053 - CORE_M, rc)            # the ruling clipped to the cap disk
            assert abs(pts[:, 4].min() - lo) < 1e-3 + 1e-6 and abs(pts[:, 4].max() - hi) < 1e-3 + 1e-6, pts[:, 4]
            assert np.all(np.hypot(pts[1:, 4], pts[1:, 5]) <= rc + 1e-6)
        # 3 degrees about y: the ends' gaps are their heights above the cap's core plane
        ha = world(link, _rot_axis([0, 1, 0], np.radians(3)) @ axis_x, np.array([-0.02, 0.0, 0.053 + 0.05 + 0.0005]))
        pts = pair_manifold(ha, hb, 0.004)
        assert len(pts) >= 2, pts
        for p in pts[1:]:
            # the core point on A: the midpoint raised by half the core gap along the cap normal
            xa = p[4:7] + (p[0] + 2 * CORE_M) / 2 * np.array([0, 0, 1.0])
            assert abs(xa[2] - (0.053 - CORE_M) - 2 * CORE_M - p[0]) < 2e-6
        assert pts[:, 0].max() - pts[:, 0].min() > 1e-3  # (the GJK point sits at the low end)
        # 10 degrees: outside RIM_DEG
        ha = world(link, _rot_axis([0, 1, 0], np.radians(10)) @ axis_x, np.array([-0.02, 0.0, 0.053 + 0.05 + 0.001]))
        assert len(pair_manifold(ha, hb, 0.004)) <= 1
        lib.zbo_set_pair_manifold_mode(2)
        ha = world(link, axis_x, np.array([-0.02, 0.0, 0.053 + 0.05 + 0.001]))
        assert len(pair_manifold(ha, hb, 0.004)) == 1
    finally:
        lib.zbo_set_pair_manifold_mode(2)


def test_ruling_on_face_falls_through_to_side_by_side():
    """with self_manifold 3 a pair whose ruling-on-face test keeps only its GJK point is still
    tested as a side-by-side pair, so mode 3 loses no side-by-side pair of mode 2 (each one is a
    side-by-side or a ruling-on-face pair in mode 3), on random folds (zbo_pair_classes)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fullstate import random_states, task_cfg
    from oracle.pyoracle import OracleSim
    n, res = 60_000, {}
    for sm in (2, 3):
        cfg = task_cfg("v2")
        cfg.self_manifold = sm
        o = OracleSim(n, cfg, seed=1)
        st = random_states("v2", o, n, seed=5)
        st[13:19] = np.random.default_rng(100).uniform(-np.pi, np.pi, (6, n)).astype(np.float32)
        o.set_state(st)
        res[sm] = o.pair_classes()
    a, b = res[2], res[3]
    rim2 = a[:, 2] > 0
    assert rim2.sum() >= 5
    assert np.all((b[rim2, 2] + b[rim2, 8]) >= a[rim2, 2])  # every mode-2 rim pair kept as rim or rim-on-face
    assert (b[:, 5] < a[:, 5]).sum() <= 1e-4 * n           # points removed only where rim-on-face wins
