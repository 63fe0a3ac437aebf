"""Self-collision GJK on the GPU (gjk_quad, run by the 4 lanes of a DPP quad) against the oracle's
hull_pair (oracle/zbot_oracle.c), through the C ABI's test entry zb_gjk_pairs.

The robot's own link shapes at random relative poses around contact (separated, touching,
penetrating less than 2 CORE_M, and overlapping cores: the separating-axis estimate), cold
(hull centre difference) and warm (a given start direction, as the step kernels pass the pair's
contact normal of the previous substep). Contact flags must agree away from the margin; where
both report a contact the separation agrees to 2e-5 m (GJK_TOL 1e-5 plus fp32 rounding), the normal
to 2e-3 and the point to 1e-4 m. A pair may miss the normal / point bound (nearly flat closest
features, where fp32 rounding changes GJK's path and the normal is poorly determined although the
distance is not; at most 2 % of the contacts) only if the GPU's answer is itself a converged one
-- the separating gap of the two cores along the GPU's normal (float64, exact circle supports) is
within 2e-5 m of its distance and its point lies midway between the core surfaces along that
normal -- or the oracle's own answer spreads by half the GPU's deviation under 1e-6 relative
perturbations of the hulls and the start direction.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import pyoracle
from tests.test_oracle_selfcollision import CORE_M, _quat, _rot, core_circles, rim_points, sat_gap, world
from zbot_lab_amd import model as zm

pytestmark = pytest.mark.gpu
MARGIN = 0.004


def _pairs(n, seed):
    rm = zm.load_model()
    cores = [core_circles(np.asarray(rm.circles[l], np.float64)) for l in range(zm.NUM_LINKS)]
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 2, 2, 9), np.float32)
    for k in range(n):
        la, lb = rng.integers(0, zm.NUM_LINKS, size=2)
        ha = world(cores[la], _rot(_quat(rng)), np.zeros(3))
        # offsets from overlapping to ~2 cm apart along a random direction
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        hb = world(cores[lb], _rot(_quat(rng)), d * rng.uniform(0.05, 0.14))
        out[k, 0], out[k, 1] = ha, hb
    return out


def _oracle(pairs, v0=None):
    res = np.zeros((len(pairs), 9), np.float32)
    vp = None if v0 is None else np.ascontiguousarray(v0, np.float32)
    pyoracle.lib().zbo_gjk_pairs(np.ascontiguousarray(pairs, np.float32).ravel(), None if vp is None else vp.ctypes.data,
                                 len(pairs), MARGIN, res.ravel(), None)
    return res


def _gpu(pairs, v0=None):
    import torch
    from zbot_lab_amd import _native as nat
    P = torch.from_numpy(np.ascontiguousarray(pairs)).cuda()
    V = None if v0 is None else torch.from_numpy(np.ascontiguousarray(v0, np.float32)).cuda()
    out = torch.zeros(len(pairs), 9, device="cuda")
    nat.check(nat.lib().zb_gjk_pairs(nat.ptr(P), nat.ptr(V), len(pairs), MARGIN, nat.ptr(out), None), "zb_gjk_pairs")
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _spread(pairs, v0, k, o):
    """largest change of the oracle's normal and point of pair k under 1e-6 relative perturbations
    of its hulls and start direction"""
    rng = np.random.default_rng(k)
    dn = dx = 0.0
    for _ in range(6):
        p = pairs[k:k + 1] * (1 + 1e-6 * rng.standard_normal(pairs[k:k + 1].shape)).astype(np.float32)
        v = None if v0 is None else v0[k:k + 1] * (1 + 1e-6 * rng.standard_normal((1, 3))).astype(np.float32)
        r = _oracle(p.astype(np.float32), v)[0]
        if r[0] == 1:
            dn = max(dn, np.abs(r[2:5] - o[k, 2:5]).max())
            dx = max(dx, np.abs(r[5:8] - o[k, 5:8]).max())
    return dn, dx


def _converged(pair, r):
    """the GPU's contact of one pair is a converged GJK answer: the gap along its normal is within
    2e-5 m of its distance, and its point is midway between the core surfaces along the normal"""
    ha, hb = pair[0].astype(np.float64), pair[1].astype(np.float64)
    n = r[2:5].astype(np.float64)
    n /= np.linalg.norm(n)
    d = float(r[1]) + 2 * CORE_M
    if abs(sat_gap(ha, hb, n) - d) > 2e-5:
        return False
    xa, xb = r[5:8] + n * d / 2, r[5:8] - n * d / 2
    return (abs(min(rim_points(ha, 4096) @ n) - xa @ n) < 5e-5 and abs(max(rim_points(hb, 4096) @ n) - xb @ n) < 5e-5)


def _compare(g, o, pairs, v0=None):
    edge = np.abs(o[:, 1] - MARGIN) < 1e-4  # contact decided at the margin: either answer is right
    flag_ok = (g[:, 0] == o[:, 0]) | edge
    assert flag_ok.all(), np.where(~flag_ok)[0][:20]
    both = (g[:, 0] == 1) & (o[:, 0] == 1)
    deep = both & (o[:, 1] <= -2 * CORE_M + 1e-6)
    assert (np.abs(g[both, 1] - o[both, 1]) < 2e-5).all(), np.abs(g[both, 1] - o[both, 1]).max()
    en = np.abs(g[:, 2:5] - o[:, 2:5]).max(axis=1)
    ex = np.abs(g[:, 5:8] - o[:, 5:8]).max(axis=1)
    off = both & ((en >= 2e-3) | (ex >= 1e-4))
    unexplained = []
    for k in np.nonzero(off)[0]:
        if not deep[k] and _converged(pairs[k], g[k]):
            continue
        dn, dx = _spread(pairs, v0, k, o)
        if not ((en[k] < 2e-3 or dn >= 0.5 * en[k]) and (ex[k] < 1e-4 or dx >= 0.5 * ex[k])):
            unexplained.append((int(k), float(en[k]), dn, float(ex[k]), dx))
    assert not unexplained, unexplained[:10]
    assert off.sum() <= 0.02 * both.sum(), (off.sum(), both.sum())
    return both.sum(), deep.sum()


def test_gjk_quad_matches_oracle_cold():
    pairs = _pairs(4000, seed=11)
    o = _oracle(pairs)
    g = _gpu(pairs)
    nb, nd = _compare(g, o, pairs)
    assert nb - nd > 200 and nd > 20, (nb, nd)  # exact contacts and overlapping cores both exercised
    # iteration counts agree except where a stopping test sits at its threshold
    assert (g[:, 8] == o[:, 8]).mean() > 0.95


def test_gjk_quad_matches_oracle_warm():
    pairs = _pairs(2000, seed=12)
    o0 = _oracle(pairs)
    rng = np.random.default_rng(1)
    # the previous substep's normal: the converged one, turned by a few degrees
    v0 = o0[:, 2:5] + rng.normal(size=(len(pairs), 3)).astype(np.float32) * 0.05
    v0[o0[:, 0] == 0] = rng.normal(size=((o0[:, 0] == 0).sum(), 3))
    o = _oracle(pairs, v0)
    g = _gpu(pairs, v0)
    _compare(g, o, pairs, v0)


def _face_pairs(n, seed):
    """Face-to-face link pairs: two flat stacks (parallel circles) with the upper one tilted up to 12
    degrees, offset in the plane up to 6 cm and gapped -3 .. +4 mm (lens, containment and apart)."""
    from tests.test_oracle_selfcollision import _flat_link
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 2, 2, 9), np.float32)
    for k in range(n):
        tilt = rng.uniform(0, np.radians(12))
        ax = rng.normal(size=3)
        ax[2] = 0
        ax /= np.linalg.norm(ax)
        q = np.concatenate([[np.cos(tilt / 2)], np.sin(tilt / 2) * ax])
        ra, rb = rng.choice([0.05, 0.04]), rng.choice([0.05, 0.04])
        off = rng.uniform(-0.06, 0.06, 2)
        out[k, 0] = world(_flat_link(ra), _rot(q), np.array([off[0], off[1], 0.053 + rng.uniform(-0.003, 0.004)]))
        out[k, 1] = world(_flat_link(rb), np.eye(3), np.zeros(3))
    return out


def _rot_axis(axis, ang):
    axis = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def _rim_pairs(n, seed):
    """Two flat links lying side by side (axes along x, one above the other), A tilted by up to 8
    degrees about a random axis, shifted along the axis by up to 3 cm, gap -3 .. 4 mm, the whole
    configuration rotated at random: rulings within and beyond the 5-degree rim threshold."""
    from tests.test_oracle_selfcollision import _flat_link
    rng = np.random.default_rng(seed)
    lie = _rot_axis([0, 1, 0], np.pi / 2)
    out = np.zeros((n, 2, 2, 9), np.float32)
    for k in range(n):
        ra, rb = rng.uniform(0.035, 0.05, 2)
        tilt = _rot_axis(rng.normal(size=3), np.radians(rng.uniform(0, 8)))
        G = _rot(_quat(rng))
        pa = np.array([rng.uniform(-0.03, 0.03), 0.0, ra + rb + rng.uniform(-0.003, 0.004)])
        ha = world(_flat_link(ra), G @ tilt @ lie, G @ pa)
        hb = world(_flat_link(rb), G @ lie, np.zeros(3))
        out[k, 0], out[k, 1] = ha, hb
    return out


def _compare_manifolds(pairs, label, ntol_multi, gjk_first=False, mode=2):
    """zb_pair_manifold_mode vs zbo_pair_manifold (self_manifold ``mode``): counts and (for agreeing
    counts) points."""
    import ctypes as C
    import torch
    from zbot_lab_amd import _native as nat
    n = len(pairs)
    ref = np.zeros((n, 29), np.float32)
    lib = pyoracle.lib()
    lib.zbo_set_pair_manifold_mode.argtypes = [C.c_int]
    lib.zbo_set_pair_manifold_mode(mode)
    try:
        for k in range(n):
            pts = np.zeros(28, np.float32)
            c = lib.zbo_pair_manifold(np.ascontiguousarray(pairs[k, 0]).ravel(), np.ascontiguousarray(pairs[k, 1]).ravel(),
                                      MARGIN, pts)
            ref[k, 0] = c
            ref[k, 1:] = pts
    finally:
        lib.zbo_set_pair_manifold_mode(2)
    P = torch.from_numpy(np.ascontiguousarray(pairs)).cuda()
    out = torch.zeros(n, 29, device="cuda")
    nat.check(nat.lib().zb_pair_manifold_mode(nat.ptr(P), n, MARGIN, mode, nat.ptr(out), None), "zb_pair_manifold_mode")
    got = out.cpu().numpy()
    same = got[:, 0] == ref[:, 0]
    print(f"\n{label} pairs {n}: oracle counts {np.bincount(ref[:, 0].astype(int), minlength=5).tolist()}, "
          f"GPU counts {np.bincount(got[:, 0].astype(int), minlength=5).tolist()}, count agreement {same.mean():.4f}")
    bad = []
    for k in np.nonzero(same & (ref[:, 0] > 0))[0]:
        c = int(ref[k, 0])
        g, r = got[k, 1:1 + 7 * c].reshape(c, 7), ref[k, 1:1 + 7 * c].reshape(c, 7)
        # (rim manifolds: the first point is the GJK point with GJK's own normal)
        ntol = np.full(c, 2e-3 if c == 1 else ntol_multi)
        if gjk_first:
            ntol[0] = 2e-3
        if not (np.abs(g[:, 0] - r[:, 0]).max() <= 2e-5 and (np.abs(g[:, 1:4] - r[:, 1:4]).max(axis=1) <= ntol).all()
                and np.abs(g[:, 4:7] - r[:, 4:7]).max() <= 1e-4):
            bad.append((int(k), c, float(np.abs(g - r).max())))
    print(f"pairs outside the point bounds: {len(bad)} {bad[:8]}")
    return ref, got, same, bad


def test_gpu_rim_manifold_matches_oracle():
    """The rim manifold (self_manifold 2: side-by-side rulings, the GJK point + the overlap's ends)
    of quad_manifold (zb_pair_manifold) against the oracle's rim_manifold on 4000 side-by-side pairs:
    the same number of points in the same order for >= 99 % (a ruling within fp32 rounding of the
    5-degree thresholds or an end within rounding of the 1 mm rule may go either way), separations
    to 2e-5 m, normals to 5e-4, points to 1e-4 m."""
    ref, got, same, bad = _compare_manifolds(_rim_pairs(4000, 31), "rim manifold", 5e-4, gjk_first=True)
    assert (ref[:, 0] >= 2).sum() >= 1000 and (ref[:, 0] == 3).sum() >= 40  # (parallel rulings: GJK ends at one end)
    assert same.mean() >= 0.99
    assert len(bad) <= 0.01 * same.sum(), bad[:20]


def _rimface_pairs(n, seed):
    """A link lying on its side over an upright link's cap: the lying link tilted by up to 8 degrees
    about a random axis, shifted over the cap by up to 4 cm, gap -3 .. 4 mm, the whole configuration
    rotated at random: rulings within and beyond the 5-degree threshold, stretches inside and across
    the cap's rim, and the GJK point at either end."""
    from tests.test_oracle_selfcollision import _flat_link
    rng = np.random.default_rng(seed)
    lie = _rot_axis([0, 1, 0], np.pi / 2)
    out = np.zeros((n, 2, 2, 9), np.float32)
    for k in range(n):
        ra, rb = rng.uniform(0.035, 0.05, 2)
        tilt = _rot_axis(rng.normal(size=3), np.radians(rng.uniform(0, 8)))
        G = _rot(_quat(rng))
        pa = np.array([rng.uniform(-0.04, 0.02), rng.uniform(-0.02, 0.02), 0.053 + ra + rng.uniform(-0.003, 0.004)])
        ha = world(_flat_link(ra), G @ tilt @ lie, G @ pa)
        hb = world(_flat_link(rb), G, np.zeros(3))
        out[k, 0], out[k, 1] = (ha, hb) if k % 2 == 0 else (hb, ha)   # the face on B, then on A
    return out


def test_gpu_ruling_on_face_manifold_matches_oracle():
    """The ruling-on-face manifold (self_manifold 3, round 5: the GJK point + the ends of the lying
    link's ruling over the cap's disk) of quad_manifold (zb_pair_manifold_mode) against the oracle's
    rim_face_manifold on 4000 pairs, the face on either hull: the same number of points in the same
    order for >= 99 %, separations to 2e-5 m, the ends' normals (the cap's exact normal) to 5e-4,
    points to 1e-4 m."""
    ref, got, same, bad = _compare_manifolds(_rimface_pairs(4000, 41), "ruling-on-face manifold", 5e-4,
                                             gjk_first=True, mode=3)
    assert (ref[:, 0] >= 2).sum() >= 1000 and (ref[:, 0] == 3).sum() >= 100, np.bincount(ref[:, 0].astype(int))
    assert same.mean() >= 0.99
    assert len(bad) <= 0.01 * same.sum(), bad[:20]


def test_gpu_face_manifold_matches_oracle():
    """quad_manifold (zb_pair_manifold) against the oracle's face_manifold (zbo_pair_manifold) on
    face-to-face pairs and on random robot link pairs: the same number of points in the same order,
    separations to 2e-5 m, points to 1e-4 m, away from the decision edges (a sample within 1e-5 m of
    the margin or of the other disk's rim, or a face within 1e-4 of the 15-degree threshold, may go
    either way in fp32)."""
    import torch
    from zbot_lab_amd import _native as nat
    pairs = np.concatenate([_face_pairs(3000, 21), _pairs(1000, 22)])
    n = len(pairs)
    ref = np.zeros((n, 29), np.float32)
    for k in range(n):
        pts = np.zeros(28, np.float32)
        c = pyoracle.lib().zbo_pair_manifold(np.ascontiguousarray(pairs[k, 0]).ravel(), np.ascontiguousarray(pairs[k, 1]).ravel(),
                                             MARGIN, pts)
        ref[k, 0] = c
        ref[k, 1:] = pts
    P = torch.from_numpy(np.ascontiguousarray(pairs)).cuda()
    out = torch.zeros(n, 29, device="cuda")
    nat.check(nat.lib().zb_pair_manifold(nat.ptr(P), n, MARGIN, nat.ptr(out), None), "zb_pair_manifold")
    got = out.cpu().numpy()
    same = got[:, 0] == ref[:, 0]
    multi = ref[:, 0] >= 2
    print(f"\nmanifold pairs {n}: oracle counts {np.bincount(ref[:, 0].astype(int), minlength=5).tolist()}, "
          f"GPU counts {np.bincount(got[:, 0].astype(int), minlength=5).tolist()}, count agreement {same.mean():.4f}")
    assert multi.sum() >= 500 and (ref[:, 0] == 4).sum() >= 100
    assert same.mean() >= 0.99
    bad = []
    for k in np.nonzero(same & (ref[:, 0] > 0))[0]:
        c = int(ref[k, 0])
        g, r = got[k, 1:1 + 7 * c].reshape(c, 7), ref[k, 1:1 + 7 * c].reshape(c, 7)
        # one-point pairs carry GJK's normal (poorly determined for nearly flat closest features,
        # tests above); face manifolds A's exact face normal
        ntol = 2e-3 if c == 1 else 2e-5
        if not (np.abs(g[:, 0] - r[:, 0]).max() <= 2e-5 and np.abs(g[:, 1:4] - r[:, 1:4]).max() <= ntol
                and np.abs(g[:, 4:7] - r[:, 4:7]).max() <= 1e-4):
            bad.append((int(k), c, float(np.abs(g - r).max())))
    print(f"pairs outside the point bounds: {len(bad)} {bad[:8]}")
    assert len(bad) <= 0.01 * same.sum(), bad[:20]
