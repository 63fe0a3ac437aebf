"""Physical invariants of the oracle integrator (its algorithm is the HIP kernel's; PhysX itself is
not available, so these pin the physics)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from helpers import S, perturbed_states
from zbot_lab_amd import model as zm


def _sim(n, cfg=None, model_edit=None, double=False):
    from oracle.pyoracle import OracleSim
    s = OracleSim(n, cfg or zm.TaskCfg(), double=double)
    if model_edit:
        model_edit(s._m)
        s.lib.zbo_destroy(s.h)
        s.h = s.lib.zbo_create(C.byref(s._m), C.byref(s._c), n, 0)
    return s


def _airborne(n, seed=0, **kw):
    st = perturbed_states(n, seed=seed, **kw)
    st[S["ROOT_POS"] + 2] += 2.0
    return st


def test_free_fall():
    n = 8
    s = _sim(n)
    st = _airborne(n, jqd_sigma=0.0, vel=0.0, tilt=0.0)
    s.set_state(st)
    tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy()
    k = 20
    s.physics_substeps(tg, k)
    out = s.get_state()
    dt, g = 0.005, 9.81
    np.testing.assert_allclose(out[S["ROOT_LINVEL"] + 2], -g * dt * k, rtol=1e-4)
    np.testing.assert_allclose(out[S["ROOT_POS"] + 2] - st[S["ROOT_POS"] + 2], -g * dt * dt * k * (k + 1) / 2, rtol=1e-4)
    np.testing.assert_allclose(out[S["JOINT_VEL"]:S["JOINT_VEL"] + 6], 0, atol=1e-4)


def test_momentum_first_order_without_gravity_and_contact():
    """Free-floating chain, drives active (internal forces only): spatial momentum is conserved up
    to the first-order error of semi-implicit Euler in generalised coordinates (M(q) changes
    within the step) - the drift must halve when dt halves and stay < 5 % of |p| over 0.1 s (strong drive transients)."""
    drift = []
    for dt in (0.005, 0.0025):
        n = 8
        # self collision off: the strong drive transients fold links into each other, and contact
        # is what the title excludes (impulses are internal, but not first order in dt)
        s = _sim(n, zm.TaskCfg(gravity=0.0, sim_dt=dt, enable_self_collision=False), double=True)
        st = _airborne(n, seed=3, jqd_sigma=2.0, vel=0.5)
        s.set_state(st)
        em0 = s.energy_momentum()
        tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy()
        s.physics_substeps(tg, int(round(0.1 / dt)))
        em1 = s.energy_momentum()
        drift.append((np.abs(em1[:, 1:4] - em0[:, 1:4]).max(), np.abs(em1[:, 4:7] - em0[:, 4:7]).max(),
                      np.abs(em0[:, 1:4]).max()))
    (p1, l1, pn), (p2, l2, _) = drift
    assert p1 < 0.05 * pn
    assert 1.6 < p1 / p2 < 2.4 and 1.6 < l1 / l2 < 2.4, drift


def test_energy_without_drives_gravity_contact():
    """No drives, gravity or contact (self collision off: it is inelastic, e = 0): kinetic energy
    drifts only at first order in dt (< 3 % over 0.5 s at dt = 5 ms, halving with dt)."""
    def no_drive(m):
        m.kp = 0.0
        m.kd = 0.0
    errs = []
    for dt in (0.005, 0.0025):
        n = 16
        s = _sim(n, zm.TaskCfg(gravity=0.0, sim_dt=dt, enable_self_collision=False), model_edit=no_drive,
                 double=True)
        st = _airborne(n, seed=5, jqd_sigma=1.0, vel=0.2)
        s.set_state(st)
        e0 = s.energy_momentum()[:, 0]
        s.physics_substeps(st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy(), int(round(0.5 / dt)))
        errs.append(np.abs(s.energy_momentum()[:, 0] / e0 - 1).max())
    assert errs[0] < 0.03 and 1.6 < errs[0] / errs[1] < 2.4, errs


def test_pd_step_response():
    n = 4
    s = _sim(n, zm.TaskCfg(gravity=0.0))
    st = _airborne(n, seed=7, jq_sigma=0.0, jqd_sigma=0.0, vel=0.0, tilt=0.0)
    s.set_state(st)
    tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy()
    tg[:, 2] += 0.2
    s.physics_substeps(tg, 200)   # 1 s
    out = s.get_state()
    q = out[S["JOINT_POS"] + 2]
    np.testing.assert_allclose(q, tg[:, 2], atol=0.01)
    assert np.abs(out[S["JOINT_VEL"]:S["JOINT_VEL"] + 6]).max() < 0.05


def test_standing_at_default_pose_is_stable():
    n = 8
    s = _sim(n)
    s.reset()
    st = s.get_state()
    st[S["EP_LEN"]] = 0
    s.set_state(st)
    for _ in range(250):  # 5 s of zero actions
        _, r, term, trunc = s.step(np.zeros((n, 6), np.float32))
        assert not term.any()
    p, _ = s.link_poses()
    np.testing.assert_allclose(p[:, 6, 2], 0.2545, atol=2e-3)
    out = s.get_state()
    assert np.abs(out[S["JOINT_VEL"]:S["JOINT_VEL"] + 6]).max() < 0.1
    # both feet carry the weight: contact-sensor F_z history sums to ~m g
    fz = out[S["FEET_FZ_HIST"]:S["FEET_FZ_HIST"] + 2]
    np.testing.assert_allclose(fz.sum(axis=0), 3.005 * 9.81, rtol=0.05)


def test_joint_wrap():
    def no_drive(m):
        m.kp = 0.0
        m.kd = 0.0
    n = 2
    s = _sim(n, zm.TaskCfg(gravity=0.0), model_edit=no_drive)
    st = _airborne(n, jq_sigma=0.0, jqd_sigma=0.0, vel=0.0)
    st[S["JOINT_POS"] + 3] = 6.27
    st[S["JOINT_VEL"] + 3] = 15.0
    s.set_state(st)
    tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy()
    tg[:, 3] = 6.27
    s.physics_substeps(tg, 1)
    q = s.get_state()[S["JOINT_POS"] + 3]
    assert (q < 0).all() and (q > -2 * np.pi).all()    # crossed +2pi -> wrapped by 4pi


def test_velocity_limit():
    n = 2
    s = _sim(n, zm.TaskCfg(gravity=0.0))
    st = _airborne(n, jq_sigma=0.0, jqd_sigma=0.0, vel=0.0)
    s.set_state(st)
    tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy()
    tg[:, 5] += 3.0   # saturating step on the distal joint
    s.physics_substeps(tg, 3)
    assert np.abs(s.get_state()[S["JOINT_VEL"]:S["JOINT_VEL"] + 6]).max() <= 20.0 + 1e-4


def test_random_rollout_sane():
    from oracle.pyoracle import OracleSim
    n = 64
    s = OracleSim(n, seed=3)
    s.reset()
    rng = np.random.default_rng(0)
    died = 0
    for _ in range(200):
        obs, r, te, tr = s.step(rng.normal(size=(n, 6)).astype(np.float32))
        assert np.isfinite(obs).all() and np.isfinite(r).all()
        died += te.sum()
    st = s.get_state()
    assert np.isfinite(st).all()
    assert 0 < died < n * 200 * 0.2


def test_static_friction_raised_to_dynamic():
    """Per-link friction draws with mu_dynamic > mu_static (stand-up / manager DR draw the two
    independently): the combined static coefficient is raised to the dynamic one (PhysX material
    combine), so such a world behaves exactly like one with mu_static = mu_dynamic."""
    from oracle.pyoracle import OracleSim
    n = 16
    rng = np.random.default_rng(7)
    mu_s = rng.uniform(0.3, 0.6, size=(n, zm.NUM_LINKS)).astype(np.float32)
    mu_d = rng.uniform(0.7, 1.0, size=(n, zm.NUM_LINKS)).astype(np.float32)
    runs = []
    for ms in (mu_s, mu_d):
        s = OracleSim(n, zm.TaskCfg.standup(), seed=3)
        s.reset()
        s.set_link_friction(ms, mu_d)
        a_rng = np.random.default_rng(1)
        for _ in range(40):
            s.step(a_rng.normal(size=(n, 6)).astype(np.float32))
        runs.append(s.get_state())
    np.testing.assert_array_equal(runs[0][:25], runs[1][:25])  # physics rows bit-identical
    # control: static coefficients raised above the dynamic ones change the motion
    s = OracleSim(n, zm.TaskCfg.standup(), seed=3)
    s.reset()
    s.set_link_friction(np.minimum(mu_d + 0.5, 2.0), mu_d)
    a_rng = np.random.default_rng(1)
    for _ in range(40):
        s.step(a_rng.normal(size=(n, 6)).astype(np.float32))
    assert not np.array_equal(s.get_state()[:25], runs[1][:25])


def _tgs_cfg(mode, **kw):
    return zm.TaskCfg(solver_mode=mode, **kw)


def test_tgs_refresh_standing_is_stable():
    """solver_mode 2 (TGS with the per-position-iteration refresh of the ground contacts,
    zbot_cfg.py:637-638): 5 s of zero actions from the default pose stay upright with both feet
    carrying the weight, as with the other solves."""
    n = 8
    s = _sim(n, _tgs_cfg(2))
    s.reset()
    st = s.get_state()
    st[S["EP_LEN"]] = 0
    s.set_state(st)
    for _ in range(250):
        _, r, term, trunc = s.step(np.zeros((n, 6), np.float32))
        assert not term.any()
    p, _ = s.link_poses()
    np.testing.assert_allclose(p[:, 6, 2], 0.2545, atol=2e-3)
    out = s.get_state()
    assert np.abs(out[S["JOINT_VEL"]:S["JOINT_VEL"] + 6]).max() < 0.1
    fz = out[S["FEET_FZ_HIST"]:S["FEET_FZ_HIST"] + 2]
    np.testing.assert_allclose(fz.sum(axis=0), 3.005 * 9.81, rtol=0.05)


def test_tgs_refresh_touches_ground_contacts_only():
    """The refresh re-evaluates ground contacts only: airborne envs (self contacts allowed) step
    bit-identically under modes 1 and 2, and so does every env with a single sub-iteration (no
    refresh point); envs resting on the ground differ, by less than the solve's own convergence
    scale."""
    n = 32
    st = _airborne(n, seed=11, jqd_sigma=3.0, vel=0.5)
    tg = st[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy() + 0.3
    outs = []
    for mode in (1, 2):
        s = _sim(n, _tgs_cfg(mode))
        s.set_state(st)
        s.physics_substeps(tg, 4)
        outs.append(s.get_state())
    np.testing.assert_array_equal(outs[0], outs[1])
    ground = perturbed_states(n, seed=12)
    outs = []
    for mode, iters in ((1, 1), (2, 1), (1, 4), (2, 4)):
        s = _sim(n, _tgs_cfg(mode, solver_iterations=iters))
        s.set_state(ground)
        s.physics_substeps(ground[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy(), 4)
        outs.append(s.get_state())
    np.testing.assert_array_equal(outs[0], outs[1])
    d = np.abs(outs[3] - outs[2])
    assert d.max() > 0  # the refresh acts on ground contacts
    v = S["JOINT_VEL"]
    assert d[v:v + 6].max() < 0.5, d[v:v + 6].max()


def test_tgs_self_refresh_touches_self_contacts_only():
    """solver_mode 3 adds the refresh of the self contacts (body-fixed anchors carried to each
    sub-iteration's pose): on ground-only states it steps bit-identically to mode 2, on constructed
    self-contact folds (airborne, tests/fullstate.constructed_states) it differs from mode 2; with a
    single sub-iteration (no refresh point) modes 2 and 3 agree there too."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from fullstate import constructed_states, self_manifold, task_cfg
    from oracle.pyoracle import OracleSim
    n = 32
    ground = perturbed_states(n, seed=12)
    outs = []
    for mode in (2, 3):  # (self collision off: the ground contacts alone)
        s = _sim(n, _tgs_cfg(mode, solver_iterations=4, enable_self_collision=False))
        s.set_state(ground)
        s.physics_substeps(ground[S["JOINT_POS"]:S["JOINT_POS"] + 6].T.copy(), 4)
        outs.append(s.get_state())
    np.testing.assert_array_equal(outs[0], outs[1])
    with self_manifold(2):
        st, _ = constructed_states("v2", "face", 64, seed=3)
    a = np.random.default_rng(608).normal(size=(64, 6)).astype(np.float32)
    res = {}
    for mode, iters in ((2, 1), (3, 1), (2, 4), (3, 4)):
        cfg = task_cfg("v2")
        cfg.self_manifold, cfg.solver_mode, cfg.solver_iterations = 2, mode, iters
        o = OracleSim(64, cfg, seed=1)
        o.set_state(st)
        o.contact_activity()
        o.step(a)
        res[mode, iters] = (o.get_state(), o.contact_activity()[:, 1] > 0)
    np.testing.assert_array_equal(res[2, 1][0], res[3, 1][0])
    diff = (res[3, 4][0] != res[2, 4][0]).any(axis=0)
    loaded = res[2, 4][1] | res[3, 4][1]
    assert loaded.sum() >= 10 and (diff & loaded).sum() >= 0.9 * loaded.sum()  # the refresh acts on the loaded ones
    assert np.isfinite(res[3, 4][0]).all()
