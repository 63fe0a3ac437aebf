"""Full-state MDP parity of the HIP kernels (libzbot.so, through the C ABI) vs the CPU oracle, all
four tasks: every persistent state row — physics, p_delta / actions, sensor histories and timers,
feet latches / step lengths / last forces, integrators, commands / timers, counters and every
per-term episode sum — randomised to valid values, then compared row by row after the step, with
obs, reward and both flags (reference: v2.py:371-459,509-543; v4.py:880-1095; standup.py:571-703;
zbotlab_manager mdp/*).

Each env outside tolerance must be explained: the GPU's deviation must lie within twice the envelope
of perturbed oracle runs at that env (rounding-scale perturbations of its physics state before each
step, GJK's stopping tolerance, the sensor force at its tolerance; it sits at a contact-margin /
sensor-threshold / drive-clamp discontinuity, tests/fullstate.py). Unexplained envs fail and are
printed with their worst rows; the outlier count is reported and bounded, and over the
contact-active envs the outlier fraction and median err/tol are bounded by the f64 oracle's own
(the rounding-noise baseline).
"""
from __future__ import annotations

import numpy as np
import pytest

from fullstate import TOL, TASKS, compare, perturb_physics, random_states, row_groups, solver_mode, task_cfg

pytestmark = pytest.mark.gpu
K_SENS = 8


def _sims(task, n, seed):
    import torch
    from oracle.pyoracle import OracleSim
    from zbot_lab_amd.sim import ZbotSim
    cfg = task_cfg(task)
    return ZbotSim(n, cfg, device="cuda:0", seed=seed), OracleSim(n, cfg, seed=seed), cfg, torch


def _run_oracle(task, n, seed, st, actions, rng=None, scale=1.0, wc=None, double=False, activity=False):
    """The oracle from state ``st``; with ``rng`` the physics rows are perturbed at ~1e-6 (x scale)
    before every step (rounding-level noise injected along the whole trajectory, as the GPU's own
    rounding differences are). ``double``: the f64 build (the rounding-noise baseline, or the
    stand-in device of tests/test_fullstate_machinery.py). ``activity``: also return the per-env
    loaded ground / self contact counts over the run."""
    from oracle.pyoracle import OracleSim
    o = OracleSim(n, task_cfg(task), seed=seed, double=double)
    # multi-step runs: the GPU's fast-math rounding (v_rcp / v_rsq, reassociated sums) differs from
    # the oracle's by more than 1e-6 per step once it passes through 80 substeps of contact solves
    rel, ab = (1e-6 * scale, 1e-7 * scale) if len(actions) == 1 else (1e-5, 1e-6)
    o.set_state(st if rng is None else perturb_physics(st, rng, rel, ab))
    if wc is not None:  # walking v2: the solver's self-contact cache the GPU started from
        o.set_contact_cache(wc)
    o.contact_activity(clear=True)
    out = []
    for k, a in enumerate(actions):
        if rng is not None and k > 0:  # (the solver's contact cache survives the perturbation)
            wc = o.get_contact_cache()
            o.set_state(perturb_physics(o.get_state(), rng, rel, ab))
            o.set_contact_cache(wc)
        out.append(o.step(a))
    if activity:
        return o.get_state(), out, o.contact_activity()
    return o.get_state(), out


# the perturbed-oracle runs, by family (the explained-outlier envelope, tests/fullstate.py)
SENS_FAMILIES = ("1e-6", "1e-5", "1e-4", "gjk_tol", "face_cos", "sensor_force")


def _sensitivity(task, n, seed, st, actions, so, obs_o, rew_o, fl_o, before, nsteps, wc=None):
    """Per family of perturbed oracle runs, the max over its runs of each env's error ratio vs the
    unperturbed oracle (dict family -> [n]):
    * "1e-6" / "1e-5" / "1e-4": physics rows x (1 +- scale) before every step (multi-step runs
      perturb at 1e-5 in all three families). 1e-6 is the GPU / oracle rounding scale; 1e-5 the
      size of their difference after a step without contact (~4e-5 m/s after 4
      substeps); 1e-4 stands for the GPU injecting its rounding differences in every substep and
      solver sweep, which a perturbation of the initial state alone must exceed to spread as far
      through a violent impact. Envs explained only at 1e-4 are counted and reported separately.
    * "gjk_tol": GJK's stopping tolerance scaled by 1/4, 1/2, 2 and 4 (where GJK stops is a
      discontinuity of the self-contact normal, as the margin is of contact activation; the fp32
      kernel and oracle can stop one iteration apart).
    * "face_cos": the self-contact manifold's face-alignment threshold (15 degrees) moved by -+ 0.5
      degree: where a pair switches between one point and a face manifold is a discontinuity of the
      contact set (oracle zbo_set_face_cos).
    * "sensor_force": the sensors see the contact forces scaled by 1 -+ 7 % (the force comparison
      tolerance, 0.05 N + 2 %, at the 1 N is_contact threshold): an env whose air / contact timers,
      touchdown latch, undesired-contact death or force-flagged reward terms flip there sits at a
      sensor threshold the two sides' forces straddle within tolerance. Those runs count the
      non-force rows only (the scaled forces themselves differ by design)."""
    from oracle.pyoracle import lib
    rng = np.random.default_rng(1234)
    fam = {f: np.zeros(n) for f in SENS_FAMILIES}
    scales = [(1.0, "1e-6")] * (K_SENS // 2) + [(10.0, "1e-5")] * (K_SENS // 4) \
        + [(100.0, "1e-4")] * (K_SENS - K_SENS // 2 - K_SENS // 4)
    runs = [(rng, None, None, sc, f, None) for sc, f in scales]
    runs += [(None, t, None, 1.0, "gjk_tol", None) for t in (0.25e-5, 0.5e-5, 2e-5, 4e-5)]
    runs += [(None, None, None, 1.0, "face_cos", c) for c in (np.cos(np.radians(14.5)), np.cos(np.radians(15.5)))]
    runs += [(None, None, s, 1.0, "sensor_force", None) for s in (0.93, 1.07)]
    force_rows = row_groups(task)["force"] + row_groups(task).get("fsum", [])
    for r_, tol, fs, scale, f, fc in runs:
        if tol is not None:
            lib().zbo_set_gjk_tol(tol)
        if fs is not None:
            lib().zbo_set_sensor_force_scale(fs)
        if fc is not None:
            lib().zbo_set_face_cos(float(fc))
        try:
            sk, outs = _run_oracle(task, n, seed, st, actions, r_, scale, wc)
        finally:
            if tol is not None:
                lib().zbo_set_gjk_tol(0.0)
            if fs is not None:
                lib().zbo_set_sensor_force_scale(1.0)
            if fc is not None:
                lib().zbo_set_face_cos(0.0)
        ob, rw, te, tr = outs[-1]
        r, rows, *_ = compare(task, sk, so, ob, obs_o, rw, rew_o, (te, tr), fl_o, before, nsteps)
        if fs is not None:
            rows = rows.copy()
            rows[force_rows] = 0.0
            r = np.maximum(rows.max(axis=0), np.abs(rw - rew_o) / (2e-3 + 2e-3 * np.abs(rew_o)))
            r[(te != fl_o[0]) | (tr != fl_o[1])] = np.inf
        fam[f] = np.maximum(fam[f], r)
    return fam


def _refine(task, n, seed, st, actions, so, obs_o, rew_o, fl_o, before, nsteps, wc=None, k=32, rseed=4321,
            record=None):
    """A second, larger draw of the rounding-scale families (k runs: 3/4 at 1e-6, 1/4 at 1e-5, a new
    random stream) for a check that still has unexplained envs after the first K_SENS draws: the
    envelope is a maximum over random perturbations, and a discrete event (a contact switching on,
    a sensor threshold) is reached by some perturbation directions only. ``record`` (env indices):
    also return the range of every state row / obs / reward over the draws (the unperturbed oracle
    included) and the set of flag pairs the draws produced, per recorded env (``_members``)."""
    rng = np.random.default_rng(rseed)
    fam = {"1e-6": np.zeros(n), "1e-5": np.zeros(n)}
    rec = None
    if record is not None:
        ids = np.asarray(record, int)
        s0, o0, r0 = so[:, ids].astype(np.float64), obs_o[ids].astype(np.float64), rew_o[ids].astype(np.float64)
        rec = dict(ids=ids, st_lo=s0.copy(), st_hi=s0.copy(), obs_lo=o0.copy(), obs_hi=o0.copy(), rew_lo=r0.copy(),
                   rew_hi=r0.copy(), flags=[{(bool(fl_o[0][e]), bool(fl_o[1][e]))} for e in ids])
    for j in range(k):
        scale, f = (1.0, "1e-6") if j < 3 * k // 4 else (10.0, "1e-5")
        sk, outs = _run_oracle(task, n, seed, st, actions, rng, scale, wc)
        ob, rw, te, tr = outs[-1]
        r = compare(task, sk, so, ob, obs_o, rw, rew_o, (te, tr), fl_o, before, nsteps)[0]
        fam[f] = np.maximum(fam[f], r)
        if rec is not None:
            ids = rec["ids"]
            rec["st_lo"] = np.minimum(rec["st_lo"], sk[:, ids])
            rec["st_hi"] = np.maximum(rec["st_hi"], sk[:, ids])
            rec["obs_lo"] = np.minimum(rec["obs_lo"], ob[ids])
            rec["obs_hi"] = np.maximum(rec["obs_hi"], ob[ids])
            rec["rew_lo"] = np.minimum(rec["rew_lo"], rw[ids])
            rec["rew_hi"] = np.maximum(rec["rew_hi"], rw[ids])
            for j_, e in enumerate(ids):
                rec["flags"][j_].add((bool(te[e]), bool(tr[e])))
    return (fam, rec) if record is not None else fam


def _members(rec, sg, obs_g, rew_g, fl_g, tol, ratio_rows, obs_o, rew_o):
    """The deep-draw rule (membership): for each recorded env, every state row, obs entry and the
    reward outside tolerance must lie inside the range the oracle's draws produced for that value,
    widened by that value's tolerance, and the GPU's flag pair must be one the draws produced. A
    value the oracle never reaches under rounding-scale perturbations is a mismatch however chaotic
    the env is elsewhere. Returns [(env, ok, the first failing values)]."""
    a, r = TOL["obs"]
    out = []
    for j, e in enumerate(rec["ids"]):
        why = []
        for k in np.nonzero(ratio_rows[:, e] > 1)[0]:
            lo, hi = rec["st_lo"][k, j] - tol[k, e], rec["st_hi"][k, j] + tol[k, e]
            if not lo <= sg[k, e] <= hi:
                why.append(f"row {k} {sg[k, e]:.6g} not in [{lo:.6g}, {hi:.6g}]")
        to = a + r * np.abs(obs_o[e])
        for c in np.nonzero(np.abs(obs_g[e] - obs_o[e]) > to)[0]:
            lo, hi = rec["obs_lo"][j, c] - to[c], rec["obs_hi"][j, c] + to[c]
            if not lo <= obs_g[e, c] <= hi:
                why.append(f"obs {c} {obs_g[e, c]:.6g} not in [{lo:.6g}, {hi:.6g}]")
        tr_ = 2e-3 + 2e-3 * abs(rew_o[e])
        if abs(rew_g[e] - rew_o[e]) > tr_ and not rec["rew_lo"][j] - tr_ <= rew_g[e] <= rec["rew_hi"][j] + tr_:
            why.append(f"reward {rew_g[e]:.6g} not in [{rec['rew_lo'][j] - tr_:.6g}, {rec['rew_hi'][j] + tr_:.6g}]")
        if (bool(fl_g[0][e]), bool(fl_g[1][e])) not in rec["flags"][j]:
            why.append(f"flags {(bool(fl_g[0][e]), bool(fl_g[1][e]))} not in {sorted(rec['flags'][j])}")
        out.append((int(e), not why, why[:3]))
    return out


def _explained(ratio, sens):
    """The parity rule: an env outside tolerance is explained only when the GPU's deviation lies
    within twice the envelope of the perturbed-oracle runs (its error ratio <= 2 x the largest
    ratio those runs reach at that env). No other pass: an env the perturbations move past the
    tolerance is still unexplained if the GPU moves it further."""
    return ratio <= 2 * sens


def _report(task, label, ratio, ratio_rows, err, tol, flags_bad, fam, names):
    sens = np.max(np.stack([fam[f] for f in SENS_FAMILIES]), axis=0)
    bad = np.nonzero(ratio > 1)[0]
    good = ratio <= 1
    groups = row_groups(task)
    expl = _explained(ratio[bad], sens[bad])
    at6 = _explained(ratio[bad], fam["1e-6"][bad])
    no4 = np.max(np.stack([fam[f][bad] for f in SENS_FAMILIES if f != "1e-4"]), axis=0)
    only4 = expl & ~_explained(ratio[bad], no4)
    print(f"\n[{task} {label}] envs {len(ratio)}, outside tolerance {len(bad)} "
          f"({len(bad) / len(ratio):.2%}), explained {int(expl.sum())} (by the 1e-6 runs alone "
          f"{int(at6.sum())}, only with the 1e-4 runs {int(only4.sum())}), unexplained {int((~expl).sum())}")
    for cls, rows in groups.items():
        if rows:
            w = ratio_rows[rows][:, good].max() if good.any() else 0.0
            print(f"  {cls:9s} worst err/tol over in-tolerance envs {w:.3f}")
    # unexplained envs first, then the rest
    order = sorted(range(len(bad)), key=lambda i: (bool(expl[i]), int(bad[i])))
    for i in order[:16]:
        e = bad[i]
        worst = np.argsort(-ratio_rows[:, e])[:4]
        rows = ", ".join(f"{names.get(int(k), k)}: {err[k, e]:.3g}/{tol[k, e]:.2g}" for k in worst)
        fs = " ".join(f"{f}={fam[f][e]:.3g}" for f in SENS_FAMILIES)
        print(f"  env {e}: ratio {ratio[e]:.3g} flags_differ {bool(flags_bad[e])} envelope [{fs}] | {rows}")
    return bad


def _row_names(task):
    names = {}
    for cls, rows in row_groups(task).items():
        for j, k in enumerate(rows):
            names[k] = f"{cls}[{j}]"
    return names


# Aggregate bound over the contact-active envs (an env with a loaded contact in any substep of the
# run), against the f64 oracle as the near-exact result: the device's outlier fraction and median
# err/tol measured from the f64 result must stay within the f32 oracle's own (two f32
# implementations of one algorithm, each against the f64 one):
# frac <= AGG_FRAC_K x baseline + AGG_FRAC_ABS and median <= AGG_MED_K x baseline + AGG_MED_ABS.
AGG_FRAC_K, AGG_FRAC_ABS = 2.0, 0.005
# multi-step checks (20 steps of standing contact): the contact solve's per-substep rounding excess
# over the f32 oracle (1.35-1.67x, tools/error_budget.py) compounds, and the outlier fraction then
# moves with code generation alone: PGS v2 1.76-2.73 %, v4 1.66-2.25 % over six builds of one source
# (f32 oracle 1.07 / 0.68 %). 3x keeps >= 11 % headroom on every build measured;
# the one-step checks, where the device's factor is 0.7-1.3x, stay at 2x.
AGG_FRAC_K_MULTI = 3.0
# at most this many envs still unexplained after the 32-run refinement get a deep draw of
# REFINE_DEEP_RUNS rounding-scale runs (a quarter of that for multi-step checks); more fail at once
REFINE_DEEP_MAX, REFINE_DEEP_RUNS = 4, 1024
AGG_MED_K, AGG_MED_ABS = 4.0, 0.02


def _record_stats(task, label, n, **kw):
    """ZB_PARITY_STATS=<file>: append one JSON line per check (the library under test, the check, its
    aggregate numbers) -- the build-flag A/B of DESIGN.md §6 reads them (scripts/parity_ab.py)."""
    import json
    import os
    path = os.environ.get("ZB_PARITY_STATS")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"lib": os.environ.get("ZBOT_LIB", "libzbot.so"), "task": task, "check": label,
                                "envs": n, **kw}) + "\n")


def _aggregate(ratio, active):
    r = ratio[active]
    return (float((r > 1).mean()) if len(r) else 0.0), (float(np.median(np.minimum(r, 1e6))) if len(r) else 0.0)


def _check(task, label, n, seed, st, actions, g_out, sg, torch, wc=None, stats=None):
    """Every env within tolerance or explained (``_explained``), and the contact-active aggregate
    within the f64 baseline. Returns the number of envs outside tolerance; ``stats`` (a dict)
    receives the aggregate numbers."""
    so, outs, act = _run_oracle(task, n, seed, st, actions, wc=wc, activity=True)
    ob_o, rw_o, te_o, tr_o = outs[-1]
    ob_g, rw_g, te_g, tr_g = g_out
    nsteps = len(actions)
    ratio, ratio_rows, err, tol, flags_bad = compare(task, sg, so, ob_g, ob_o, rw_g, rw_o, (te_g, tr_g), (te_o, tr_o), st,
                                                     nsteps)
    bad = np.nonzero(ratio > 1)[0]
    fam = {f: np.zeros(n) for f in SENS_FAMILIES}
    if len(bad):
        fam = _sensitivity(task, n, seed, st, actions, so, ob_o, rw_o, (te_o, tr_o), st, nsteps, wc)
    _report(task, label, ratio, ratio_rows, err, tol, flags_bad, fam, _row_names(task))
    sens = np.max(np.stack([fam[f] for f in SENS_FAMILIES]), axis=0)
    # the aggregate: the device and the f32 oracle, each against the f64 oracle (near-exact)
    sd, outs_d = _run_oracle(task, n, seed, st, actions, wc=wc, double=True)
    ob_d, rw_d, te_d, tr_d = outs_d[-1]
    ref_d = (ob_d, rw_d, (te_d, tr_d))
    ratio_gd, rows_gd = compare(task, sg, sd, ob_g, ob_d, rw_g, rw_d, (te_g, tr_g), ref_d[2], st, nsteps)[:2]
    ratio_od, rows_od = compare(task, so, sd, ob_o, ob_d, rw_o, rw_d, (te_o, tr_o), ref_d[2], st, nsteps)[:2]
    ratio_do = compare(task, sd, so, ob_d, ob_o, rw_d, rw_o, ref_d[2], (te_o, tr_o), st, nsteps)[0]
    active = act.sum(axis=1) > 0
    frac, med = _aggregate(ratio_gd, active)
    frac_o, med_o = _aggregate(ratio_od, active)
    frac_g, med_g = _aggregate(ratio, active)
    frac_x, med_x = _aggregate(ratio_do, active)
    print(f"  contact-active envs {int(active.sum())} of {n}, against the f64 oracle: device outliers {frac:.2%} "
          f"median err/tol {med:.3g}; f32 oracle {frac_o:.2%} / {med_o:.3g}  (device vs f32 oracle "
          f"{frac_g:.2%} / {med_g:.3g}; f64 vs f32 oracle {frac_x:.2%} / {med_x:.3g})")
    # which quantities carry the device's error against f64: per row class, the median over the
    # contact-active envs of the class's worst err/tol, device and f32 oracle
    groups = {}
    for cls, rows in row_groups(task).items():
        if rows and active.any():
            g_ = float(np.median(np.minimum(rows_gd[rows][:, active].max(axis=0), 1e6)))
            o_ = float(np.median(np.minimum(rows_od[rows][:, active].max(axis=0), 1e6)))
            groups[cls] = (g_, o_)
    print("  by class, median worst err/tol vs f64 (device / f32 oracle): "
          + ", ".join(f"{c} {g_:.3g} / {o_:.3g}" for c, (g_, o_) in groups.items()))
    # the f32 oracle's own outlier count against f64 on the same states: the rounding-noise baseline of
    # the per-check outlier caps (test_full_state_tgs)
    nbad_f32 = int((ratio_do > 1).sum())
    if stats is not None:
        stats.update(frac=frac, med=med, frac_f32=frac_o, med_f32=med_o, active=int(active.sum()), nbad=len(bad),
                     nbad_f32=nbad_f32)
    _record_stats(task, label, n, frac=frac, med=med, frac_f32=frac_o, med_f32=med_o, frac_vs_f32=frac_g,
                  med_vs_f32=med_g, active=int(active.sum()), nbad=len(bad), groups=groups)
    unexplained = [int(e) for e in bad if not _explained(ratio[e], sens[e])]
    ndeep = 0
    if unexplained:
        fam2 = _refine(task, n, seed, st, actions, so, ob_o, rw_o, (te_o, tr_o), st, nsteps, wc)
        for f, v in fam2.items():
            fam[f] = np.maximum(fam[f], v)
        sens = np.max(np.stack([fam[f] for f in SENS_FAMILIES]), axis=0)
        still = [e for e in unexplained if not _explained(ratio[e], sens[e])]
        print(f"  refined envelope (32 more rounding-scale runs) for {len(unexplained)} unexplained envs: "
              + ", ".join(f"env {e} ratio {ratio[e]:.3g} envelope {sens[e]:.3g}" for e in unexplained[:8])
              + f"; still unexplained {len(still)}")
        if 0 < len(still) <= REFINE_DEEP_MAX:
            # a rare discrete event: the oracle's own output can jump by tens of newtons at the
            # rounding scale in ~0.1-1 % of draws (env 6192 of the 65 536-env check), which
            # 8 + 32 draws miss. Draw it properly for the few envs still left, and explain an env only
            # by membership: each of its out-of-tolerance values inside the range the draws reach
            k = REFINE_DEEP_RUNS if nsteps == 1 else REFINE_DEEP_RUNS // 4
            _, rec = _refine(task, n, seed, st, actions, so, ob_o, rw_o, (te_o, tr_o), st, nsteps, wc, k=k,
                             rseed=8642, record=still)
            mem = _members(rec, sg, ob_g, rw_g, (te_g, tr_g), tol, ratio_rows, ob_o, rw_o)
            print(f"  deep draw ({k} more rounding-scale runs, membership rule) for {len(still)} envs: "
                  + "; ".join(f"env {e} ratio {ratio[e]:.3g} " + ("member" if ok else "NOT member: " + ", ".join(w))
                              for e, ok, w in mem))
            still = [e for e, ok, _ in mem if not ok]
            ndeep = len(mem)
        unexplained = still
    print(f"  sent to the deep draw: {ndeep} envs")
    if stats is not None:
        stats["deep_draw"] = ndeep
    assert not unexplained, f"{task}: {len(unexplained)} envs outside tolerance where the oracle is stable: {unexplained[:20]}"
    k_frac = AGG_FRAC_K if nsteps == 1 else AGG_FRAC_K_MULTI
    assert frac <= k_frac * frac_o + AGG_FRAC_ABS, \
        f"{task}: contact-active outlier fraction {frac:.3%} vs the f32 oracle's {frac_o:.3%} (both against f64)"
    assert med <= AGG_MED_K * med_o + AGG_MED_ABS, \
        f"{task}: contact-active median err/tol {med:.3g} vs the f32 oracle's {med_o:.3g} (both against f64)"
    return len(bad)


@pytest.mark.parametrize("task", TASKS)
def test_full_state_one_step(gpu, task):
    n, seed = 2048, 17
    g, o, cfg, torch = _sims(task, n, seed)
    st = random_states(task, o, n, seed=101)
    g.set_state(torch.from_numpy(st).cuda())
    a = np.random.default_rng(7).normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    sg = g.get_state().cpu().numpy()
    nbad = _check(task, "one step from random full states", n, seed, st, [a], g_out, sg, torch)
    assert nbad <= 0.02 * n


@pytest.mark.parametrize("task", TASKS)
def test_full_state_zero_action_standing(gpu, task):
    """20 zero-action steps from (near-)standing states with random MDP carry: every row at the end."""
    n, seed, steps = 1024, 5, 20
    g, o, cfg, torch = _sims(task, n, seed)
    st = random_states(task, o, n, seed=202, standing=True)
    g.set_state(torch.from_numpy(st).cuda())
    a = np.zeros((n, 6), np.float32)
    at = torch.from_numpy(a).cuda()
    for _ in range(steps):
        obs, rew, te, tr = g.step(at)
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    sg = g.get_state().cpu().numpy()
    nbad = _check(task, f"{steps} zero-action steps from standing", n, seed, st, [a] * steps, g_out, sg, torch)
    assert nbad <= 0.05 * n


@pytest.mark.parametrize("stage", ["step0", "step1"])
def test_full_state_v2_stage(gpu, stage):
    """The first stages of the staged v2 recipe (v2.py:78-110; step0 adds feet_force_diff /
    feet_force_sum and the feet_force_sum row; each stage advances only its active terms'
    buffers): one step from random full states and 20 zero-action steps from standing, every row
    (feet_force_sum included) under the full-state rule."""
    task = f"v2:{stage}"
    n, seed = 2048, 29
    g, o, cfg, torch = _sims(task, n, seed)
    if stage == "step0":  # the feet-force terms on, step_length (its latches) off
        assert cfg.pack().reward_active >> 13 == 3 and "step_length" not in cfg.reward_weights
    st = random_states(task, o, n, seed=121)
    g.set_state(torch.from_numpy(st).cuda())
    a = np.random.default_rng(9).normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    sg = g.get_state().cpu().numpy()
    nbad = _check(task, "one step from random full states", n, seed, st, [a], g_out, sg, torch)
    assert nbad <= 0.02 * n
    n, seed, steps = 1024, 7, 20
    g, o, cfg, torch = _sims(task, n, seed)
    st = random_states(task, o, n, seed=222, standing=True)
    g.set_state(torch.from_numpy(st).cuda())
    at = torch.zeros(n, 6, device="cuda:0")
    for _ in range(steps):
        obs, rew, te, tr = g.step(at)
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    nbad = _check(task, f"{steps} zero-action steps from standing", n, seed, st, [np.zeros((n, 6), np.float32)] * steps,
                  g_out, g.get_state().cpu().numpy(), torch)
    assert nbad <= 0.05 * n


def test_full_state_deep_overlap(gpu):
    """One step from states whose links interpenetrate deeper than 2 CORE_M (the rounded cores
    intersect): both sides take the separating-axis penetration estimate (normal and depth over the
    centre difference and the four circle normals, point at the mean hull centre), so away from the
    switch (the core distance crossing 1e-6, GJK's overlap tests) and the axis choice every row
    agrees under the same explained-outlier rule; no state is set aside."""
    from oracle.pyoracle import OracleSim
    task, seed, pool = "v2", 31, 8192
    o = OracleSim(pool, task_cfg(task), seed=seed)
    st = random_states(task, o, pool, seed=404)
    rng = np.random.default_rng(405)
    st[13:19] += rng.normal(0, 0.6, (6, pool)).astype(np.float32)  # fold links into each other
    o.set_state(st)
    deep = np.nonzero(o.self_min_sep() <= -2 * 0.004 + 1e-6)[0]
    assert len(deep) >= 512, len(deep)
    ids = deep[:512]
    n = len(ids)
    st = np.ascontiguousarray(st[:, ids])
    g, _, cfg, torch = _sims(task, n, seed)
    g.set_state(torch.from_numpy(st).cuda())
    a = np.random.default_rng(406).normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    sg = g.get_state().cpu().numpy()
    nbad = _check(task, "one step from deep self-overlap", n, seed, st, [a], g_out, sg, torch)
    assert nbad <= 0.05 * n


@pytest.mark.parametrize("mode", [1, 2, 3], ids=["tgs", "tgs-refresh", "tgs-refresh-self"])
@pytest.mark.parametrize("task", ["v2", "standup"])
def test_full_state_tgs(gpu, task, mode):
    """The TGS-style contact solve (zb_task_cfg.solver_mode 1: per-sub-iteration re-linearised
    biases, pose from the mean sub-iteration velocity; mode 2 also re-evaluates every ground
    contact's point, separation and Jacobian rows at each sub-iteration's pose, mode 3 every self
    contact's too): one step from random
    full states and 20 zero-action steps from standing, every row under the same explained-outlier
    rule."""
    with solver_mode(mode):
        n, seed = 2048, 19
        g, o, cfg, torch = _sims(task, n, seed)
        assert cfg.solver_mode == mode
        st = random_states(task, o, n, seed=111)
        g.set_state(torch.from_numpy(st).cuda())
        a = np.random.default_rng(8).normal(size=(n, 6)).astype(np.float32)
        obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
        g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
        nbad = _check(task, f"TGS mode {mode}: one step from random full states", n, seed, st, [a], g_out,
                      g.get_state().cpu().numpy(), torch)
        assert nbad <= 0.02 * n
        n, seed, steps = 1024, 6, 20
        g, o, cfg, torch = _sims(task, n, seed)
        st = random_states(task, o, n, seed=212, standing=True)
        g.set_state(torch.from_numpy(st).cuda())
        at = torch.zeros(n, 6, device="cuda:0")
        for _ in range(steps):
            obs, rew, te, tr = g.step(at)
        g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
        stats = {}
        nbad = _check(task, f"TGS mode {mode}: {steps} zero-action steps from standing", n, seed, st,
                      [np.zeros((n, 6), np.float32)] * steps, g_out, g.get_state().cpu().numpy(), torch, stats=stats)
        # the envs outside tolerance (device against the f32 oracle), bounded by the f32 oracle's own count
        # against f64 on the same states -- two f32 implementations each differ from exact arithmetic
        # by their rounding -- with the aggregate rule's multi-step factor (round 5
        # had a hand-set 8.5 % cap here). Every env outside tolerance is still explained per env by
        # _check. The count moves with code generation alone: v2 mode 2 69 -> 81 envs (f32 oracle 36)
        # from a branch-free rewrite of selects whose arithmetic is unchanged
        assert nbad <= AGG_FRAC_K_MULTI * stats["nbad_f32"] + 0.005 * n, (nbad, stats["nbad_f32"])


@pytest.mark.parametrize("task", TASKS)
def test_full_state_contact_cache(gpu, task):
    """The persistent self-contact cache (the first substep's GJK warm start):
    from folded states one oracle step after random joint angles (self contacts present) and the
    oracle's cache of those states, set into the GPU handle, one step on both sides; every state row under the
    full-state rule (the oracle run from the same cache), and the cache after the step: pair codes
    identical in >= 99 % of the (slot, env) entries, normals within 2e-3 (95 %) / 5e-2 (99 %) where
    the codes agree."""
    from oracle.pyoracle import OracleSim
    seed, n = 23, 2048
    o = OracleSim(n, task_cfg(task), seed=seed)
    rng = np.random.default_rng(77)
    st = random_states(task, o, n, seed=78)
    st[13:19] += rng.normal(0, 1.5, (6, n)).astype(np.float32)  # folded: links in contact
    o.set_state(st)
    o.step(rng.normal(size=(n, 6)).astype(np.float32))  # one step leaves its self contacts in the cache
    st, wc = o.get_state(), o.get_contact_cache()
    hot = (wc[3::4] >= 1).any(axis=0)
    assert hot.sum() >= 50, hot.sum()
    g, _, cfg, torch = _sims(task, n, seed)
    g.set_state(torch.from_numpy(st).cuda())
    g.set_contact_cache(torch.from_numpy(wc).cuda())
    np.testing.assert_array_equal(g.get_contact_cache().cpu().numpy(), wc)
    a = rng.normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    sg, wg = g.get_state().cpu().numpy(), g.get_contact_cache().cpu().numpy()
    _check(task, "one step from a folded state with its contact cache", n, seed, st, [a], g_out, sg, torch, wc=wc)
    o2 = OracleSim(n, task_cfg(task), seed=seed)
    o2.set_state(st)
    o2.set_contact_cache(wc)
    o2.step(a)
    wo = o2.get_contact_cache()
    same = wg[3::4] == wo[3::4]
    assert same.mean() >= 0.99, same.mean()
    both = same & (wo[3::4] >= 1)
    assert both.sum() >= 50, both.sum()
    dn = np.abs(np.stack([wg[k::4] for k in range(3)]) - np.stack([wo[k::4] for k in range(3)])).max(axis=0)
    # (normals of slowly converging pairs -- GJK stopping one iteration apart -- differ more)
    assert (dn[both] <= 2e-3).mean() >= 0.95 and (dn[both] <= 5e-2).mean() >= 0.99, np.sort(dn[both])[-10:]
    # the in-kernel auto-reset invalidates a resetting env's entries
    assert (wg[3::4][:, g_out[2] | g_out[3]] == -1).all()


@pytest.mark.parametrize("kind", ["face", "rim", "rimface"])
@pytest.mark.parametrize("task", ["v2", "standup"])
def test_full_state_face_manifold(gpu, task, kind):
    """The self-contact manifold (zb_task_cfg.self_manifold 2) on 512 constructed
    gentle folds per case (tests/fullstate.constructed_states: the joint angles of a seed fold from
    tests/golden/manifold_seeds.npz plus 3 mrad of jitter, the class checked by the oracle's
    per-pair classes): "face" -- one link pair cap on cap (up to 4 points), "rim" -- one pair side by
    side (the GJK point + the two ends of the rulings' overlap), "rimface" -- one link lying on
    another's cap (self_manifold 3: the GJK point + the ends of the ruling over the cap disk), no
    overlapping cores anywhere; one step on both sides under the full-state rule, with the
    contact-active aggregate against the f64 oracle over all 512 envs."""
    from fullstate import constructed_states, self_manifold
    seed, n = 43, 512
    mode = 3 if kind == "rimface" else 2
    with self_manifold(mode):
        st, which = constructed_states(task, kind, n, seed=606)
        g, o, cfg, torch = _sims(task, n, seed)
        assert cfg.self_manifold == mode
        o.set_state(st)
        pc = o.pair_classes()
        assert (pc[:, {"face": 1, "rim": 2, "rimface": 8}[kind]] > 0).all() and (pc[:, 3] == 0).all()
        _manifold_step(task, kind, n, seed, st, which, pc, g, torch)


def _manifold_step(task, kind, n, seed, st, which, pc, g, torch):
    print(f"\n[{task} {kind}] {n} constructed envs from {len(np.unique(which))} seed folds; self points per env "
          f"{pc[:, 5].mean():.2f}")
    g.set_state(torch.from_numpy(st).cuda())
    a = np.random.default_rng(608).normal(size=(n, 6)).astype(np.float32)
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    g_out = (obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy())
    nbad = _check(task, f"one step from constructed {kind}-manifold folds", n, seed, st, [a], g_out,
                  g.get_state().cpu().numpy(), torch)
    assert nbad <= 0.05 * n


@pytest.mark.parametrize("kind", ["face", "rim"])
@pytest.mark.parametrize("task", ["v2", "standup"])
def test_full_state_self_refresh(gpu, task, kind):
    """The TGS refresh of the self contacts (zb_task_cfg.solver_mode 3: each self contact's two
    body-fixed anchors carried to every sub-iteration's pose, the separation and rows re-evaluated
    there) on 512 constructed gentle folds per case (cap on cap / side by side, as in
    test_full_state_face_manifold): one step on both sides under the full-state rule."""
    from fullstate import constructed_states, self_manifold, solver_mode
    seed, n = 47, 512
    with self_manifold(2), solver_mode(3):
        st, which = constructed_states(task, kind, n, seed=616)
        g, o, cfg, torch = _sims(task, n, seed)
        assert cfg.solver_mode == 3 and cfg.self_manifold == 2
        o.set_state(st)
        pc = o.pair_classes()
        _manifold_step(task, f"{kind} (self refresh)", n, seed, st, which, pc, g, torch)
