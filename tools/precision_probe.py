#!/usr/bin/env python3
"""CPU probe of where a single-precision implementation's error against exact arithmetic comes from
(VERDICT r5 item 1). Builds variants of the f32 oracle (oracle/zbot_oracle.c,
compiled here into /tmp, never into the repo) that each adopt one of the device kernel's numerical
choices, and measures each variant against the f64 oracle on the parity suite's states: the outlier
fraction and median err/tol over the contact-active envs, and the median per state-row class.

variants: base (the oracle as built by oracle/Makefile); fast_math (-ffast-math); fma
(-ffp-contract=fast -mfma); kernel_form (the free velocity as L^-1((M + A) u + dt (tau - C)), the
kernel's RNEA-suffix form, instead of L^T u + L^-1 dt (tau - C)); tanh_r (the kernel's round-5
single-precision tanh polynomial for the actions); sincos_r (the kernel's sin / cos polynomials in
FK and the root's exponential map). Usage: python tools/precision_probe.py [variant ...]
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "oracle", "zbot_oracle.c")
CFLAGS = ["-O2", "-fPIC", "-std=c11", "-fopenmp", "-I", os.path.join(ROOT, "include"), "-shared"]

TANH_R = r'''
static float tanh_r(float x) {
  const float ax = fabsf(x);
  if (ax < 0.625f) {
    const float z = x * x;
    return fmaf(fmaf(fmaf(fmaf(fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f), z, -5.37397155531e-2f), z,
                          1.33314422036e-1f), z, -3.33332819422e-1f), z * x, x);
  }
  const float e = expf(2.f * fminf(ax, 20.f));
  return copysignf(1.f - 2.f / (e + 1.f), x);
}
'''
SINCOS_R = r'''
static void sincos_r(float x, float* sn, float* cs) {
  const float kf = rintf(x * 0.636619772367581343f);
  const int k = (int)kf;
  float r = fmaf(-kf, 1.57079637050628662f, x);
  r = fmaf(kf, 4.37113900018624283e-8f, r);
  const float z = r * r;
  const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
  const float cp = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f), z,
                             -0.5f), z, 1.f);
  const float s0 = (k & 1) ? cp : sp, c0 = (k & 1) ? sp : cp;
  *sn = (k & 2) ? -s0 : s0;
  *cs = ((k + 1) & 2) ? -c0 : c0;
}
static float sin_r(float x) { float s, c; sincos_r(x, &s, &c); return s; }
static float cos_r(float x) { float s, c; sincos_r(x, &s, &c); return c; }
'''


def _patch(src: str, variant: str) -> tuple[str, list]:
    if variant == "fast_math":
        return src, ["-ffast-math"]
    if variant == "fma":
        return src, ["-ffp-contract=fast", "-mfma"]
    flags = ["-ffp-contract=off"]
    if variant == "kernel_form":
        old = "    lt_mul(L, u, w);\n    fwd_sub(L, b, z);\n    for (int a = 0; a < NV; ++a) w[a] += z[a];"
        new = ("    { real y[NV]; for (int a = 0; a < NV; ++a) { real t = 0; for (int c = 0; c < NV; ++c) t += Mw[a][c] * u[c];"
               " y[a] = t + b[a]; } fwd_sub(L, y, w); (void)z; }")
        assert old in src
        return src.replace(old, new), flags
    if variant == "tanh_r":
        i = src.index("static void cholesky(")
        src = src[:i] + TANH_R + src[i:]
        src = src.replace("act[j] = (real)tanh((double)action[j]);", "act[j] = (real)tanh_r((float)action[j]);")
        return src.replace("real a = (real)tanh((double)actions[i]);", "real a = (real)tanh_r((float)actions[i]);"), flags
    if variant == "sincos_r":
        i = src.index("static inline real sqrtr")
        src = src[:i] + SINCOS_R + src[i:]
        for a, b in (("(real)cos((double)h), 0, 0, (real)sin((double)h)", "(real)cos_r((float)h), 0, 0, (real)sin_r((float)h)"),
                     ("(real)sin((double)(0.5 * th)) / th * T", "(real)sin_r((float)(0.5 * th)) / th * T"),
                     ("(real)cos((double)(0.5 * th))", "(real)cos_r((float)(0.5 * th))")):
            assert a in src
            src = src.replace(a, b)
        return src, flags
    return src, flags  # base


def build(variant: str, out_dir: str) -> str:
    src, flags = _patch(open(SRC).read(), variant)
    c = os.path.join(out_dir, f"zo_{variant}.c")
    open(c, "w").write(src)
    so = os.path.join(out_dir, variant, "libzbot_oracle.so")
    os.makedirs(os.path.dirname(so), exist_ok=True)
    subprocess.run(["gcc", *CFLAGS, *flags, "-o", so, c, "-lm"], check=True)
    return so


CHECKS = [("v4", "20 zero-action steps from standing", True, 20, 202, 1024, 5),
          ("v2", "20 zero-action steps from standing", True, 20, 202, 1024, 5),
          ("v2", "one step from random full states", False, 1, 101, 2048, 17),
          ("standup", "20 zero-action steps from standing", True, 20, 202, 1024, 5)]


def measure(so: str) -> list[str]:
    """Runs in a child process (one oracle library per process)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import pyoracle
    build_dir = pyoracle.BUILD
    pyoracle.BUILD = os.path.dirname(so)
    pyoracle._LIBS[False] = pyoracle._load(False)
    pyoracle.BUILD = build_dir
    from fullstate import compare, random_states, row_groups, task_cfg
    from oracle.pyoracle import OracleSim
    lines = []
    for task, label, standing, steps, sseed, n, seed in CHECKS:
        st = random_states(task, OracleSim(n, task_cfg(task), seed=seed), n, seed=sseed, standing=standing)
        acts = ([np.zeros((n, 6), np.float32)] * steps if standing
                else [np.random.default_rng(7).normal(size=(n, 6)).astype(np.float32)])
        res = {}
        for dbl in (False, True):
            o = OracleSim(n, task_cfg(task), seed=seed, double=dbl)
            o.set_state(st)
            o.contact_activity(clear=True)
            for a in acts:
                out = o.step(a)
            res[dbl] = (o.get_state(), out, o.contact_activity())
        (s32, o32, act), (s64, o64, _) = res[False], res[True]
        r, rows = compare(task, s32, s64, o32[0], o64[0], o32[1], o64[1], (o32[2], o32[3]), (o64[2], o64[3]), st,
                          steps)[:2]
        a = act.sum(axis=1) > 0
        g = {c: float(np.median(np.minimum(rows[rr][:, a].max(axis=0), 1e6))) for c, rr in row_groups(task).items() if rr}
        lines.append(f"  {task} {label}: outliers {(r[a] > 1).mean():.2%}, median err/tol "
                     f"{np.median(np.minimum(r[a], 1e6)):.3g} | " + ", ".join(f"{k} {v:.3g}" for k, v in g.items()))
    return lines


def main(variants):
    if len(variants) == 2 and variants[0] == "--measure":
        print("\n".join(measure(variants[1])), flush=True)
        return
    tmp = tempfile.mkdtemp(prefix="zbo_probe_")
    for v in variants or ["base", "fast_math", "fma", "kernel_form", "tanh_r", "sincos_r"]:
        so = build(v, tmp)
        print(f"[{v}] f32 oracle variant against the f64 oracle", flush=True)
        subprocess.run([sys.executable, os.path.abspath(__file__), "--measure", so], check=True)


if __name__ == "__main__":
    main(sys.argv[1:])
