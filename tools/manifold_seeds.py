"""Seed poses for the constructed self-contact manifold states (tests/test_gpu_fullstate.py,
tests/test_fullstate_machinery.py): joint angles of gentle folds in which one link pair touches
cap on cap (the face manifold), side by side (the rim manifold), or with overlapping cores (the
separating-axis branch), and no other pair overlaps.

Searched once over uniformly random joint angles with the CPU oracle's per-pair classes
(zbo_pair_classes): of 4 M folds, ~90 are a gentle cap-on-cap contact and ~370 a gentle side-by-side
one (a face pair almost always comes with deep overlaps elsewhere, so uniform sampling at test time
finds few gentle ones: VERDICT r4). The tests then build their envs from these seeds directly --
each seed's joint angles plus a small jitter, kept when the class survives -- instead of sampling.

Writes tests/golden/manifold_seeds.npz: {face, rim, deep, rimface}: [k, 6] joint angles (float32).
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from fullstate import random_states, task_cfg  # noqa: E402
from oracle.pyoracle import OracleSim  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "manifold_seeds.npz")
POOL, ROUNDS, MAX_SEEDS = 500_000, 8, 256


def classify(pc: np.ndarray) -> dict:
    """Gentle classes from zbo_pair_classes rows (self_manifold 3): no overlapping cores except the deep
    class's one."""
    gentle = pc[:, 3] == 0
    return {"face": gentle & (pc[:, 1] > 0), "rim": gentle & (pc[:, 2] > 0),
            "deep": (pc[:, 3] == 1) & (pc[:, 0] <= 2), "rimface": gentle & (pc[:, 8] > 0)}


def main():
    cfg = task_cfg("v2")
    cfg.self_manifold = 3
    o = OracleSim(POOL, cfg, seed=1)
    base = random_states("v2", o, POOL, seed=5)
    seeds = {k: [] for k in ("face", "rim", "deep", "rimface")}
    for r in range(ROUNDS):
        st = base.copy()
        st[13:19] = np.random.default_rng(100 + r).uniform(-np.pi, np.pi, (6, POOL)).astype(np.float32)
        o.set_state(st)
        for k, m in classify(o.pair_classes()).items():
            seeds[k].extend(st[13:19, m].T.tolist())
    out = {k: np.array(v[:MAX_SEEDS], np.float32) for k, v in seeds.items()}
    np.savez_compressed(OUT, **out)
    print("wrote", os.path.normpath(OUT), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
