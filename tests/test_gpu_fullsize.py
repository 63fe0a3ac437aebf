"""BASELINE.json's full sizes (4096 envs = configs[1], 8192 = one GPU's shard of configs[2]'s 65 536,
and 65 536 on one GPU) through the C ABI, checked by properties that do not depend on N:

* full-state parity: one step of N envs from random full states on the GPU vs the CPU oracle run on
  a spread sample of the same env columns (envs are independent, so a sample is an exact
  sub-problem), every state row / obs / reward / flag under the explained-outlier rule of
  tests/test_gpu_fullstate.py — covers the grid / XCD-aware workgroup renumbering and the last
  partial workgroup at the real launch sizes (4096, 8192, 65 536);
* permutation equivariance: permuting the env columns of the state and the action rows permutes every
  output bit-for-bit (no cross-env leakage between the 16-lane teams of a wave or between workgroups);
* shard equivalence: the two halves of an N-env state stepped in two handles of N/2 give the same
  bits as one handle of N (what the env-sharded multi-GPU bench relies on);
* determinism + sanity over a 100-step random-action rollout from a full reset: two handles with the
  same seed agree bit-for-bit, everything stays finite, episode lengths stay in [0, 999].
"""
from __future__ import annotations

import numpy as np
import pytest

from helpers import S, perturbed_states
from zbot_lab_amd import model as zm

pytestmark = pytest.mark.gpu


def _sim(n, seed=0):
    from zbot_lab_amd.sim import ZbotSim
    return ZbotSim(n, zm.TaskCfg(), device="cuda:0", seed=seed)


def _step(g, a):
    import torch
    obs, rew, te, tr = g.step(torch.from_numpy(a).cuda())
    return obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy().copy(), tr.cpu().numpy().copy()


def _sample(n, k=1024, seed=0):
    """k env ids spread over [0, n): both ends, workgroup / XCD boundaries, and random fill."""
    rng = np.random.default_rng(seed)
    ids = {0, 1, 2, 3, 4, n - 1, n - 2, n - 5, n // 2, n // 2 - 1, n // 8, n // 8 - 1}
    ids |= set(rng.choice(n, size=k - len(ids) - 8, replace=False).tolist())
    while len(ids) < k:
        ids.add(int(rng.integers(0, n)))
    return np.array(sorted(ids), dtype=np.int64)


@pytest.mark.parametrize("n", [4096, 8192, 65536])
def test_full_state_headline_sizes(gpu, n):
    """Walking v2 at BASELINE's sizes (4096 = configs[1], 8192 = one GPU's shard of configs[2],
    65 536 on one GPU): one step of all n envs from random full states (every persistent row: sensor
    histories, timers, feet latches, step lengths, integrators, episode sums), then every state row,
    obs, reward and both flags of a spread sample of 1024 env columns against the oracle run on
    those columns (envs are independent, so the sample is an exact sub-problem), under the
    full-state rule of tests/test_gpu_fullstate.py: every env inside tolerance or explained."""
    import torch
    import test_gpu_fullstate as F
    from fullstate import random_states, task_cfg
    from oracle.pyoracle import OracleSim
    task, seed = "v2", 29
    st = random_states(task, OracleSim(n, task_cfg(task), seed=seed), n, seed=300 + n)
    a = np.random.default_rng(n).normal(size=(n, 6)).astype(np.float32)
    g = _sim(n, seed=seed)
    g.set_state(torch.from_numpy(st).cuda())
    obs, rew, te, tr = _step(g, a)
    sg = g.get_state().cpu().numpy()
    g.close()
    ids = _sample(n)
    sub = lambda x: np.ascontiguousarray(x[:, ids])  # noqa: E731
    g_out = (np.ascontiguousarray(obs[ids]), rew[ids].copy(), te[ids].copy(), tr[ids].copy())
    nbad = F._check(task, f"one step of {n} envs, sampled columns", len(ids), seed, sub(st),
                    [np.ascontiguousarray(a[ids])], g_out, sub(sg), torch)
    assert nbad <= 0.02 * len(ids)


@pytest.mark.parametrize("task,mode", [("v2", 0), ("v2", 1), ("v2", 2), ("v2", 3), ("v4", 0), ("manager", 0)],
                         ids=["v2-pgs", "v2-tgs", "v2-tgs-refresh", "v2-tgs-refresh-self", "v4-pgs", "manager-pgs"])
def test_full_state_4096_every_solver(gpu, task, mode):
    """configs[1]'s size, every column: one step of 4096 envs from random full states against the
    oracle run on ALL 4096 columns under the full-state rule, for the benchmarked walking v2 PGS
    solve, v2's TGS-style solves (modes 1-3), v4 and the manager. (v4's and the manager's command resampling
    draws from a counter-based generator keyed on the env index, so a column subset would not be
    the same sub-problem there.)"""
    import torch
    import test_gpu_fullstate as F
    from fullstate import random_states, solver_mode, task_cfg
    from oracle.pyoracle import OracleSim
    from zbot_lab_amd.sim import ZbotSim
    n, seed = 4096, 37
    with solver_mode(mode):
        cfg = task_cfg(task)
        st = random_states(task, OracleSim(n, cfg, seed=seed), n, seed=500)
        a = np.random.default_rng(n + 1).normal(size=(n, 6)).astype(np.float32)
        g = ZbotSim(n, cfg, device="cuda:0", seed=seed)
        g.set_state(torch.from_numpy(st).cuda())
        g_out = _step(g, a)
        sg = g.get_state().cpu().numpy()
        g.close()
        nbad = F._check(task, f"one step of {n} envs ({['PGS', 'TGS', 'TGS refresh', 'TGS refresh + self'][mode]}, every column)", n, seed, st, [a], g_out,
                        sg, torch)
    assert nbad <= 0.02 * n


def test_permutation_equivariance_65536(gpu):
    import torch
    n = 65536
    st = perturbed_states(n, seed=61)
    a = np.random.default_rng(3).normal(size=(n, 6)).astype(np.float32)
    perm = np.random.default_rng(4).permutation(n)
    g1, g2 = _sim(n), _sim(n)
    g1.set_state(torch.from_numpy(st).cuda())
    g2.set_state(torch.from_numpy(np.ascontiguousarray(st[:, perm])).cuda())
    out1 = _step(g1, a)
    out2 = _step(g2, np.ascontiguousarray(a[perm]))
    te1, tr1 = out1[2], out1[3]
    assert not (te1 | tr1).all()  # no full-reset episode-length draw (that one is keyed by env index)
    for x1, x2 in zip(out1, out2):
        np.testing.assert_array_equal(x1[perm], x2)
    np.testing.assert_array_equal(g1.get_state().cpu().numpy()[:, perm], g2.get_state().cpu().numpy())
    g1.close()
    g2.close()


def test_shard_equivalence_8192(gpu):
    import torch
    n = 8192
    st = perturbed_states(n, seed=71)
    a = np.random.default_rng(5).normal(size=(n, 6)).astype(np.float32)
    g = _sim(n)
    h = [_sim(n // 2), _sim(n // 2)]
    g.set_state(torch.from_numpy(st).cuda())
    for r in range(2):
        h[r].set_state(torch.from_numpy(np.ascontiguousarray(st[:, r * n // 2:(r + 1) * n // 2])).cuda())
    for k in range(5):
        ak = np.roll(a, k, axis=0)
        full = _step(g, ak)
        parts = [_step(h[r], np.ascontiguousarray(ak[r * n // 2:(r + 1) * n // 2])) for r in range(2)]
        for x, p0, p1 in zip(full, parts[0], parts[1]):
            np.testing.assert_array_equal(x, np.concatenate([p0, p1]))
    sg = g.get_state().cpu().numpy()
    np.testing.assert_array_equal(sg, np.concatenate([x.get_state().cpu().numpy() for x in h], axis=1))
    for x in [g] + h:
        x.close()


def test_rollout_determinism_and_sanity_65536(gpu):
    import torch
    n, steps = 65536, 100
    g1, g2 = _sim(n, seed=42), _sim(n, seed=42)
    for x in (g1, g2):
        x.reset(None)
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(42)
    done = 0
    for k in range(steps):
        a = torch.randn(n, 6, device="cuda:0", generator=gen)
        o1, r1, t1, u1 = g1.step(a)
        o2, r2, t2, u2 = g2.step(a)
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(t1, t2) and torch.equal(u1, u2), k
        assert torch.isfinite(o1).all() and torch.isfinite(r1).all(), k
        done += int((t1 | u1).sum())
    s1, s2 = g1.get_state(), g2.get_state()
    assert torch.equal(s1, s2)
    ep = s1[S["EP_LEN"]]
    assert float(ep.min()) >= 0 and float(ep.max()) <= 999
    assert torch.isfinite(s1).all()
    assert done > 0  # random actions topple some robots within 2 s
    g1.close()
    g2.close()


@pytest.mark.parametrize("task", ["standup", "v4", "manager"])
def test_rollout_determinism_other_tasks_65536(gpu, task):
    """Same bit-for-bit determinism for the other tasks' kernels (their own epilogues, counter-based
    draws and curriculum state) over a 60-step random-action rollout."""
    import torch
    from zbot_lab_amd.sim import ZbotSim
    cfg = {"standup": zm.TaskCfg.standup, "v4": zm.TaskCfg.walking_v4, "manager": zm.TaskCfg.manager_flat}[task]()
    n, steps = 65536, 60
    g1, g2 = ZbotSim(n, cfg, device="cuda:0", seed=7), ZbotSim(n, cfg, device="cuda:0", seed=7)
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(7)
    for k in range(steps):
        a = torch.randn(n, 6, device="cuda:0", generator=gen)
        o1, r1, t1, u1 = g1.step(a)
        o2, r2, t2, u2 = g2.step(a)
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(t1, t2) and torch.equal(u1, u2), k
        assert torch.isfinite(o1).all() and torch.isfinite(r1).all(), k
    assert torch.equal(g1.get_state(), g2.get_state())
    g1.close()
    g2.close()
