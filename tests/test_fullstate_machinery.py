"""CPU check of the full-state parity machinery (tests/fullstate.py) that test_gpu_fullstate.py runs
against the HIP kernels: with the f64 oracle standing in for the device, every env agrees or is an
explained discontinuity; and a planted error of the size a wrong weight / latch / integrator would
cause is reported as unexplained."""
from __future__ import annotations

import re

import numpy as np
import pytest

import test_gpu_fullstate as T
from fullstate import TASKS, random_states, row_groups, task_cfg


def _device_f64(task, n, seed, st, actions):
    from oracle.pyoracle import OracleSim
    d = OracleSim(n, task_cfg(task), seed=seed, double=True)
    d.set_state(st)
    for a in actions:
        out = d.step(a)
    return out, d.get_state()


@pytest.mark.parametrize("task", TASKS)
def test_f64_oracle_passes_full_state_check(oracle_lib, task):
    from oracle.pyoracle import OracleSim
    n, seed = 256, 17
    st = random_states(task, OracleSim(n, task_cfg(task), seed=seed), n, seed=101)
    a = np.random.default_rng(7).normal(size=(n, 6)).astype(np.float32)
    out, sg = _device_f64(task, n, seed, st, [a])
    assert T._check(task, "f64 oracle as device", n, seed, st, [a], out, sg, None) <= 0.02 * n


@pytest.mark.parametrize("task", TASKS)
def test_planted_errors_are_unexplained(oracle_lib, task):
    from oracle.pyoracle import OracleSim
    n, seed = 256, 17
    st = random_states(task, OracleSim(n, task_cfg(task), seed=seed), n, seed=101)
    a = np.random.default_rng(7).normal(size=(n, 6)).astype(np.float32)
    out, sg = _device_f64(task, n, seed, st, [a])
    g = row_groups(task)
    sg = sg.copy()
    # plant into envs where the oracle is stable (no contact discontinuity nearby) and that do not
    # reset in the step, so every planted error must be reported as unexplained
    so, outs = T._run_oracle(task, n, seed, st, [a])
    ob_o, rw_o, te_o, tr_o = outs[-1]
    sens = T._sensitivity(task, n, seed, st, [a], so, ob_o, rw_o, (te_o, tr_o), st, 1)
    calm = [int(e) for e in np.nonzero((sens < 0.3) & ~(te_o | tr_o))[0]]
    envs = [calm[k] for k in (1, 10, 20, 30)]
    sg[g["sums"][0], envs[0]] += 2e-2            # a per-term episode sum off by a weight-sized error
    sg[g["exact"][0], envs[1]] += 1e-3           # p_delta / raw action carry
    if g["kin"]:
        sg[g["kin"][0], envs[2]] += 5e-3          # a latch / integrator
    sg[g["phys_vel"][3], envs[3]] += 0.1         # a joint velocity
    with pytest.raises(AssertionError, match="oracle is stable") as ei:
        T._check(task, "planted", n, seed, st, [a], out, sg, None)
    listed = {int(v) for v in re.findall(r"\d+", str(ei.value).split(":")[-1].split("\n")[0])}
    for e in envs if g["kin"] else envs[:2] + envs[3:]:
        assert e in listed, (e, listed)
