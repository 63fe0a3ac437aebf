"""Non-finite guard of the step kernels (zbot_sim.hip `phys_bad`): the product build
uses -ffast-math, which folds isfinite away, so the kernels test the exponent bits of the physics
state after the substeps. An env whose state went inf / NaN ends its episode as `died` with a
finite reward and is reset; no other env is touched (compared bit for bit with a run that never
had the bad envs). All four step kernels (walking v2, stand-up, v4, manager).
"""
from __future__ import annotations

import numpy as np
import pytest

from zbot_lab_amd import model as zm

pytestmark = pytest.mark.gpu

TASKS = {"walking": lambda: zm.TaskCfg(), "standup": lambda: zm.TaskCfg.standup(),
         "v4": lambda: zm.TaskCfg.walking_v4(), "manager": lambda: zm.TaskCfg.manager_flat()}


def _penalty(task, cfg):
    """The reward of a poisoned env: -terminal_penalty, or for the manager task its is_terminated
    term alone (weight x step_dt)."""
    if task == "manager":
        return cfg.pack().stage_scales[0][zm.M_REWARD_TERMS.index("termination_penalty")] * cfg.sim_dt * cfg.decimation
    return -cfg.terminal_penalty


@pytest.mark.parametrize("task", sorted(TASKS))
def test_non_finite_state_is_reset(gpu, task):
    import torch
    from zbot_lab_amd.sim import ZbotSim
    n = 256
    cfg = TASKS[task]()
    clean, bad = ZbotSim(n, cfg, device="cuda:0", seed=3), ZbotSim(n, cfg, device="cuda:0", seed=3)
    st = clean.get_state().cpu().numpy()
    poisoned = [5, 77, 200]
    st_bad = st.copy()
    st_bad[0, poisoned[0]] = np.nan          # root position
    st_bad[20, poisoned[1]] = np.inf         # a joint velocity
    st_bad[4, poisoned[2]] = -np.nan         # root quaternion
    clean.set_state(torch.from_numpy(st).cuda())
    bad.set_state(torch.from_numpy(st_bad).cuda())
    a = torch.from_numpy(np.random.default_rng(0).normal(size=(n, 6)).astype(np.float32)).cuda()
    oc, rc, tc, uc = [x.cpu().numpy() for x in clean.step(a)]
    ob, rb, tb, ub = [x.cpu().numpy() for x in bad.step(a)]
    sb = bad.get_state().cpu().numpy()
    assert np.isfinite(ob).all() and np.isfinite(rb).all() and np.isfinite(sb).all()
    assert tb[poisoned].all(), "poisoned envs must terminate"
    np.testing.assert_allclose(rb[poisoned], _penalty(task, cfg), rtol=1e-6)
    keep = np.setdiff1d(np.arange(n), poisoned)
    np.testing.assert_array_equal(ob[keep], oc[keep])
    np.testing.assert_array_equal(rb[keep], rc[keep])
    np.testing.assert_array_equal(sb[:, keep], clean.get_state().cpu().numpy()[:, keep])
    # the next step runs normally from the reset state
    ob2, rb2, _, _ = [x.cpu().numpy() for x in bad.step(a)]
    assert np.isfinite(ob2).all() and np.isfinite(rb2).all()
