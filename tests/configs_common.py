"""Shared checks of BASELINE.json configs[0] (C1: zbot-6b-walking-v2, 4 envs, random actions, 1000
steps): per-step invariants that hold on the CPU oracle and on the HIP path alike."""
from __future__ import annotations

import numpy as np

from zbot_lab_amd import model as zm

S = zm.S


def c1_step_invariants(k, st_before, st_after, obs, rew, te, tr, log_counts):
    """DirectRLEnv bookkeeping of one v2 step (v2.py:384-459; DirectRLEnv.step order)."""
    assert np.isfinite(st_after).all() and np.isfinite(obs).all() and np.isfinite(rew).all(), k
    q = st_after[S["ROOT_QUAT"]:S["ROOT_QUAT"] + 4]
    np.testing.assert_allclose(np.linalg.norm(q, axis=0), 1.0, atol=1e-5)
    ep0 = st_before[S["EP_LEN"]]
    ep1 = st_after[S["EP_LEN"]]
    done = te | tr
    np.testing.assert_array_equal(tr, ep0 + 1 >= 999)                   # time_out = ep_len >= max - 1
    if done.all():   # every env reset in one call: episode_length_buf ~ U{0..999} (v2.py:418-422)
        assert ((ep1 >= 0) & (ep1 < 1000)).all(), k
    else:
        assert (ep1[done] == 0).all() and (ep1[~done] == ep0[~done] + 1).all(), k
    assert (st_after[S["EP_SUMS"]:S["EP_SUMS"] + 13][:, done] == 0).all()  # _reset_idx zeroes the sums
    assert (st_after[S["P_DELTA"]:S["P_DELTA"] + 6][:, done] == 0).all()
    assert (np.abs(st_after[S["P_DELTA"]:S["P_DELTA"] + 6]) <= np.pi + 1e-6).all()
    assert (obs[:, 22] == 1.0).all()                                      # joint_speed_limit
    np.testing.assert_allclose(obs[:, 4:10], (st_after[S["JOINT_POS"]:S["JOINT_POS"] + 6]
                                              - zm.load_model().default_joint_pos[:, None]).T, atol=1e-5)
    if done.any():                                                        # Episode_Termination/* counts
        assert int(log_counts[0]) == int(te.sum()) and int(log_counts[1]) == int(tr.sum()), k
    assert (rew[te] < -10).all() or not te.any()                          # -20 terminal penalty dominates
