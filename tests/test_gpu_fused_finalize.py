"""Fused step-end finalisation of the walking v2 kernel (zbot_sim.hip `finalize_body`):
the step kernel's last workgroup folds the episode log, advances the counters and applies the
full-reset episode-length draw (v2.py:418-422) instead of a separate zb_finalize_kernel launch.
Compared bit for bit with the two-launch path (ZB_FUSED_FINALIZE=0 at create) on the same inputs:
observations, rewards, flags, every state row and the log counts bit for bit, the log means to
float-atomic rounding, at 4096 envs (all 8 XCDs,
1024 workgroups) through individual resets and a full reset.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from zbot_lab_amd import model as zm

pytestmark = pytest.mark.gpu


def _make(n, cfg, fused):
    from zbot_lab_amd.sim import ZbotSim
    old = os.environ.get("ZB_FUSED_FINALIZE")
    os.environ["ZB_FUSED_FINALIZE"] = "1" if fused else "0"
    try:
        return ZbotSim(n, cfg, device="cuda:0", seed=11)
    finally:
        if old is None:
            del os.environ["ZB_FUSED_FINALIZE"]
        else:
            os.environ["ZB_FUSED_FINALIZE"] = old


@pytest.mark.parametrize("n", [4096, 1000])
def test_fused_finalize_matches_two_launches(gpu, n):
    import torch
    cfg = zm.TaskCfg(episode_length_s=0.4)  # 20-step episodes: time-outs within the run
    fz, sp = _make(n, cfg, True), _make(n, cfg, False)
    ep_row, L = zm.S["EP_LEN"], cfg.max_episode_length
    rng = np.random.default_rng(5)
    full_seen = False
    for k in range(60):
        if k == 7:  # every env times out on the next step: the full-reset draw
            for s in (fz, sp):
                st = s.get_state().clone()
                st[ep_row] = float(L - 1)
                s.set_state(st)
        a = torch.from_numpy(rng.normal(size=(n, 6)).astype(np.float32)).cuda()
        of, rf, tf, uf = [x.cpu().numpy() for x in fz.step(a)]
        os_, rs, ts, us = [x.cpu().numpy() for x in sp.step(a)]
        np.testing.assert_array_equal(of, os_, err_msg=f"obs, step {k}")
        np.testing.assert_array_equal(rf, rs, err_msg=f"reward, step {k}")
        np.testing.assert_array_equal(tf, ts, err_msg=f"terminated, step {k}")
        np.testing.assert_array_equal(uf, us, err_msg=f"truncated, step {k}")
        sf, ss = fz.get_state().cpu().numpy(), sp.get_state().cpu().numpy()
        np.testing.assert_array_equal(sf, ss, err_msg=f"state, step {k}")
        # (float atomics into the accumulator slots add in arrival order: not bit-reproducible)
        np.testing.assert_allclose(fz.log_buffer.cpu().numpy(), sp.log_buffer.cpu().numpy(), rtol=1e-5,
                                   atol=1e-7, err_msg=f"log means, step {k}")
        np.testing.assert_array_equal(fz.read_log()[1].cpu().numpy(), sp.read_log()[1].cpu().numpy(),
                                      err_msg=f"log counts, step {k}")
        if k == 7:
            assert (uf.astype(bool) | tf.astype(bool)).all(), "every env must reset at step 7"
            full_seen = len(np.unique(sf[ep_row])) > 1  # the draw spreads the episode lengths
    assert full_seen, "the full-reset draw did not run"
    # the next launch sees a cleared accumulator and done counter: a further step still agrees
    a = torch.zeros(n, 6, device="cuda:0")
    assert np.array_equal(fz.step(a)[0].cpu().numpy(), sp.step(a)[0].cpu().numpy())
