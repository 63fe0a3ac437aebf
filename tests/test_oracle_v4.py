"""zbot-6b-walking-v4 (commands, events, curricula): the oracle pinned to the reference's own code.

Golden file: tests/golden/mdp_v4.npz, written by tools/gen_v4_goldens.py, which imports
``zbot_direct_6dof_bipedal_env_v4.py`` (v4.py) from the reference with stub isaaclab / gymnasium
packages and records: the MDP over 16 calls (32 envs; stage 0, then 1 from call 6, then 3 from
call 11 — the stage weights set by the module's own my_curriculum), ``resample_commands`` on given
draws, ``my_curriculum`` transitions, ``range_curriculum`` cases and the ``_reset_idx`` log.
Isaac Lab's math helpers are absent; the generator restates them. fp32 both sides: 1e-5, flags exact.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from zbot_lab_amd import model as zm

GOLD = os.path.join(os.path.dirname(__file__), "golden", "mdp_v4.npz")
FRAME_KEYS = ("body_link_pos_w", "body_link_quat_w", "body_link_lin_vel_w", "body_com_lin_vel_w", "joint_vel",
              "joint_acc", "applied_torque", "net_forces_w_history", "current_air_time", "current_contact_time",
              "last_air_time", "last_contact_time")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD, allow_pickle=False))


def test_golden_metadata(gold):
    assert list(gold["term_names"]) == zm.V4_REWARD_TERMS
    cfg = zm.TaskCfg.walking_v4()
    ws = cfg.stage_weights()
    np.testing.assert_allclose(gold["weights_stage0"], [ws[0][k] for k in zm.V4_REWARD_TERMS])
    np.testing.assert_allclose(gold["weights_stage3"], [ws[3][k] for k in zm.V4_REWARD_TERMS])
    assert cfg.max_episode_length == int(gold["max_episode_length"]) == 1000
    assert int(gold["observation_space"]) == zm.V4_OBS_DIM
    np.testing.assert_allclose(gold["interval_range_s"], cfg.cmd_interval_s)
    np.testing.assert_allclose(gold["limit_yaw_ranges"], cfg.range_limit_yaw)
    np.testing.assert_allclose(gold["limit_ranges"], cfg.range_limit_vel)
    assert 0.1 < gold["died"].mean() < 0.9 and 0.05 < gold["time_out"].mean() < 0.5
    assert list(gold["stage"]) == [0] * 6 + [1] * 5 + [3] * 5


def test_mdp_matches_reference(gold, oracle_lib):
    cfg = zm.TaskCfg.walking_v4()
    T, N = gold["reward"].shape
    state = dict(commands=gold["init_commands"], target_yaw=gold["init_target_heading_yaw"],
                 feet_down_pos=gold["init_feet_down_pos_last"], feet_step_len=gold["init_feet_step_length"],
                 feet_f_last=gold["init_feet_contact_forces_last"], ep_sums=np.zeros((N, 15), np.float32))
    for t in range(T):
        frame = {k: gold["frame_" + k][t + 1] for k in FRAME_KEYS}
        out = oracle_lib.v4_mdp_eval(cfg, int(gold["stage"][t]), frame, gold["episode_length_buf"][t],
                                     gold["tanh_actions"][t], gold["prev_actions"][t], state)
        np.testing.assert_array_equal(out["died"], gold["died"][t])
        np.testing.assert_array_equal(out["time_out"], gold["time_out"][t])
        np.testing.assert_allclose(out["cur_yaw"], gold["current_yaw"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(out["heading_err"], gold["heading_err"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(out["terms"], gold["terms"][t], rtol=2e-5, atol=1e-6)
        np.testing.assert_allclose(out["reward"], gold["reward"][t], rtol=2e-5, atol=1e-5)
        np.testing.assert_allclose(out["feet_step_len"], gold["feet_step_length"][t], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(out["feet_down_pos"], gold["feet_down_pos_last"][t], rtol=0, atol=0)
        np.testing.assert_allclose(out["feet_f_last"], gold["feet_contact_forces_last"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(out["ep_sums"], gold["episode_sums"][t], rtol=2e-5, atol=1e-5)
        state = dict(commands=gold["init_commands"], target_yaw=gold["init_target_heading_yaw"],
                     feet_down_pos=gold["feet_down_pos_last"][t], feet_step_len=gold["feet_step_length"][t],
                     feet_f_last=gold["feet_contact_forces_last"][t], ep_sums=gold["episode_sums"][t])


def test_observation_layout_matches_reference(gold):
    """obs = [base quat, joint_pos - default, joint_vel, actions, commands[:, 0], heading_err]."""
    q0 = np.array([0.312, 0.837, -2.02, 2.02, -0.837, -0.312], np.float32)
    for t in range(gold["reward"].shape[0]):
        exp = np.concatenate([gold["frame_body_link_quat_w"][t + 1][:, 6], gold["frame_joint_pos"][t + 1] - q0,
                              gold["frame_joint_vel"][t + 1], gold["tanh_actions"][t],
                              gold["init_commands"][:, :1], gold["heading_err"][t][:, None]], axis=1)
        np.testing.assert_allclose(gold["obs"][t], exp, atol=1e-7)


def test_resample_commands_matches_reference(gold, oracle_lib):
    for c in range(len(gold["resample_params"])):
        cmd, tgt = oracle_lib.v4_commands_from_draws(gold["resample_params"][c], gold["resample_sign_u"][c],
                                                     gold["resample_u_vel"][c], gold["resample_u_yaw"][c],
                                                     gold["resample_cur"][c])
        np.testing.assert_allclose(cmd, gold["resample_cmd"][c], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(tgt, gold["resample_target"][c], rtol=1e-6, atol=2e-6)


def test_my_curriculum_matches_reference(gold, oracle_lib):
    cfg = zm.TaskCfg.walking_v4()
    prob_of_stage = [1.0, 1.0, 0.8, 0.6]
    for steps, st0, st1, prob in gold["my_curriculum_cases"]:
        io = [st0, 1.0, 0.3, 0.3, -0.1, 0.1]
        out = oracle_lib.curriculum_probe(cfg, int(steps), io, run_my=True, run_range=False)
        assert int(out[0]) == int(st1), (steps, st0)
        if int(st1) != int(st0):  # the reference sets prob_pos on the transition only
            assert out[1] == pytest.approx(prob) and prob == pytest.approx(prob_of_stage[int(st1)])


def test_range_curriculum_matches_reference(gold, oracle_lib):
    cfg = zm.TaskCfg.walking_v4()
    for steps, nbuf, vmean, ymean, vlo, vhi, ylo, yhi in gold["range_curriculum_cases"]:
        io = [0, 1.0, 0.3, 0.3, -0.45, 0.45]
        out = oracle_lib.curriculum_probe(cfg, int(steps), io, run_my=False, run_range=True, ring_n=int(nbuf),
                                          ring_vel=vmean, ring_yaw=ymean)
        np.testing.assert_allclose(out[2:], [vlo, vhi, ylo, yhi], rtol=0, atol=1e-7)


def test_episode_log_matches_reference(gold):
    dt = np.float32(gold["step_dt"])
    dur = np.maximum(gold["log_ep_len"].astype(np.float32) * dt, dt)
    np.testing.assert_allclose((gold["log_sums"] / dur[:, None]).mean(axis=0), gold["log_means"], rtol=1e-5, atol=1e-7)
    assert list(gold["log_counts"]) == [int(gold["log_terminated"].sum()), int((~gold["log_terminated"]).sum())]
    # curriculum entries are the values before the events: stage, velocity range, yaw lower bound
    np.testing.assert_allclose(gold["log_curriculum"], [1, 0.25, 0.3, -0.15], rtol=1e-6)
    np.testing.assert_allclose(gold["reset_feet_contact_forces_last"], 15.0)
    np.testing.assert_allclose(gold["reset_feet_step_length"], 0.0)


def test_reset_pose_matches_reference(gold, oracle_lib):
    smp = gold["pose_samples"][:, [0, 1, 3, 5]]
    pos, quat = oracle_lib.su_pose_from_samples(smp, body_frame=True, robot=zm.load_model())
    np.testing.assert_allclose(pos, gold["pose_out"][:, :3] - gold["env_origins"], atol=2e-6)
    np.testing.assert_allclose(quat, gold["pose_out"][:, 3:7], atol=2e-6)
    np.testing.assert_allclose(gold["pose_current_yaw"], gold["pose_samples"][:, 5])


# ----------------------------------------------------------------------------- oracle simulator
def _sim(n, seed=0, **kw):
    from oracle.pyoracle import OracleSim
    return OracleSim(n, zm.TaskCfg.walking_v4(**kw), seed=seed)


def test_v4_state_and_commands(oracle_lib):
    s = _sim(256, seed=4)
    st = s.get_state()
    V4 = zm.V4
    assert st.shape == (zm.V4_STATE_DIM, 256)
    np.testing.assert_allclose(st[V4["COMMANDS"]], 0.3)                 # velocity_range (0.3, 0.3), prob_pos 1
    assert np.abs(st[V4["COMMANDS"] + 1]).max() <= 0.1 + 1e-6
    left = st[V4["INTERVAL_LEFT"]]
    assert left.min() >= 3.0 and left.max() <= 6.0 and left.std() > 0.5
    np.testing.assert_allclose(st[V4["FEET_F_LAST"]:V4["FEET_F_LAST"] + 2], 15.0)
    yaw = st[V4["CURRENT_YAW"]]
    assert np.abs(yaw).max() <= 3.14 + 1e-6 and yaw.std() > 1.0
    d = st[V4["TARGET_YAW"]] - yaw - st[V4["COMMANDS"] + 1]
    np.testing.assert_allclose(np.angle(np.exp(1j * d)), 0, atol=1e-5)   # target = wrap(yaw + cmd)
    obs = s.observe()
    assert obs.shape == (256, 24)
    np.testing.assert_allclose(obs[:, 22], 0.3)
    np.testing.assert_allclose(obs[:, 23], st[V4["COMMANDS"] + 1], atol=1e-5)


def test_v4_rollout_interval_and_log(oracle_lib):
    n = 64
    s = _sim(n, seed=1)
    s.reset()
    rng = np.random.default_rng(0)
    V4 = zm.V4
    left0 = s.get_state()[V4["INTERVAL_LEFT"]].copy()
    for k in range(60):
        obs, rew, te, tr = s.step(rng.normal(size=(n, 6)).astype(np.float32))
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
    left = s.get_state()[V4["INTERVAL_LEFT"]]
    # 60 steps = 1.2 s: every timer moved down by 1.2 s unless it fired (then redrawn in [3, 6))
    fired = left > left0 - 1.2 + 1e-4
    np.testing.assert_allclose(left[~fired], left0[~fired] - 1.2, atol=1e-4)
    means, counts = s.read_log(full=True)
    assert means.shape == (zm.LOG_LEN,) and np.isfinite(means).all()
    np.testing.assert_allclose(means[17:20], [0.3, 0.3, -0.1])
    assert s.read_curriculum() == (0, 60)


def test_v4_curriculum_in_sim(oracle_lib):
    n = 32
    s = _sim(n, seed=2, stage_scale=0.02)   # stages at 12 / 24 / 144 x 0.02 = 0 / 0 / 2 steps... scaled
    s.reset()
    a = np.zeros((n, 6), np.float32)
    stages = []
    for k in range(12):
        s.step(a)
        stages.append(s.read_curriculum()[0])
    assert stages == sorted(stages) and stages[-1] == 3
