"""Host-side API mirrors of the reference interfaces: registry, DirectRLEnv 5-tuple, rsl_rl VecEnv.

CPU part: the wrapper / registry logic on a fake env. GPU part (marked): the real env."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import zbot_lab_amd
from zbot_lab_amd import model as zm
from zbot_lab_amd.rl import PPORunnerCfgV2, RslRlVecEnvWrapper
from zbot_lab_amd.tasks import load_cfg, spec


class FakeEnv:
    def __init__(self, n=4):
        self.num_envs = n
        self.device = torch.device("cpu")
        self.max_episode_length = 1000
        self.cfg = object()
        from zbot_lab_amd import spaces
        self.single_action_space = spaces.Box(-np.inf, np.inf, (6,))
        self._ep = torch.zeros(n, dtype=torch.long)
        self.last_action = None

    @property
    def unwrapped(self):
        return self

    @property
    def episode_length_buf(self):
        return self._ep

    @episode_length_buf.setter
    def episode_length_buf(self, v):
        self._ep = v

    def reset(self):
        return {"policy": torch.zeros(self.num_envs, 23)}, {}

    def get_observations(self):
        return {"policy": torch.zeros(self.num_envs, 23)}

    def step(self, a):
        self.last_action = a
        term = torch.tensor([True, False, False, False])
        trunc = torch.tensor([False, True, False, False])
        return {"policy": torch.ones(self.num_envs, 23)}, torch.ones(self.num_envs), term, trunc, {"log": {}}

    def seed(self, s):
        return s

    def close(self):
        pass


def test_registry_matches_reference_registration():
    assert "zbot-6b-walking-v2" in zbot_lab_amd.registered()
    s = spec("zbot-6b-walking-v2")
    assert s.entry_point.endswith("ZbotDirectEnvV2")
    cfg = load_cfg("zbot-6b-walking-v2")
    assert cfg.decimation == 4 and cfg.action_space == 6 and cfg.observation_space == 23
    assert cfg.scene.num_envs == 4096 and cfg.scene.env_spacing == 4.0
    assert abs(cfg.sim.dt - 1 / 200) < 1e-12 and cfg.termination_height == 0.22
    assert list(cfg.reward_cfg["reward_scales"]) == zm.REWARD_TERMS[:13]   # step4 (v2.py:190-206)
    agent = load_cfg("zbot-6b-walking-v2", "rsl_rl_cfg_entry_point")
    assert isinstance(agent, PPORunnerCfgV2)
    d = agent.to_dict()
    assert d["num_steps_per_env"] == 24 and d["policy"]["actor_hidden_dims"] == [128, 128, 128]
    assert d["algorithm"]["desired_kl"] == 0.01 and d["algorithm"]["num_mini_batches"] == 4


def test_standup_registration_and_cfg():
    """zbot-6b-standup-v0 (reference __init__.py:111-119, Zbot6SUpEnvCfg standup.py:191-447)."""
    from zbot_lab_amd.rl import Zbot6SUpEnvPPOCfg
    s = spec("zbot-6b-standup-v0")
    assert s.entry_point.endswith("Zbot6SUpEnv")
    cfg = load_cfg("zbot-6b-standup-v0")
    assert cfg.episode_length_s == 6.0 and cfg.observation_space == 22 and cfg.action_space == 6
    assert list(cfg.reward_cfg["reward_scales"]) == zm.SU_REWARD_TERMS
    pm = cfg.events.physics_material.params
    assert pm["static_friction_range"] == (0.6, 1.0) and pm["num_buckets"] == 64
    t = cfg.task_cfg()
    assert t.task == zm.TASK_STANDUP_V0 and t.max_episode_length == 300 and t.terminal_penalty == 2.0
    c = t.pack()
    assert c.num_stages == 2 and c.stage_steps[1] == 24000 and c.task == 1
    assert list(c.stage_scales[0][:4]) == [10.0, -1.0, -1.0, 0.0]     # weights; x step_dt in the kernel
    assert list(c.stage_scales[1][:4]) == [10.0, -2.0, -1.0, 2.0]
    np.testing.assert_allclose(np.array(c.reset_pose_range), [[-0.5, 0.5], [-0.5, 0.5], [-0.7854, 0.7854],
                                                              [-3.14, 3.14]], rtol=1e-6)
    cfg.events.my_curric = None                                       # play-script variant: no curriculum
    assert cfg.task_cfg().pack().num_stages == 1
    agent = load_cfg("zbot-6b-standup-v0", "rsl_rl_cfg_entry_point")
    assert isinstance(agent, Zbot6SUpEnvPPOCfg)
    assert agent.to_dict()["policy"]["actor_hidden_dims"] == [256, 256, 128]
    assert agent.experiment_name == "zbot_6b_flat_direct_standup"


def test_walking_v4_registration_and_cfg():
    """zbot-6b-walking-v4 (reference __init__.py:91-99, Zbot6SEnvV4Cfg v4.py:443-686)."""
    from zbot_lab_amd.rl import Zbot6SEnvV4PPOCfg
    assert spec("zbot-6b-walking-v4").entry_point.endswith("Zbot6SEnvV4")
    cfg = load_cfg("zbot-6b-walking-v4")
    assert cfg.observation_space == 24 and cfg.contact_history_length == 3 and cfg.termination_height == 0.20
    assert list(cfg.reward_cfg["reward_scales"]) == zm.V4_REWARD_TERMS
    c = cfg.task_cfg().pack()
    assert c.task == zm.TASK_WALKING_V4 and c.num_stages == 4 and list(c.stage_steps) == [0, 12000, 24000, 144000]
    assert list(c.stage_prob_pos) == pytest.approx([1.0, 1.0, 0.8, 0.6])
    assert (c.range_start_steps, c.range_period_steps, c.range_min_buffer) == (48000, 12000, 20)
    assert list(c.range_limit_yaw) == [-0.5, 0.5] and c.undesired_force_threshold == 0.5
    assert list(c.cmd_vel_range) == pytest.approx([0.3, 0.3]) and c.reset_pose_body_frame == 1
    agent = load_cfg("zbot-6b-walking-v4", "rsl_rl_cfg_entry_point")
    assert isinstance(agent, Zbot6SEnvV4PPOCfg) and agent.max_iterations == 2000
    assert agent.to_dict()["policy"]["critic_hidden_dims"] == [256, 256, 128]


def test_manager_registration_and_cfg():
    """zbot-6b-walking-m-v0 / -m-play-v0 (zbotlab_manager/config/zbot6b_manager/__init__.py:18-36):
    the manager cfg compiles to TaskCfg.manager_flat(); unsupported terms raise instead of being
    dropped; Zbot6BFlatPPORunnerCfg (agents/rsl_rl_ppo_cfg.py:40-49)."""
    import dataclasses
    from zbot_lab_amd import model as zm
    from zbot_lab_amd.envs.manager_flat import DoneTerm, EventTerm, RewTerm
    assert {"zbot-6b-walking-m-v0", "zbot-6b-walking-m-play-v0"} <= set(zbot_lab_amd.tasks.registered())
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-m-v0")
    # (the env's solver default is the product configuration, DESIGN.md §3.6: TGS, mode 1; the raw ABI
    # mirror TaskCfg keeps the C struct's PGS default)
    assert dataclasses.asdict(cfg.task_cfg()) == dataclasses.asdict(zm.TaskCfg.manager_flat(solver_mode=1))
    assert cfg.task_cfg().self_manifold == 2
    cfg.rewards.feet_slide.weight = -3.0
    cfg.commands.base_velocity.ranges.lin_vel_x = (-0.2, 0.2)
    t = cfg.task_cfg()
    assert t.reward_weights["feet_slide"] == -3.0 and t.cmd_vel_range == (-0.2, 0.2)
    play = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-m-play-v0")
    assert play.scene.num_envs == 64 and not play.task_cfg().obs_corruption
    assert play.task_cfg().cmd_vel_range == (-0.3, 0.3)
    for edit in (lambda c: setattr(c.rewards, "gait", RewTerm("feet_gait", 0.5)),
                 lambda c: setattr(c.terminations, "base_contact", DoneTerm("illegal_contact")),
                 lambda c: setattr(c.events, "push_robot", EventTerm("push_by_setting_velocity", "interval")),
                 lambda c: setattr(c.rewards.track_lin_vel_xy_exp, "params", {"std": 0.4}),
                 lambda c: setattr(c.commands.base_velocity, "heading_command", True)):
        c = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-m-v0")
        edit(c)
        with pytest.raises(NotImplementedError):
            c.task_cfg()
    c = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-m-v0")
    c.curriculum.lin_vel_cmd_levels = None
    assert c.task_cfg().pack().range_period_steps <= 0
    ppo = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-m-v0", "rsl_rl_cfg_entry_point").to_dict()
    assert ppo["max_iterations"] == 1000 and ppo["experiment_name"] == "zbot_6b_flat_mana_v1"
    assert ppo["policy"]["actor_hidden_dims"] == [128, 128, 128] and ppo["algorithm"]["entropy_coef"] == 0.01


def test_vecenv_wrapper_contract():
    env = FakeEnv()
    w = RslRlVecEnvWrapper(env, clip_actions=1.0)
    assert w.num_envs == 4 and w.num_actions == 6 and w.max_episode_length == 1000
    obs, rew, dones, extras = w.step(torch.full((4, 6), 3.0))
    assert torch.equal(dones, torch.tensor([1, 1, 0, 0]))
    assert torch.equal(extras["time_outs"], torch.tensor([False, True, False, False]))
    assert env.last_action.max() == 1.0           # clip_actions applied
    w.episode_length_buf = torch.full((4,), 7)
    assert (w.episode_length_buf == 7).all()
    assert w.get_observations()["policy"].shape == (4, 23)


def test_grid_env_origins():
    from zbot_lab_amd.envs import grid_env_origins
    o = grid_env_origins(16, 4.0)
    assert o.shape == (16, 3)
    d = torch.cdist(o, o) + torch.eye(16) * 100
    assert abs(d.min().item() - 4.0) < 1e-6


@pytest.mark.gpu
def test_env_step_contract_gpu(gpu):
    env = zbot_lab_amd.make("zbot-6b-walking-v2", num_envs=256)
    obs, extras = env.reset()
    assert obs["policy"].shape == (256, 23) and obs["policy"].device.type == "cuda"
    ep = env.episode_length_buf
    assert ep.dtype == torch.long and 0 <= ep.min() and ep.max() <= 999 and len(ep.unique()) > 100
    term_buf = env.reset_terminated
    for _ in range(50):
        a = torch.randn(256, 6, device="cuda")
        obs, rew, term, trunc, extras = env.step(a)
    assert term is term_buf                              # persistent, mutated in place
    assert rew.shape == (256,) and rew.dtype == torch.float32 and torch.isfinite(rew).all()
    assert term.dtype == torch.bool and trunc.dtype == torch.bool
    assert set(extras["log"]) >= {"Episode_Reward/step_length", "Episode_Termination/body_contact"}
    assert torch.allclose(obs["policy"][:, 22], torch.ones(256, device="cuda"))
    env.episode_length_buf = torch.full((256,), 998, device="cuda")
    _, _, _, trunc, _ = env.step(torch.zeros(256, 6, device="cuda"))
    assert trunc.all()                                   # 998 + 1 >= max_episode_length - 1
    w = RslRlVecEnvWrapper(env)
    o, r, d, ex = w.step(torch.zeros(256, 6, device="cuda"))
    assert d.dtype == torch.long and "time_outs" in ex
    env.close()
