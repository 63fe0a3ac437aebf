"""§8(f)1 remainder on CPU: checkpoint resolution (``get_checkpoint_path`` as train.py:165-166 /
play.py:110 call it), resume round trip (iteration counter, weights, Adam moments, learning rate),
the adaptive learning rate after a load, the TorchScript export of play.py:172-174, and
the cfg YAML dumps of train.py:199-200."""
from __future__ import annotations

import os

import pytest
import torch
import yaml

from test_ppo import ToyVecEnv
from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2, dump_yaml, export_policy_as_jit, get_checkpoint_path


def _touch(p):
    os.makedirs(os.path.dirname(p), exist_ok=True)
    open(p, "w").close()


def test_get_checkpoint_path_picks_newest_run_and_highest_model(tmp_path):
    root = tmp_path / "exp"
    for run in ("2025-01-01_10-00-00", "2025-01-02_09-00-00_step2", "2024-12-31_23-59-59"):
        for it in (0, 50, 999, 1000):
            _touch(str(root / run / f"model_{it}.pt"))
    _touch(str(root / "2025-01-02_09-00-00_step2" / "params" / "env.yaml"))
    p = get_checkpoint_path(str(root), ".*", "model_.*.pt")
    assert p.endswith(os.path.join("2025-01-02_09-00-00_step2", "model_1000.pt"))  # 1000 after 999
    p = get_checkpoint_path(str(root), "2025-01-01.*", "model_50.pt")
    assert p.endswith(os.path.join("2025-01-01_10-00-00", "model_50.pt"))
    with pytest.raises(ValueError):
        get_checkpoint_path(str(root), "nope.*")
    with pytest.raises(ValueError):
        get_checkpoint_path(str(tmp_path / "missing"))


def _runner(log_dir=None, seed=0):
    torch.manual_seed(seed)
    cfg = PPORunnerCfgV2()
    cfg.num_steps_per_env = 8
    cfg.save_interval = 1000
    return OnPolicyRunner(ToyVecEnv(n=32), cfg.to_dict(), log_dir=log_dir, device="cpu")


def test_resume_round_trip_restores_iteration_weights_optimizer_and_lr(tmp_path):
    r1 = _runner(str(tmp_path))
    r1.learn(6)
    lr1 = r1.alg.learning_rate
    ck = tmp_path / "model_6.pt"
    assert ck.exists()
    r2 = _runner(None, seed=123)  # different init: everything must come from the checkpoint
    r2.load(str(ck))
    assert r2.current_learning_iteration == 6
    for a, b in zip(r1.alg.policy.state_dict().values(), r2.alg.policy.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    s1, s2 = r1.alg.optimizer.state_dict()["state"], r2.alg.optimizer.state_dict()["state"]
    for k in s1:
        for name in ("exp_avg", "exp_avg_sq", "step"):
            torch.testing.assert_close(torch.as_tensor(s1[k][name]), torch.as_tensor(s2[k][name]), rtol=0, atol=0)
    assert r2.alg.learning_rate == pytest.approx(lr1, rel=0, abs=0)
    assert r2.alg.optimizer.param_groups[0]["lr"] == pytest.approx(lr1, rel=0, abs=0)
    log = r2.learn(2)  # continues the iteration counter like rsl_rl
    assert [rec["iteration"] for rec in log] == [6, 7]
    assert r2.current_learning_iteration == 8


def test_learning_rate_applied_after_load_follows_adaptive_rule(tmp_path):
    """after load the rate Adam applies must be the one the adaptive-KL rule updates."""
    r1 = _runner(str(tmp_path))
    r1.learn(2)
    r2 = _runner(None)
    r2.load(str(tmp_path / "model_2.pt"))
    alg = r2.alg
    lr0 = alg.learning_rate
    with torch.no_grad():
        obs = r2.env.get_observations()["policy"]
        for _ in range(r2.num_steps_per_env):
            alg.act(obs, obs)
            alg._tr["mu"] = alg._tr["mu"] + 10.0  # force a large KL: lr / 1.5 per minibatch
            alg.process_env_step(torch.randn(32), torch.zeros(32), {})
        alg.compute_returns(obs)
    alg.update()
    n_mb = alg.num_learning_epochs * alg.num_mini_batches
    expect = max(lr0 / 1.5 ** n_mb, 1e-5)
    assert alg.learning_rate == pytest.approx(expect, rel=1e-5)
    applied = alg.optimizer.param_groups[0]["lr"]
    assert float(applied) == pytest.approx(alg.learning_rate, rel=1e-6)


def test_jit_export_equals_act_inference_bitwise(tmp_path):
    r = _runner(None)
    r.learn(2)
    pol = r.get_inference_policy()
    path = export_policy_as_jit(r.alg.policy, None, str(tmp_path / "exported"), "policy.pt")
    m = torch.jit.load(path)
    obs = torch.randn(257, 23, generator=torch.Generator().manual_seed(3))
    with torch.inference_mode():
        torch.testing.assert_close(m(obs), pol(obs), rtol=0, atol=0)
    m.reset()


def test_dump_yaml_of_env_and_agent_cfg(tmp_path):
    from zbot_lab_amd.envs.walking_v2 import ZbotDirectEnvCfgV2
    dump_yaml(str(tmp_path / "params" / "env.yaml"), ZbotDirectEnvCfgV2())
    dump_yaml(str(tmp_path / "params" / "agent.yaml"), PPORunnerCfgV2())
    env = yaml.safe_load(open(tmp_path / "params" / "env.yaml"))
    agent = yaml.safe_load(open(tmp_path / "params" / "agent.yaml"))
    assert env["decimation"] == 4 and env["episode_length_s"] == 20.0
    assert agent["num_steps_per_env"] == 24 and agent["algorithm"]["learning_rate"] == 1e-3
    assert agent["load_checkpoint"] == "model_.*.pt"
