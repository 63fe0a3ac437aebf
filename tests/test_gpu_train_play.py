"""The reference's train -> resume -> play recipe end to end on the MI355X simulator (§8(f)1:
train.py:165-166,193-205, play.py:150-200): a short run, a resumed run that continues the
iteration counter from the newest checkpoint, cfg dumps, then play with the TorchScript export,
whose output must match ``act_inference``."""
from __future__ import annotations

import importlib.util
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "scripts", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_train_resume_play(gpu, tmp_path):
    train, play = _script("train"), _script("play")
    root = str(tmp_path / "logs")
    common = ["--task", "zbot-6b-walking-v2", "--num_envs", "512", "--log_root", root, "--log-every", "100"]
    s1 = train.main(common + ["--max_iterations", "3", "--run_name", "step1"])
    assert s1["last_iteration"] == 3 and s1["resumed_from"] is None
    assert os.path.exists(os.path.join(s1["log_dir"], "model_3.pt"))
    assert os.path.exists(os.path.join(s1["log_dir"], "params", "agent.yaml"))
    s2 = train.main(common + ["--max_iterations", "2", "--run_name", "step2", "--resume", "--load_run", ".*step1"])
    assert s2["resumed_from"].endswith(os.path.join(os.path.basename(s1["log_dir"]), "model_3.pt"))
    assert s2["last_iteration"] == 5
    assert os.path.exists(os.path.join(s2["log_dir"], "model_5.pt"))
    out = play.main(["--task", "zbot-6b-walking-v2", "--num_envs", "256", "--log_root", root, "--num_steps", "60"])
    assert out["checkpoint"].endswith("model_5.pt")
    assert out["exported_jit"] and os.path.exists(out["exported_jit"])
    m = torch.jit.load(out["exported_jit"]).cuda()
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2, RslRlVecEnvWrapper
    import zbot_lab_amd
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    cfg.scene.num_envs = 64
    env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-walking-v2", cfg=cfg))
    r = OnPolicyRunner(env, PPORunnerCfgV2().to_dict(), log_dir=None, device="cuda:0", use_graph=False)
    r.load(out["checkpoint"])
    pol = r.get_inference_policy()
    obs = env.get_observations()["policy"]
    with torch.inference_mode():  # bitwise on the CPU (test_resume_export); a TorchScript fuser may
        torch.testing.assert_close(m(obs), pol(obs), rtol=1e-6, atol=1e-6)  # re-fuse ELU on the GPU
    env.close()
