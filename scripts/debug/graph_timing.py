import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import zbot_lab_amd
from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper
from zbot_lab_amd.rl.cfg import PPORunnerCfgV2
import torch.nn as nn
class _F(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())
    @staticmethod
    def backward(ctx, go):
        x, w = ctx.saved_tensors
        gx = go @ w if ctx.needs_input_grad[0] else None
        B = x.shape[0]; S = int(os.environ.get("SPLITK", "1"))
        gw = torch.bmm(go.view(S, B // S, -1).transpose(1, 2), x.view(S, B // S, -1)).sum(0)
        return gx, gw, go.sum(0)
if int(os.environ.get("SPLITK", "1")) > 1:
    def fwd(self, x):
        return _F.apply(x, self.weight, self.bias) if torch.is_grad_enabled() else nn.functional.linear(x, self.weight, self.bias)
    nn.Linear.forward = fwd
if os.environ.get("BLAS") == "rocblas":
    torch.backends.cuda.preferred_blas_library("cublas")
env_cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2"); env_cfg.scene.num_envs = 4096
env = RslRlVecEnvWrapper(zbot_lab_amd.make("zbot-6b-walking-v2", cfg=env_cfg))
r = OnPolicyRunner(env, PPORunnerCfgV2().to_dict(), log_dir=None, device="cuda:0", use_graph=True, graph_update=True)
r.learn(2)
def t(f, n=10):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
print("SPLITK", os.environ.get("SPLITK"), "BLAS", os.environ.get("BLAS"))
print("rollout graph ms", t(r._graph.replay))
print("update graph ms", t(r._update_graph.replay))
print("compute_returns ms", t(lambda: r.alg.compute_returns(r._g_obs)))
def eager():
    r.alg.update_steps()
print("eager update ms", t(eager, 3))
print("sample", float(r.alg.policy.actor[0].weight.sum()))
