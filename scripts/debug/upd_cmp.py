import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import zbot_lab_amd
from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper
from zbot_lab_amd.tasks import load_cfg
task = os.environ.get("TASK", "zbot-6b-standup-v0")
cfg = load_cfg(task); cfg.scene.num_envs = 4096
env = RslRlVecEnvWrapper(zbot_lab_amd.make(task, cfg=cfg))
agent = load_cfg(task, "rsl_rl_cfg_entry_point")
r = OnPolicyRunner(env, agent.to_dict(), log_dir=None, device="cuda:0", use_graph=True, graph_update=True)
r.learn(1, init_at_random_ep_len=True)
alg = r.alg
params = list(alg.policy.parameters())
def snapshot():
    st = [{k: v.clone() for k, v in alg.optimizer.state[p].items()} for p in params]
    return [p.detach().clone() for p in params], st, alg.lr_t.clone()
def restore(snap):
    ps, st, lr = snap
    with torch.no_grad():
        for p, v, s_ in zip(params, ps, st):
            p.copy_(v)
            for k, t in s_.items():
                alg.optimizer.state[p][k].copy_(t)
        alg.lr_t.copy_(lr)
cur = lambda: torch.cat([p.detach().flatten() for p in params]).clone()
for it in range(8):
    with torch.no_grad():
        r._graph.replay()
        alg.compute_returns(r._g_obs)
    alg.draw_minibatch_indices()
    snap = snapshot()
    r._update_graph.replay(); alg.storage.clear(); torch.cuda.synchronize(); g = cur(); lrg = float(alg.lr_t)
    restore(snap); alg.update_steps(); torch.cuda.synchronize(); e = cur(); lre = float(alg.lr_t)
    print(it, "graph-eager max", float((g - e).abs().max()), "moved", float((e - torch.cat([v.flatten() for v in snap[0]])).abs().max()), "lr", lrg, lre, "std", float(alg.policy.std.mean()), flush=True)
