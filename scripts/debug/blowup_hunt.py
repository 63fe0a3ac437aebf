"""Train like scripts/train.py (HIP graphs on) and catch the first env step whose state blows up:
every step's pre-step state and actions are recorded into a ring inside the rollout graph; after
each iteration the final state is checked; the offending step's inputs go to gpurun_out/blowup.npz."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import zbot_lab_amd
from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper
from zbot_lab_amd.tasks import load_cfg
task = os.environ.get("TASK", "zbot-6b-standup-v0")
cfg = load_cfg(task); cfg.scene.num_envs = int(os.environ.get("N", "4096"))
agent = load_cfg(task, "rsl_rl_cfg_entry_point")
agent.seed = int(os.environ.get("SEED", agent.seed))
cfg.seed = agent.seed
torch.manual_seed(agent.seed)
env = zbot_lab_amd.make(task, cfg=cfg)
T = agent.num_steps_per_env
N = env.num_envs
D = env.sim.state_dim
ring = torch.zeros(T, D, N, device="cuda:0")
acts = torch.zeros(T, N, 6, device="cuda:0")
k = [0]
orig = env.step
def step(a):
    ring[k[0] % T].copy_(env.sim.get_state()); acts[k[0] % T].copy_(a); k[0] += 1
    return orig(a)
env.step = step
def bad_of(st):
    return (~torch.isfinite(st).all(0)) | (st.abs().max(0).values > 1e3)
r = OnPolicyRunner(RslRlVecEnvWrapper(env), agent.to_dict(), log_dir=None, device="cuda:0")
for it in range(int(os.environ.get("ITERS", "400"))):
    r.learn(1, init_at_random_ep_len=(it == 0))
    fin = env.sim.get_state()
    b = bad_of(fin)
    if bool(b.any()):
        for t in range(T):
            post = ring[t + 1] if t + 1 < T else fin
            bb = bad_of(post) & ~bad_of(ring[t])
            if bool(bb.any()):
                ids = torch.nonzero(bb).flatten()[:32]
                print(f"blow-up: iteration {it} step {t} envs {ids.tolist()}", flush=True)
                np.savez("gpurun_out/blowup.npz", pre=ring[t][:, ids].cpu().numpy(), post=post[:, ids].cpu().numpy(),
                         actions=acts[t][ids].cpu().numpy(), ids=ids.cpu().numpy(), it=it, t=t,
                         prev=ring[t - 1][:, ids].cpu().numpy() if t > 0 else ring[t][:, ids].cpu().numpy(),
                         prev_actions=acts[t - 1][ids].cpu().numpy() if t > 0 else acts[t][ids].cpu().numpy(),
                         ring=ring[:, :, ids].cpu().numpy(), ring_actions=acts[:, ids].cpu().numpy())
                sys.exit(0)
        print("bad at iteration start?", it, flush=True)
        sys.exit(1)
    if it % 25 == 0:
        print(it, r.log[-1]["mean_reward"], r.log[-1]["mean_noise_std"], flush=True)
print("no blow-up")
