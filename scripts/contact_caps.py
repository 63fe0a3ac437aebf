#!/usr/bin/env python3
"""Contact-cap hit rates: how often an env-substep has more
than ZB_MAX_CONTACTS candidates (the cap selects the deepest), more than 18 self contacts, and self
contacts on overlapping cores (the separating-axis penetration estimate), per task and situation:

* stand-up from its lying start (ZBOT_6S_CFG_2, zbot_cfg.py:741-744; random actions),
* walking v2 random actions,
* trained-policy rollouts (a short PPO run of the task's own runner cfg, then the deterministic
  policy).

Needs the diagnostic build (python -m zbot_lab_amd.build --stamps; counters of zb_read_stamp_hist).
ZBOT_LIB selects another build for an A/B (e.g. one with -DZB_MAX_CONTACTS=16, with its
termination rate and stand-up outcome). Prints one JSON line per situation.
Usage (GPU box): ZBOT_LIB=libzbot_stamps.so python scripts/contact_caps.py [N] [ITERS]
"""
import ctypes as C
import json
import os
import sys
import time

os.environ.setdefault("ZBOT_LIB", "libzbot_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zbot_lab_amd  # noqa: E402
from zbot_lab_amd import _native as nat  # noqa: E402
from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper  # noqa: E402

CAP0 = 128


def read_counters():
    h = (C.c_uint64 * 136)()
    nat.check(nat.lib().zb_read_stamp_hist(h), "zb_read_stamp_hist (diagnostic build)")
    c = [int(x) for x in h[CAP0:CAP0 + 7]]
    n = max(c[0], 1)
    return {"env_substeps": c[0], "over_max_contacts": c[1] / n, "over_18_self": c[2] / n,
            "deep_self_contacts_per_env_substep": c[3] / n, "env_substeps_with_deep_self": c[4] / n,
            "self_contacts_per_env_substep": c[5] / n, "ground_candidates_per_env_substep": c[6] / n}


def rollout(env, steps, policy=None, seed=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    obs = env.get_observations()
    obs = obs["policy"] if isinstance(obs, dict) else obs
    died = 0
    for _ in range(steps):
        a = policy(obs) if policy is not None else torch.randn(env.num_envs, 6, device="cuda", generator=g)
        obs, _, dones, extras = env.step(a)
        obs = obs["policy"] if isinstance(obs, dict) else obs
        died += int((dones & ~extras["time_outs"]).sum()) if "time_outs" in extras else int(dones.sum())
    return died


def situation(task, n, label, steps, train_iters=0, seed=1):
    cfg = zbot_lab_amd.tasks.load_cfg(task)
    cfg.scene.num_envs = n
    env = RslRlVecEnvWrapper(zbot_lab_amd.make(task, cfg=cfg))
    policy, t_train = None, 0.0
    if train_iters:
        agent = zbot_lab_amd.tasks.load_cfg(task, "rsl_rl_cfg_entry_point")
        agent.max_iterations = train_iters
        agent.seed = seed
        torch.manual_seed(seed)
        runner = OnPolicyRunner(env, agent.to_dict(), log_dir=None, device="cuda:0")
        t0 = time.perf_counter()
        runner.learn(train_iters, init_at_random_ep_len=True)
        t_train = time.perf_counter() - t0
        policy = runner.get_inference_policy()
        env.reset()
    torch.cuda.synchronize()
    read_counters()  # reset after construction / training
    with torch.no_grad():
        died = rollout(env, steps, policy, seed)
    torch.cuda.synchronize()
    rec = dict(task=task, situation=label, envs=n, steps=steps, train_iterations=train_iters,
               train_s=round(t_train, 1), lib=os.environ["ZBOT_LIB"],
               died_per_1000_env_steps=1000.0 * died / (n * steps), **read_counters())
    print(json.dumps(rec), flush=True)
    env.close()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    situation("zbot-6b-standup-v0", n, "lying start, random actions (first 50 steps)", 50)
    situation("zbot-6b-walking-v2", n, "random actions", 300)
    situation("zbot-6b-standup-v0", n, "trained policy", 300, train_iters=iters)
    situation("zbot-6b-walking-v2", n, "trained policy", 300, train_iters=iters)


if __name__ == "__main__":
    main()
