#!/usr/bin/env python3
"""Train with PPO — the reference's ``scripts/rsl_rl/train.py`` flow on the MI355X simulator.

Same CLI names as the reference (``--task``, ``--num_envs``, ``--seed``, ``--max_iterations``,
``--distributed``; train.py:19-33) and the same sequence (train.py:125-205): agent cfg from the task
registry, seed + rank per process, env on ``cuda:{local_rank}``, ``RslRlVecEnvWrapper``,
``OnPolicyRunner(env, agent_cfg.to_dict(), log_dir, device)``,
``learn(max_iterations, init_at_random_ep_len=True)``. Multi-GPU: launch with
``torchrun --nproc-per-node G --master-addr 127.0.0.1 scripts/train.py --distributed``; the process
group is ``nccl`` (RCCL) on GPUs and PPO all-reduces gradients per minibatch.

Prints one JSON line per iteration (``--log-every``) and a final summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser(description="Train an RL agent with PPO (zbot_lab_amd).")
    ap.add_argument("--task", default="zbot-6b-walking-v2")
    ap.add_argument("--num_envs", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--max_iterations", type=int, default=None)
    ap.add_argument("--distributed", action="store_true")
    ap.add_argument("--log_dir", default=None)
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()

    import zbot_lab_amd
    from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper

    env_cfg = zbot_lab_amd.tasks.load_cfg(args.task)
    agent_cfg = zbot_lab_amd.tasks.load_cfg(args.task, "rsl_rl_cfg_entry_point")
    if args.num_envs is not None:
        env_cfg.scene.num_envs = args.num_envs
    if args.max_iterations is not None:
        agent_cfg.max_iterations = args.max_iterations
    if args.seed is not None:
        agent_cfg.seed = args.seed

    rank, local_rank = 0, 0
    if args.distributed:  # train.py:125-132: device per local rank, seed + rank
        import torch.distributed as dist
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if args.device == "cuda" else "gloo"
        kw = {"device_id": torch.device("cuda", local_rank)} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
        rank = dist.get_rank()
        agent_cfg.seed += rank
    device = f"cuda:{local_rank}" if args.device == "cuda" else "cpu"
    if args.device == "cuda":
        torch.cuda.set_device(local_rank)
    env_cfg.sim.device = device
    agent_cfg.device = device
    env_cfg.seed = agent_cfg.seed
    torch.manual_seed(agent_cfg.seed)

    env = zbot_lab_amd.make(args.task, cfg=env_cfg)
    env = RslRlVecEnvWrapper(env, clip_actions=agent_cfg.clip_actions)
    runner = OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=args.log_dir, device=device)
    t0 = time.perf_counter()
    done = 0
    while done < agent_cfg.max_iterations:
        n = min(args.log_every, agent_cfg.max_iterations - done)
        log = runner.learn(n, init_at_random_ep_len=(done == 0))
        done += n
        if rank == 0:
            rec = dict(log[-1])
            rec["elapsed_s"] = time.perf_counter() - t0
            print(json.dumps(rec), flush=True)
    wall = time.perf_counter() - t0
    if rank == 0:
        world = int(os.environ.get("WORLD_SIZE", "1")) if args.distributed else 1
        steps = agent_cfg.max_iterations * agent_cfg.num_steps_per_env * env.num_envs * world
        print(json.dumps({"summary": True, "iterations": agent_cfg.max_iterations, "wall_s": wall,
                          "env_steps_per_s": steps / wall, "s_per_iteration": wall / agent_cfg.max_iterations,
                          "final_mean_reward": runner.log[-1]["mean_reward"],
                          "final_mean_episode_length": runner.log[-1]["mean_episode_length"]}), flush=True)
    env.close()
    if args.distributed:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
