#!/usr/bin/env python3
"""Train with PPO — the reference's ``scripts/rsl_rl/train.py`` flow on the MI355X simulator.

Same CLI names as the reference (``--task``, ``--num_envs``, ``--seed``, ``--max_iterations``,
``--distributed``, train.py:19-33; rsl_rl group ``--experiment_name --run_name --resume --load_run
--checkpoint``, cli_args.py:16-40) and the same sequence (train.py:110-205):

* agent cfg from the task registry, CLI overrides (cli_args.py:60-90), seed + rank per process;
* log dir ``logs/rsl_rl/<experiment_name>/<%Y-%m-%d_%H-%M-%S>[_<run_name>]`` (train.py:138-147);
* with ``--resume`` the checkpoint is resolved *before* the new log dir exists
  (``get_checkpoint_path(log_root, load_run, load_checkpoint)``, train.py:165-166) and loaded into
  the runner (train.py:193-196): weights, optimizer state, learning rate and iteration counter;
* ``params/env.yaml`` and ``params/agent.yaml`` dumps (train.py:199-200; the pickles are skipped);
* ``runner.learn(max_iterations, init_at_random_ep_len=True)`` (train.py:205), one call.

Multi-GPU: ``torchrun --nproc-per-node G --master-addr 127.0.0.1 scripts/train.py --distributed``;
the process group is ``nccl`` (RCCL) on GPUs and PPO all-reduces gradients per minibatch.
Prints one JSON line every ``--log-every`` iterations (and appends every iteration's record to
``<log_dir>/train_log.jsonl``) and a final summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import datetime

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import zbot_lab_amd  # noqa: E402,F401  (before torch: sets HIP's graph capture mode, zbot_lab_amd/__init__.py)
import torch  # noqa: E402



def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Train an RL agent with PPO (zbot_lab_amd).")
    ap.add_argument("--task", default="zbot-6b-walking-v2")
    ap.add_argument("--num_envs", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--max_iterations", type=int, default=None)
    ap.add_argument("--distributed", action="store_true")
    ap.add_argument("--device", default="cuda")
    g = ap.add_argument_group("rsl_rl")
    g.add_argument("--experiment_name", default=None)
    g.add_argument("--run_name", default=None)
    g.add_argument("--resume", action="store_true", default=False)
    g.add_argument("--load_run", default=None)
    g.add_argument("--checkpoint", default=None)
    ap.add_argument("--log_root", default=os.path.join("logs", "rsl_rl"),
                    help="parent of the experiment folders (reference: logs/rsl_rl)")
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--reward_cfg", default=None,
                    help="zbot-6b-walking-v2 reward stage (step0 / step1 / step1_v1 / step1_v2 / step2 / step3 / step4 = v2.py:77-206); the reference "
                         "edits the active reward_cfg in v2.py between its chained 2000-iteration runs")
    ap.add_argument("--env", action="append", default=[], metavar="PATH=VALUE",
                    help="env cfg override by dotted path, e.g. solver.iterations=8 (simulator ablations)")
    return ap


def update_rsl_rl_cfg(agent_cfg, args):
    """cli_args.update_rsl_rl_cfg (cli_args.py:60-90)."""
    if args.seed is not None:
        if args.seed == -1:
            import random
            args.seed = random.randint(0, 10000)
        agent_cfg.seed = args.seed
    if args.resume:
        agent_cfg.resume = True
    if args.load_run is not None:
        agent_cfg.load_run = args.load_run
    if args.checkpoint is not None:
        agent_cfg.load_checkpoint = args.checkpoint
    if args.run_name is not None:
        agent_cfg.run_name = args.run_name
    if args.experiment_name is not None:
        agent_cfg.experiment_name = args.experiment_name
    return agent_cfg


def main(argv=None) -> dict:
    args = build_parser().parse_args(argv)

    import zbot_lab_amd
    from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper, dump_yaml, get_checkpoint_path

    env_cfg = zbot_lab_amd.tasks.load_cfg(args.task)
    agent_cfg = update_rsl_rl_cfg(zbot_lab_amd.tasks.load_cfg(args.task, "rsl_rl_cfg_entry_point"), args)
    if args.num_envs is not None:
        env_cfg.scene.num_envs = args.num_envs
    if args.max_iterations is not None:
        agent_cfg.max_iterations = args.max_iterations
    if args.reward_cfg is not None:
        from zbot_lab_amd.envs.walking_v2 import REWARD_CFGS
        env_cfg.reward_cfg = REWARD_CFGS[args.reward_cfg]
    zbot_lab_amd.tasks.apply_env_overrides(env_cfg, args.env)

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

    log_root_path = os.path.abspath(os.path.join(args.log_root, agent_cfg.experiment_name))
    log_dir = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    if agent_cfg.run_name:
        log_dir += f"_{agent_cfg.run_name}"
    log_dir = os.path.join(log_root_path, log_dir)
    resume_path = None
    if agent_cfg.resume:  # resolved before this run's folder exists (train.py:165-166)
        resume_path = get_checkpoint_path(log_root_path, agent_cfg.load_run, agent_cfg.load_checkpoint)

    env = zbot_lab_amd.make(args.task, cfg=env_cfg)
    env = RslRlVecEnvWrapper(env, clip_actions=agent_cfg.clip_actions)
    runner = OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=log_dir if rank == 0 else None, device=device)
    if resume_path is not None:
        if rank == 0:
            print(f"[INFO]: Loading model checkpoint from: {resume_path}", flush=True)
        runner.load(resume_path)
    if rank == 0:
        dump_yaml(os.path.join(log_dir, "params", "env.yaml"), env_cfg)
        dump_yaml(os.path.join(log_dir, "params", "agent.yaml"), agent_cfg)
        print(f"[INFO] Logging experiment in directory: {log_dir}", flush=True)

    t0 = time.perf_counter()
    jsonl = open(os.path.join(log_dir, "train_log.jsonl"), "a") if rank == 0 else None
    start = runner.current_learning_iteration

    def on_iteration(rec: dict) -> None:
        if jsonl is None:
            return
        rec = dict(rec, elapsed_s=time.perf_counter() - t0)
        jsonl.write(json.dumps(rec) + "\n")
        k = rec["iteration"] - start + 1
        if k % args.log_every == 0 or k == agent_cfg.max_iterations:
            jsonl.flush()
            print(json.dumps(rec), flush=True)

    runner.learn(num_learning_iterations=agent_cfg.max_iterations, init_at_random_ep_len=True,
                 callback=on_iteration)
    wall = time.perf_counter() - t0
    summary = {}
    if rank == 0:
        jsonl.close()
        world = int(os.environ.get("WORLD_SIZE", "1")) if args.distributed else 1
        steps = agent_cfg.max_iterations * agent_cfg.num_steps_per_env * env.num_envs * world
        summary = {"summary": True, "log_dir": log_dir, "resumed_from": resume_path,
                   "iterations": agent_cfg.max_iterations, "last_iteration": runner.current_learning_iteration,
                   "wall_s": wall, "env_steps_per_s": steps / wall, "s_per_iteration": wall / agent_cfg.max_iterations,
                   "final_mean_reward": runner.log[-1]["mean_reward"],
                   "final_mean_episode_length": runner.log[-1]["mean_episode_length"]}
        print(json.dumps(summary), flush=True)
    env.close()
    if args.distributed:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return summary


if __name__ == "__main__":
    main()
