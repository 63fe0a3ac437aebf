#!/usr/bin/env python3
"""Play a trained policy — the reference's ``scripts/rsl_rl/play.py`` flow on the MI355X simulator.

Sequence (play.py:85-200): resolve the checkpoint (``--checkpoint <file>``, else
``get_checkpoint_path(logs/rsl_rl/<experiment>, --load_run, load_checkpoint)``), build the env and
``RslRlVecEnvWrapper``, ``OnPolicyRunner(..., log_dir=None)``, ``runner.load``,
``runner.get_inference_policy``, export the actor to ``<run>/exported/policy.pt`` with
``export_policy_as_jit`` (ONNX needs the absent ``onnx`` package), then roll the policy out under
``torch.inference_mode``. There is no viewer, so the loop runs ``--num_steps`` steps and prints one
JSON summary: mean reward per step, finished episodes (length, return, termination split) and the
gait: the root's mean forward (+x, the heading the v2 rewards hold, v2.py:320-327) velocity and the
mean forward distance per finished episode.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import zbot_lab_amd  # noqa: E402,F401  (before torch: sets HIP's graph capture mode, zbot_lab_amd/__init__.py)
import torch  # noqa: E402



def _posture(env, st, max_envs: int = 512) -> dict:
    """Posture at the end of the rollout from the final states (the robot model's FK on the host):
    base link height (v2 dies below 0.22 m, v2.py:405; the stand-up task's standing height) and
    how upright the feet are (foot z axis . world z; foot_1's sole normal is -z, v2.py:341-343)."""
    import numpy as np

    from zbot_lab_amd import model as zm
    rm = env.sim.robot
    n = min(st.shape[1], max_envs)
    bz, up = [], []
    for e in range(n):
        _, links = rm.fk(st[0:3, e], st[3:7, e], st[13:19, e])
        bz.append(links[rm.base_link].p[2])
        up.append([zm.qrot(links[li].q, np.array([0.0, 0.0, sg]))[2] for li, sg in ((0, 1.0), (11, -1.0))])
    bz, up = np.asarray(bz), np.asarray(up)
    return {"final_base_z_mean": float(bz.mean()), "final_base_z_quantiles_10_50_90": np.quantile(bz, [0.1, 0.5, 0.9]).tolist(),
            "final_frac_base_z_ge_0.20": float((bz >= 0.20).mean()),
            "final_feet_up_alignment_mean": up.mean(axis=0).tolist(), "posture_envs": n}


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser(description="Play a checkpoint of an RL agent (zbot_lab_amd).")
    ap.add_argument("--task", default="zbot-6b-walking-v2")
    ap.add_argument("--num_envs", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--experiment_name", default=None)
    ap.add_argument("--load_run", default=None)
    ap.add_argument("--checkpoint", default=None, help="checkpoint file (else resolved under the log root)")
    ap.add_argument("--log_root", default=os.path.join("logs", "rsl_rl"))
    ap.add_argument("--num_steps", type=int, default=1000)
    ap.add_argument("--env", action="append", default=[], metavar="PATH=VALUE",
                    help="env cfg override by dotted path (as scripts/train.py --env)")
    ap.add_argument("--no_export", action="store_true")
    ap.add_argument("--fresh_episodes", action="store_true",
                    help="start every env at episode step 0 (the posture summary then describes step --num_steps)")
    args = ap.parse_args(argv)

    import zbot_lab_amd
    from zbot_lab_amd import model as zm
    from zbot_lab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper, export_policy_as_jit, get_checkpoint_path

    env_cfg = zbot_lab_amd.tasks.load_cfg(args.task)
    agent_cfg = zbot_lab_amd.tasks.load_cfg(args.task, "rsl_rl_cfg_entry_point")
    if args.num_envs is not None:
        env_cfg.scene.num_envs = args.num_envs
    zbot_lab_amd.tasks.apply_env_overrides(env_cfg, args.env)
    if args.seed is not None:
        agent_cfg.seed = args.seed
    if args.experiment_name is not None:
        agent_cfg.experiment_name = args.experiment_name
    if args.load_run is not None:
        agent_cfg.load_run = args.load_run
    device = "cuda:0" if args.device == "cuda" else args.device
    env_cfg.sim.device = device
    agent_cfg.device = device
    env_cfg.seed = agent_cfg.seed

    log_root_path = os.path.abspath(os.path.join(args.log_root, agent_cfg.experiment_name))
    if args.checkpoint and os.path.isfile(args.checkpoint):
        resume_path = os.path.abspath(args.checkpoint)
    else:
        if args.checkpoint:
            agent_cfg.load_checkpoint = args.checkpoint
        resume_path = get_checkpoint_path(log_root_path, agent_cfg.load_run, agent_cfg.load_checkpoint)
    print(f"[INFO]: Loading model checkpoint from: {resume_path}", flush=True)

    env = RslRlVecEnvWrapper(zbot_lab_amd.make(args.task, cfg=env_cfg), clip_actions=agent_cfg.clip_actions)
    runner = OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=None, device=agent_cfg.device)
    runner.load(resume_path)
    policy = runner.get_inference_policy(device=env.unwrapped.device)
    exported = None
    if not args.no_export:
        exported = export_policy_as_jit(runner.alg.policy, normalizer=None,
                                        path=os.path.join(os.path.dirname(resume_path), "exported"),
                                        filename="policy.pt")

    sim = env.unwrapped.sim
    n = env.num_envs
    dt = env.unwrapped.step_dt
    x_row = zm.S["ROOT_POS"]
    if args.fresh_episodes:
        env.unwrapped.episode_length_buf = torch.zeros_like(env.unwrapped.episode_length_buf)
    obs = env.get_observations()
    obs = obs["policy"] if hasattr(obs, "keys") else obs
    x_prev = sim.get_state()[x_row].clone()
    x_start = x_prev.clone()
    rew_sum = torch.zeros((), device=sim.device)
    ep_ret = torch.zeros(n, device=sim.device)
    ep_len = torch.zeros(n, device=sim.device)
    fin = torch.zeros(5, device=sim.device)  # episodes, length sum, return sum, distance sum, time-outs
    vel_sum = torch.zeros((), device=sim.device)
    vel_cnt = torch.zeros((), device=sim.device)
    # walking v2's contact sensor (state rows FEET_AIR_CUR / FEET_AIR_LAST): the gait's air time --
    # foot-steps in the air, touchdowns (last_air_time refreshed) and the air time they end
    gait = sim.state_dim == zm.STATE_DIM and args.task.startswith("zbot-6b-walking-v2")
    air = torch.zeros(3, device=sim.device)  # airborne foot-steps, touchdowns, air time at touchdown
    a_last = sim.get_state()[zm.S["FEET_AIR_LAST"]:zm.S["FEET_AIR_LAST"] + 2].clone() if gait else None
    with torch.inference_mode():
        for _ in range(args.num_steps):
            actions = policy(obs)
            obs_d, rew, dones, extras = env.step(actions)
            obs = obs_d["policy"] if hasattr(obs_d, "keys") else obs_d
            stt = sim.get_state()
            x = stt[x_row]
            d = dones > 0
            if gait:
                cur = stt[zm.S["FEET_AIR_CUR"]:zm.S["FEET_AIR_CUR"] + 2]
                last = stt[zm.S["FEET_AIR_LAST"]:zm.S["FEET_AIR_LAST"] + 2]
                td = (last != a_last) & (last > 0) & ~d
                air += torch.stack([(cur > 0).sum().float(), td.sum().float(), torch.where(td, last, 0.0).sum()])
                a_last = last.clone()
            alive = ~d
            vel_sum += torch.where(alive, (x - x_prev) / dt, 0.0).sum()
            vel_cnt += alive.sum()
            ep_ret += rew
            ep_len += 1
            rew_sum += rew.sum()
            fin += torch.stack([d.sum().float(), torch.where(d, ep_len, 0.0).sum(), torch.where(d, ep_ret, 0.0).sum(),
                                torch.where(d, x_prev - x_start, 0.0).sum(),
                                (d & extras["time_outs"].bool()).sum().float()])
            x_start = torch.where(d, x, x_start)
            ep_ret.masked_fill_(d, 0.0)
            ep_len.masked_fill_(d, 0.0)
            x_prev = x.clone()
    f = fin.tolist()
    posture = _posture(env.unwrapped, sim.get_state().cpu().numpy())
    out = {"task": args.task, "checkpoint": resume_path, "exported_jit": exported, "num_envs": n,
           "num_steps": args.num_steps, "mean_reward_per_step": float(rew_sum) / (n * args.num_steps),
           "episodes_finished": int(f[0]), "time_outs": int(f[4]),
           "mean_episode_length": f[1] / f[0] if f[0] else None,
           "mean_episode_return": f[2] / f[0] if f[0] else None,
           "mean_forward_distance_per_episode_m": f[3] / f[0] if f[0] else None,
           "mean_forward_velocity_m_s": float(vel_sum) / max(float(vel_cnt), 1.0), **posture}
    if gait:
        a = air.tolist()
        out.update(airborne_foot_fraction=a[0] / (2 * n * args.num_steps), touchdowns_per_env_s=a[1] / (n * args.num_steps * dt),
                   mean_air_time_at_touchdown_s=a[2] / a[1] if a[1] else None)
    print(json.dumps(out), flush=True)
    env.close()
    return out


if __name__ == "__main__":
    main()
