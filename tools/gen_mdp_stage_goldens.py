"""Golden vectors for every stage of the reference's staged v2 reward recipe (build container only).

The reference keeps its curriculum as commented-out ``reward_cfg`` blocks in
``zbot_direct_6dof_bipedal_env_v2.py`` (v2.py:77-206: step0 "just stepping walk base", step1 v0 "use
this" / v1 / v2, step2, step3, and the active step4), switched by editing the file between chained
``--resume`` runs (README.md:69). This script reads those blocks from the reference source as text
(the weights come from the file, not from this repo's transcription in
``zbot_lab_amd/envs/walking_v2.py``), then for each stage constructs the reference's own
``ZbotDirectEnvV2`` with that ``reward_cfg`` (stub isaaclab / gymnasium packages, as in
tools/gen_mdp_goldens.py) and drives ``_pre_physics_step -> _get_dones -> _get_rewards ->
_get_observations`` over the same seeded synthetic robot / contact frames and actions.

The persistent buffers start from random non-zero values (feet_force_sum, base_heading_x_sum,
base_pos_y_err_sum, the step-length latches), so a stage that leaves a stateful term out proves that
its buffer does not move (the reference updates them inside ``_reward_<name>`` only, v2.py:484-533,
563-571), and step0's ``feet_force_diff`` sees both signs of ``feet_force_sum`` (it reads the
integrator before ``feet_force_sum`` updates it: dict order).

Writes ``tests/golden/mdp_v2_stages.npz`` (data only; no reference code leaves this container).
"""
from __future__ import annotations

import ast
import importlib.util
import os
import re
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_mdp_goldens as G  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "mdp_v2_stages.npz")
STAGES = {"step0": "just stepping walk base 2000 step0", "step1": "2000 step1 v0 use this",
          "step1_v1": "2000 step1 v1", "step1_v2": "2000 step1 v2", "step2": "2000 step2",
          "step3": "2000 step3", "step4": "2000 step4"}


def stage_cfgs_from_source(path: str) -> dict:
    """{stage: {term: weight}} from the reward_cfg blocks of the reference's v2 file (commented or
    not): each block follows a ``#   train reward ... <stage>`` marker line."""
    lines = open(path).read().split("\n")
    out = {}
    for name, marker in STAGES.items():
        start = next(i for i, l in enumerate(lines) if l.strip().lstrip("#").strip().endswith(marker))
        body, depth, opened = [], 0, False
        for l in lines[start + 1:]:
            t = re.sub(r"^\s*(#\s?)*", "", l)          # uncomment
            t = re.sub(r"#.*$", "", t).rstrip()        # inline comments
            if not opened:
                if t.startswith("reward_cfg"):
                    t = t.split("=", 1)[1]
                    opened = True
                else:
                    continue
            body.append(t)
            depth += t.count("{") - t.count("}")
            if opened and depth == 0:
                break
        out[name] = ast.literal_eval("\n".join(body))["reward_scales"]
    return out


def main():
    G.install_stubs()
    scales = stage_cfgs_from_source(G.REF)
    rng = np.random.default_rng(20261018)
    N, T = G.N, G.T
    robot, sensor = G._Robot(), G._Sensor()
    q0 = np.array([0.312, 0.837, -2.02, 2.02, -0.837, -0.312], np.float32)
    robot.data.default_joint_pos = torch.from_numpy(np.tile(q0, (N, 1)))
    robot.data.GRAVITY_VEC_W = torch.tensor([0.0, 0.0, -1.0]).repeat(N, 1)
    origins = rng.normal(0, 4.0, (N, 3)).astype(np.float32)
    origins[:, 2] = 0
    G.FAKES.update(robot=robot, sensor=sensor, terrain=G._Cfg(env_origins=torch.from_numpy(origins)))
    frames = [G.make_frame(rng, origins) for _ in range(T + 1)]
    actions = [rng.normal(0, 1.5, (N, 6)).astype(np.float32) for _ in range(T)]
    init = {
        "feet_down_pos_last": rng.normal(0, 0.2, (N, 2, 3)).astype(np.float32),
        "feet_contact_forces_last": rng.uniform(0, 20, (N, 2)).astype(np.float32),
        "feet_step_length": rng.normal(0, 0.05, (N, 2)).astype(np.float32),
        "feet_force_sum": rng.normal(0, 0.02, N).astype(np.float32),
        "base_heading_x_sum": rng.uniform(-0.5, 0.5, N).astype(np.float32),
        "base_pos_y_err_sum": rng.uniform(-0.5, 0.5, N).astype(np.float32),
        "episode_length_buf": rng.integers(975, 999, N).astype(np.int32),
    }
    spec = importlib.util.spec_from_file_location("ref_zbot_v2", G.REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)

    # the frames as v2 reads them: bodies 0 / 6 / 11 (feet, base) of the link arrays, every body of the
    # sensor history (feet F_z, undesired |F|)
    out = {f"frame_{k}": np.stack([fr[k] for fr in frames]) for k in frames[0] if k != "current_contact_time"}
    for k in ("body_link_pos_w", "body_link_quat_w", "body_com_lin_vel_w"):
        out[f"frame_{k}"] = np.ascontiguousarray(out[f"frame_{k}"][:, :, [0, 6, 11]])
    out["frame_last_air_time"] = np.ascontiguousarray(out["frame_last_air_time"][:, :, [0, 11]])
    out["actions"] = np.stack(actions)
    out.update({f"init_{k}": v for k, v in init.items()})
    out["env_origins"] = origins
    out["default_joint_pos"] = q0
    out["stages"] = np.array(list(STAGES))
    for stage in STAGES:
        cfg = ref.ZbotDirectEnvCfgV2()
        cfg.reward_cfg = {"reward_scales": dict(scales[stage])}   # (v2.py:251 scales the dict in place)
        env = ref.ZbotDirectEnvV2(cfg)
        names = list(env.reward_scales.keys())
        captured = {}
        for name in names:
            fn = env.reward_functions[name]

            def wrap(fn=fn, name=name):
                def g():
                    v = fn()
                    captured[name] = v.detach().clone()
                    return v
                return g
            env.reward_functions[name] = wrap()
        G.apply_frame(robot, sensor, frames[0])
        env.episode_length_buf[:] = torch.from_numpy(init["episode_length_buf"].astype(np.int64))
        env.feet_down_pos_last[:] = torch.from_numpy(init["feet_down_pos_last"])
        env.feet_contact_forces_last[:] = torch.from_numpy(init["feet_contact_forces_last"])
        env.feet_step_length[:] = torch.from_numpy(init["feet_step_length"])
        env.feet_force_sum[:] = torch.from_numpy(init["feet_force_sum"])
        env.base_heading_x_sum[:] = torch.from_numpy(init["base_heading_x_sum"])
        env.base_pos_y_err_sum[:] = torch.from_numpy(init["base_pos_y_err_sum"])
        env._get_observations()
        rec = {k: [] for k in ("reward", "terms", "died", "time_out", "obs", "feet_force_sum", "heading_sum",
                               "y_err_sum", "feet_step_length", "feet_down_pos_last", "feet_contact_forces_last",
                               "episode_sums", "prev_actions")}
        for t in range(T):
            env._pre_physics_step(torch.from_numpy(actions[t]))
            G.apply_frame(robot, sensor, frames[t + 1])
            env.episode_length_buf += 1
            died, tout = env._get_dones()
            env.reset_terminated[:] = died
            env.reset_time_outs[:] = tout
            rec["prev_actions"].append(env._previous_actions.numpy().copy())
            r = env._get_rewards()
            obs = env._get_observations()["policy"]
            rec["reward"].append(r.numpy().copy())
            rec["terms"].append(np.stack([captured[k].numpy() * float(env.reward_scales[k]) for k in names], axis=1))
            rec["died"].append(died.numpy().copy())
            rec["time_out"].append(tout.numpy().copy())
            rec["obs"].append(obs.numpy().copy())
            rec["feet_force_sum"].append(env.feet_force_sum.numpy().copy())
            rec["heading_sum"].append(env.base_heading_x_sum.numpy().copy())
            rec["y_err_sum"].append(env.base_pos_y_err_sum.numpy().copy())
            rec["feet_step_length"].append(env.feet_step_length.numpy().copy())
            rec["feet_down_pos_last"].append(env.feet_down_pos_last.numpy().copy())
            rec["feet_contact_forces_last"].append(env.feet_contact_forces_last.numpy().copy())
            rec["episode_sums"].append(np.stack([env._episode_sums[k].numpy() for k in names], axis=1))
        for k, v in rec.items():
            out[f"{stage}/{k}"] = np.stack(v)
        out[f"{stage}/term_names"] = np.array(names)
        out[f"{stage}/weights"] = np.array([float(scales[stage][k]) for k in names], np.float64)
        out[f"{stage}/scales_x_step_dt"] = np.array([float(env.reward_scales[k]) for k in names], np.float64)
        print(stage, names, "died", np.mean(out[f"{stage}/died"]))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print("wrote", os.path.normpath(OUT), os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
