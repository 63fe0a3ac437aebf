#!/usr/bin/env python3
"""Throughput benchmark: zbot-6b-walking-v2 random-action env-steps/s on MI355X.

Contract: every GPU rank owns ``--envs-per-gpu`` envs (default 4096
= configs[1] at N=1; weak scaling across ranks, no data-path collective — envs are independent),
starts from the default pose with a full reset (episode_length_buf ~ U{0..999}), feeds
``randn(N, 6)`` actions (seed 42 + rank) through the DirectRLEnv ``step()`` (kernel + Python:
obs, reward, dones, auto-reset, episode log), W untimed warm-up steps, then K timed steps
bracketed by barrier + synchronize; the max time over ranks is used. Prints ONE JSON line.

``roofline``: the dominant kernel is ``zb_step_kernel``; its per-launch time is measured in this
process with hipEvents on the launch stream (libzbot ``zb_profile_begin/end``). Algorithmic bytes
per env-step = 946 B: 87 fp32 persistent state read + written, the 16-float
self-contact cache read + written (128 B), actions 24 B, obs 92 B, reward 4 B, two flag bytes. ``cpu_baseline``: the C oracle (same model + algorithm,
OpenMP over envs) on all of this host's cores available to the process and on one thread, on a
bounded sample, with nproc / affinity / cgroup quota / CPU model stated.

``--task v4`` measures zbot-6b-walking-v4 (commands / events / curricula; ``zb_v4_step_kernel``, 918 B
per env-step: 81 state rows read, 85 written, actions, obs 96 B, reward, flags, the contact cache) at
4096 envs. ``--task manager`` measures zbot-6b-walking-m-v0 (the manager-based flat env on
ZBOT_6S_V2_CFG; ``zb_m_step_kernel``, 962 B per env-step: 76 state rows read + written, 24 static /
dynamic friction coefficients read, actions 24 B, obs 100 B, reward, flags, the contact cache) at 4096
envs with the startup friction randomisation. ``--task standup`` measures the stand-up task instead
(zbot-6b-standup-v0, 32768 envs, friction randomisation on; kernel
``zb_su_step_kernel``, 686 B per env-step: 43 fp32 state rows read + written, 24 static / dynamic
friction coefficients read, actions 24 B, obs 88 B, reward, flags, the contact cache).

``--rehearsal`` (with N ranks under torch.distributed.run on a one-GPU box): every rank on cuda:0,
gloo for the barrier and the timing reduction (RCCL cannot place two ranks on one device). The line
then reports ``n_gpus`` 1 and the rank count under ``config.rehearsal_ranks``: it is a one-GPU
measurement of the N-rank plumbing, never a multi-GPU result.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# = 946: SURVEY.md §8d's 794 + the contact cache + round 5's three rows (step0's feet_force_sum
# and the episode sums of its two terms, v2.py:78-92, 238)
BYTES_PER_ENV_STEP = 794 + 2 * 16 * 4 + 2 * 3 * 4
WC_BYTES = 2 * 16 * 4  # the contact cache read + written
SU_BYTES_PER_ENV_STEP = 2 * 43 * 4 + 24 * 4 + 24 + 88 + 4 + 2 + WC_BYTES  # = 686, stand-up task
V4_BYTES_PER_ENV_STEP = 81 * 4 + 85 * 4 + 24 + 96 + 4 + 2 + WC_BYTES       # = 918, walking v4
M_BYTES_PER_ENV_STEP = 76 * 4 + 76 * 4 + 24 * 4 + 24 + 100 + 4 + 2 + WC_BYTES  # = 962, manager flat env


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=500)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--task", choices=("walking", "standup", "v4", "manager"), default="walking")
    p.add_argument("--envs-per-gpu", type=int, default=None, help="default 4096 (walking) / 32768 (standup, C5)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--event-stride", type=int, default=8,
                   help="the roofline's kernel time: HIP start / stop events on every N-th timed step launch (the "
                        "event dispatch adds ~5.7 us to the step it brackets: 1 = every step, 4.3 %% slower)")
    p.add_argument("--action-pool", type=int, default=64, help="distinct pre-drawn randn action batches cycled")
    # ablation knobs (the reported line uses the defaults)
    p.add_argument("--solver-iterations", type=int, default=None)
    p.add_argument("--no-self-collision", action="store_true")
    p.add_argument("--self-manifold", type=int, default=None, help="zb_task_cfg.self_manifold (0 / 1 / 2 / 3)")
    p.add_argument("--solver-mode", type=int, default=None,
                   help="zb_task_cfg.solver_mode (0 PGS, 1 TGS, 2 TGS + ground refresh, 3 + self refresh)")
    p.add_argument("--rehearsal", action="store_true",
                   help="N ranks share cuda:0 over gloo (one-GPU box rehearsal; reports n_gpus 1)")
    return p.parse_args()


ENVS_PER_WORKGROUP = 4         # zb_step_kernel: one 64-lane workgroup = 4 envs x 16 lanes


VALU_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector peak (256 CUs x 4 SIMDs x 64 FLOP/clk x 2.4 GHz)
VALU_LANE_OPS_PEAK_T = 39.3   # one wave64 VALU instruction per SIMD per 4 cycles: 256 x 4 x 16 lanes x 2.4 GHz
ROOFLINE_PMC = "roofline_pmc.json"


def pmc_entry(num_envs: int, kernel: str = "zb_step_kernel"):
    """The PMC-derived numbers of the dominant kernel for this grid (work-items = 64 per workgroup of 4
    envs) from the tracked ``roofline_pmc.json`` (written by scripts/prof_summary.py from the rocprofv3
    passes committed under profiles/<round>/; it travels to the GPU box, profiles/ does not). None when
    no pass covers this kernel and grid."""
    here = os.path.dirname(os.path.abspath(__file__))
    grid = -(-num_envs // ENVS_PER_WORKGROUP) * 64
    try:
        db = json.load(open(os.path.join(here, ROOFLINE_PMC)))
    except (OSError, ValueError):
        return None
    return db.get(f"{kernel}@{grid}")


def pmc_traffic(num_envs: int, kernel: str = "zb_step_kernel"):
    """HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (separate rocprofv3 passes, KiB). Calibrated for
    this kernel's access patterns (team loads and staged stores under the XCD-aware workgroup mapping,
    tools/calib, profiles/r1i_calib): FETCH_SIZE counts 1/2 of the bytes read (the guide's gfx950 tally),
    WRITE_SIZE the bytes written. Returns (bytes, source) or (None, None)."""
    e = pmc_entry(num_envs, kernel)
    if e is None or "traffic_bytes" not in e:
        return None, None
    return e["traffic_bytes"], e["source"]


def pmc_issue(num_envs: int, kernel: str = "zb_step_kernel"):
    """VALU issue fraction of the dominant kernel (same grid): the quad-cycles a wave spends issuing VALU
    instructions (SQ_ACTIVE_INST_VALU) over its resident quad-cycles (SQ_WAVE_CYCLES), plus VALU
    instructions per wave. With one wave per SIMD (4096 envs) this is the SIMD's VALU utilisation -- the
    kernel's real bound."""
    e = pmc_entry(num_envs, kernel)
    if e is None or "issue_frac" not in e:
        return None
    return {"bound": "valu-issue", "frac": e["issue_frac"], "wait_any_frac": e.get("wait_any_frac"),
            "valu_insts_per_wave": e.get("valu_insts_per_wave"), "waves": e.get("waves"), "source": e["source"]}


def valu_roofline(num_envs: int, kernel_s: float, kernel: str = "zb_step_kernel"):
    """The VALU half of the roofline: VALU lane-instructions per launch (SQ_INSTS_VALU x 64 lanes, inactive
    lanes included) over the kernel time measured in this run. ``achieved`` counts every lane-instruction
    as an FMA (2 FLOP) -- an upper bound on the FP32 rate -- against the 157.3 TF vector peak (which
    assumes packed FMAs); ``issue_frac_device`` is the lane-instruction rate against the chip's
    non-packed issue rate (39.3 T lane-instructions/s)."""
    e = pmc_entry(num_envs, kernel)
    if e is None or "valu_insts_per_wave" not in e or not kernel_s:
        return None
    lane_ops = e["valu_insts_per_wave"] * e["waves"] * 64.0
    tflops = 2.0 * lane_ops / kernel_s / 1e12
    return {"bound": "valu", "achieved": tflops, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s (upper bound)",
            "frac": tflops / VALU_PEAK_TFLOPS, "lane_ops_per_env_step": lane_ops / num_envs,
            "issue_frac_device": lane_ops / kernel_s / 1e12 / VALU_LANE_OPS_PEAK_T, "source": e["source"]}


def host_cpu_info() -> dict:
    """nproc / affinity / cgroup CPU quota / model name of this host (the GPU box's host cores)."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_limit": None,
            "model": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_cpu_limit"] = float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def _time_oracle(sim, acts, seconds: float):
    sim.step(acts[0])  # warm
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        sim.step(acts[steps % len(acts)])
        steps += 1
    return steps, time.perf_counter() - t0


def cpu_baseline(num_envs: int, seconds: float, task: str = "walking") -> dict:
    """Time the C oracle (test infrastructure, used here only as the CPU baseline) on every host core
    this process may use and on one thread. The all-core leg runs at
    the affinity count and, when the cgroup grants fewer CPUs, also at that quota; the faster is
    ``value`` and its thread count is ``cores``."""
    import numpy as np
    from oracle.pyoracle import OracleSim, lib as oracle_lib
    from zbot_lab_amd import model as zm
    info = host_cpu_info()
    cands = {info["affinity"]}
    if info["cgroup_cpu_limit"]:
        cands.add(max(1, int(info["cgroup_cpu_limit"])))
    cfg = {"standup": zm.TaskCfg.standup, "v4": zm.TaskCfg.walking_v4,
           "manager": zm.TaskCfg.manager_flat}.get(task, zm.TaskCfg)()
    rng = np.random.default_rng(42)
    acts = [rng.standard_normal((num_envs, 6)).astype(np.float32) for _ in range(8)]
    legs = {}
    for th in sorted(cands):
        oracle_lib().zbo_set_threads(th)
        sim = OracleSim(num_envs, cfg, seed=0)
        sim.reset()
        steps, dt = _time_oracle(sim, acts, seconds / (len(cands) + 1))
        legs[th] = (num_envs * steps / dt, steps, dt)
    n1 = max(64, num_envs // 16)
    oracle_lib().zbo_set_threads(1)
    sim1 = OracleSim(n1, cfg, seed=0)
    sim1.reset()
    steps1, dt1 = _time_oracle(sim1, [a[:n1] for a in acts], seconds / (len(cands) + 1))
    best = max(legs, key=lambda t: legs[t][0])
    v, steps, dt = legs[best]
    return {"value": v, "unit": "env-steps/s", "cores": best, "kind": "port",
            "single_thread": {"value": n1 * steps1 / dt1, "cores": 1,
                              "sample": f"{steps1} steps x {n1} envs, {dt1:.1f} s"},
            "by_threads": {str(t): legs[t][0] for t in sorted(legs)},
            "host": info,
            "sample": f"{steps} steps x {num_envs} envs of the C oracle (oracle/zbot_oracle.c, OpenMP "
                      f"{best} threads), random actions, {dt:.1f} s"}


def launch_plan(gpus: int, environ, argv: list[str], port: int | None = None) -> list[str] | None:
    """How ``bench.py --gpus N`` runs (reference multi-GPU entry: ``train.py:125-132``, one process
    per GPU). Returns None when this process is the worker (N = 1 without a launcher, or a rank
    started by torch.distributed.run whose WORLD_SIZE equals N), or the child command line that a
    plain ``python bench.py --gpus N`` (N > 1, no WORLD_SIZE) spawns: torch.distributed.run with N
    local ranks on 127.0.0.1. Raises ValueError when --gpus and WORLD_SIZE disagree (a SCALE run
    must never time fewer GPUs than it reports)."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise ValueError(f"--gpus {gpus} but WORLD_SIZE={ws}: launch one rank per GPU")
        return None
    if gpus == 1:
        return None
    if port is None:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def run_launcher(cmd: list[str]) -> int:
    """Parent of an N-GPU run: it never touches the GPU and never execs (the box forbids replacing
    a process); the ranks' output passes through (rank 0 prints the JSON line) and the parent exits
    with the launcher's code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def rank_plan(environ, rehearsal: bool = False) -> dict:
    """Process-group and device plan of one bench rank (reference: train.py:125-132, one process per
    GPU): rank / world from the launcher's env; with world > 1 the backend is "nccl" (= RCCL over
    xGMI on ROCm) bound to device cuda:LOCAL_RANK, or, in a --rehearsal, "gloo" with every rank on
    cuda:0 and host-side reductions. ``n_gpus`` is what the JSON line reports."""
    world = int(environ.get("WORLD_SIZE", "1"))
    rank = int(environ.get("RANK", "0"))
    local_rank = int(environ.get("LOCAL_RANK", "0"))
    share = world > 1 and rehearsal
    if share:
        local_rank = 0
    backend = None if world == 1 else ("gloo" if share else "nccl")
    return {"world": world, "rank": rank, "local_rank": local_rank, "share": share, "backend": backend,
            "device": f"cuda:{local_rank}", "reduce_device": "cpu" if share else f"cuda:{local_rank}",
            "n_gpus": 1 if share else world}


def init_group(plan: dict, dist_mod=None):
    """Initialise the process group of ``plan`` (None for one rank). RCCL gets the rank's device so
    its communicator binds to that GPU at init."""
    if plan["backend"] is None:
        return None
    if dist_mod is None:
        import torch.distributed as dist_mod
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if plan["backend"] == "nccl":
        dist_mod.init_process_group("nccl", device_id=torch.device(plan["device"]))
    else:
        dist_mod.init_process_group(plan["backend"])
    return dist_mod


def main():
    args = parse()
    cmd = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if cmd is not None:
        sys.exit(run_launcher(cmd))
    plan = rank_plan(os.environ, args.rehearsal)
    world, rank, local_rank, share = plan["world"], plan["rank"], plan["local_rank"], plan["share"]
    dist = init_group(plan)
    torch.cuda.set_device(local_rank)
    dev = torch.device(plan["device"])

    from zbot_lab_amd.envs import (Zbot6BFlatEnvCfg, Zbot6SEnvV4, Zbot6SEnvV4Cfg, Zbot6SUpEnv, Zbot6SUpEnvCfg,
                                   ZbotDirectEnvCfgV2, ZbotDirectEnvV2, ZbotManagerBasedRLEnv)
    standup = args.task == "standup"
    v4 = args.task == "v4"
    mgr = args.task == "manager"
    cfg = (Zbot6SUpEnvCfg() if standup else Zbot6SEnvV4Cfg() if v4 else Zbot6BFlatEnvCfg() if mgr
           else ZbotDirectEnvCfgV2())
    cfg.scene.num_envs = args.envs_per_gpu or (32768 if standup else 4096)
    cfg.sim.device = str(dev)
    cfg.seed = 42 + rank
    if args.solver_iterations is not None:
        cfg.solver.iterations = args.solver_iterations
    if args.self_manifold is not None:
        cfg.solver.self_manifold = args.self_manifold
    if args.solver_mode is not None:
        cfg.solver.mode = args.solver_mode
    if args.no_self_collision:
        cfg.solver.self_collision = False
    env = (Zbot6SUpEnv(cfg) if standup else Zbot6SEnvV4(cfg) if v4 else ZbotManagerBasedRLEnv(cfg) if mgr
           else ZbotDirectEnvV2(cfg))
    n = env.num_envs
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    pool = [torch.randn(n, 6, device=dev, generator=gen) for _ in range(max(1, args.action_pool))]

    for k in range(args.warmup):
        env.step(pool[k % len(pool)])
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    env.sim.profile_begin(args.steps, stride=max(1, args.event_stride))
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        env.step(pool[k % len(pool)])
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, kern_n = env.sim.profile_end()

    rdev = plan["reduce_device"]  # (gloo reduces host tensors)
    t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
    per_rank = torch.tensor([n * args.steps / elapsed], dtype=torch.float64, device=rdev)
    coll_world = 1
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gathered = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(gathered, per_rank)
        per_rank = torch.cat(gathered)
        coll_world = dist.get_world_size()
    elapsed = float(t.item())
    per_rank_rates = [float(v) for v in per_rank.tolist()]
    total_steps = n * world * args.steps
    value = total_steps / elapsed

    if rank == 0:
        kern_s = kern_ms / 1e3 / max(kern_n, 1)
        kname = ("zb_su_step_kernel" if standup else "zb_v4_step_kernel" if v4 else "zb_m_step_kernel" if mgr
                 else "zb_step_kernel")
        bpe = (SU_BYTES_PER_ENV_STEP if standup else V4_BYTES_PER_ENV_STEP if v4 else M_BYTES_PER_ENV_STEP if mgr
               else BYTES_PER_ENV_STEP)
        traffic, traffic_src = pmc_traffic(n, kname)
        achieved = n * bpe / kern_s / 1e9
        workload = (f"zbot-6b-standup-v0 (C5), {n} envs/GPU x {world} GPU, friction DR, random-action throughput"
                    if standup else f"zbot-6b-walking-v4, {n} envs/GPU x {world} GPU, commands + curricula, "
                    "random-action throughput" if v4 else
                    f"zbot-6b-walking-m-v0 (ManagerBasedRLEnv flat), {n} envs/GPU x {world} GPU, friction DR, "
                    "random-action throughput" if mgr else
                    f"zbot-6b-walking-v2, {n} envs/GPU x {world} GPU, random-action throughput")
        out = {
            "metric": "env-steps/sec at 4096/65536 envs, 1->8 GPUs; % HBM roofline",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": plan["n_gpus"],
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: default-pose starts, full reset, randn(N,6) actions seeded 42+rank",
            "config": {"workload": workload,
                       "envs_per_gpu": n, "total_envs": n * world, "decimation": 4, "sim_dt": 0.005,
                       "solver": {"mode": cfg.solver.mode, "iterations": cfg.solver.iterations,
                                  "self_manifold": cfg.solver.self_manifold,
                                  "self_collision": cfg.solver.self_collision},
                       "parallelism": f"env-sharded x{world} (replicas, no collective)",
                       "collective": {"backend": plan["backend"], "world_size": coll_world},
                       "per_rank_env_steps_per_s": per_rank_rates,
                       **({"rehearsal_ranks": world, "rehearsal": "all ranks on cuda:0, gloo collectives"}
                          if share else {})},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kname, "kernel_ms": kern_s * 1e3,
                         "kernel_timing": f"HIP events on every {max(1, args.event_stride)}th timed launch "
                                          f"({kern_n} launches)",
                         "bytes_per_env_step": bpe, "issue": pmc_issue(n, kname),
                         "valu": valu_roofline(n, kern_s, kname)},
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(min(n, 4096), args.cpu_baseline_seconds, args.task)
        print(json.dumps(out), flush=True)
    env.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
