"""Multi-GPU launch plumbing (CPU): ``bench.py --gpus N`` spawns N ranks through
torch.distributed.run (reference multi-GPU entry ``scripts/rsl_rl/train.py:125-132``) or runs as a
rank whose WORLD_SIZE must equal N; the PPO runner keeps the update eager when the world is > 1
(no captured RCCL all-reduce until a multi-GPU run proves it), rehearsed with gloo."""
from __future__ import annotations

import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_plan_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, ["--steps", "5"]) is None


def test_launch_plan_spawns_one_rank_per_gpu():
    cmd = bench.launch_plan(2, {}, ["--gpus", "2", "--steps", "7"], port=29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "7"]  # the ranks see the same arguments
    assert os.path.basename(cmd[-5]) == "bench.py"
    assert bench.launch_plan(8, {}, ["--gpus", "8"]) is not None


def test_launch_plan_rank_under_launcher():
    # the driver's SCALE command: torch.distributed.run ... bench.py --gpus N (WORLD_SIZE = N)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, ["--gpus", "4"]) is None


@pytest.mark.parametrize("gpus,ws", [(2, "1"), (8, "4"), (1, "2")])
def test_launch_plan_mismatch_fails_loudly(gpus, ws):
    with pytest.raises(ValueError):
        bench.launch_plan(gpus, {"WORLD_SIZE": ws}, [])


def test_launch_plan_rejects_zero():
    with pytest.raises(ValueError):
        bench.launch_plan(0, {}, [])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _runner_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_ppo import ToyVecEnv
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2
    cfg = PPORunnerCfgV2().to_dict()
    r_default = OnPolicyRunner(ToyVecEnv(n=8), cfg, log_dir=None, device="cpu", use_graph=True)
    r_forced = OnPolicyRunner(ToyVecEnv(n=8), cfg, log_dir=None, device="cpu", use_graph=True, graph_update=True)
    q.put((rank, r_default.is_distributed, r_default.use_graph, r_default.graph_update, r_forced.graph_update))
    dist.destroy_process_group()


def test_runner_update_graph_default_multi_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_runner_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, is_dist, use_graph, graph_update, forced in out:
        assert is_dist and use_graph          # rollout graph unaffected
        # world > 1: graphs on either side of each minibatch's all-reduce (PPO.capture_update_segments,
        # after the first eager update; a runner without the fused driver drops back to eager there)
        assert graph_update is True
        assert forced is True


def test_runner_update_graph_follows_rollout_graph_single_rank(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_ppo import ToyVecEnv
    from zbot_lab_amd.rl import OnPolicyRunner, PPORunnerCfgV2
    r = OnPolicyRunner(ToyVecEnv(n=8), PPORunnerCfgV2().to_dict(), log_dir=None, device="cpu", use_graph=True)
    assert r.graph_update is True


def test_rank_plan_single_rank():
    p = bench.rank_plan({})
    assert p["backend"] is None and p["n_gpus"] == 1 and p["device"] == "cuda:0"
    assert bench.init_group(p, dist_mod=object()) is None  # no process group for one rank


@pytest.mark.parametrize("rank", [0, 3, 7])
def test_rank_plan_scale_run_binds_rccl_to_the_local_gpu(rank):
    """The driver's SCALE command (torch.distributed.run, 8 ranks): backend "nccl" (RCCL), each rank's
    communicator bound at init to cuda:LOCAL_RANK, device-side reductions, n_gpus = WORLD_SIZE."""
    env = {"WORLD_SIZE": "8", "RANK": str(rank), "LOCAL_RANK": str(rank)}
    p = bench.rank_plan(env)
    assert p["backend"] == "nccl" and p["n_gpus"] == 8 and not p["share"]
    assert p["device"] == f"cuda:{rank}" and p["reduce_device"] == f"cuda:{rank}"

    calls = []

    class FakeDist:
        def init_process_group(self, backend, **kw):
            calls.append((backend, kw))

    bench.init_group(p, dist_mod=FakeDist())
    (backend, kw), = calls
    assert backend == "nccl" and str(kw["device_id"]) == f"cuda:{rank}"


def test_rank_plan_rehearsal_reports_one_gpu():
    """--rehearsal: every rank on cuda:0 over gloo; the line reports n_gpus 1 (never a multi-GPU
    result), and only the explicit flag turns it on (an environment variable does not)."""
    env = {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1", "ZB_BENCH_SHARE_GPU": "1"}
    assert bench.rank_plan(env)["backend"] == "nccl"        # no flag: a real 2-GPU rank
    p = bench.rank_plan(env, rehearsal=True)
    assert p["backend"] == "gloo" and p["device"] == "cuda:0" and p["reduce_device"] == "cpu"
    assert p["n_gpus"] == 1 and p["share"]
    calls = []

    class FakeDist:
        def init_process_group(self, backend, **kw):
            calls.append((backend, kw))

    bench.init_group(p, dist_mod=FakeDist())
    assert calls == [("gloo", {})]
