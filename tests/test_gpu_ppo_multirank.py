"""The multi-GPU PPO update (PPO._update_steps_fused's world > 1 branch: the fused minibatch kernels
fill every ``.grad``, then the flattened-gradient all-reduce with the KL mean in the bucket, the
adaptive rate rule, clipping, torch's Adam and a re-pack of the weight images; reference
``scripts/rsl_rl/train.py:125-132``) against the torch statement of the same multi-rank update
(ZBOT_PPO_FUSED=0), from one snapshot.

RCCL cannot place two ranks on one device, so the two ranks share cuda:0 and reduce over gloo (the
same arrangement as ``bench.py --rehearsal``): the collective is gloo's, everything else is the
product path. Each rank owns different rollout data, so the all-reduce carries real differences;
both ranks must end with bit-identical parameters in each mode, and the fused ranks must match the
torch ranks to the fp32 summation-order tolerances of tests/test_gpu_ppo_fused.py.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, fused, q):
    os.environ["ZBOT_PPO_FUSED"] = "1" if fused else "0"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from zbot_lab_amd.rl.ppo import PPO, ActorCritic
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = "cuda:0"
        torch.manual_seed(11 + rank)  # different init per rank: the broadcast unifies them
        pol = ActorCritic(23, 23, 6, actor_hidden_dims=[128, 128, 128], critic_hidden_dims=[128, 128, 128])
        alg = PPO(pol, device=dev, multi_gpu_cfg={"global_rank": rank, "world_size": world})
        alg.broadcast_parameters()
        envs, steps = 512, 24
        alg.init_storage(envs, steps, 23, 23, 6)
        st = alg.storage
        g = torch.Generator(device=dev).manual_seed(100 + rank)  # rank-specific rollouts
        for t in (st.observations, st.critic_observations, st.actions, st.rewards, st.mu):
            t.copy_(torch.randn(t.shape, device=dev, generator=g))
        st.sigma.copy_(0.5 + torch.rand(st.sigma.shape, device=dev, generator=g))
        st.dones.copy_((torch.rand(st.dones.shape, device=dev, generator=g) < 0.05).float())
        with torch.no_grad():
            pol.update_distribution(st.observations.flatten(0, 1))
            lp = pol.get_actions_log_prob(st.actions.flatten(0, 1)).view(steps, envs, 1)
            st.actions_log_prob.copy_(lp + 0.3 * torch.randn(lp.shape, device=dev, generator=g))
            st.values.copy_(pol.evaluate(st.critic_observations.flatten(0, 1)).view(steps, envs, 1)
                            + 0.3 * torch.randn(st.values.shape, device=dev, generator=g))
        st.step = steps
        alg.compute_returns(st.critic_observations[-1])
        st.step = steps
        alg.generator = torch.Generator(device=dev).manual_seed(99)  # the same shuffle on both ranks
        p0 = torch.cat([p.detach().flatten() for p in pol.parameters()]).clone()
        alg.draw_minibatch_indices()
        alg.update_steps()
        torch.cuda.synchronize()
        steps_ = sorted({float(alg.optimizer.state[p]["step"]) for p in pol.parameters()})
        q.put((rank, fused, alg._fused is not None, p0.cpu().numpy(),
               torch.cat([p.detach().flatten() for p in pol.parameters()]).cpu().numpy(),
               float(alg.lr_t), alg.update_sums.cpu().numpy(), steps_))
    finally:
        dist.destroy_process_group()


def _run(fused: bool):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + (os.getpid() + (7 if fused else 0)) % 900
    ps = [ctx.Process(target=_worker, args=(r, 2, port, fused, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=240) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0, p.exitcode
    return out


def test_two_rank_fused_update_matches_torch_update(gpu):
    fu, to = _run(True), _run(False)
    assert all(o[2] for o in fu) and not any(o[2] for o in to)  # the fused driver ran / did not run
    for out in (fu, to):  # replicas stay identical: the same averaged gradients, rate and Adam step
        np.testing.assert_array_equal(out[0][3], out[1][3])
        np.testing.assert_array_equal(out[0][4], out[1][4])
        assert out[0][5] == out[1][5] and out[0][7] == out[1][7] == [20.0]
    np.testing.assert_array_equal(fu[0][3], to[0][3])  # the same broadcast snapshot
    p0, pf, pt = fu[0][3], fu[0][4], to[0][4]
    moved, d = np.abs(pt - p0), np.abs(pf - pt)
    print(f"\n2-rank fused vs torch update: max |dp| {d.max():.3g} (99.9% {np.quantile(d, 0.999):.3g}), "
          f"max move {moved.max():.3g}, lr {fu[0][5]:.4g} / {to[0][5]:.4g}, sums {fu[0][6]} / {to[0][6]}")
    assert moved.max() > 0
    assert np.quantile(d, 0.999) <= 1e-3 * moved.max()
    assert d.max() <= 0.05 * moved.max()
    assert abs(fu[0][5] - to[0][5]) <= 1e-7 + 1e-5 * to[0][5]
    # (update_sums are rank-local losses in both paths: rsl_rl logs the local minibatch losses)
    for r in range(2):
        np.testing.assert_allclose(fu[r][6], to[r][6], rtol=1e-4, atol=1e-6)


def _seg_worker(rank, world, port, q):
    """Two updates from one snapshot: the second eager, then again with the minibatch segments captured
    as HIP graphs on either side of the all-reduce (PPO.capture_update_segments)."""
    os.environ["ZBOT_PPO_FUSED"] = "1"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from zbot_lab_amd.rl.ppo import PPO, ActorCritic
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = "cuda:0"
        torch.manual_seed(11 + rank)
        pol = ActorCritic(23, 23, 6, actor_hidden_dims=[128, 128, 128], critic_hidden_dims=[128, 128, 128])
        alg = PPO(pol, device=dev, multi_gpu_cfg={"global_rank": rank, "world_size": world})
        alg.broadcast_parameters()
        envs, steps = 512, 24
        alg.init_storage(envs, steps, 23, 23, 6)
        st = alg.storage
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        for t in (st.observations, st.critic_observations, st.actions, st.rewards, st.mu):
            t.copy_(torch.randn(t.shape, device=dev, generator=g))
        st.sigma.copy_(0.5 + torch.rand(st.sigma.shape, device=dev, generator=g))
        st.dones.copy_((torch.rand(st.dones.shape, device=dev, generator=g) < 0.05).float())
        with torch.no_grad():
            pol.update_distribution(st.observations.flatten(0, 1))
            st.actions_log_prob.copy_(pol.get_actions_log_prob(st.actions.flatten(0, 1)).view(steps, envs, 1))
            st.values.copy_(pol.evaluate(st.critic_observations.flatten(0, 1)).view(steps, envs, 1))
        st.step = steps
        alg.compute_returns(st.critic_observations[-1])

        def update(seed):
            alg.generator = torch.Generator(device=dev).manual_seed(seed)
            alg.draw_minibatch_indices()
            alg.update_steps()
            torch.cuda.synchronize()

        update(99)  # the eager first update (the driver, its Adam state and the bucket now exist)
        assert alg._fused is not None and alg._flat is not None
        opt = alg.optimizer
        ps = list(pol.parameters())
        snap = ([p.detach().clone() for p in ps],
                [{k: v.clone() for k, v in opt.state[p].items()} for p in ps], alg.lr_t.clone())

        def restore():
            for p, v in zip(ps, snap[0]):
                p.data.copy_(v)
            for p, d in zip(ps, snap[1]):
                for k, v in d.items():
                    opt.state[p][k].copy_(v)
            alg.lr_t.copy_(snap[2])

        update(7)
        eager = (torch.cat([p.detach().flatten() for p in ps]).cpu().numpy(), float(alg.lr_t),
                 alg.update_sums.cpu().numpy())
        restore()
        ok = alg.capture_update_segments()
        update(7)
        graphed = (torch.cat([p.detach().flatten() for p in ps]).cpu().numpy(), float(alg.lr_t),
                   alg.update_sums.cpu().numpy())
        q.put((rank, ok, len(alg._seg_pre or []), eager, graphed))
    finally:
        dist.destroy_process_group()


def test_two_rank_update_graph_segments_match_eager(gpu):
    """with world > 1 the update graph is split at the all-reduce (graph -> all-reduce
    -> graph per minibatch); on two gloo ranks sharing cuda:0 the graphed update is bit-identical to the
    eager one from the same snapshot, and both ranks stay identical."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + (os.getpid() + 13) % 900
    ps = [ctx.Process(target=_seg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=240) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0, p.exitcode
    for rank, ok, npre, eager, graphed in out:
        assert ok and npre == 4
        np.testing.assert_array_equal(eager[0], graphed[0])
        assert eager[1] == graphed[1]
        np.testing.assert_array_equal(eager[2], graphed[2])
    np.testing.assert_array_equal(out[0][3][0], out[1][3][0])
