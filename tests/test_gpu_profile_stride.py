"""zb_profile_stride (bench.py --event-stride): HIP events bracket only every stride-th zb_step
launch, so the roofline's kernel time is a sample of the timed steps, not a probe on every one (the
event dispatch adds ~5.7 us to the step it brackets)."""
from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stride,steps,expect", [(1, 20, 20), (8, 100, 13), (8, 7, 1)])
def test_profile_stride_samples_every_nth_launch(gpu, stride, steps, expect):
    import torch
    from zbot_lab_amd import model as zm
    from zbot_lab_amd.sim import ZbotSim
    n = 1024
    sim = ZbotSim(n, zm.TaskCfg(solver_mode=1, self_manifold=3), device="cuda:0", seed=1)
    sim.reset()
    g = torch.Generator(device="cuda:0").manual_seed(2)
    sim.profile_begin(steps, stride=stride)
    for _ in range(steps):
        sim.step(torch.randn(n, zm.ACT_DIM, device="cuda:0", generator=g))
    ms, count = sim.profile_end()
    assert count == expect
    assert 0.0 < ms / count < 10.0  # (milliseconds per timed launch of a 1024-env step)
    # a later profile_begin starts counting launches afresh
    sim.profile_begin(4, stride=stride)
    for _ in range(3):
        sim.step(torch.zeros(n, zm.ACT_DIM, device="cuda:0"))
    ms, count = sim.profile_end()
    assert count == 1 if stride > 1 else count == 3
    sim.close()
