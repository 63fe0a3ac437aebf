"""Where the time between two env steps goes (GPU box): the bench's DirectRLEnv ``step()`` vs the
allocation-free ``step_into`` vs a HIP graph of G captured ``step_into`` calls, all on the same
env and action pool, each timed over K steps with events on the current stream.

    python scripts/step_gaps.py            # N=4096, K=500, G=16

rocprofv3's start-to-start time of zb_step_kernel is 132 us against a 117 us kernel (r3z
kernel_gaps.txt): ~4 us of it is the finalize launch, the rest gaps between the two launches of
a step and the next step. This script separates host-side cost (Python / allocation / ctypes)
from the kernel-boundary cost that a graph keeps.
"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import zbot_lab_amd  # noqa: E402,F401  (before torch: HIP graph settings)
import torch  # noqa: E402

from zbot_lab_amd.tasks import load_cfg, make  # noqa: E402


def timed(fn, k):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    fn(k)
    e1.record()
    host = (time.perf_counter() - t0) * 1e6 / k
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k, host


def main():
    n, K, G = int(os.environ.get("N", "4096")), int(os.environ.get("K", "500")), int(os.environ.get("G", "16"))
    cfg = load_cfg("zbot-6b-walking-v2")
    cfg.scene.num_envs = n
    env = make("zbot-6b-walking-v2", cfg)
    env.reset()
    gen = torch.Generator(device="cuda")
    gen.manual_seed(42)
    pool = [torch.randn(n, 6, device="cuda", generator=gen) for _ in range(G)]
    sim = env.sim
    obs = torch.empty(n, sim.obs_dim, device="cuda")
    rew = torch.empty(n, device="cuda")

    def plain(k):
        for i in range(k):
            env.step(pool[i % G])

    def into(k):
        for i in range(k):
            sim.step_into(pool[i % G], obs, rew)

    plain(50)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        into(G)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        into(G)

    def graph(k):
        for _ in range(k // G):
            g.replay()

    for name, fn in (("env.step()", plain), ("step_into", into), (f"graph of {G} steps", graph),
                     ("env.step() again", plain)):
        gpu, host = timed(fn, K)
        print(f"{name:22s} {gpu:8.2f} us per step on the GPU clock, host enqueue {host:8.2f} us per step, "
              f"{n / gpu:8.2f} M env-steps/s")


if __name__ == "__main__":
    main()
