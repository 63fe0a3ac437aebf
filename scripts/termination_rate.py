#!/usr/bin/env python3
"""Random-action termination rate of zbot-6b-walking-v2: N envs x T steps of
randn actions from the default pose, seeded; prints terminations (died) per 1000 env-steps and the
env-steps/s of the run. ZBOT_LIB selects the library (e.g. a build with another self-collision
shape) for A/B comparisons."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zbot_lab_amd  # noqa: E402


def main():
    n, steps = int(os.environ.get("N", "4096")), int(os.environ.get("STEPS", "1000"))
    cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
    cfg.scene.num_envs = n
    env = zbot_lab_amd.make("zbot-6b-walking-v2", cfg=cfg)
    env.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    died = torch.zeros((), device="cuda", dtype=torch.int64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        _, _, term, trunc, _ = env.step(torch.randn(n, 6, device="cuda", generator=g))
        died += term.sum()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"lib": os.environ.get("ZBOT_LIB", "libzbot.so"), "envs": n, "steps": steps,
                      "died_per_1000_env_steps": 1000.0 * died.item() / (n * steps),
                      "env_steps_per_s": n * steps / dt}))


if __name__ == "__main__":
    main()
