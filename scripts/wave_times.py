"""Per-wave timing of zb_step_kernel (diagnostic build with per-workgroup records, GPU box):

    python -m zbot_lab_amd.build --stamps -DZB_STAMPS_NO_CAPS --out=libzbot_stamps_t.so
    ZBOT_LIB=libzbot_stamps_t.so python scripts/wave_times.py

For each of K launches (after a warm-up) the start / end of every workgroup (one wave each) on the
100 MHz constant clock: the dispatch spread (last wave start - first), the span (last end - first
start), the wave durations (median, p99, max) and the phase breakdown of the slowest 1 % of waves
against the median wave (phase cycles from the same launch). Answers where the launch's tail
(span vs mean wave) comes from.
"""
import ctypes as C
import os
import sys

import numpy as np

os.environ.setdefault("ZBOT_LIB", "libzbot_stamps_t.so")
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import zbot_lab_amd  # noqa: E402,F401  (before torch: HIP graph settings)
import torch  # noqa: E402

from zbot_lab_amd import _native as nat  # noqa: E402
from zbot_lab_amd.tasks import load_cfg, make  # noqa: E402

NAMES = ["prologue", "ground", "self-collision", "rnea+crba", "chol+drives", "contact rows", "pgs", "post",
         "mdp stores", "fk(substep)", "mdp loads", "mdp fk", "mdp rewards+reset"]
TICK_NS = 10.0  # s_memrealtime: 100 MHz


def main():
    task = os.environ.get("TASK", "zbot-6b-walking-v2")
    cfg = load_cfg(task)
    cfg.scene.num_envs = int(os.environ.get("N", "4096"))
    env = make(task, cfg)
    env.reset()
    n = env.num_envs
    waves = (n + 3) // 4
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    for _ in range(30):
        env.step(torch.randn(n, 6, device="cuda", generator=g))
    torch.cuda.synchronize()
    # SAVE_STATE=f.npy keeps the post-warm-up state; LOAD_STATE=f.npy replays every timed launch
    # from it (identical physics work per launch, whatever the library does with its stores)
    if os.environ.get("SAVE_STATE"):
        np.save(os.environ["SAVE_STATE"], env.sim.get_state().cpu().numpy())
    st0 = None
    if os.environ.get("LOAD_STATE"):
        st0 = torch.from_numpy(np.load(os.environ["LOAD_STATE"])).cuda()
    K = int(os.environ.get("K", "20"))
    rec = np.zeros((waves, 23), np.uint64)
    spread, span, durs, slow_ph, med_ph, timeline = [], [], [], [], [], []
    for _ in range(K):
        if st0 is not None:
            env.sim.set_state(st0)
        env.step(torch.randn(n, 6, device="cuda", generator=g))
        torch.cuda.synchronize()
        nat.check(nat.lib().zb_read_wave_times(rec.ctypes.data_as(C.c_void_p), waves), "zb_read_wave_times")
        t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
        ph = rec[:, 2:15].astype(np.float64)
        sub = rec[:, 15:19].astype(np.int64)
        d = (t1 - t0) * TICK_NS / 1e3  # us
        spread.append((t0.max() - t0.min()) * TICK_NS / 1e3)
        span.append((t1.max() - t0.min()) * TICK_NS / 1e3)
        durs.append(d)
        order = np.argsort(d)
        k = max(1, waves // 100)
        if not timeline:  # the absolute timeline of the 5 slowest and 3 median waves of the first launch
            base = t0.min()
            for w in list(order[-5:]) + list(order[waves // 2 - 1: waves // 2 + 2]):
                marks = [t0[w]] + list(sub[w]) + [t1[w]]
                timeline.append(f"  wg {w:5d} xcd {w % 8}: " + " ".join(f"{(x - base) * TICK_NS / 1e3:7.1f}" for x in marks))
        slow_ph.append(ph[order[-k:]].mean(axis=0))
        med_ph.append(ph[order[waves // 2 - k // 2: waves // 2 + k // 2 + 1]].mean(axis=0))
    durs = np.concatenate(durs)
    print(f"{task} {n} envs, {waves} waves x {K} launches")
    print(f"dispatch spread (last wave start - first) us: median {np.median(spread):.2f} max {np.max(spread):.2f}")
    print(f"span (last end - first start) us: median {np.median(span):.2f}")
    print(f"wave duration us: mean {durs.mean():.2f} median {np.median(durs):.2f} p90 {np.percentile(durs, 90):.2f} "
          f"p99 {np.percentile(durs, 99):.2f} max {durs.max():.2f}")
    hist, edges = np.histogram(durs, bins=12)
    print("duration histogram:", " ".join(f"{edges[i]:.0f}-{edges[i + 1]:.0f}:{h}" for i, h in enumerate(hist)))
    sp, mp = np.mean(slow_ph, axis=0), np.mean(med_ph, axis=0)
    print(f"{'phase (cycles per wave per step)':34s} {'median waves':>12s} {'slowest 1%':>12s} {'extra':>10s}")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:32s} {mp[i]:12.0f} {sp[i]:12.0f} {sp[i] - mp[i]:10.0f}")
    print(f"  {'total':32s} {mp.sum():12.0f} {sp.sum():12.0f} {sp.sum() - mp.sum():10.0f}")
    print("timeline (us from the launch's first wave start): start, end of substeps 1-4, end")
    print("\n".join(timeline))


if __name__ == "__main__":
    main()
