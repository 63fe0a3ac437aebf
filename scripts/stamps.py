"""Per-phase cycle breakdown of zb_step_kernel (diagnostic build libzbot_stamps.so, GPU box)."""
import os, sys, ctypes as C
os.environ.setdefault("ZBOT_LIB", "libzbot_stamps.so")
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import torch
from zbot_lab_amd import _native as nat
from zbot_lab_amd.tasks import load_cfg, make
names = ["prologue(pre+cache)", "ground", "self-collision", "inertia+rnea+crba", "chol+drives",
         "contact rows", "pgs", "post(solve,forces,integrate)", "mdp stores", "fk(substep)", "mdp loads", "mdp fk", "mdp rewards+reset"]
task = os.environ.get("TASK", "zbot-6b-walking-v2")
cfg = load_cfg(task); cfg.scene.num_envs = int(os.environ.get("N", "4096"))
env = make(task, cfg); env.reset()
print(task, env.num_envs, "envs")
g = torch.Generator(device="cuda"); g.manual_seed(42)
for k in range(30): env.step(torch.randn(env.num_envs, 6, device="cuda", generator=g))
torch.cuda.synchronize()
buf = (C.c_uint64 * 16)(); nat.lib().zb_read_stamps(buf)
nat.lib().zb_read_stamp_hist((C.c_uint64 * 136)())  # reset the histograms after the warm-up
steps = 100
for k in range(steps): env.step(torch.randn(env.num_envs, 6, device="cuda", generator=g))
torch.cuda.synchronize()
nat.lib().zb_read_stamps(buf)
waves = (env.num_envs + 3) // 4  # one wave per 4 envs (16 lanes per env)
tot = sum(buf[k] for k in range(len(names)))
calls, its, wmax = buf[13], buf[14], buf[15]
print(f"self collision: {calls / waves / steps / 4:.1f} GJK calls per wave per substep, {its / max(calls, 1):.2f} "
      f"iterations per call; slowest wave of one launch {wmax:.0f} cycles (mean {tot / waves / steps:.0f})")
print(f"cycles per wave per step: {tot / waves / steps:.0f}")
for k in range(len(names)):
    print(f"  {names[k]:32s} {buf[k] / waves / steps:10.0f}  {100 * buf[k] / tot:5.1f} %")
slow = (C.c_uint64 * 16)(); nat.lib().zb_read_stamps_slowest(slow)
hist = (C.c_uint64 * 136)(); nat.lib().zb_read_stamp_hist(hist)
print("waves by the largest GJK pair count of one env in one substep:",
      {k: hist[k] for k in range(64) if hist[k]})
print("waves by the largest per-lane GJK iteration sum over the step (bin of 4):",
      {4 * k: hist[64 + k] for k in range(64) if hist[64 + k]})
print("slowest wave of one launch, by phase:")
for k in range(len(names)):
    print(f"  {names[k]:32s} {slow[k]:10.0f}")
