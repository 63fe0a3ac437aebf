"""Build libzbot.so in-tree for gfx950 (``python -m zbot_lab_amd.build``)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "zbot_sim.hip")
OUT = os.path.join(HERE, "libzbot.so")
ARCH = os.environ.get("ZBOT_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


STAMPS_OUT = os.path.join(HERE, "libzbot_stamps.so")


def build(force: bool = False, verbose: bool = False, stamps: bool = False, defines: tuple = (),
          out: str | None = None, flags: tuple = ()) -> str:
    """defines / out: an experiment variant (e.g. ``-DZB_GJK_TOL=3e-5f`` into ``libzbot_x.so``),
    selected at run time with ZBOT_LIB=<file name>."""
    out = os.path.join(HERE, out) if out else (STAMPS_OUT if stamps else OUT)
    deps = [SRC, os.path.join(ROOT, "include", "zbot.h"), os.path.abspath(__file__)]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    # -fno-slp-vectorize: packing scalar f32 math into v_pk_* pairs forces aligned register pairs
    # and shuffles; on this register-bound kernel it costs ~1.1 KB/lane of scratch spills.
    # -fno-hip-fp32-correctly-rounded-divide-sqrt: f32 '/' and sqrtf as v_rcp/v_sqrt sequences
    # (<= 2.5 ulp, OpenCL precision) instead of the ~10-instruction correctly rounded expansions.
    # -ffast-math: a / b as v_rcp * a, 1 / sqrt as v_rsq, sqrt without the denormal rescaling
    # (-freciprocal-math -fapprox-func: ~570 fewer frexp / ldexp / cndmask instructions, +3 %),
    # multiplications by the mass matrix's structural zeros folded and sums reassociated
    # (finite / no-signed-zeros / associative: +2 % more). No code path relies on inf / NaN (the
    # disk projection clamps |l| away from 0); the GPU parity suite is unchanged.
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize",
           "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-ffast-math", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp", SRC]
    if stamps:
        cmd.insert(1, "-DZB_STAMPS")
    for d in defines:
        cmd.insert(1, f"-D{d}")
    cmd[1:1] = list(flags)
    if verbose:
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


PPO_SRC = os.path.join(HERE, "csrc", "ppo_mlp.hip")
PPO_OUT = os.path.join(HERE, "libzbot_ppo.so")


def build_ppo(force: bool = False) -> str:
    """libzbot_ppo.so: the fused PPO minibatch update (fp32 MFMA, include/zbot_ppo.h). Plain -O3:
    no fast-math (expf / logf / division as torch computes them)."""
    deps = [PPO_SRC, os.path.join(ROOT, "include", "zbot_ppo.h"), os.path.abspath(__file__)]
    if not force and os.path.exists(PPO_OUT) and all(os.path.getmtime(PPO_OUT) >= os.path.getmtime(d) for d in deps):
        return PPO_OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-I", os.path.join(ROOT, "include"),
           "-o", PPO_OUT + ".tmp", PPO_SRC]
    subprocess.run(cmd, check=True)
    os.replace(PPO_OUT + ".tmp", PPO_OUT)
    return PPO_OUT


if __name__ == "__main__":
    defs = tuple(a[2:] for a in sys.argv[1:] if a.startswith("-D"))
    outs = [a[6:] for a in sys.argv[1:] if a.startswith("--out=")]
    flags = tuple(a[8:] for a in sys.argv[1:] if a.startswith("--flags="))
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv, stamps="--stamps" in sys.argv,
                defines=defs, out=outs[0] if outs else None, flags=flags))
    if not defs and not outs and not flags and "--stamps" not in sys.argv:
        print(build_ppo(force="--force" in sys.argv))
