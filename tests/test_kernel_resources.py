"""Occupancy budget of the step kernels, read from the built libzbot.so's gfx950 code object
(no GPU needed): <= 20 KB of LDS per workgroup and <= 256 VGPRs + AGPRs, so that two waves share
a SIMD once a launch has more than one wave per SIMD (the LDS diet). Scratch: at most
one dword in the walking v2 (the benchmarked kernel) and stand-up kernels with the default PGS solve
(round 4, with the self-contact manifold: one loop-invariant value stored before the substep loop and
reloaded once in the epilogue); the v4 / manager kernels and the TGS instantiations
spill a few registers (<= 64 B per lane)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "zbot_lab_amd", os.environ.get("ZBOT_LIB", "libzbot.so"))
LLVM = "/opt/rocm/lib/llvm/bin"
STEP_KERNELS = ("zb_step_kernel", "zb_su_step_kernel", "zb_v4_step_kernel", "zb_m_step_kernel")
LDS_PER_CU = 160 * 1024


def _kernel_metadata(tmp_path):
    tools = [shutil.which("objcopy"), os.path.join(LLVM, "clang-offload-bundler"), os.path.join(LLVM, "llvm-readobj")]
    if not os.path.exists(LIB) or not all(t and os.path.exists(t) for t in tools):
        pytest.skip("libzbot.so or the ROCm binary tools are missing")
    fat, co = str(tmp_path / "fatbin.bin"), str(tmp_path / "co.elf")
    subprocess.run([tools[0], "-O", "binary", "--only-section=.hip_fatbin", LIB, fat], check=True)
    subprocess.run([tools[1], "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([tools[2], "--notes", co], check=True, capture_output=True, text=True).stdout
    kernels, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "agpr_count" and line.lstrip().startswith("-"):  # first field of a kernel's entry
            cur = {}
        if key == "name" and not val.endswith(".kd"):
            kernels[val] = cur
        elif key in ("group_segment_fixed_size", "vgpr_count", "agpr_count", "private_segment_fixed_size"):
            cur[key] = int(val)
    return kernels


def test_step_kernels_fit_two_waves_per_simd(tmp_path):
    kernels = _kernel_metadata(tmp_path)
    found = 0
    for name, md in kernels.items():
        short = next((k for k in STEP_KERNELS if f"{len(k)}{k}" in name), None)
        if short is None:
            continue
        found += 1
        tgs = "ILb1E" in name  # template argument kTgs
        lds = md["group_segment_fixed_size"]
        regs = md["vgpr_count"] + md.get("agpr_count", 0)
        scratch = md.get("private_segment_fixed_size", 0)
        assert lds <= LDS_PER_CU // 8, f"{short}: {lds} B of LDS per one-wave workgroup (> 20 KB: one wave per SIMD)"
        assert regs <= 256, f"{short}: {regs} VGPRs + AGPRs (> 256: one wave per SIMD)"
        if short in ("zb_step_kernel", "zb_su_step_kernel") and not tgs:
            assert scratch <= 8, f"{short}: {scratch} B of scratch per lane (register spill)"
        assert scratch <= 64, f"{short}{' (TGS)' if tgs else ''}: {scratch} B of scratch per lane"
    assert found == 2 * len(STEP_KERNELS), sorted(kernels)  # PGS and TGS instantiations
