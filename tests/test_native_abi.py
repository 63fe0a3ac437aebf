"""C ABI: libzbot.so (HIP, gfx950) loads on a CPU-only host and exports every entry point declared
in include/zbot.h; the oracle exports the same surface with the zbo_ prefix. No compute here."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zbot.h")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(zb_\w+)\s*\(", text, re.M)))


def test_header_declares_the_abi():
    syms = header_symbols()
    for s in ("zb_create", "zb_destroy", "zb_reset", "zb_step", "zb_observe", "zb_read_log", "zb_get_state",
              "zb_set_state", "zb_last_error", "zb_physics_substeps", "zb_profile_begin", "zb_profile_end"):
        assert s in syms


def test_library_builds_and_exports_every_header_symbol():
    from zbot_lab_amd import build
    path = build.build()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (zb_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    from zbot_lab_amd import _native
    assert set(_native.EXPORTED) == set(header_symbols())


def test_library_loads_without_gpu():
    from zbot_lab_amd import _native
    L = _native.lib()
    assert L.zb_last_error() is not None
    # error path: invalid arguments are reported, not crashed on
    h = C.c_void_p()
    rc = L.zb_create(None, None, 0, 0, 0, C.byref(h))
    assert rc < 0 and b"zb_create" in L.zb_last_error()


def test_gfx950_code_object_present():
    from zbot_lab_amd import build
    path = build.build()
    data = open(path, "rb").read()
    assert b"gfx950" in data


def test_struct_layout_matches_header():
    """ctypes mirrors of zb_model / zb_task_cfg have the C sizes (compiled probe)."""
    import tempfile
    from zbot_lab_amd import model as zm
    src = '#include <stdio.h>\n#include "zbot.h"\nint main(){printf("%zu %zu\\n", sizeof(zb_model), sizeof(zb_task_cfg));}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        a, b = map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split())
    assert a == C.sizeof(zm.ZbModel) and b == C.sizeof(zm.ZbTaskCfg)


def test_oracle_exports_mirror():
    from oracle import pyoracle
    L = pyoracle.lib()
    for s in header_symbols():
        if s in ("zb_last_error", "zb_num_envs", "zb_profile_begin", "zb_profile_end", "zb_profile_stride", "zb_create", "zb_destroy",
                 "zb_read_stamps", "zb_read_stamps_slowest", "zb_read_stamp_hist", "zb_read_wave_times",
                 "zb_set_log_buffers", "zb_set_log_accumulator", "zb_set_done_buffer"):
            continue
        assert hasattr(L, "zbo_" + s[3:]), s


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from zbot_lab_amd import _native
    from zbot_lab_amd.sim import ZbotSim
    with pytest.raises(_native.ZbotError):
        ZbotSim(4, device="cuda:0")
    with pytest.raises(_native.ZbotError):
        ZbotSim(4, device="cpu")


def test_ppo_library_exports_and_struct_layouts():
    """libzbot_ppo.so (include/zbot_ppo.h) exports every declared entry point, its ctypes structs have
    the C sizes, and the host-side shape check answers without a GPU."""
    import tempfile
    from zbot_lab_amd import build
    from zbot_lab_amd.rl import fused
    path = build.build_ppo()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    text = open(os.path.join(ROOT, "include", "zbot_ppo.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(zbp_\w+)\s*\(", text, re.M))
    assert declared == set(fused.EXPORTED)
    assert declared <= set(re.findall(r"\bT (zbp_\w+)", out))
    assert b"gfx950" in open(path, "rb").read()
    src = ('#include <stdio.h>\n#include "zbot_ppo.h"\nint main(){printf("%zu %zu %zu %zu %zu\\n", sizeof(zbp_net), '
           'sizeof(zbp_batch), sizeof(zbp_loss_cfg), sizeof(zbp_params), sizeof(zbp_act_io));}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        sizes = list(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    assert sizes == [C.sizeof(fused.Net), C.sizeof(fused.Batch), C.sizeof(fused.LossCfg), C.sizeof(fused.Params),
                     C.sizeof(fused.ActIO)]
    L = fused.lib()
    n = fused.Net()
    n.n_layers = 4
    for i, dd in enumerate([23, 128, 128, 128, 6]):
        n.dim[i] = dd
    for i in range(4):
        n.w[i] = n.b[i] = 16  # non-null; not dereferenced by the shape check
    m = fused.Net.from_buffer_copy(n)
    m.dim[4] = 1
    assert L.zbp_workspace_floats(C.byref(n), C.byref(m), 24576) > 0
    n.dim[2] = 100  # hidden dims must be multiples of 32
    assert L.zbp_workspace_floats(C.byref(n), C.byref(m), 24576) < 0


def test_create_rejects_weighted_term_without_active_bit():
    """a walking-v2 cfg whose weighted term has its reward_active bit clear (e.g. a C caller that
    zero-initialises the struct) is refused before any HIP call, instead of silently freezing that term's
    buffers (include/zbot.h reward_active)."""
    from zbot_lab_amd import _native
    from zbot_lab_amd import model as zm
    L = _native.lib()
    m = zm.load_model()
    mc = zm.pack_model(m)
    c = zm.TaskCfg().pack()
    c.reward_active = 0
    h = C.c_void_p()
    rc = L.zb_create(C.byref(mc), C.byref(c), 4, 0, 0, C.byref(h))
    assert rc < 0 and b"reward_active" in L.zb_last_error()
