"""ctypes binding of ``libzbot.so`` (the HIP simulator's C ABI, ``include/zbot.h``).

The library is built in-tree by ``__graft_entry__.build()`` / ``python -m zbot_lab_amd.build``.
There is no fallback: if the library or a GPU is missing, :func:`lib` raises. Argument meaning
and error behaviour follow ``include/zbot.h``; a negative return code becomes ``ZbotError`` with
the library's ``zb_last_error()`` text.
"""
from __future__ import annotations

import ctypes as C
import os

from . import model as zm

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, os.environ.get("ZBOT_LIB", "libzbot.so"))


class ZbotError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libzbot.so (raises ZbotError if it is missing — no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ZbotError(f"{LIB_PATH} not built: run `python -m zbot_lab_amd.build` (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.zb_last_error.restype = C.c_char_p
    L.zb_create.argtypes = [C.POINTER(zm.ZbModel), C.POINTER(zm.ZbTaskCfg), C.c_int, C.c_int, C.c_uint64,
                            C.POINTER(P)]
    L.zb_destroy.argtypes = [P]
    L.zb_num_envs.argtypes = [P]
    L.zb_reset.argtypes = [P, P, C.c_int, P]
    L.zb_step.argtypes = [P, P, P, P, P, P, P]
    L.zb_observe.argtypes = [P, P, P]
    L.zb_read_log.argtypes = [P, P, P, P]
    L.zb_set_log_buffers.argtypes = [P, P, P]
    L.zb_set_log_accumulator.argtypes = [P, P]
    L.zb_set_done_buffer.argtypes = [P, P]
    L.zb_get_state.argtypes = [P, P, P]
    L.zb_set_state.argtypes = [P, P, P]
    L.zb_get_contact_cache.argtypes = [P, P, P]
    L.zb_set_contact_cache.argtypes = [P, P, P]
    L.zb_physics_substeps.argtypes = [P, P, C.c_int, P, P, P]
    L.zb_profile_begin.argtypes = [P, C.c_int]
    L.zb_profile_stride.argtypes = [P, C.c_int]
    L.zb_profile_end.argtypes = [P, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    L.zb_read_stamps.argtypes = [P]
    L.zb_read_stamps.restype = C.c_int
    L.zb_read_stamps_slowest.argtypes = [P]
    L.zb_read_stamps_slowest.restype = C.c_int
    L.zb_read_stamp_hist.argtypes = [P]
    L.zb_read_stamp_hist.restype = C.c_int
    L.zb_read_wave_times.argtypes = [P, C.c_int]
    L.zb_read_wave_times.restype = C.c_int
    L.zb_state_dim.argtypes = [P]
    L.zb_set_link_friction.argtypes = [P, P, P]
    L.zb_set_link_friction_sd.argtypes = [P, P, P, P]
    L.zb_read_curriculum.argtypes = [P, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    L.zb_gjk_pairs.argtypes = [P, P, C.c_int, C.c_float, P, P]
    L.zb_pair_manifold.argtypes = [P, C.c_int, C.c_float, P, P]
    L.zb_pair_manifold_mode.argtypes = [P, C.c_int, C.c_float, C.c_int, P, P]
    for name in ("zb_create", "zb_num_envs", "zb_reset", "zb_step", "zb_observe", "zb_read_log", "zb_set_log_buffers", "zb_set_log_accumulator", "zb_set_done_buffer",
                 "zb_get_state", "zb_set_state", "zb_get_contact_cache", "zb_set_contact_cache", "zb_physics_substeps",
                 "zb_profile_begin", "zb_profile_end", "zb_profile_stride",
                 "zb_state_dim", "zb_set_link_friction", "zb_set_link_friction_sd", "zb_read_curriculum", "zb_gjk_pairs", "zb_pair_manifold", "zb_pair_manifold_mode"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


EXPORTED = ["zb_create", "zb_destroy", "zb_last_error", "zb_num_envs", "zb_reset", "zb_step", "zb_observe",
            "zb_read_log", "zb_set_log_buffers", "zb_set_log_accumulator", "zb_set_done_buffer", "zb_get_state", "zb_set_state", "zb_get_contact_cache",
            "zb_set_contact_cache", "zb_physics_substeps", "zb_profile_begin", "zb_profile_stride",
            "zb_profile_end", "zb_read_stamps", "zb_read_stamps_slowest", "zb_read_stamp_hist", "zb_read_wave_times", "zb_state_dim", "zb_set_link_friction", "zb_set_link_friction_sd",
            "zb_read_curriculum", "zb_gjk_pairs", "zb_pair_manifold", "zb_pair_manifold_mode"]


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().zb_last_error()
        raise ZbotError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def ptr(t) -> C.c_void_p:
    """Device pointer of a contiguous torch tensor (or None)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ZbotError("tensor passed to libzbot must be contiguous")
    return C.c_void_p(t.data_ptr())
