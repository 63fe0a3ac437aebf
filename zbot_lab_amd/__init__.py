"""zbot_lab_amd — MI355X-native batched simulator for the ZBOT-6 ``zbot-6b-walking-v2`` task.

Hot path: one fused HIP kernel per policy step (``csrc/zbot_sim.hip`` -> ``libzbot.so``, C ABI in
``include/zbot.h``). Host side mirrors the reference's DirectRLEnv / rsl_rl VecEnv interfaces.
"""
import os as _os
import sys as _sys

# HIP graphs: ROCm's "packet capture" graph mode (the CLR default) makes the captured PPO update
# replay with wrong results from its second replay on (tests/test_ppo.py
# ::test_gpu_update_graph_matches_eager fails with DEBUG_CLR_GRAPH_PACKET_CAPTURE=1). Narrowed in
# tools/graph_repro/clip_repro.py: a captured large GEMM (1024x512, K = 8192) followed by a
# reduction over its output replays wrong under packet capture -- no kernel of this package is
# involved. The runtime reads the switch once, when HIP initialises --
# which any HIP call does, torch.cuda.is_available() / device_count() included, even while
# torch.cuda.is_initialized() is still False. GRAPHS_SAFE is therefore True only when the switch
# is certain to have been read as "0": it was in the process environment at launch
# (/proc/self/environ: scripts/train.py and play.py re-launch nothing, they set it before
# importing torch), or torch was not imported yet when this package set it. Otherwise the PPO
# runner runs eagerly.
def _launch_env(name: str):
    try:
        with open("/proc/self/environ", "rb") as f:
            for kv in f.read().split(b"\0"):
                k, _, v = kv.partition(b"=")
                if k.decode(errors="replace") == name:
                    return v.decode(errors="replace")
    except OSError:
        pass
    return None


_KNOB = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
_torch_first = "torch" in _sys.modules
if not _torch_first:
    _os.environ.setdefault(_KNOB, "0")
GRAPHS_SAFE = _os.environ.get(_KNOB) == "0" and (not _torch_first or _launch_env(_KNOB) == "0")

from . import model  # noqa: F401
from .tasks import make, register, registered  # noqa: F401

__all__ = ["make", "register", "registered", "model"]
