"""zbot_lab_amd — MI355X-native batched simulator for the ZBOT-6 ``zbot-6b-walking-v2`` task.

Hot path: one fused HIP kernel per policy step (``csrc/zbot_sim.hip`` -> ``libzbot.so``, C ABI in
``include/zbot.h``). Host side mirrors the reference's DirectRLEnv / rsl_rl VecEnv interfaces.
"""
import os as _os
import sys as _sys

# HIP graphs: ROCm's "packet capture" graph mode (the CLR default) leaves a replayed graph with
# kernel arguments that later eager launches of the same kernels overwrite -- a captured PPO update
# or rollout then silently computes with another launch's arguments (tests/test_ppo.py
# ::test_gpu_update_graph_matches_eager). The runtime reads the switch once, when HIP
# initialises, so it is set here, before anything touches the GPU. GRAPHS_SAFE records whether that
# worked (False when the GPU was initialised before this import without the switch); the PPO runner
# then runs eagerly.
_torch = _sys.modules.get("torch")
_late = _torch is not None and getattr(_torch, "cuda", None) is not None and _torch.cuda.is_initialized()
if not _late:
    _os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
GRAPHS_SAFE = _os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0"

from . import model  # noqa: F401
from .tasks import make, register, registered  # noqa: F401

__all__ = ["make", "register", "registered", "model"]
