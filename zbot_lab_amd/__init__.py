"""zbot_lab_amd — MI355X-native batched simulator for the ZBOT-6 ``zbot-6b-walking-v2`` task.

Hot path: one fused HIP kernel per policy step (``csrc/zbot_sim.hip`` -> ``libzbot.so``, C ABI in
``include/zbot.h``). Host side mirrors the reference's DirectRLEnv / rsl_rl VecEnv interfaces.
"""
from . import model  # noqa: F401
from .tasks import make, register, registered  # noqa: F401

__all__ = ["make", "register", "registered", "model"]
