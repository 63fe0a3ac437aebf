from .vecenv import RslRlVecEnvWrapper  # noqa: F401
from .cfg import PPORunnerCfgV2  # noqa: F401
