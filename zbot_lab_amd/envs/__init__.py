from .walking_v2 import ZbotDirectEnvCfgV2, ZbotDirectEnvV2, grid_env_origins  # noqa: F401
from .standup_v0 import Zbot6SUpEnv, Zbot6SUpEnvCfg  # noqa: F401
