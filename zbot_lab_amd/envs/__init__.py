from .walking_v2 import ZbotDirectEnvCfgV2, ZbotDirectEnvV2, grid_env_origins  # noqa: F401
from .standup_v0 import Zbot6SUpEnv, Zbot6SUpEnvCfg  # noqa: F401
from .walking_v4 import Zbot6SEnvV4, Zbot6SEnvV4Cfg  # noqa: F401
from .manager_flat import ZbotManagerBasedRLEnv, Zbot6BFlatEnvCfg, Zbot6BFlatEnvCfg_PLAY  # noqa: F401
