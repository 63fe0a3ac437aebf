from .walking_v2 import ZbotDirectEnvCfgV2, ZbotDirectEnvV2, grid_env_origins  # noqa: F401
