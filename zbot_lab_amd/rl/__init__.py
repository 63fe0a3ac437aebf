from .vecenv import RslRlVecEnvWrapper  # noqa: F401
from .cfg import PPORunnerCfgV2, Zbot6SEnvV4PPOCfg, Zbot6SUpEnvPPOCfg  # noqa: F401
from .ppo import PPO, ActorCritic, RolloutStorage  # noqa: F401
from .runner import OnPolicyRunner  # noqa: F401
from .export import dump_yaml, export_policy_as_jit, get_checkpoint_path  # noqa: F401
