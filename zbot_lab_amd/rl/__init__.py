from .vecenv import RslRlVecEnvWrapper  # noqa: F401
from .cfg import PPORunnerCfgV2  # noqa: F401
from .ppo import PPO, ActorCritic, RolloutStorage  # noqa: F401
from .runner import OnPolicyRunner  # noqa: F401
