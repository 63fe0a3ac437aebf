"""``PPORunnerCfgV2`` (reference ``source/zbot/zbot/tasks/zbot6b_direct/agents/rsl_rl_ppo_cfg.py:65-91``) and
``Zbot6SUpEnvPPOCfg`` (same file, 264-289), ``Zbot6SEnvV4PPOCfg`` (206-233) and the manager env's
``Zbot6BFlatPPORunnerCfg`` (``zbotlab_manager/config/zbot6b_manager/agents/rsl_rl_ppo_cfg.py:11-49``).

Consumed by ``zbot_lab_amd.rl.OnPolicyRunner`` (``agent_cfg.to_dict()``, as ``train.py:192``)."""
from __future__ import annotations

from dataclasses import asdict, dataclass, field


@dataclass
class RslRlPpoActorCriticCfg:
    class_name: str = "ActorCritic"
    init_noise_std: float = 1.0
    actor_hidden_dims: list = field(default_factory=lambda: [128, 128, 128])
    critic_hidden_dims: list = field(default_factory=lambda: [128, 128, 128])
    activation: str = "elu"
    actor_obs_normalization: bool = False
    critic_obs_normalization: bool = False


@dataclass
class RslRlPpoAlgorithmCfg:
    class_name: str = "PPO"
    value_loss_coef: float = 1.0
    use_clipped_value_loss: bool = True
    clip_param: float = 0.2
    entropy_coef: float = 0.005
    num_learning_epochs: int = 5
    num_mini_batches: int = 4
    learning_rate: float = 1.0e-3
    schedule: str = "adaptive"
    gamma: float = 0.99
    lam: float = 0.95
    desired_kl: float = 0.01
    max_grad_norm: float = 1.0


@dataclass
class PPORunnerCfgV2:
    class_name: str = "OnPolicyRunner"
    seed: int = 42
    device: str = "cuda:0"
    num_steps_per_env: int = 24
    max_iterations: int = 1000
    save_interval: int = 100
    experiment_name: str = "zbot_6b_flat_direct_v2"
    empirical_normalization: bool = False
    clip_actions: float | None = None
    # RslRlOnPolicyRunnerCfg load / logging fields (cli_args.py:76-85 writes them)
    run_name: str = ""
    resume: bool = False
    load_run: str = ".*"
    load_checkpoint: str = "model_.*.pt"
    logger: str = "tensorboard"
    policy: RslRlPpoActorCriticCfg = field(default_factory=RslRlPpoActorCriticCfg)
    algorithm: RslRlPpoAlgorithmCfg = field(default_factory=RslRlPpoAlgorithmCfg)

    def to_dict(self) -> dict:
        return asdict(self)


@dataclass
class Zbot6SUpEnvPPOCfg(PPORunnerCfgV2):
    """rsl_rl_ppo_cfg.py:264-289: the stand-up task's [256, 256, 128] actor / critic."""
    experiment_name: str = "zbot_6b_flat_direct_standup"
    policy: RslRlPpoActorCriticCfg = field(default_factory=lambda: RslRlPpoActorCriticCfg(
        actor_hidden_dims=[256, 256, 128], critic_hidden_dims=[256, 256, 128]))


@dataclass
class Zbot6SEnvV4PPOCfg(PPORunnerCfgV2):
    """rsl_rl_ppo_cfg.py:206-233: v4's [256, 256, 128] actor / critic, 2000 iterations."""
    max_iterations: int = 2000
    save_interval: int = 1000
    experiment_name: str = "zbot_6b_flat_direct_v4"
    policy: RslRlPpoActorCriticCfg = field(default_factory=lambda: RslRlPpoActorCriticCfg(
        actor_hidden_dims=[256, 256, 128], critic_hidden_dims=[256, 256, 128]))


@dataclass
class Zbot6BFlatPPORunnerCfg(PPORunnerCfgV2):
    """zbotlab_manager agents/rsl_rl_ppo_cfg.py:11-49: Zbot6BRoughPPORunnerCfg (entropy 0.01, 24 steps)
    with the flat overrides (1000 iterations, [128, 128, 128] actor / critic)."""
    max_iterations: int = 1000
    save_interval: int = 100
    experiment_name: str = "zbot_6b_flat_mana_v1"
    algorithm: RslRlPpoAlgorithmCfg = field(default_factory=lambda: RslRlPpoAlgorithmCfg(entropy_coef=0.01))
