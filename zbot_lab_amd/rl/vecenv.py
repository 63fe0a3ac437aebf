"""rsl_rl VecEnv adapter for the DirectRLEnv-compatible envs.

Mirrors ``isaaclab_rl.rsl_rl.RslRlVecEnvWrapper`` as the reference uses it (``scripts/rsl_rl/
train.py:181``, rsl-rl-lib >= 3.0.1, ``train.py:59-71``): ``get_observations()`` returns the
observation groups (a ``TensorDict`` when tensordict is installed, else a dict),
``step(a) -> (obs, rew, dones = terminated | truncated, extras)`` with ``extras["time_outs"]``.
"""
from __future__ import annotations

import torch

try:  # rsl-rl-lib 3.x hands TensorDicts around; optional here
    from tensordict import TensorDict as _TensorDict
except ImportError:  # pragma: no cover - not installed in this image
    _TensorDict = None


def _as_obs(obs: dict, num_envs: int):
    if _TensorDict is not None:
        return _TensorDict(obs, batch_size=[num_envs])
    return obs


class RslRlVecEnvWrapper:
    def __init__(self, env, clip_actions: float | None = None):
        self.env = env
        self.clip_actions = clip_actions
        self.num_envs = env.unwrapped.num_envs
        self.device = env.unwrapped.device
        self.max_episode_length = env.unwrapped.max_episode_length
        self.num_actions = env.unwrapped.single_action_space.shape[0]
        self.cfg = env.unwrapped.cfg
        # the native sim writes terminated | truncated as int64 into a registered buffer inside its step
        # kernel (zb_set_done_buffer), so step() returns that instead of two torch launches per step
        sim = getattr(env.unwrapped, "sim", None)
        self._dones = sim.done_buffer() if hasattr(sim, "done_buffer") else None
        self.env.reset()

    @property
    def unwrapped(self):
        return self.env.unwrapped

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self.env.unwrapped.episode_length_buf

    @episode_length_buf.setter
    def episode_length_buf(self, value: torch.Tensor) -> None:
        self.env.unwrapped.episode_length_buf = value

    def seed(self, seed: int = -1) -> int:
        return self.env.unwrapped.seed(seed)

    def get_observations(self):
        return _as_obs(self.env.unwrapped.get_observations(), self.num_envs)

    def reset(self):
        obs, extras = self.env.reset()
        return _as_obs(obs, self.num_envs), extras

    def step(self, actions: torch.Tensor):
        if self.clip_actions is not None:
            actions = torch.clamp(actions, -self.clip_actions, self.clip_actions)
        obs, rew, terminated, truncated, extras = self.env.step(actions)
        dones = self._dones if self._dones is not None else (terminated | truncated).to(dtype=torch.long)
        extras["time_outs"] = truncated
        return _as_obs(obs, self.num_envs), rew, dones, extras

    def close(self):
        return self.env.close()
