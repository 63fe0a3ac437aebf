"""Task registry: ``make("zbot-6b-walking-v2")`` like ``gym.make`` on the reference's registration
(``source/zbot/zbot/tasks/zbot6b_direct/__init__.py:41-49``; ``zbot-6b-standup-v0`` 111-119;
``zbot-6b-walking-v4`` 91-99; ``zbot-6b-walking-m-v0`` / ``-m-play-v0``:
``zbotlab_manager/config/zbot6b_manager/__init__.py:18-36``; the rough variants need the terrain
generator and are out of scope)."""
from __future__ import annotations

import importlib
from dataclasses import dataclass, field


@dataclass
class EnvSpec:
    id: str
    entry_point: str
    kwargs: dict = field(default_factory=dict)


_REGISTRY: dict[str, EnvSpec] = {}


def register(id: str, entry_point: str, kwargs: dict | None = None, disable_env_checker: bool = True) -> None:
    _REGISTRY[id] = EnvSpec(id, entry_point, dict(kwargs or {}))


def _load(ref):
    if not isinstance(ref, str):
        return ref
    mod, name = ref.split(":")
    return getattr(importlib.import_module(mod), name)


def spec(id: str) -> EnvSpec:
    if id not in _REGISTRY:
        raise KeyError(f"unknown task {id!r}; registered: {sorted(_REGISTRY)}")
    return _REGISTRY[id]


def load_cfg(id: str, key: str = "env_cfg_entry_point"):
    ref = spec(id).kwargs[key]
    obj = _load(ref)
    return obj() if isinstance(obj, type) else obj


def make(id: str, cfg=None, render_mode=None, **kwargs):
    s = spec(id)
    env_cls = _load(s.entry_point)
    cfg = cfg if cfg is not None else load_cfg(id)
    return env_cls(cfg, render_mode=render_mode, **kwargs)


def registered() -> list[str]:
    return sorted(_REGISTRY)


register(
    id="zbot-6b-walking-v2",
    entry_point="zbot_lab_amd.envs.walking_v2:ZbotDirectEnvV2",
    kwargs={
        "env_cfg_entry_point": "zbot_lab_amd.envs.walking_v2:ZbotDirectEnvCfgV2",
        "rsl_rl_cfg_entry_point": "zbot_lab_amd.rl.cfg:PPORunnerCfgV2",
    },
)

register(
    id="zbot-6b-standup-v0",
    entry_point="zbot_lab_amd.envs.standup_v0:Zbot6SUpEnv",
    kwargs={
        "env_cfg_entry_point": "zbot_lab_amd.envs.standup_v0:Zbot6SUpEnvCfg",
        "rsl_rl_cfg_entry_point": "zbot_lab_amd.rl.cfg:Zbot6SUpEnvPPOCfg",
    },
)

register(
    id="zbot-6b-walking-v4",
    entry_point="zbot_lab_amd.envs.walking_v4:Zbot6SEnvV4",
    kwargs={
        "env_cfg_entry_point": "zbot_lab_amd.envs.walking_v4:Zbot6SEnvV4Cfg",
        "rsl_rl_cfg_entry_point": "zbot_lab_amd.rl.cfg:Zbot6SEnvV4PPOCfg",
    },
)

register(
    id="zbot-6b-walking-m-v0",
    entry_point="zbot_lab_amd.envs.manager_flat:ZbotManagerBasedRLEnv",
    kwargs={
        "env_cfg_entry_point": "zbot_lab_amd.envs.manager_flat:Zbot6BFlatEnvCfg",
        "rsl_rl_cfg_entry_point": "zbot_lab_amd.rl.cfg:Zbot6BFlatPPORunnerCfg",
    },
)

register(
    id="zbot-6b-walking-m-play-v0",
    entry_point="zbot_lab_amd.envs.manager_flat:ZbotManagerBasedRLEnv",
    kwargs={
        "env_cfg_entry_point": "zbot_lab_amd.envs.manager_flat:Zbot6BFlatEnvCfg_PLAY",
        "rsl_rl_cfg_entry_point": "zbot_lab_amd.rl.cfg:Zbot6BFlatPPORunnerCfg",
    },
)


def apply_env_overrides(env_cfg, overrides):
    """``--env a.b=v``: set attribute path a.b of the env cfg; v parsed as a Python literal
    (bool / int / float / tuple) when it is one. Unknown paths raise, so a typo cannot silently
    train the unmodified cfg."""
    import ast
    for item in overrides:
        path, _, raw = item.partition("=")
        try:
            val = ast.literal_eval(raw)
        except (ValueError, SyntaxError):
            val = raw
        *parents, leaf = path.split(".")
        obj = env_cfg
        for a in parents:
            obj = getattr(obj, a)
        if not hasattr(obj, leaf):
            raise AttributeError(f"--env {item}: {type(obj).__name__} has no field {leaf!r}")
        setattr(obj, leaf, val)
    return env_cfg
