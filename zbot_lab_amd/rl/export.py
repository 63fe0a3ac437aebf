"""Checkpoint resolution, cfg dumps and policy export used by ``scripts/train.py`` / ``scripts/play.py``.

Restates the Isaac Lab helpers the reference scripts call (their package is absent here):
``isaaclab_tasks.utils.get_checkpoint_path`` (``train.py:165-166``, ``play.py:110``),
``isaaclab.utils.io.dump_yaml`` (``train.py:199-200``) and
``isaaclab_rl.rsl_rl.export_policy_as_jit`` (``play.py:172-174``). ONNX export
(``play.py:175``) needs the ``onnx`` package, which this image does not have.
"""
from __future__ import annotations

import copy
import dataclasses
import os
import re

import torch
import torch.nn as nn


def get_checkpoint_path(log_path: str, run_dir: str = ".*", checkpoint: str = ".*", other_dirs=None,
                        sort_alpha: bool = True) -> str:
    """Newest run folder under ``log_path`` whose name matches ``run_dir`` (alphabetical order, i.e. the
    time-stamped names sort by time), then the highest-numbered file in it matching ``checkpoint``
    (names compared zero-padded to 15 characters, so ``model_1000.pt`` sorts after ``model_999.pt``)."""
    try:
        runs = [os.path.join(log_path, r.name) for r in os.scandir(log_path) if r.is_dir() and re.match(run_dir, r.name)]
    except FileNotFoundError:
        runs = []
    if not runs:
        raise ValueError(f"No runs present in the directory: '{log_path}' match: '{run_dir}'.")
    runs.sort() if sort_alpha else runs.sort(key=os.path.getmtime)
    run_path = os.path.join(runs[-1], *other_dirs) if other_dirs else runs[-1]
    ckpts = [f for f in os.listdir(run_path) if re.match(checkpoint, f)]
    if not ckpts:
        raise ValueError(f"No checkpoints in the directory: '{run_path}' match '{checkpoint}'.")
    ckpts.sort(key=lambda m: f"{m:0>15}")
    return os.path.join(run_path, ckpts[-1])


def _plain(obj):
    if dataclasses.is_dataclass(obj) and not isinstance(obj, type):
        return {f.name: _plain(getattr(obj, f.name)) for f in dataclasses.fields(obj)}
    if hasattr(obj, "to_dict"):
        return _plain(obj.to_dict())
    if isinstance(obj, dict):
        return {str(k): _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    if isinstance(obj, (int, float, str, bool)) or obj is None:
        return obj
    if hasattr(obj, "__dict__"):
        return {k: _plain(v) for k, v in vars(obj).items() if not k.startswith("_") and not callable(v)}
    return repr(obj)


def dump_yaml(filename: str, data) -> None:
    """Write a cfg object (dataclass / configclass-like / dict) as YAML, creating the folder."""
    import yaml
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    with open(filename, "w") as f:
        yaml.safe_dump(_plain(data), f, default_flow_style=False, sort_keys=False)


def _plain_linears(m: nn.Module) -> nn.Module:
    """Copy of ``m`` with every ``nn.Linear`` subclass (the PPO's split-K training layer) replaced by
    a plain ``nn.Linear`` holding the same weights, so TorchScript sees the standard module."""
    m = copy.deepcopy(m)
    for name, child in list(m.named_children()):
        if isinstance(child, nn.Linear) and type(child) is not nn.Linear:
            lin = nn.Linear(child.in_features, child.out_features, bias=child.bias is not None)
            lin.load_state_dict(child.state_dict())
            setattr(m, name, lin)
        else:
            setattr(m, name, _plain_linears(child))
    return m


class _TorchPolicyExporter(nn.Module):
    """actor(normalizer(obs)) as a self-contained TorchScript module (rsl_rl's deterministic policy)."""

    def __init__(self, policy, normalizer=None):
        super().__init__()
        self.actor = _plain_linears(policy.actor).cpu()
        self.normalizer = copy.deepcopy(normalizer).cpu() if normalizer is not None else nn.Identity()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.actor(self.normalizer(x))

    @torch.jit.export
    def reset(self) -> None:
        pass


def export_policy_as_jit(policy, normalizer=None, path: str = ".", filename: str = "policy.pt") -> str:
    os.makedirs(path, exist_ok=True)
    out = os.path.join(path, filename)
    mod = _TorchPolicyExporter(policy, normalizer).eval()
    torch.jit.script(mod).save(out)
    return out
