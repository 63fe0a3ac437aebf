"""HIP graph capture mode: GRAPHS_SAFE is True only when HIP is certain to read
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 -- the package set it before torch was imported, or it was in the
process environment at launch; torch imported first (which may already have initialised HIP, e.g.
through torch.cuda.is_available()) without it at launch gives False, and the PPO runner runs
eagerly. The training / play scripts import the package before torch."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _safe(code: str, env_extra: dict | None = None) -> bool:
    env = {k: v for k, v in os.environ.items() if k != "DEBUG_CLR_GRAPH_PACKET_CAPTURE"}
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, "-c", code + "; import zbot_lab_amd as z; print(z.GRAPHS_SAFE)"],
                         cwd=ROOT, env=env, capture_output=True, text=True, check=True).stdout.split()
    return out[-1] == "True"


def test_package_first_is_safe():
    assert _safe("import sys")


def test_torch_first_without_launch_env_is_not_safe():
    assert not _safe("import torch; torch.cuda.is_available()")


def test_torch_first_with_launch_env_is_safe():
    assert _safe("import torch", {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0"})


def test_packet_capture_requested_is_not_safe():
    assert not _safe("import sys", {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"})


def test_scripts_import_the_package_before_torch():
    for name in ("train.py", "play.py"):
        src = open(os.path.join(ROOT, "scripts", name)).read()
        assert src.index("import zbot_lab_amd") < src.index("import torch"), name
