"""Loaders of the in-tree native extensions (built by ``llm_mcp_amd.build``).

Both raise a clear error when the extension is missing instead of degrading
to a Python fallback; ``ensure_built()`` compiles them in place first."""
from __future__ import annotations

import importlib
import os

_mods: dict[str, object] = {}


def ensure_built(force: bool = False) -> None:
    from . import build
    build.build_all(force=force)


def _load(name: str):
    if name not in _mods:
        try:
            _mods[name] = importlib.import_module(f"llm_mcp_amd.{name}")
        except ImportError:
            if os.environ.get("LMX_AUTOBUILD", "1") != "1":
                raise
            ensure_built()
            _mods[name] = importlib.import_module(f"llm_mcp_amd.{name}")
    return _mods[name]


def runtime():
    """C++ runtime: JobQueue, BlockManager, Scheduler."""
    return _load("_lmx_runtime")


def kernels():
    """gfx950 HIP kernels (import torch first: shares its HIP runtime)."""
    import torch  # noqa: F401  (loads libamdhip64 before the extension)
    return _load("_lmx_kernels")
