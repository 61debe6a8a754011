"""Loader for the in-tree HIP extension ``llmtrain/ops/_llmtrain_hip.so``.

The shared object is built by ``python -m llmtrain.ops.build`` (hipcc, ``--offload-arch=gfx950``)
and registers its kernels as ``torch.ops.llmtrain_hip.*`` through ``TORCH_LIBRARY``, so every
kernel shows up under its own name in ``rocprofv3 --kernel-trace`` and in ``torch.profiler``.

On a GPU box a missing or unloadable extension is a hard error (:func:`require`): the fused path
never silently falls back to eager PyTorch.
"""

from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

__all__ = ["EXT_PATH", "is_loaded", "load", "require"]

EXT_PATH = Path(__file__).with_name("_llmtrain_hip.so")
DEBUG_EXT_PATH = Path(__file__).with_name("_llmtrain_hip_debug.so")
_lock = threading.Lock()
_state: dict[str, object] = {"loaded": False, "error": None}


def load() -> bool:
    """Try to load the extension once; returns whether it is available."""
    with _lock:
        if _state["loaded"]:
            return True
        if _state["error"] is not None:
            return False
        default = DEBUG_EXT_PATH if os.environ.get("LLMTRAIN_DEBUG_KERNELS", "0") == "1" else EXT_PATH
        path = Path(os.environ.get("LLMTRAIN_HIP_EXT") or default)  # empty: the default
        if not path.exists():
            _state["error"] = f"{path} not found (build it with `python -m llmtrain.ops.build`)"
            return False
        try:
            torch.ops.load_library(str(path))
        except (OSError, RuntimeError) as exc:
            _state["error"] = f"failed to load {path}: {exc}"
            return False
        _state["loaded"] = True
        return True


def is_loaded() -> bool:
    return bool(_state["loaded"])


def require() -> None:
    """Raise unless the HIP extension is loaded (called before any GPU kernel launch)."""
    if not load():
        raise RuntimeError(f"llmtrain HIP extension unavailable: {_state['error']}")
