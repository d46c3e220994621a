"""Loader for the native gfx950 extension ``ml_trainer_amd._C``.

Policy (no silent fallbacks on the GPU): when a device tensor reaches an op that
has a HIP kernel, the extension MUST be importable -- :func:`require_native`
raises with build instructions otherwise. Pure-torch code paths exist only for
CPU tensors (the reference's CPU/gloo plumbing config, BASELINE.json config 1).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

_C = None
_err: Optional[BaseException] = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        _C = importlib.import_module("ml_trainer_amd._C")
    except BaseException as e:  # ImportError, OSError (undefined symbol), ...
        _err = e
        if os.environ.get("MLT_AUTOBUILD", "0") == "1":
            from ml_trainer_amd.build import build
            build(verbose=True)
            _err = None
            _C = importlib.import_module("ml_trainer_amd._C")
    return _C


def native_available() -> bool:
    return _load() is not None


def require_native():
    """Return the extension module or raise loudly (GPU paths)."""
    mod = _load()
    if mod is None:
        raise RuntimeError(
            "ml_trainer_amd native extension is not built/importable "
            f"({_err!r}). Build it with `python -m ml_trainer_amd.build` "
            "(hipcc --offload-arch=gfx950) before running on an MI355X.")
    return mod


def use_native(t) -> bool:
    """True when `t` lives on the GPU: the HIP kernel is then mandatory."""
    if getattr(t, "is_cuda", False):
        require_native()
        return True
    return False
