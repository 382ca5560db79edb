"""C++ control plane (search methods, scheduler) compiled in-tree by determined_amd._build."""

import importlib
import importlib.util
import os
from typing import Any, Optional

_mod: Optional[Any] = None
_err: Optional[BaseException] = None


def load() -> Any:
    """Return the compiled ``_native`` module (building it on first use if needed)."""
    global _mod, _err
    if _mod is not None:
        return _mod
    alt = os.environ.get("DAMD_NATIVE_PATH")  # e.g. the sanitizer build (python -m determined_amd._build --sanitize)
    if alt:
        spec = importlib.util.spec_from_file_location("determined_amd._native._native", alt)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)  # type: ignore[union-attr]
        _mod = mod
        return _mod
    try:
        _mod = importlib.import_module("determined_amd._native._native")
    except ImportError as e:
        _err = e
        from determined_amd import _build

        _build.build_native()
        _mod = importlib.import_module("determined_amd._native._native")
    return _mod
