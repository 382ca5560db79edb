"""Hand-written CDNA4 (gfx950) HIP kernels and their torch-facing wrappers.

The kernels live in ``determined_amd/csrc`` and are compiled in-tree into
``determined_amd/ops/_hip_ops*.so`` by ``determined_amd._build`` (driven from
``__graft_entry__.build``).  GPU tensors ALWAYS go through the HIP path: if the
extension is missing on a machine with a GPU the call raises instead of silently
falling back.  CPU tensors use an exact PyTorch reference implementation of the same
math (that is what the CPU test-suite exercises).
"""

import importlib
import importlib.util
import os
from typing import Any, Optional

_ext: Optional[Any] = None
_err: Optional[BaseException] = None


def _load() -> Optional[Any]:
    global _ext, _err
    if _ext is not None or _err is not None:
        return _ext
    try:
        import torch  # noqa: F401  (loads libtorch/libamdhip64 before the extension)

        alt = os.environ.get("DAMD_HIP_OPS_PATH")  # A/B runs: another build of the same extension
        if alt:
            spec = importlib.util.spec_from_file_location("determined_amd.ops._hip_ops", alt)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)  # type: ignore[union-attr]
            _ext = mod
        else:
            _ext = importlib.import_module("determined_amd.ops._hip_ops")
    except BaseException as e:  # ImportError, OSError from a bad .so, ...
        _err = e
        if os.environ.get("DAMD_AUTOBUILD", "0") == "1":
            from determined_amd import _build

            _build.build_hip_ops()
            _err = None
            _ext = importlib.import_module("determined_amd.ops._hip_ops")
    return _ext


def available() -> bool:
    return _load() is not None


def ext() -> Any:
    """Return the compiled extension or raise loudly (used for every GPU tensor)."""
    e = _load()
    if e is None:
        raise RuntimeError(
            "determined_amd HIP kernels are not built (run `python -m determined_amd._build`); "
            f"import error: {_err!r}"
        )
    return e


_DISABLED = frozenset(f.strip() for f in os.environ.get("DAMD_DISABLE_FUSIONS", "").split(",") if f.strip())


def fusion_enabled(name: str) -> bool:
    """Model-level fusions can be switched off for A/B measurements with
    ``DAMD_DISABLE_FUSIONS=stem_conv,stem_stats,stem_pool,split_grad,avgpool,igemm_conv,conv_stats,bn_conv,bn_prologue,bn_lazy_bwd,
    compact_shortcut_grad,bn_residual_fold`` (the replacement is the
    plain PyTorch / MIOpen composition, never a silent eager fallback of a kernel)."""
    return name not in _DISABLED


def conv_sk_timeouts(device=None) -> int:
    """Number of stream-K hand-off time-outs on ``device`` since the last check (resets the counter and
    the flag buffers; syncs the device).  0 without the extension or a GPU."""
    import torch

    if _ext is None or not torch.cuda.is_available():
        return 0
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    return int(_ext.conv_sk_timeouts(torch.empty(0, device=dev), True))


def conv_health_check(device=None) -> None:
    """Raise if any stream-K convolution on ``device`` timed out waiting for a partial tile
    (conv_igemm.hip sk_gather: such a tile is written as NaN, never silently wrong).  Syncs the
    device; called after conv tuning and at the trainer's reporting boundaries.  On a time-out the
    flag buffers are reset and the stream-K configs are excluded from later tuning choices."""
    import torch

    if _ext is None or not torch.cuda.is_available():
        return
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    n = conv_sk_timeouts(dev)
    if n:
        from determined_amd.ops import conv as _conv

        _conv.exclude_stream_k()
        raise RuntimeError(f"{n} stream-K convolution hand-off(s) timed out on {dev}: the affected output tiles "
                           "were written as NaN; stream-K configs are now excluded from the tuning choices")


from determined_amd.ops.optim import FusedAdamW, FusedSGD, fused_clip_grad_norm_  # noqa: E402
from determined_amd.ops.norm import (  # noqa: E402
    FusedLayerNorm,
    FusedRMSNorm,
    layer_norm,
    rms_norm,
)
from determined_amd.ops.scaler import DeviceGradScaler  # noqa: E402
from determined_amd.ops.bn import BatchNormAct2d  # noqa: E402

__all__ = [
    "available",
    "conv_health_check",
    "conv_sk_timeouts",
    "ext",
    "FusedAdamW",
    "FusedSGD",
    "fused_clip_grad_norm_",
    "FusedLayerNorm",
    "FusedRMSNorm",
    "layer_norm",
    "rms_norm",
    "DeviceGradScaler",
    "BatchNormAct2d",
]
