"""Causal self-attention entry point used by the transformer models.

GPU: flash attention through PyTorch's ROCm SDPA with the composable_kernel (CK) backend
selected -- CK's FMHA kernels are native CDNA MFMA code, tiled for 64-wide waves, and never
materialise the [T, T] score matrix.  CPU: the math reference.

All model code calls ``causal_attention`` so the backend can be swapped for a hand-written
kernel without touching the models.
"""

import torch
import torch.nn.functional as F

_configured = False


def _configure() -> None:
    global _configured
    if _configured:
        return
    _configured = True
    if torch.version.hip is not None and hasattr(torch.backends.cuda, "preferred_rocm_fa_library"):
        try:
            torch.backends.cuda.preferred_rocm_fa_library("ck")
        except Exception:  # pragma: no cover - older builds without CK FMHA
            pass


def causal_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, dropout_p: float = 0.0) -> torch.Tensor:
    """``softmax(q k^T / sqrt(d) + causal_mask) v`` for ``[B, H, T, D]`` tensors."""
    if q.is_cuda:
        _configure()
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=True)
