"""Route a HuggingFace encoder's hot ops through determined_amd's MI355X kernels.

``accelerate(model)`` (BERT / RoBERTa-style encoders, ``transformers`` 5.x):

* attention -> ``csrc/attention.hip`` flash attention (non-causal, key-padding mask, in-kernel
  attention-probability dropout), registered as the ``"damd"`` attention implementation through
  ``AttentionInterface`` together with a mask function that hands the kernel its uint8 key mask
  (built once per forward, ``None`` for unpadded batches);
* ``BertSelfOutput`` / ``BertOutput`` (dense -> dropout -> LayerNorm(. + residual)) -> the dense GEMM
  followed by ONE ``csrc/norm.hip`` kernel doing residual add + dropout + LayerNorm (its backward
  emits both gradients in one pass);
* every other ``nn.LayerNorm`` (embeddings, MLM head) -> ``FusedLayerNorm``.

Shapes the kernels do not serve (CPU, fp32, head dim not in {64, 128}, cross attention with
different lengths) fall back to PyTorch SDPA with the equivalent boolean mask.  Reference: the
HF Trainer path of ``harness/determined/transformers/_hf_callback.py`` runs the stock modules.
"""

import types
from typing import Any, Optional

import torch
from torch import nn

from determined_amd.ops.attention import _supported, flash_attention, key_mask
from determined_amd.ops.norm import FusedLayerNorm, residual_dropout_layer_norm

NAME = "damd"


def _damd_mask(batch_size: int, q_length: int, kv_length: int, q_offset: int = 0, kv_offset: int = 0,
               attention_mask: Optional[torch.Tensor] = None, **kwargs: Any) -> Optional[torch.Tensor]:
    """Mask interface for the ``"damd"`` attention: None when no key is padded, else the kernels'
    uint8 key mask (one check per model forward, like the flash-attention-2 mask function)."""
    if attention_mask is None:
        return None
    am = attention_mask[:, -kv_length:]
    if am.dim() != 2:
        return am
    # (inside a graph capture the all-valid shortcut would be a host sync: always pass the mask there)
    capturing = am.is_cuda and torch.cuda.is_current_stream_capturing()
    if am.shape[1] == kv_length and not capturing and bool(am.all()):
        return None
    return key_mask(am.bool())


def _damd_attention(module: nn.Module, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                    attention_mask: Optional[torch.Tensor], dropout: float = 0.0, scaling: Optional[float] = None,
                    is_causal: Optional[bool] = None, **kwargs: Any):
    causal = bool(getattr(module, "is_causal", False) if is_causal is None else is_causal)
    same_len = query.shape[2] == key.shape[2]
    kernel_mask = attention_mask is None or (attention_mask.dtype == torch.uint8 and attention_mask.dim() == 2)
    if same_len and kernel_mask:
        km = attention_mask
        q, k, v = (t if t.stride(-1) == 1 else t.contiguous() for t in (query, key, value))
        if _supported(q, k, v):
            o = flash_attention(q, k, v, causal=causal, scale=scaling, key_padding=km,
                                dropout_p=dropout if module.training else 0.0)
            return o.transpose(1, 2), None
    # fallback: SDPA with a boolean [B, 1, 1|Tq, Tk] mask
    mask = attention_mask
    if mask is not None and mask.dtype == torch.uint8 and mask.dim() == 2:
        mask = mask[:, None, None, : key.shape[2]].bool()
    o = torch.nn.functional.scaled_dot_product_attention(query, key, value, attn_mask=mask,
                                                         dropout_p=dropout if module.training else 0.0,
                                                         is_causal=causal and mask is None, scale=scaling)
    return o.transpose(1, 2).contiguous(), None


def register() -> None:
    from transformers import AttentionInterface
    from transformers.masking_utils import AttentionMaskInterface

    AttentionInterface.register(NAME, _damd_attention)
    AttentionMaskInterface.register(NAME, _damd_mask)


def _fused_output_forward(self, hidden_states: torch.Tensor, input_tensor: torch.Tensor) -> torch.Tensor:
    h = self.dense(hidden_states)
    if h.dtype != input_tensor.dtype:  # autocast: bf16 GEMM output, fp32 residual stream (as in the stock add)
        h = h.to(input_tensor.dtype)
    _, y = residual_dropout_layer_norm(input_tensor, h, self.LayerNorm, self.dropout.p, self.training)
    return y


def _to_fused(ln: nn.LayerNorm) -> FusedLayerNorm:
    f = FusedLayerNorm(ln.normalized_shape, eps=ln.eps, bias=ln.bias is not None,
                       device=ln.weight.device, dtype=ln.weight.dtype)
    with torch.no_grad():
        f.weight.copy_(ln.weight)
        if ln.bias is not None:
            f.bias.copy_(ln.bias)
    return f


def accelerate(model: nn.Module) -> nn.Module:
    """Swap in the fused kernels (in place; returns ``model``).  Parameters keep their names, so
    checkpoints stay loadable by the stock modules."""
    register()
    if hasattr(model, "set_attn_implementation"):
        model.set_attn_implementation(NAME)
    else:
        model.config._attn_implementation = NAME
    for name, mod in list(model.named_modules()):
        cls = type(mod).__name__
        if cls.endswith("SelfOutput") or (cls.endswith("Output") and hasattr(mod, "dense")
                                          and isinstance(getattr(mod, "LayerNorm", None), nn.LayerNorm)):
            mod.LayerNorm = _to_fused(mod.LayerNorm)
            mod.forward = types.MethodType(_fused_output_forward, mod)
    for name, mod in list(model.named_modules()):
        for child_name, child in list(mod.named_children()):
            if isinstance(child, nn.LayerNorm) and len(child.normalized_shape) == 1:
                setattr(mod, child_name, _to_fused(child))
    return model
