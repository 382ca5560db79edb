"""ResNet-50 training step used by bench.py and the rocprof profiles.

Variants:
* ``bf16_master`` (default): every parameter and activation in bf16 (channels-last), bf16
  gradients all-reduced over RCCL (half the xGMI bytes of fp32), fp32 master weights and
  momentum updated by the fused SGD kernel, which writes the bf16 copy back in-pass.
* ``bf16_fp32bn``: as above but BatchNorm affine params kept in fp32 (MIOpen mixed BN).
* ``amp``: fp32 parameters + ``torch.autocast(bfloat16)`` (conv weights re-cast every step).
"""

from typing import Any, Callable, Dict, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from determined_amd.models.resnet import resnet50


def param_groups(model: nn.Module, weight_decay: float):
    decay, no_decay = [], []
    for n, p in model.named_parameters():
        (no_decay if p.ndim <= 1 else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]


def make_model(variant: str, device: torch.device) -> nn.Module:
    model = resnet50().to(device)
    if variant == "bf16_master":
        model = model.to(torch.bfloat16)
    elif variant == "bf16_fp32bn":
        for m in model.modules():
            if not isinstance(m, nn.BatchNorm2d):
                for p in m.parameters(recurse=False):
                    p.data = p.data.to(torch.bfloat16)
    return model.to(memory_format=torch.channels_last)


def synthetic_batch(batch: int, dtype: torch.dtype, device: torch.device, seed: int = 0):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn(batch, 3, 224, 224, generator=g, device=device, dtype=torch.float32)
    x = x.to(dtype).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), generator=g, device=device)
    return x, y


def build_step(batch: int = 256, variant: str = "bf16_master", bucket_mb: float = 16.0,
               use_harness: bool = True) -> Tuple[Callable[[], None], Dict[str, Any]]:
    device = torch.device("cuda", torch.cuda.current_device())
    if use_harness:
        from determined_amd.benchmarks._harness_step import harness_step

        return harness_step(batch=batch, variant=variant, bucket_mb=bucket_mb, device=device)

    from determined_amd.ops import FusedSGD
    from determined_amd.parallel.ddp import DistributedDataParallel

    model = make_model(variant, device)
    ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_mb)
    opt = FusedSGD(param_groups(model, 1e-4), lr=0.1, momentum=0.9, master_weights=True)
    in_dtype = torch.float32 if variant == "amp" else torch.bfloat16
    batches = [synthetic_batch(batch, in_dtype, device, seed=s) for s in range(2)]
    state: Dict[str, Any] = {"i": 0, "loss": None}

    def step() -> None:
        x, y = batches[state["i"] % len(batches)]
        state["i"] += 1
        if variant == "amp":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = ddp(x)
        else:
            out = ddp(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        ddp.finish()
        opt.step()
        ddp.zero_grad()
        state["loss"] = loss.detach()

    state["last_loss"] = lambda: state["loss"].item()
    return step, state
