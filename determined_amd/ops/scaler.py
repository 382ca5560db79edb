"""Dynamic loss scaler whose state never leaves the GPU.

With the fused optimizers the AMP unscale, the non-finite check and the skip-on-overflow
all happen inside the optimizer's finalize/update kernels (csrc/optim.hip), so a scaled
fp16 step costs no host synchronisation (``torch.cuda.amp.GradScaler.step`` performs a
``.item()`` per step).  For other optimizers we fall back to torch's foreach unscale,
which does sync.  Reference counterpart: ``PyTorchTrialContext.wrap_scaler``
(``harness/determined/pytorch/_pytorch_context.py:505``).
"""

from typing import Any, Dict, Optional

import torch


class DeviceGradScaler:
    def __init__(
        self,
        init_scale: float = 2.0**16,
        growth_factor: float = 2.0,
        backoff_factor: float = 0.5,
        growth_interval: int = 2000,
        enabled: bool = True,
    ) -> None:
        self._enabled = enabled
        self._init_scale = init_scale
        self._growth_factor = growth_factor
        self._backoff_factor = backoff_factor
        self._growth_interval = growth_interval
        self._scale: Optional[torch.Tensor] = None
        self._growth_tracker: Optional[torch.Tensor] = None
        self._found_inf: Optional[torch.Tensor] = None
        self._inv_scale: Optional[torch.Tensor] = None
        self._unscaled: set = set()  # ids of optimizers unscale_()d since the last update()

    def is_enabled(self) -> bool:
        return self._enabled

    def _lazy_init(self, device: torch.device) -> None:
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=device)
            self._growth_tracker = torch.zeros((1,), dtype=torch.int32, device=device)
        if self._found_inf is None:
            self._found_inf = torch.zeros((1,), dtype=torch.int32, device=device)
            self._inv_scale = torch.empty((1,), dtype=torch.float32, device=device)

    def scale(self, outputs: torch.Tensor) -> torch.Tensor:
        if not self._enabled:
            return outputs
        self._lazy_init(outputs.device)
        assert self._scale is not None
        return outputs * self._scale.to(outputs.dtype)

    def get_scale(self) -> float:
        return float(self._scale.item()) if self._scale is not None else self._init_scale

    def unscale_(self, optimizer: torch.optim.Optimizer) -> None:
        """Divide the optimizer's gradients by the scale now (before gradient clipping) and record
        non-finite values; the following :meth:`step` then only applies the skip decision."""
        if not self._enabled or self._scale is None:
            return
        assert self._inv_scale is not None and self._found_inf is not None
        if id(optimizer) in self._unscaled:
            raise RuntimeError("unscale_() has already been called on this optimizer since the last update()")
        torch.reciprocal(self._scale, out=self._inv_scale)
        found = torch.zeros((1,), dtype=torch.float32, device=self._scale.device)
        grads = [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
        if grads:
            torch._amp_foreach_non_finite_check_and_unscale_(grads, found, self._inv_scale)
        self._found_inf.copy_(torch.maximum(self._found_inf, found.to(torch.int32)))
        self._unscaled.add(id(optimizer))

    def step(self, optimizer: torch.optim.Optimizer, *args: Any, **kwargs: Any) -> Optional[float]:
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        from determined_amd.ops.optim import _FusedBase

        assert self._scale is not None and self._inv_scale is not None and self._found_inf is not None
        fused = isinstance(optimizer, _FusedBase) and any(p.is_cuda for g in optimizer.param_groups for p in g["params"])
        if id(optimizer) in self._unscaled:  # gradients already unscaled and checked (unscale_)
            if fused:  # the skip decision stays on the device
                return optimizer.step(*args, found_inf=self._found_inf, **kwargs)
            if int(self._found_inf.item()) == 0:
                return optimizer.step(*args, **kwargs)
            return None
        torch.reciprocal(self._scale, out=self._inv_scale)
        if fused:
            self._found_inf.zero_()
            return optimizer.step(*args, grad_scale=self._inv_scale, found_inf=self._found_inf,
                                  check_finite=True, **kwargs)
        # Generic optimizer: torch's foreach unscale + a host-side skip decision.
        found = torch.zeros((1,), dtype=torch.float32, device=self._scale.device)
        grads = [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
        if grads:
            torch._amp_foreach_non_finite_check_and_unscale_(grads, found, self._inv_scale)
        self._found_inf.copy_(found.to(torch.int32))
        if float(found.item()) == 0.0:
            return optimizer.step(*args, **kwargs)
        return None

    def update(self, new_scale: Optional[float] = None) -> None:
        if not self._enabled or self._scale is None:
            return
        self._unscaled.clear()
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
            return
        assert self._growth_tracker is not None and self._found_inf is not None
        torch._amp_update_scale_(
            self._scale,
            self._growth_tracker,
            self._found_inf.float(),
            self._growth_factor,
            self._backoff_factor,
            self._growth_interval,
        )
        self._found_inf.zero_()  # unscale_() accumulates into it until the next update()

    def state_dict(self) -> Dict[str, Any]:
        if not self._enabled:
            return {}
        return {
            "scale": self.get_scale(),
            "growth_factor": self._growth_factor,
            "backoff_factor": self._backoff_factor,
            "growth_interval": self._growth_interval,
            "_growth_tracker": int(self._growth_tracker.item()) if self._growth_tracker is not None else 0,
        }

    def load_state_dict(self, state: Dict[str, Any]) -> None:
        if not state:
            return
        self._init_scale = float(state["scale"])
        self._growth_factor = float(state["growth_factor"])
        self._backoff_factor = float(state["backoff_factor"])
        self._growth_interval = int(state["growth_interval"])
        if self._scale is not None:
            self._scale.fill_(self._init_scale)
            assert self._growth_tracker is not None
            self._growth_tracker.fill_(int(state.get("_growth_tracker", 0)))
