"""Whole-step HIP-graph capture (MI355X-native replacement for a tracing compiler's launch fusion).

A training step of a mid-sized model is ~1000 kernel launches; when the kernels are short, the host
launch path, not the GPU, sets the step time (BERT-base at batch 64 x 128 under autocast: 72.5% kernel
busy, ``profiles/bert_base_mlm_b64_s128_1gpu_r4.txt``).  ``GraphedStep`` records the step once into a
hipGraph (PyTorch-ROCm's ``torch.cuda.CUDAGraph``) and replays it with one launch per step.

What a captured step needs, and what this framework provides for it:

* every random draw on the device: the dropout kernels (``csrc/attention.hip``, ``csrc/norm.hip``) read
  their seed from a device tensor drawn by ``torch.randint(..., device="cuda")``, which PyTorch's
  graph-safe generator advances on every replay -- each replay drops a fresh pattern;
* no host synchronisation inside the step (``transformers.accelerate``'s mask function skips its
  all-valid shortcut while capturing);
* static memory: the inputs are fixed tensors the caller refills before each replay, gradients stay
  allocated (``zero_grad(set_to_none=False)`` inside the step), the fused optimizers keep their step
  counter on the device (``ops.optim``).  Hyperparameters passed by value (learning rate, betas) are
  frozen at capture: call :meth:`GraphedStep.recapture` after changing them.

Reference counterpart: none -- the reference relies on eager PyTorch / DeepSpeed kernels
(harness/determined/pytorch/_pytorch_trial.py ``_train_batch``).
"""

from typing import Any, Callable, Optional

import torch


class GraphedStep:
    """``step = GraphedStep(fn); out = step()`` runs ``fn`` ``warmup`` times eagerly on a side stream (kernel
    selection, lazy allocations, optimizer state), captures one call into a graph, and from then on every
    call replays the graph and returns the captured call's (static) outputs."""

    def __init__(self, fn: Callable[[], Any], warmup: int = 3, pool: Optional[Any] = None) -> None:
        self._fn = fn
        self._warmup = warmup
        self._pool = pool
        self._graph: Optional[torch.cuda.CUDAGraph] = None
        self._out: Any = None

    @property
    def captured(self) -> bool:
        return self._graph is not None

    def capture(self) -> None:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self._warmup):
                self._fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self._pool):
            self._out = self._fn()
        self._graph = graph

    def recapture(self) -> None:
        """Capture again (after a hyperparameter change), without the warm-up runs."""
        self._warmup, warm = 0, self._warmup
        try:
            self._graph = None
            self.capture()
        finally:
            self._warmup = warm

    def __call__(self) -> Any:
        if self._graph is None:
            self.capture()
        self._graph.replay()
        return self._out
