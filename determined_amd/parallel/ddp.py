"""Data-parallel gradient engine: flat gradient buckets + RCCL all-reduce overlapped with backward.

Replaces the reference's DDP/Horovod wrapping (``PyTorchTrialContext.wrap_model`` ->
``torch.nn.parallel.DistributedDataParallel`` / ``hvd.DistributedOptimizer``;
reference ``harness/determined/pytorch/_pytorch_context.py:285`` and ``horovod.py``).

MI355X design points:

* After ``backward`` every parameter's ``.grad`` is a strided view into a flat per-bucket
  buffer (memory format preserved, so channels-last conv weights stay dense).  Buckets are
  ready-made RCCL send buffers and the fused multi-tensor optimizer sees stable grad
  pointers (its chunk table is built once).
* ``zero_grad()`` does not memset anything: it drops ``.grad`` so autograd hands each fresh
  gradient over without an accumulate kernel; when the last gradient of a bucket arrives
  the bucket is filled with ONE multi-tensor copy (``_foreach_copy_``) and its all-reduce
  is issued immediately.  (Accumulating into pre-set views instead costs one ``grad +=``
  launch per parameter: 161 launches / 2.1 ms per ResNet-50 step, measured.)
* ProcessGroupNCCL (= RCCL on ROCm) runs each all-reduce on its own HIP stream after
  waiting on the compute stream, so communication of bucket k overlaps the backward kernels
  that produce buckets k+1...; ``finish()`` only makes the compute stream wait on the RCCL
  stream (no host blocking).
* Bucket order is re-derived from the hook order observed in the first backward, so later
  iterations launch collectives in true gradient-ready order.
* Bucket size defaults to 16 MiB (first bucket 2 MiB): on an 8-GPU xGMI node a ring
  all-reduce of S bytes moves 2*(7/8)*S per rank over point-to-point links; 16 MiB keeps
  each collective bandwidth-bound (>> its ~20-40 us launch/latency floor) while leaving
  enough buckets (ResNet-50 bf16: 51 MB of grads -> 4-5 collectives) to overlap backward.
* The LAST bucket (the earliest layers' gradients, ready only when the backward ends) is capped
  at ``last_bucket_mb`` (2 MiB) too: its all-reduce cannot overlap anything, so it should be
  small -- a 16 MiB tail bucket holding layer3/layer2 weights of ResNet-50 would wait for the
  stem's gradient and then run fully exposed.
* Averaging uses ``ReduceOp.AVG`` on RCCL (no separate divide kernel); gloo (CPU tests)
  falls back to SUM + in-place divide.
"""

import contextlib
import logging
from typing import Dict, Iterator, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from determined_amd.utils.tensor import is_dense

logger = logging.getLogger("determined_amd.parallel.ddp")

MiB = 1 << 20


class _Bucket:
    __slots__ = ("params", "offsets", "views", "numel", "buffer", "pending", "work", "dtype", "index",
                 "copy_dst", "copy_src", "arrived")

    def __init__(self, index: int, params: List[nn.Parameter], dtype: torch.dtype, device: torch.device) -> None:
        self.index = index
        self.params = params
        self.dtype = dtype
        self.offsets: List[int] = []
        n = 0
        for p in params:
            self.offsets.append(n)
            # keep each view 16-byte aligned so vectorised kernels take the fast path
            align = max(1, 16 // p.element_size())
            n += (p.numel() + align - 1) // align * align
        self.numel = n
        self.buffer = torch.zeros(n, dtype=dtype, device=device)
        self.views = [_grad_view(self.buffer, off, p) for p, off in zip(params, self.offsets)]
        self.pending = len(params)
        self.work = None
        self.copy_dst: List[torch.Tensor] = []
        self.copy_src: List[torch.Tensor] = []
        self.arrived = [False] * len(params)


def _grad_view(buf: torch.Tensor, offset: int, p: torch.Tensor) -> torch.Tensor:
    flat = buf.narrow(0, offset, p.numel())
    return flat.as_strided(p.shape, p.stride()) if is_dense(p) else flat.view(p.shape)


class DistributedDataParallel(nn.Module):
    """Wraps ``module``; gradients are averaged across ``process_group`` during backward."""

    def __init__(
        self,
        module: nn.Module,
        process_group: Optional[dist.ProcessGroup] = None,
        bucket_cap_mb: float = 16.0,
        first_bucket_mb: float = 2.0,
        last_bucket_mb: float = 2.0,
        broadcast_buffers: bool = False,
        average: bool = True,
        reorder_after_first_step: bool = True,
    ) -> None:
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.bucket_cap = int(bucket_cap_mb * MiB)
        self.first_bucket_cap = int(first_bucket_mb * MiB)
        self.last_bucket_cap = int(min(last_bucket_mb, bucket_cap_mb) * MiB)
        self.broadcast_buffers = broadcast_buffers
        self.average = average
        self._reorder = reorder_after_first_step
        self._sync_enabled = True
        self._observed: List[nn.Parameter] = []
        self._steps = 0
        backend = dist.get_backend(process_group) if dist.is_initialized() else "none"
        self._use_avg = backend == "nccl"
        self._params = [p for p in module.parameters() if p.requires_grad]
        self._hooks = []
        self._sync_module_states()
        self._build_buckets(list(reversed(self._params)))
        for p in self._params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(p)))

    # -- construction -----------------------------------------------------------------------
    def _sync_module_states(self) -> None:
        if self.world_size <= 1:
            return
        src = dist.get_global_rank(self.process_group, 0) if self.process_group else 0
        tensors = [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]
        by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.reshape(-1) for t in ts])
            dist.broadcast(flat, src=src, group=self.process_group)
            off = 0
            for t in ts:
                t.copy_(flat[off : off + t.numel()].view_as(t))
                off += t.numel()

    def _build_buckets(self, order: List[nn.Parameter]) -> None:
        old: Dict[int, torch.Tensor] = {}
        for b in getattr(self, "_buckets", []):
            for p, v in zip(b.params, b.views):
                old[id(p)] = v.clone()
        self._buckets: List[_Bucket] = []
        self._slot: Dict[int, Tuple[_Bucket, int]] = {}
        cur: List[nn.Parameter] = []
        cur_bytes = 0
        cap = self.first_bucket_cap

        def flush() -> None:
            nonlocal cur, cur_bytes, cap
            if cur:
                b = _Bucket(len(self._buckets), cur, cur[0].dtype, cur[0].device)
                self._buckets.append(b)
                for i, p in enumerate(cur):
                    self._slot[id(p)] = (b, i)
                cur, cur_bytes = [], 0
                cap = self.bucket_cap

        # the tail (last-ready gradients) forms its own small bucket: peel it off the end first
        order = list(order)
        tail: List[nn.Parameter] = []
        tail_bytes = 0
        while order and self.last_bucket_cap > 0:
            p = order[-1]
            nbytes = p.numel() * p.element_size()
            if tail and (p.dtype != tail[0].dtype or p.device != tail[0].device
                         or tail_bytes + nbytes > self.last_bucket_cap):
                break
            tail.insert(0, order.pop())
            tail_bytes += nbytes
        for p in order:
            nbytes = p.numel() * p.element_size()
            if cur and (p.dtype != cur[0].dtype or p.device != cur[0].device or cur_bytes + nbytes > cap):
                flush()
            cur.append(p)
            cur_bytes += nbytes
        flush()
        cur, cur_bytes = tail, tail_bytes
        flush()
        for b in self._buckets:
            for p, v in zip(b.params, b.views):
                if id(p) in old:
                    v.copy_(old[id(p)])
                elif p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v

    # -- hooks ------------------------------------------------------------------------------
    def _make_hook(self, p: nn.Parameter):
        def hook(param: torch.Tensor) -> None:
            self._on_grad_ready(p)

        return hook

    def _on_grad_ready(self, p: nn.Parameter) -> None:
        b, i = self._slot[id(p)]
        v = b.views[i]
        g = p.grad
        if g is not None and g.data_ptr() != v.data_ptr():
            # fresh gradient handed over by autograd: copy into the bucket with the others
            b.copy_dst.append(v)
            b.copy_src.append(g)
            p.grad = v
        elif g is None:
            v.zero_()
            p.grad = v
        if self._steps == 0 and self._reorder:
            self._observed.append(p)
        if not b.arrived[i]:
            b.arrived[i] = True
            b.pending -= 1
        if b.pending == 0:
            self._complete(b)

    def _flush_copies(self, b: _Bucket) -> None:
        if b.copy_dst:
            torch._foreach_copy_(b.copy_dst, b.copy_src)
            b.copy_dst = []
            b.copy_src = []

    def _complete(self, b: _Bucket) -> None:
        self._flush_copies(b)
        if self._sync_enabled and self.world_size > 1 and b.work is None:
            op = dist.ReduceOp.AVG if (self.average and self._use_avg) else dist.ReduceOp.SUM
            b.work = dist.all_reduce(b.buffer, op=op, group=self.process_group, async_op=True)

    # -- public API -------------------------------------------------------------------------
    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.world_size > 1 and self._sync_enabled:
            self.sync_buffers()
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self) -> Iterator[None]:
        """Accumulate gradients locally (gradient aggregation); no collectives are issued."""
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev
            self._reset_arrivals()
            if self._steps == 0:  # bucket order is learned from the first SYNCED backward
                self._observed = []

    def _reset_arrivals(self) -> None:
        for b in self._buckets:
            for i, p in enumerate(b.params):
                if not b.arrived[i] and p.grad is None:
                    b.views[i].zero_()
                    p.grad = b.views[i]
            self._flush_copies(b)
            b.arrived = [False] * len(b.params)
            b.pending = len(b.params)

    def finish(self) -> None:
        """Complete gradient averaging for this step (call once after the last backward)."""
        for b in self._buckets:
            if b.pending > 0:  # params that received no gradient this step
                for i, p in enumerate(b.params):
                    if not b.arrived[i] and (p.grad is None or p.grad.data_ptr() != b.views[i].data_ptr()):
                        if p.grad is not None:
                            b.copy_dst.append(b.views[i])
                            b.copy_src.append(p.grad)
                        else:
                            b.views[i].zero_()
                        p.grad = b.views[i]
                b.pending = 0
                self._complete(b)
        if self.world_size > 1:
            for b in self._buckets:
                if b.work is not None:
                    b.work.wait()  # stream-level wait: compute stream waits on the RCCL stream
                    if self.average and not self._use_avg:
                        b.buffer.div_(self.world_size)
                    b.work = None
        for b in self._buckets:
            b.arrived = [False] * len(b.params)
            b.pending = len(b.params)
        if self._steps == 0 and self._reorder and self._observed:
            seen = {id(p) for p in self._observed}
            order = self._observed + [p for p in reversed(self._params) if id(p) not in seen]
            self._observed = []
            self._build_buckets(order)
        self._steps += 1

    def zero_grad(self, set_to_none: bool = True) -> None:
        """Drop gradients; the next backward refills the buckets without a memset."""
        for b in self._buckets:
            if set_to_none:
                for p in b.params:
                    p.grad = None
            else:
                b.buffer.zero_()

    def grad_buffers(self) -> List[torch.Tensor]:
        return [b.buffer for b in self._buckets]

    def sync_buffers(self) -> None:
        bufs = [b for b in self.module.buffers() if b.is_floating_point()]
        if not bufs or self.world_size <= 1:
            return
        for t in bufs:
            dist.broadcast(t, src=0, group=self.process_group)

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)
