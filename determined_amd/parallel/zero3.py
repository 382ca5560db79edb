"""ZeRO stage 3: parameters partitioned across data-parallel ranks, gathered per module on use
(DeepSpeed ``zero_optimization.stage: 3``; the reference reaches it through
``harness/determined/pytorch/deepspeed/_deepspeed_context.py`` -> ``deepspeed.initialize``).

Layout (per parameter dtype, see ``zero.py`` for stages 0-2):

* every module that directly owns trainable parameters is a *gather unit*; its parameters form
  one bucket laid out like the stage-2 buckets (padded so each rank's chunk is 16-byte aligned).
  Rank ``r`` permanently stores only chunk ``r`` of every bucket in one flat shard buffer
  ``PS``; the optimizer's fragments alias ``PS`` (and the gradient shard ``GS``), so the fused
  AdamW/SGD kernels update the shard in place and nothing is written back;
* outside of use a parameter's ``.data`` is an empty placeholder.  A forward pre-hook on the
  owning module issues ``all_gather_into_tensor`` of the unit (RCCL), binds the parameters to
  views of the gathered buffer and prefetches the next unit of the recorded forward order, so
  the next gather overlaps this module's compute;
* the forward post-hook wraps the module's outputs in an identity autograd node whose backward
  re-gathers the unit *before* the module's own backward runs (the saved parameter tensors
  share the parameter's TensorImpl, so re-binding ``.data`` is enough) and pins it until all of
  its gradients have arrived;
* each parameter's gradient is copied into the unit's full-size gradient buffer; when the unit
  is complete it is ``reduce_scatter``-ed straight into this rank's ``GS`` chunk (fp32
  accumulation across micro-batches when ``gradient_accumulation_steps > 1``), and the full
  buffers are dropped as soon as their collective is done (at most ``max_inflight`` live);
* gathered units stay resident up to ``stage3_max_live_parameters`` elements (LRU eviction,
  never evicting a pinned unit); units smaller than ``stage3_param_persistence_threshold``
  are never evicted during a step.  The optimizer step invalidates every gathered copy.

Parameters used outside their owning module's ``forward`` (e.g. a tied LM head calling
``F.linear(h, self.wte.weight)`` in the parent) must be registered with
``register_external_parameter(module, param)`` -- or the model can expose
``zero3_external_parameters() -> [(module, param), ...]`` -- exactly as with DeepSpeed.
"""

import contextlib
from typing import Any, Dict, Iterator, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from determined_amd.parallel.zero import _ALIGN_BYTES, ZeroEngine, _Bucket

RELEASED, INFLIGHT, AVAILABLE = 0, 1, 2


class _Space3:
    """Partitioned flat storage for one parameter dtype: shard buffers + per-unit buckets."""

    def __init__(self, units: List[List[nn.Parameter]], dtype: torch.dtype, grad_dtype: torch.dtype, world: int,
                 rank: int, device: torch.device, global_index: Dict[int, int]) -> None:
        self.dtype = dtype
        self.grad_dtype = grad_dtype
        self.world = world
        self.rank = rank
        align = max(1, _ALIGN_BYTES // torch.empty((), dtype=dtype).element_size())
        align = max(align, _ALIGN_BYTES // torch.empty((), dtype=grad_dtype).element_size(), 4)
        self.buckets: List[_Bucket] = []
        start = 0
        for params in units:
            b = _Bucket(len(self.buckets), params, [global_index[id(q)] for q in params], start, world, align)
            start += b.numel
            self.buckets.append(b)
        self.numel = start
        shard = 0
        for b in self.buckets:
            b.shard_off = shard
            shard += b.chunk
            # stage-3 runtime state
            b.state = RELEASED
            b.full = None
            b.gfull = None
            b.gwork = None
            b.pin = 0
            b.bw_pin = False
            b.last_use = 0
            b.reduced = False  # reduce-scattered during the current micro-batch
        self.shard_numel = shard
        self.PS = torch.zeros(shard, dtype=dtype, device=device)
        self.GS = torch.zeros(shard, dtype=grad_dtype, device=device)
        self.slot: Dict[int, Tuple[_Bucket, int]] = {}
        self.shape: Dict[int, torch.Size] = {}
        self.placeholder = torch.empty(0, dtype=dtype, device=device)
        with torch.no_grad():
            for b in self.buckets:
                full = torch.zeros(b.numel, dtype=dtype, device=device)
                for i, (p, off) in enumerate(zip(b.params, b.offsets)):
                    full.narrow(0, off, p.numel()).copy_(p.data.reshape(-1))
                    self.slot[id(p)] = (b, i)
                    self.shape[id(p)] = p.shape
                self.PS.narrow(0, b.shard_off, b.chunk).copy_(full.narrow(0, rank * b.chunk, b.chunk))
                del full

    def drop_full_params(self) -> None:
        """Swap every parameter's storage for the empty placeholder (after fragments are bound:
        ``_Bucket.fragments`` reads parameter sizes)."""
        for b in self.buckets:
            for p in b.params:
                p.data = self.placeholder

    def shard(self, buf: torch.Tensor, b: _Bucket) -> torch.Tensor:
        return buf.narrow(0, b.shard_off, b.chunk)


class _PreBackward(torch.autograd.Function):
    """Identity on a module's outputs; its backward re-gathers the module's units first."""

    @staticmethod
    def forward(ctx, engine: "Zero3Engine", units: Any, *ts: torch.Tensor) -> Any:  # type: ignore[override]
        ctx.engine = engine
        ctx.units = units
        out = tuple(t.view_as(t) for t in ts)
        return out if len(out) > 1 else out[0]

    @staticmethod
    def backward(ctx, *grads: torch.Tensor) -> Any:  # type: ignore[override]
        ctx.engine._pre_backward(ctx.units)
        return (None, None) + grads


class Zero3Engine(ZeroEngine):
    """``ZeroEngine`` with parameter partitioning (stage 3); same DeepSpeed-style surface."""

    def __init__(self, model: nn.Module, config: Any, *args: Any, **kwargs: Any) -> None:
        self._external: Dict[int, List[nn.Parameter]] = {}
        raw = (config.raw.get("zero_optimization") or {}) if hasattr(config, "raw") else {}
        self.max_live_numel = int(raw.get("stage3_max_live_parameters", 1_000_000_000))
        self.persist_numel = int(raw.get("stage3_param_persistence_threshold", 100_000))
        self.prefetch_numel = int(raw.get("stage3_prefetch_bucket_size", 50_000_000))
        self.max_inflight = 4
        ext = getattr(model, "zero3_external_parameters", None)
        if callable(ext):
            for mod, p in ext():
                self._external.setdefault(id(mod), []).append(p)
        super().__init__(model, config, *args, **kwargs)

    # ------------------------------------------------------------------ construction
    def _build_spaces(self) -> None:
        trainable = {id(p) for p in self._params}
        seen: set = set()
        units_by_dtype: Dict[torch.dtype, List[List[nn.Parameter]]] = {}
        self._units_of_module: Dict[int, List[Tuple[_Space3, _Bucket]]] = {}
        self._unit_modules: List[nn.Module] = []
        owner: Dict[int, Tuple[nn.Module, torch.dtype, int]] = {}
        for m in self.module.modules():
            by_dt: Dict[torch.dtype, List[nn.Parameter]] = {}
            for p in m.parameters(recurse=False):
                if id(p) in trainable and id(p) not in seen:
                    seen.add(id(p))
                    by_dt.setdefault(p.dtype, []).append(p)
            if by_dt:
                self._unit_modules.append(m)
            for dt, ps in by_dt.items():
                lst = units_by_dtype.setdefault(dt, [])
                for p in ps:
                    owner[id(p)] = (m, dt, len(lst))
                lst.append(ps)
        self.spaces: List[_Space3] = []  # type: ignore[assignment]
        space_of_dt: Dict[torch.dtype, _Space3] = {}
        for dt, units in units_by_dtype.items():
            gdt = self.config.grad_accum_dtype or self.config.communication_dtype or \
                (torch.float32 if self.config.gas > 1 else dt)
            sp = _Space3(units, dt, gdt, self._shard_world, self._shard_rank, self.device, self._pindex)
            self.spaces.append(sp)
            space_of_dt[dt] = sp
        self._space_of: Dict[int, _Space3] = {}  # type: ignore[assignment]
        for sp in self.spaces:
            for b in sp.buckets:
                for p in b.params:
                    self._space_of[id(p)] = sp
        for m in self._unit_modules:
            lst: List[Tuple[_Space3, _Bucket]] = []
            for p in m.parameters(recurse=False):
                if id(p) in self._space_of:
                    sp = self._space_of[id(p)]
                    b = sp.slot[id(p)][0]
                    if all(b is not x for _, x in lst):
                        lst.append((sp, b))
            self._units_of_module[id(m)] = lst
        self._tick = 0
        self._live: List[Tuple[_Space3, _Bucket]] = []
        self._live_numel = 0
        self._trace: List[Tuple[_Space3, _Bucket]] = []
        self._trace_done = False
        self._inflight: List[Tuple[Any, torch.Tensor, Optional[torch.Tensor], torch.Tensor, bool]] = []

    def _fragment_views(self, sp: Any, b: _Bucket, boff: int, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
        off = b.shard_off + (boff - self._shard_rank * b.chunk)
        return sp.PS.narrow(0, off, n), sp.GS.narrow(0, off, n)

    def _install_hooks(self) -> None:
        for sp in self.spaces:
            sp.drop_full_params()
        super()._install_hooks()
        mods = {id(m): m for m in self._unit_modules}
        for mid in self._external:
            for m in self.module.modules():
                if id(m) == mid:
                    mods[mid] = m
        mods[id(self.module)] = self.module
        for m in mods.values():
            self._hooks.append(m.register_forward_pre_hook(self._pre_forward))
            self._hooks.append(m.register_forward_hook(self._post_forward))

    def register_external_parameter(self, module: nn.Module, param: nn.Parameter) -> None:
        """``param`` is used in ``module.forward`` although another module owns it."""
        first = id(module) not in self._external and id(module) not in self._units_of_module \
            and module is not self.module
        self._external.setdefault(id(module), []).append(param)
        if first:
            self._hooks.append(module.register_forward_pre_hook(self._pre_forward))
            self._hooks.append(module.register_forward_hook(self._post_forward))

    def _units_for(self, module: nn.Module) -> List[Tuple[_Space3, _Bucket]]:
        units = list(self._units_of_module.get(id(module), []))
        for p in self._external.get(id(module), []):
            sp = self._space_of.get(id(p))
            if sp is not None:
                b = sp.slot[id(p)][0]
                if all(b is not x for _, x in units):
                    units.append((sp, b))
        return units

    # ------------------------------------------------------------------ gather / release
    def _fetch(self, sp: _Space3, b: _Bucket) -> None:
        if b.state != RELEASED:
            return
        full = torch.empty(b.numel, dtype=sp.dtype, device=self.device)
        mine = sp.shard(sp.PS, b)
        if self._shard_world > 1:
            b.gwork = dist.all_gather_into_tensor(full, mine, group=self.process_group, async_op=True)
        else:
            full.copy_(mine)
        b.full = full
        b.state = INFLIGHT
        self._live.append((sp, b))
        self._live_numel += b.numel

    def _ensure(self, sp: _Space3, b: _Bucket) -> None:
        self._fetch(sp, b)
        if b.state == INFLIGHT:
            if b.gwork is not None:
                b.gwork.wait()
                b.gwork = None
            for p, off in zip(b.params, b.offsets):
                p.data = b.full.narrow(0, off, sp.shape[id(p)].numel()).view(sp.shape[id(p)])
            b.state = AVAILABLE
        self._tick += 1
        b.last_use = self._tick

    def _release(self, sp: _Space3, b: _Bucket) -> None:
        if b.state == RELEASED:
            return
        if b.gwork is not None:
            b.gwork.wait()
            b.gwork = None
        for p in b.params:
            p.data = sp.placeholder
        b.full = None
        b.state = RELEASED
        self._live = [(s, x) for s, x in self._live if x is not b]
        self._live_numel -= b.numel

    def _evict(self, budget: Optional[int] = None, keep_persistent: bool = True) -> None:
        budget = self.max_live_numel if budget is None else budget
        if self._live_numel <= budget:
            return
        cands = sorted((x for x in self._live if x[1].pin == 0 and x[1].state == AVAILABLE and
                        not (keep_persistent and x[1].numel < self.persist_numel)), key=lambda x: x[1].last_use)
        for sp, b in cands:
            if self._live_numel <= budget:
                break
            self._release(sp, b)

    def release_all(self) -> None:
        for sp, b in list(self._live):
            if b.pin == 0:
                self._release(sp, b)

    def _prefetch_after(self, units: List[Tuple[_Space3, _Bucket]], backward: bool) -> None:
        if not self._trace_done or not units:
            return
        pos = [i for i, (_, b) in enumerate(self._trace) if b is units[-1][1]]
        if not pos:
            return
        i = pos[0]
        step = -1 if backward else 1
        n = 0
        j = i + step
        while 0 <= j < len(self._trace) and n < self.prefetch_numel:
            sp, b = self._trace[j]
            if b.state == RELEASED:
                self._fetch(sp, b)
            n += b.numel
            j += step
            if n >= self.prefetch_numel or j - i > 2 or i - j > 2:
                break

    # ------------------------------------------------------------------ module hooks
    def _pre_forward(self, module: nn.Module, args: Any) -> None:
        units = self._units_for(module)
        for sp, b in units:
            self._fetch(sp, b)
        for sp, b in units:
            self._ensure(sp, b)
            b.pin += 1
            if not self._trace_done and all(b is not x for _, x in self._trace):
                self._trace.append((sp, b))
        self._prefetch_after(units, backward=False)

    def _post_forward(self, module: nn.Module, args: Any, out: Any) -> Any:
        units = self._units_for(module)
        for _, b in units:
            b.pin -= 1
        if module is self.module:
            self._trace_done = True
        if units and torch.is_grad_enabled():
            out = self._wrap(out, units)
        self._evict()
        return out

    def _wrap(self, out: Any, units: List[Tuple[_Space3, _Bucket]]) -> Any:
        flat: List[torch.Tensor] = []

        def collect(o: Any) -> None:
            if isinstance(o, torch.Tensor):
                if o.requires_grad and o.is_floating_point():
                    flat.append(o)
            elif isinstance(o, (list, tuple)):
                for x in o:
                    collect(x)
            elif isinstance(o, dict):
                for x in o.values():
                    collect(x)

        collect(out)
        if not flat:
            return out
        res = _PreBackward.apply(self, units, *flat)
        res = res if isinstance(res, tuple) else (res,)
        repl = {id(t): r for t, r in zip(flat, res)}

        def rebuild(o: Any) -> Any:
            if isinstance(o, torch.Tensor):
                return repl.get(id(o), o)
            if isinstance(o, tuple) and hasattr(o, "_fields"):
                return type(o)(*(rebuild(x) for x in o))
            if isinstance(o, (list, tuple)):
                return type(o)(rebuild(x) for x in o)
            if isinstance(o, dict):
                return type(o)((k, rebuild(v)) for k, v in o.items())
            return o

        return rebuild(out)

    def _pre_backward(self, units: List[Tuple[_Space3, _Bucket]]) -> None:
        for sp, b in units:
            self._fetch(sp, b)
        for sp, b in units:
            self._ensure(sp, b)
            if not b.bw_pin and not b.reduced:
                b.bw_pin = True
                b.pin += 1
        self._prefetch_after(units[:1], backward=True)
        self._evict()

    # ------------------------------------------------------------------ gradients
    def _on_grad(self, p: nn.Parameter) -> None:  # type: ignore[override]
        sp = self._space_of[id(p)]
        b, i = sp.slot[id(p)]
        g = p.grad
        if g is None:
            return
        p.grad = None
        if b.gfull is None:
            b.gfull = torch.zeros(b.numel, dtype=sp.dtype, device=self.device)
        b.gfull.narrow(0, b.offsets[i], g.numel()).copy_(g.reshape(-1))
        if not b.arrived[i]:
            b.arrived[i] = True
            b.pending -= 1
        if b.pending == 0:
            self._reduce3(sp, b)

    def _reduce3(self, sp: _Space3, b: _Bucket) -> None:
        if b.bw_pin:
            b.bw_pin = False
            b.pin -= 1
        if b.gfull is None:
            b.gfull = torch.zeros(b.numel, dtype=sp.dtype, device=self.device)
        out = sp.shard(sp.GS, b)
        first = not any(b.touched)
        b.touched = [True] * len(b.params)
        b.reduced = True
        src = b.gfull
        b.gfull = None
        if self._shard_world <= 1:
            chunk = src.narrow(0, 0, b.chunk)
            out.copy_(chunk) if first else out.add_(chunk)
            return
        op = dist.ReduceOp.AVG if self._use_avg else dist.ReduceOp.SUM
        if first and out.dtype == src.dtype:
            work = dist.reduce_scatter_tensor(out, src, op=op, group=self.process_group, async_op=True)
            self._inflight.append((work, src, None, out, True))
        else:
            tmp = torch.empty(b.chunk, dtype=src.dtype, device=self.device)
            work = dist.reduce_scatter_tensor(tmp, src, op=op, group=self.process_group, async_op=True)
            self._inflight.append((work, src, tmp, out, first))
        while len(self._inflight) > self.max_inflight:
            self._retire(self._inflight.pop(0))

    def _retire(self, item: Tuple[Any, torch.Tensor, Optional[torch.Tensor], torch.Tensor, bool]) -> None:
        work, _src, tmp, out, first = item
        work.wait()
        res = out if tmp is None else tmp
        if not self._use_avg:
            res.div_(self.world_size)
        if tmp is not None:
            out.copy_(tmp) if first else out.add_(tmp.to(out.dtype))

    def _end_backward(self) -> None:
        # every rank reduce-scatters every unit every micro-batch (collective order must match);
        # units whose gradients never arrived contribute zeros for the missing parameters
        for sp in self.spaces:
            for b in sp.buckets:
                if not b.reduced:
                    self._reduce3(sp, b)
        for sp in self.spaces:
            for b in sp.buckets:
                if b.bw_pin:
                    b.bw_pin = False
                    b.pin -= 1
                b.reduced = False
                b.arrived = [False] * len(b.params)
                b.pending = len(b.params)
        self._evict(budget=0, keep_persistent=True)

    def backward(self, loss: torch.Tensor, retain_graph: bool = False, scale_wrt_gas: bool = True) -> torch.Tensor:
        self._boundary_now = self.is_gradient_accumulation_boundary()
        if self.micro_steps % self.config.gas == 0:
            for sp in self.spaces:
                for b in sp.buckets:
                    b.touched = [False] * len(b.params)
        if scale_wrt_gas and self.config.gas > 1:
            loss = loss / self.config.gas
        loss.backward(retain_graph=retain_graph)
        self._end_backward()
        return loss

    def _finish_reduce(self) -> None:
        while self._inflight:
            self._retire(self._inflight.pop(0))

    def _gather(self) -> None:
        # the step rewrote every shard: drop all gathered copies (re-gathered lazily on use)
        self._finish_reduce()
        for sp, b in list(self._live):
            b.pin = 0
            self._release(sp, b)

    def _wait_gather(self) -> None:
        pass

    # ------------------------------------------------------------------ full-state access
    @contextlib.contextmanager
    def gathered_parameters(self, modifier_rank: Optional[int] = None) -> Iterator[None]:
        """All parameters materialised (DeepSpeed ``zero.GatheredParameters``).  With
        ``modifier_rank`` set, that rank's edits are broadcast and written back to the shards."""
        units = [(sp, b) for sp in self.spaces for b in sp.buckets]
        for sp, b in units:
            self._fetch(sp, b)
        for sp, b in units:
            self._ensure(sp, b)
            b.pin += 1
        try:
            yield
        finally:
            if modifier_rank is not None:
                with torch.no_grad():
                    for sp, b in units:
                        if self._shard_world > 1:
                            src = dist.get_global_rank(self.process_group, modifier_rank) \
                                if self.process_group is not None else modifier_rank
                            dist.broadcast(b.full, src=src, group=self.process_group)
                        sp.shard(sp.PS, b).copy_(b.full.narrow(0, self._shard_rank * b.chunk, b.chunk))
            for sp, b in units:
                b.pin -= 1
            self.release_all()

    def state_dict(self, *args: Any, **kwargs: Any) -> Dict[str, Any]:  # type: ignore[override]
        with self.gathered_parameters():
            sd = self.module.state_dict(*args, **kwargs)
            return {k: v.detach().clone() for k, v in sd.items()}

    def load_state_dict(self, sd: Dict[str, Any], strict: bool = True) -> Any:  # type: ignore[override]
        with self.gathered_parameters(modifier_rank=None):
            with torch.no_grad():
                res = self.module.load_state_dict(sd, strict=strict)
                for sp in self.spaces:
                    for b in sp.buckets:
                        sp.shard(sp.PS, b).copy_(b.full.narrow(0, self._shard_rank * b.chunk, b.chunk))
        self._refresh_master()
        return res
