"""Pipeline parallelism with a DeepSpeed-style API (``PipelineModule`` / ``engine.train_batch``),
the path the reference's DeepSpeedTrial takes when the engine is a ``deepspeed.PipelineEngine``
(reference ``harness/determined/pytorch/deepspeed/_deepspeed_trial.py`` ``use_pipeline_parallel``,
``_deepspeed_context.py`` pipeline checks).

Topology: ``world = dp * pp``; rank ``r`` is pipeline stage ``r % pp`` of data-parallel replica
``r // pp`` (consecutive ranks form one pipeline, so on one MI355X node a 2- or 4-stage pipe
sits on xGMI-adjacent GPUs).  Each rank builds only its stage's layers; the stage module is
wrapped in the ZeRO engine (stage 0/1) over the stage's data-parallel group, so gradient
all-reduce, fused AdamW and clipping are the same code as the non-pipeline path.

Schedule: fill-drain (GPipe): all ``gradient_accumulation_steps`` micro-batch forwards, then
all backwards in reverse.  Activations/gradients move with ``send``/``recv`` (RCCL P2P between
neighbouring stages); a tiny int64 header (dtype, shape) precedes every tensor.  Fill-drain is
chosen deliberately: RCCL serialises a peer pair's sends and receives in issue order, and with
fill-drain both peers issue their P2P ops in the same order, so no send/recv pairing can
deadlock; the extra activation memory of ``gas`` in-flight micro-batches is affordable with
288 GB of HBM per GPU.

Data: like DeepSpeed, the first stage reads ``inputs`` and the last stage reads ``labels`` from
the iterator of ``(inputs, labels)`` micro-batches; middle stages read nothing.  The loss
(mean over micro-batches) is broadcast from the last stage so every rank returns it.
"""

import logging
from typing import Any, Callable, Iterator, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
from torch import nn

logger = logging.getLogger("determined_amd.parallel.pipeline")

_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.bool, torch.uint8]
_HDR = 32  # int64 header slots


class LayerSpec:
    """Deferred layer construction: only the owning stage instantiates it."""

    def __init__(self, typename: Callable[..., nn.Module], *args: Any, **kwargs: Any) -> None:
        self.typename = typename
        self.args = args
        self.kwargs = kwargs

    def build(self) -> nn.Module:
        return self.typename(*self.args, **self.kwargs)


def _count_params(layer: Union[nn.Module, LayerSpec, Callable]) -> int:
    if isinstance(layer, LayerSpec):
        layer = layer.build()
    return sum(p.numel() for p in layer.parameters()) if isinstance(layer, nn.Module) else 0


def partition_balanced(weights: Sequence[int], parts: int) -> List[int]:
    """Boundaries ``[0, b1, ..., len]`` splitting ``weights`` into ``parts`` contiguous ranges
    minimising the heaviest range (binary search on the bottleneck, greedy fill)."""
    n = len(weights)
    if parts > n:
        raise ValueError(f"{n} layers cannot fill {parts} pipeline stages")
    lo, hi = max(weights), max(sum(weights), 1)

    def cuts(limit: int) -> Optional[List[int]]:
        b, acc = [0], 0
        for i, w in enumerate(weights):
            if acc + w > limit and acc > 0:
                b.append(i)
                acc = 0
            acc += w
        b.append(n)
        return b if len(b) - 1 <= parts else None

    while lo < hi:
        mid = (lo + hi) // 2
        if cuts(mid) is None:
            lo = mid + 1
        else:
            hi = mid
    b = cuts(lo) or [0, n]
    while len(b) - 1 < parts:  # split the widest range until every stage has a layer
        i = max(range(len(b) - 1), key=lambda k: b[k + 1] - b[k])
        b.insert(i + 1, (b[i] + b[i + 1]) // 2)
    return b


class PipelineModule(nn.Module):
    """Sequential layers partitioned over ``num_stages`` (``partition_method``: ``parameters``
    balances parameter counts, ``uniform`` balances layer counts, or explicit boundaries)."""

    def __init__(self, layers: Sequence[Union[nn.Module, LayerSpec, Callable]], num_stages: int,
                 loss_fn: Optional[Callable[[Any, Any], torch.Tensor]] = None,
                 partition_method: Union[str, Sequence[int]] = "parameters", stage_id: Optional[int] = None) -> None:
        super().__init__()
        self.num_stages = int(num_stages)
        if dist.is_available() and dist.is_initialized():
            world = dist.get_world_size()
            if world % self.num_stages:
                raise ValueError(f"world size {world} is not divisible by num_stages {self.num_stages}")
            self.stage_id = dist.get_rank() % self.num_stages if stage_id is None else stage_id
        else:
            if self.num_stages != 1 and stage_id is None:
                raise ValueError("a multi-stage PipelineModule needs torch.distributed (or an explicit stage_id)")
            self.stage_id = stage_id or 0
        self.loss_fn = loss_fn
        if isinstance(partition_method, str):
            w = [1] * len(layers) if partition_method == "uniform" else [max(_count_params(l), 1) for l in layers]
            self.parts = partition_balanced(w, self.num_stages)
        else:
            self.parts = list(partition_method)
            if len(self.parts) != self.num_stages + 1 or self.parts[0] != 0 or self.parts[-1] != len(layers):
                raise ValueError("explicit partition must be [0, ..., len(layers)] with num_stages+1 entries")
        lo, hi = self.parts[self.stage_id], self.parts[self.stage_id + 1]
        mods: List[nn.Module] = []
        for layer in layers[lo:hi]:
            if isinstance(layer, LayerSpec):
                layer = layer.build()
            mods.append(layer if isinstance(layer, nn.Module) else _Fn(layer))
        self.layers = nn.ModuleList(mods)

    @property
    def is_first_stage(self) -> bool:
        return self.stage_id == 0

    @property
    def is_last_stage(self) -> bool:
        return self.stage_id == self.num_stages - 1

    def forward(self, x: Any) -> Any:
        for layer in self.layers:
            x = layer(*x) if isinstance(x, tuple) and not isinstance(layer, _Fn) and len(x) > 1 else layer(x)
        return x


class _Fn(nn.Module):
    def __init__(self, fn: Callable) -> None:
        super().__init__()
        self.fn = fn

    def forward(self, *x: Any) -> Any:
        return self.fn(*x)


# ------------------------------------------------------------------------------------------ P2P
def _as_tuple(x: Any) -> Tuple[torch.Tensor, ...]:
    return x if isinstance(x, tuple) else (x,)


def _send(ts: Tuple[torch.Tensor, ...], dst: int, device: torch.device) -> None:
    hdr = torch.zeros(_HDR, dtype=torch.int64)
    hdr[0] = len(ts)
    k = 1
    for t in ts:
        shape = list(t.shape)
        if k + 2 + len(shape) > _HDR:
            raise ValueError("pipeline activations have too many tensors/dims for the P2P header")
        hdr[k] = _DTYPES.index(t.dtype)
        hdr[k + 1] = len(shape)
        hdr[k + 2 : k + 2 + len(shape)] = torch.tensor(shape, dtype=torch.int64)
        k += 2 + len(shape)
    dist.send(hdr.to(device), dst)
    for t in ts:
        dist.send(t.detach().contiguous(), dst)


def _recv(src: int, device: torch.device) -> Tuple[torch.Tensor, ...]:
    hdr = torch.empty(_HDR, dtype=torch.int64, device=device)
    dist.recv(hdr, src)
    hdr = hdr.cpu()
    out = []
    k = 1
    for _ in range(int(hdr[0])):
        dt = _DTYPES[int(hdr[k])]
        nd = int(hdr[k + 1])
        shape = [int(v) for v in hdr[k + 2 : k + 2 + nd]]
        k += 2 + nd
        t = torch.empty(shape, dtype=dt, device=device)
        dist.recv(t, src)
        out.append(t)
    return tuple(out)


# ------------------------------------------------------------------------------------------ engine
class PipelineEngine(nn.Module):
    """``train_batch(data_iter)`` / ``eval_batch(data_iter)`` over one pipeline stage."""

    is_pipe_parallel = True

    def __init__(self, module: PipelineModule, config: Any, optimizer: Any = None, model_parameters: Any = None,
                 lr_scheduler: Any = None) -> None:
        super().__init__()
        from determined_amd.parallel.zero import ZeroEngine

        if config.zero_stage > 1:
            raise ValueError("pipeline parallelism supports ZeRO stage 0 or 1 (as DeepSpeed)")
        self.pp = module.num_stages
        self.stage_id = module.stage_id
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        self.global_rank = rank
        self.dp = world // self.pp
        self.dp_rank = rank // self.pp
        self.prev_rank = rank - 1 if self.stage_id > 0 else None
        self.next_rank = rank + 1 if self.stage_id < self.pp - 1 else None
        self.last_stage_rank = self.dp_rank * self.pp + self.pp - 1
        # data-parallel group of this stage: the same stage in every replica
        self.dp_group = None
        self.pipe_group = None
        if dist.is_initialized() and world > 1:
            for s in range(self.pp):
                ranks = [d * self.pp + s for d in range(self.dp)]
                g = dist.new_group(ranks)
                if s == self.stage_id:
                    self.dp_group = g
            for d in range(self.dp):
                ranks = [d * self.pp + s for s in range(self.pp)]
                g = dist.new_group(ranks)
                if d == self.dp_rank:
                    self.pipe_group = g
        self.module_ = module
        self.loss_fn = module.loss_fn
        self.inner = ZeroEngine(module, config, optimizer=optimizer, model_parameters=model_parameters,
                                lr_scheduler=lr_scheduler, process_group=self.dp_group)
        self.device = self.inner.device
        self.config = config
        self.gas = config.gas
        self.optimizer = self.inner.optimizer
        self.lr_scheduler = self.inner.lr_scheduler
        self.global_steps = 0
        self.micro_steps = 0
        self.global_samples = 0
        self.agg_train_loss: Optional[torch.Tensor] = None

    # -- DeepSpeed-engine surface used by DeepSpeedTrial --------------------------------------
    def train_micro_batch_size_per_gpu(self) -> int:
        return self.config.micro_batch

    def gradient_accumulation_steps(self) -> int:
        return self.gas

    def train_batch_size(self) -> int:
        return self.config.train_batch_size

    def is_first_stage(self) -> bool:
        return self.stage_id == 0

    def is_last_stage(self) -> bool:
        return self.stage_id == self.pp - 1

    def get_lr(self) -> List[float]:
        return self.inner.get_lr()

    def get_global_grad_norm(self) -> Optional[float]:
        return self.inner.get_global_grad_norm()

    def zero_optimization_stage(self) -> int:
        return self.inner.stage

    def parameters(self, recurse: bool = True):  # type: ignore[override]
        return self.module_.parameters(recurse)

    def to(self, *args: Any, **kwargs: Any) -> "PipelineEngine":  # type: ignore[override]
        return self  # parameters are views into the stage engine's flat buffers

    @property
    def mpu(self) -> Any:
        """DeepSpeedTrial model-parallel unit: metrics come from the last stage, data loaders
        are built on the first and last stages."""
        from determined_amd.pytorch.deepspeed._mpu import ModelParallelUnit

        return ModelParallelUnit(data_parallel_rank=self.dp_rank, data_parallel_world_size=self.dp,
                                 should_report_metrics=self.is_last_stage(),
                                 should_build_data_loader=self.is_first_stage() or self.is_last_stage())

    # -- schedule -------------------------------------------------------------------------------
    def _load(self, data_iter: Optional[Iterator[Any]]) -> Tuple[Any, Any]:
        if not (self.is_first_stage() or self.is_last_stage()):
            return None, None
        if data_iter is None:
            raise ValueError("the first and last pipeline stages need a data iterator")
        batch = next(data_iter)
        inputs, labels = batch if isinstance(batch, (tuple, list)) and len(batch) == 2 else (batch, None)
        mv = lambda x: tuple(t.to(self.device) for t in x) if isinstance(x, (tuple, list)) else (
            x.to(self.device) if isinstance(x, torch.Tensor) else x)
        return mv(inputs), mv(labels)

    def _forward_micro(self, data_iter: Optional[Iterator[Any]], train: bool) -> Tuple[Any, Any, Any]:
        inputs, labels = self._load(data_iter)
        if self.is_first_stage():
            x = inputs
            recv = None
        else:
            recv = _recv(self.prev_rank, self.device)
            recv = tuple(t.requires_grad_(train and t.is_floating_point()) for t in recv)
            x = recv if len(recv) > 1 else recv[0]
        with torch.set_grad_enabled(train):
            out = self.module_(x)
        loss = None
        if self.is_last_stage():
            loss = self.loss_fn(out, labels) if self.loss_fn is not None else out
        else:
            _send(_as_tuple(out), self.next_rank, self.device)
        return recv, out, loss

    def train_batch(self, data_iter: Optional[Iterator[Any]] = None) -> torch.Tensor:
        self.module_.train()
        saved = []
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        for _ in range(self.gas):
            recv, out, loss = self._forward_micro(data_iter, train=True)
            if loss is not None:
                total += loss.detach().float()
            saved.append((recv, out, loss))
        for i in reversed(range(self.gas)):
            recv, out, loss = saved[i]
            self.inner.micro_steps = self.micro_steps + (self.gas - 1 - i)
            self.inner.begin_micro_backward()
            if self.is_last_stage():
                (loss / self.gas).backward()
            else:
                grads = _recv(self.next_rank, self.device)
                outs = [t for t in _as_tuple(out) if t.is_floating_point()]
                pairs = [(t, g) for t, g in zip(outs, grads) if t.requires_grad]
                if pairs:
                    torch.autograd.backward([t for t, _ in pairs], [g for _, g in pairs])
            self.inner._end_backward()
            if not self.is_first_stage():
                gs = tuple(t.grad if t.grad is not None else torch.zeros_like(t)
                           for t in recv if t.is_floating_point())
                _send(gs, self.prev_rank, self.device)
            saved[i] = None  # free this micro-batch's activations
        # optimizer step on the accumulation boundary (inner.step advances its micro counter)
        self.inner.micro_steps = self.micro_steps + self.gas - 1
        self.inner.step()
        self.micro_steps += self.gas
        self.global_steps += 1
        self.global_samples += self.config.train_batch_size
        loss = self._broadcast_loss(total / self.gas)
        self.agg_train_loss = loss
        return loss

    @torch.no_grad()
    def eval_batch(self, data_iter: Optional[Iterator[Any]] = None, num_micro_batches: Optional[int] = None
                   ) -> torch.Tensor:
        self.module_.eval()
        n = num_micro_batches or self.gas
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        for _ in range(n):
            _, _, loss = self._forward_micro(data_iter, train=False)
            if loss is not None:
                total += loss.float()
        self.module_.train()
        return self._broadcast_loss(total / n)

    def _broadcast_loss(self, loss: torch.Tensor) -> torch.Tensor:
        if self.pp > 1 and dist.is_initialized():
            loss = loss.clone()
            dist.broadcast(loss, src=self.last_stage_rank, group=self.pipe_group)
        return loss

    # -- checkpointing: every stage saves its own layers (and optimizer shard) ------------------
    def save_checkpoint(self, save_dir: str, tag: Optional[str] = None, client_state: Any = None,
                        save_latest: bool = True) -> bool:
        import os

        tag = tag or f"global_step{self.global_steps}"
        sub = os.path.join(str(save_dir), str(tag), f"pipe_stage_{self.stage_id:02d}")
        self.inner.global_steps = self.global_steps
        ok = self.inner.save_checkpoint(sub, tag="stage", client_state=client_state, save_latest=False)
        if save_latest and self.global_rank == 0:
            with open(os.path.join(str(save_dir), "latest"), "w") as f:
                f.write(str(tag))
        return ok

    def load_checkpoint(self, load_dir: str, tag: Optional[str] = None, **kw: Any) -> Tuple[Optional[str], Any]:
        import os

        if tag is None:
            latest = os.path.join(str(load_dir), "latest")
            if not os.path.exists(latest):
                return None, None
            tag = open(latest).read().strip()
        sub = os.path.join(str(load_dir), str(tag), f"pipe_stage_{self.stage_id:02d}")
        path, client = self.inner.load_checkpoint(sub, tag="stage", **kw)
        self.global_steps = self.inner.global_steps
        self.micro_steps = self.global_steps * self.gas
        return path, client

    def forward(self, *a: Any, **kw: Any) -> Any:  # pragma: no cover - pipelines run train/eval_batch
        raise RuntimeError("PipelineEngine: call train_batch(data_iter) / eval_batch(data_iter)")
