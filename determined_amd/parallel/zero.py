"""ZeRO data-parallel engine (stages 0/1/2; stage 3 in ``zero3.py``) with a DeepSpeed-style API.

The reference's ``DeepSpeedTrial`` drives a ``deepspeed.DeepSpeedEngine`` (reference
``harness/determined/pytorch/deepspeed/_deepspeed_trial.py:364`` ``_train_for_step`` calls
``engine.backward`` / ``engine.step`` once per micro-batch and checks ``engine.micro_steps``).
DeepSpeed does not exist on this image and its CUDA kernels would not be the right design for
MI355X anyway, so this module provides the engine natively:

Memory layout (one flat buffer per parameter dtype):

* every trainable parameter becomes a view into a flat parameter buffer ``P``; the flat
  buffer is cut into buckets (reverse registration order ~ gradient-ready order), each
  padded to ``world * 8`` elements so that the per-rank chunk of every bucket is 16-byte
  aligned.  Rank ``r`` owns chunk ``r`` of every bucket (interleaved ownership keeps every
  collective a single contiguous ``reduce_scatter`` / ``all_gather`` with equal shards);
* gradients are accumulated by the engine into a flat gradient buffer ``G`` (fp32 when
  accumulating over several micro-batches, the parameter dtype otherwise).  Autograd's
  gradient for each parameter is handed over in a post-accumulate hook and copied (first
  micro-batch of a window) or added (later micro-batches) with ONE multi-tensor op per
  bucket, then dropped, so no per-parameter ``.grad`` stays alive;
* on the last micro-batch of an accumulation window each completed bucket immediately
  issues its collective on RCCL's stream, overlapping the rest of backward:
  stage 2 -> ``reduce_scatter_tensor`` into this rank's gradient shard,
  stage 1 -> ``all_reduce`` (full gradients, sharded optimizer state),
  stage 0 -> ``all_reduce`` and every rank updates everything;
* the optimizer runs on *fragments*: the intersection of each parameter with the rank's
  chunk.  Fragments alias ``P`` (bf16) and the gradient shard, so the fused multi-tensor
  AdamW/SGD kernels (``csrc/optim.hip``) keep the fp32 master copy + moments for the shard
  only and write the rounded bf16 weights straight into ``P`` -- one launch for the shard;
* ``all_gather_into_tensor`` per bucket then rebuilds the full parameters (issued async,
  waited on by the next forward).

Gradient clipping uses the shard-local sum of squares from the fused norm kernel, one
scalar ``all_reduce`` and the fused finalize kernel; nothing synchronises with the host.

ZeRO-3 (parameter partitioning with per-module gather in forward/backward) is ``zero3.py``.
"""

import contextlib
import json
import logging
import math
import os
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
from torch import nn

from determined_amd.utils.tensor import is_dense

logger = logging.getLogger("determined_amd.parallel.zero")

MiB = 1 << 20
_ALIGN_BYTES = 16


# ---------------------------------------------------------------------------------------------
# config
# ---------------------------------------------------------------------------------------------
class DeepSpeedConfigError(ValueError):
    pass


def _dtype_from_str(s: Optional[str]) -> Optional[torch.dtype]:
    if s is None:
        return None
    m = {"fp32": torch.float32, "float32": torch.float32, "float": torch.float32,
         "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}
    if s not in m:
        raise DeepSpeedConfigError(f"unsupported dtype {s!r} (fp32 / bf16)")
    return m[s]


class DeepSpeedConfig:
    """The subset of the DeepSpeed JSON config this engine honours (batch sizes, optimizer,
    scheduler, bf16, zero_optimization, gradient_clipping, data types)."""

    def __init__(self, config: Union[str, os.PathLike, Dict[str, Any]], world_size: int) -> None:
        if isinstance(config, (str, os.PathLike)):
            with open(config) as f:
                config = json.load(f)
        if not isinstance(config, dict):
            raise DeepSpeedConfigError("DeepSpeed config must be a dict or a path to a JSON file")
        self.raw = dict(config)
        self.world_size = world_size
        tbs = config.get("train_batch_size")
        mb = config.get("train_micro_batch_size_per_gpu")
        gas = config.get("gradient_accumulation_steps")
        tbs = int(tbs) if tbs is not None else None
        mb = int(mb) if mb is not None else None
        gas = int(gas) if gas is not None else None
        if tbs is not None and mb is not None and gas is not None:
            if tbs != mb * gas * world_size:
                raise DeepSpeedConfigError(
                    f"train_batch_size {tbs} != train_micro_batch_size_per_gpu {mb} * "
                    f"gradient_accumulation_steps {gas} * world_size {world_size}")
        elif tbs is not None and mb is not None:
            gas = tbs // (mb * world_size)
        elif tbs is not None and gas is not None:
            mb = tbs // (gas * world_size)
        elif mb is not None and gas is not None:
            tbs = mb * gas * world_size
        elif tbs is not None:
            gas = 1
            mb = tbs // world_size
        elif mb is not None:
            gas = gas or 1
            tbs = mb * gas * world_size
        else:
            raise DeepSpeedConfigError("one of train_batch_size / train_micro_batch_size_per_gpu is required")
        if not mb or not gas or mb * gas * world_size != tbs:
            raise DeepSpeedConfigError(
                f"inconsistent batch config: train_batch_size={tbs}, micro={mb}, gas={gas}, world={world_size}")
        self.train_batch_size, self.micro_batch, self.gas = tbs, mb, gas
        if config.get("fp16", {}).get("enabled", False):
            raise DeepSpeedConfigError("fp16 is not supported: MI355X trains in bf16 (set bf16.enabled)")
        self.bf16 = bool(config.get("bf16", config.get("bfloat16", {})).get("enabled", False))
        z = config.get("zero_optimization", {}) or {}
        if isinstance(z, bool):
            z = {"stage": 1 if z else 0}
        self.zero_stage = int(z.get("stage", 0))
        if self.zero_stage not in (0, 1, 2, 3):
            raise DeepSpeedConfigError(f"zero_optimization.stage {self.zero_stage} is not supported (0-3)")
        for k in ("offload_optimizer", "offload_param"):
            dev = (z.get(k) or {}).get("device", "none")
            if dev not in (None, "none"):
                raise DeepSpeedConfigError(f"zero_optimization.{k} is not supported (HBM holds the state)")
        # DeepSpeed sizes buckets in elements; default here is 16M elements (32 MiB bf16),
        # large enough to be bandwidth-bound on xGMI rings and small enough to overlap backward.
        self.reduce_bucket_elems = int(z.get("reduce_bucket_size", 16 * MiB))
        self.allgather_bucket_elems = int(z.get("allgather_bucket_size", self.reduce_bucket_elems))
        self.overlap_comm = bool(z.get("overlap_comm", True))
        self.gradient_clipping = float(config.get("gradient_clipping", 0.0) or 0.0)
        self.optimizer = config.get("optimizer")
        self.scheduler = config.get("scheduler")
        dt = config.get("data_types", {}) or {}
        self.grad_accum_dtype = _dtype_from_str(dt.get("grad_accum_dtype"))
        self.communication_dtype = _dtype_from_str(config.get("communication_data_type"))
        self.steps_per_print = int(config.get("steps_per_print", 10))
        self.wall_clock_breakdown = bool(config.get("wall_clock_breakdown", False))
        self.prescale_gradients = bool(config.get("prescale_gradients", False))
        self.gradient_predivide_factor = float(config.get("gradient_predivide_factor", 1.0))


# ---------------------------------------------------------------------------------------------
# LR schedules (DeepSpeed "scheduler" section)
# ---------------------------------------------------------------------------------------------
class _GroupLR:
    """Base for per-step LR schedules writing ``lr`` into the optimizer's param groups."""

    def __init__(self, optimizer: Any, last_batch_iteration: int = -1) -> None:
        self.optimizer = optimizer
        self.last_batch_iteration = last_batch_iteration
        self.base_lrs = [g["lr"] for g in optimizer.param_groups]
        self._last_lr = self._apply()

    def get_lr(self) -> List[float]:
        raise NotImplementedError

    def _apply(self) -> List[float]:
        lrs = self.get_lr()
        for g, lr in zip(self.optimizer.param_groups, lrs):
            g["lr"] = lr
        return lrs

    def step(self, last_batch_iteration: Optional[int] = None) -> None:
        self.last_batch_iteration = self.last_batch_iteration + 1 if last_batch_iteration is None else \
            last_batch_iteration
        self._last_lr = self._apply()

    def get_last_lr(self) -> List[float]:
        return list(self._last_lr)

    def state_dict(self) -> Dict[str, Any]:
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.last_batch_iteration = int(sd["last_batch_iteration"])
        self._last_lr = self._apply()


def _per_group(optimizer: Any, v: Union[float, Sequence[float]]) -> List[float]:
    n = len(optimizer.param_groups)
    if isinstance(v, (list, tuple)):
        if len(v) != n:
            raise DeepSpeedConfigError(f"expected {n} values, got {len(v)}")
        return [float(x) for x in v]
    return [float(v)] * n


class WarmupLR(_GroupLR):
    """min_lr -> max_lr over ``warmup_num_steps`` (log or linear ramp), then constant."""

    def __init__(self, optimizer: Any, warmup_min_lr: Union[float, Sequence[float]] = 0.0,
                 warmup_max_lr: Union[float, Sequence[float]] = 0.001, warmup_num_steps: int = 1000,
                 warmup_type: str = "log", last_batch_iteration: int = -1) -> None:
        if warmup_type not in ("log", "linear"):
            raise DeepSpeedConfigError(f"warmup_type must be log or linear, got {warmup_type}")
        self.min_lrs = _per_group(optimizer, warmup_min_lr)
        self.max_lrs = _per_group(optimizer, warmup_max_lr)
        self.warmup_num_steps = max(2, int(warmup_num_steps))
        self.warmup_type = warmup_type
        super().__init__(optimizer, last_batch_iteration)

    def _gamma(self) -> float:
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            if self.warmup_type == "log":
                return math.log(it + 1) / math.log(self.warmup_num_steps)
            return it / self.warmup_num_steps
        return 1.0

    def get_lr(self) -> List[float]:
        if self.last_batch_iteration < 0:
            return [0.0] * len(self.min_lrs)
        g = self._gamma()
        return [lo + (hi - lo) * g for lo, hi in zip(self.min_lrs, self.max_lrs)]


class WarmupDecayLR(WarmupLR):
    """WarmupLR followed by linear decay to 0 at ``total_num_steps``."""

    def __init__(self, optimizer: Any, total_num_steps: int, warmup_min_lr: Union[float, Sequence[float]] = 0.0,
                 warmup_max_lr: Union[float, Sequence[float]] = 0.001, warmup_num_steps: int = 1000,
                 warmup_type: str = "log", last_batch_iteration: int = -1) -> None:
        self.total_num_steps = int(total_num_steps)
        super().__init__(optimizer, warmup_min_lr, warmup_max_lr, warmup_num_steps, warmup_type,
                         last_batch_iteration)
        if self.total_num_steps < self.warmup_num_steps:
            logger.warning("total_num_steps %d < warmup_num_steps %d", self.total_num_steps, self.warmup_num_steps)

    def _gamma(self) -> float:
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            return super()._gamma()
        return max(0.0, (self.total_num_steps - it) / max(1.0, self.total_num_steps - self.warmup_num_steps))


class WarmupCosineLR(_GroupLR):
    """Ratio of the base LR: ``warmup_min_ratio`` -> 1 linearly, then cosine to ``cos_min_ratio``."""

    def __init__(self, optimizer: Any, total_num_steps: int, warmup_min_ratio: float = 0.0,
                 warmup_num_steps: int = 1000, cos_min_ratio: float = 0.0001, warmup_type: str = "log",
                 last_batch_iteration: int = -1) -> None:
        self.total_num_steps = int(total_num_steps)
        self.warmup_min_ratio = float(warmup_min_ratio)
        self.warmup_num_steps = max(2, int(warmup_num_steps))
        self.cos_min_ratio = float(cos_min_ratio)
        self.warmup_type = warmup_type
        self.org_lrs = [g["lr"] for g in optimizer.param_groups]
        super().__init__(optimizer, last_batch_iteration)

    def _ratio(self) -> float:
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            if self.warmup_type == "log":
                r = math.log(it + 1) / math.log(self.warmup_num_steps)
            else:
                r = it / self.warmup_num_steps
            return self.warmup_min_ratio + (1.0 - self.warmup_min_ratio) * r
        prog = min(1.0, (it - self.warmup_num_steps) / max(1, self.total_num_steps - self.warmup_num_steps))
        return self.cos_min_ratio + (1.0 - self.cos_min_ratio) * 0.5 * (1.0 + math.cos(math.pi * prog))

    def get_lr(self) -> List[float]:
        if self.last_batch_iteration < 0:
            return [0.0] * len(self.org_lrs)
        r = self._ratio()
        return [lr * r for lr in self.org_lrs]


class OneCycle(_GroupLR):
    """Triangular cycle min->max->min over ``2 * cycle_first_step_size`` steps, then decay."""

    def __init__(self, optimizer: Any, cycle_min_lr: float, cycle_max_lr: float, cycle_first_step_size: int = 2000,
                 cycle_second_step_size: Optional[int] = None, decay_step_size: int = 0,
                 decay_lr_rate: float = 0.0, last_batch_iteration: int = -1, **_: Any) -> None:
        self.min_lr, self.max_lr = float(cycle_min_lr), float(cycle_max_lr)
        self.first = int(cycle_first_step_size)
        self.second = int(cycle_second_step_size if cycle_second_step_size is not None else self.first)
        self.decay_step_size = int(decay_step_size)
        self.decay_lr_rate = float(decay_lr_rate)
        super().__init__(optimizer, last_batch_iteration)

    def get_lr(self) -> List[float]:
        it = max(self.last_batch_iteration, 0)
        n = len(self.optimizer.param_groups)
        if it <= self.first:
            lr = self.min_lr + (self.max_lr - self.min_lr) * it / max(1, self.first)
        elif it <= self.first + self.second:
            lr = self.max_lr - (self.max_lr - self.min_lr) * (it - self.first) / max(1, self.second)
        else:
            k = it - self.first - self.second
            lr = self.min_lr
            if self.decay_step_size > 0:
                lr = self.min_lr / (1.0 + self.decay_lr_rate * (k / self.decay_step_size))
        return [lr] * n


_SCHEDULERS = {"WarmupLR": WarmupLR, "WarmupDecayLR": WarmupDecayLR, "WarmupCosineLR": WarmupCosineLR,
               "OneCycle": OneCycle}


def build_scheduler(spec: Dict[str, Any], optimizer: Any) -> Any:
    typ = spec.get("type")
    if typ not in _SCHEDULERS:
        raise DeepSpeedConfigError(f"unsupported scheduler type {typ!r} (have {sorted(_SCHEDULERS)})")
    return _SCHEDULERS[typ](optimizer, **(spec.get("params") or {}))


# ---------------------------------------------------------------------------------------------
# flat layout
# ---------------------------------------------------------------------------------------------
def _param_view(buf: torch.Tensor, offset: int, p: torch.Tensor) -> torch.Tensor:
    flat = buf.narrow(0, offset, p.numel())
    return flat.as_strided(p.shape, p.stride()) if is_dense(p) else flat.view(p.shape)


class _Bucket:
    """A contiguous range ``[start, start+numel)`` of the flat buffers of one dtype."""

    def __init__(self, index: int, params: List[nn.Parameter], pidx: List[int], start: int, world: int,
                 align: int) -> None:
        self.index = index
        self.params = params
        self.pidx = pidx
        self.start = start
        self.offsets: List[int] = []
        n = 0
        for p in params:
            self.offsets.append(n)
            n += (p.numel() + align - 1) // align * align
        unit = world * align
        self.numel = (n + unit - 1) // unit * unit
        self.chunk = self.numel // world
        self.pending = len(params)
        self.arrived = [False] * len(params)
        self.touched = [False] * len(params)  # wrote G during the current accumulation window
        self.copy_dst: List[torch.Tensor] = []
        self.copy_src: List[torch.Tensor] = []
        self.add_dst: List[torch.Tensor] = []
        self.add_src: List[torch.Tensor] = []
        self.work: Any = None
        self.gather_work: Any = None
        self.shard_off = 0  # offset of this bucket's chunk in the rank's gradient-shard buffer

    def fragments(self, rank: int) -> List[Tuple[int, int, int, int]]:
        """(local param index in bucket, start within param, end within param, bucket offset)."""
        lo, hi = rank * self.chunk, (rank + 1) * self.chunk
        out = []
        for i, (p, off) in enumerate(zip(self.params, self.offsets)):
            s, e = max(lo, off), min(hi, off + p.numel())
            if s < e:
                out.append((i, s - off, e - off, s))
        return out


class _FlatSpace:
    """Per-dtype flat parameter / gradient buffers and their buckets."""

    def __init__(self, params: List[nn.Parameter], dtype: torch.dtype, grad_dtype: torch.dtype, world: int,
                 rank: int, bucket_elems: int, device: torch.device, global_index: Dict[int, int]) -> None:
        self.dtype = dtype
        self.grad_dtype = grad_dtype
        self.world = world
        self.rank = rank
        align = max(1, _ALIGN_BYTES // torch.empty((), dtype=dtype).element_size())
        align = max(align, _ALIGN_BYTES // torch.empty((), dtype=grad_dtype).element_size(), 4)
        self.buckets: List[_Bucket] = []
        cur: List[nn.Parameter] = []
        cur_n = 0
        start = 0
        for p in reversed(params):  # ~ gradient-ready order
            if cur and cur_n + p.numel() > bucket_elems:
                b = _Bucket(len(self.buckets), cur, [global_index[id(q)] for q in cur], start, world, align)
                self.buckets.append(b)
                start += b.numel
                cur, cur_n = [], 0
            cur.append(p)
            cur_n += p.numel()
        if cur:
            b = _Bucket(len(self.buckets), cur, [global_index[id(q)] for q in cur], start, world, align)
            self.buckets.append(b)
            start += b.numel
        self.numel = start
        self.P = torch.zeros(self.numel, dtype=dtype, device=device)
        self.G = torch.zeros(self.numel, dtype=grad_dtype, device=device)
        shard = 0
        for b in self.buckets:
            b.shard_off = shard
            shard += b.chunk
        self.shard_numel = shard
        self.GS: Optional[torch.Tensor] = None
        self.slot: Dict[int, Tuple[_Bucket, int]] = {}
        self.gviews: Dict[int, torch.Tensor] = {}
        with torch.no_grad():
            for b in self.buckets:
                for i, (p, off) in enumerate(zip(b.params, b.offsets)):
                    v = _param_view(self.P, b.start + off, p)
                    v.copy_(p.data)
                    p.data = v
                    self.slot[id(p)] = (b, i)
                    self.gviews[id(p)] = _param_view(self.G, b.start + off, p)

    def bucket_slice(self, buf: torch.Tensor, b: _Bucket) -> torch.Tensor:
        return buf.narrow(0, b.start, b.numel)

    def chunk_slice(self, buf: torch.Tensor, b: _Bucket) -> torch.Tensor:
        return buf.narrow(0, b.start + self.rank * b.chunk, b.chunk)


# ---------------------------------------------------------------------------------------------
# optimizer over shard fragments
# ---------------------------------------------------------------------------------------------
class ZeroOptimizer(torch.optim.Optimizer):
    """Presents the user's param groups (for LR schedules / logging) while the real update runs
    on this rank's shard fragments with an inner (fused) optimizer."""

    def __init__(self, groups: List[Dict[str, Any]], defaults: Dict[str, Any],
                 inner_factory: Callable[[List[Dict[str, Any]]], torch.optim.Optimizer]) -> None:
        super().__init__(groups, defaults)
        self._inner_factory = inner_factory
        self.inner: Optional[torch.optim.Optimizer] = None
        self.frag_info: List[Tuple[int, int, int]] = []  # (global param index, start, end)

    def _bind(self, frag_groups: List[List[nn.Parameter]], frag_info: List[Tuple[int, int, int]]) -> None:
        spec = []
        for g, frags in zip(self.param_groups, frag_groups):
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = frags
            spec.append(d)
        self.frag_info = frag_info
        nonempty = [s for s in spec if s["params"]]
        self._group_map = [i for i, s in enumerate(spec) if s["params"]]
        self.inner = self._inner_factory(nonempty) if nonempty else None

    def _sync_hyper(self) -> None:
        if self.inner is None:
            return
        for gi, ig in zip(self._group_map, self.inner.param_groups):
            for k, v in self.param_groups[gi].items():
                if k != "params":
                    ig[k] = v

    def step(self, closure: Optional[Callable[[], float]] = None, **kw: Any) -> Optional[float]:  # type: ignore
        raise RuntimeError("call engine.step(); the ZeRO optimizer is driven by the engine")

    def zero_grad(self, set_to_none: bool = True) -> None:
        pass

    def _inner_params(self) -> List[nn.Parameter]:
        if self.inner is None:
            return []
        return [p for g in self.inner.param_groups for p in g["params"]]

    def shard_state_dict(self) -> Dict[str, Any]:
        """This rank's optimizer shard with enough layout information to re-shard on load."""
        pieces: List[Dict[str, Any]] = []
        scalars: Dict[str, Any] = {}
        if self.inner is not None:
            for frag, (pi, s, e) in zip(self._inner_params(), self.frag_info):
                st = self.inner.state.get(frag, {})
                ent: Dict[str, Any] = {"param": pi, "start": s, "end": e}
                for k, v in st.items():
                    if isinstance(v, torch.Tensor) and v.numel() == frag.numel() and v.numel() > 1 or \
                            (isinstance(v, torch.Tensor) and k in ("master", "exp_avg", "exp_avg_sq",
                                                                   "momentum_buffer")):
                        ent[k] = v.detach().reshape(-1).to("cpu", copy=True)
                    elif isinstance(v, torch.Tensor):
                        scalars[k] = v.detach().to("cpu", copy=True)
                    else:
                        scalars[k] = v
                pieces.append(ent)
        groups = [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]
        return {"pieces": pieces, "scalars": scalars, "param_groups": groups}

    def load_shard_states(self, shards: List[Dict[str, Any]]) -> None:
        """Rebuild this rank's fragment state from any number of saved shards (any world size)."""
        for g, sg in zip(self.param_groups, shards[0]["param_groups"] if shards else []):
            for k, v in sg.items():
                g[k] = v
        self._sync_hyper()
        if self.inner is None:
            return
        by_param: Dict[int, List[Dict[str, Any]]] = {}
        for sh in shards:
            for ent in sh["pieces"]:
                by_param.setdefault(int(ent["param"]), []).append(ent)
        scalars = shards[0]["scalars"] if shards else {}
        for frag, (pi, s, e) in zip(self._inner_params(), self.frag_info):
            st = self.inner.state[frag]
            if not st and hasattr(self.inner, "_init_state"):
                self.inner._init_state(frag, st)
            keys = set()
            for ent in by_param.get(pi, []):
                keys.update(k for k in ent if k not in ("param", "start", "end"))
            for k in keys:
                dst = torch.empty(e - s, dtype=torch.float32)
                filled = 0
                for ent in by_param.get(pi, []):
                    if k not in ent:
                        continue
                    a, b = max(s, int(ent["start"])), min(e, int(ent["end"]))
                    if a < b:
                        dst[a - s : b - s] = ent[k][a - int(ent["start"]) : b - int(ent["start"])].float()
                        filled += b - a
                if filled != e - s:
                    raise RuntimeError(f"optimizer checkpoint does not cover param {pi}[{s}:{e}] for {k!r}")
                ref = st.get(k)
                if isinstance(ref, torch.Tensor):
                    ref.copy_(dst.view_as(ref).to(ref.dtype))
                else:
                    st[k] = dst.view_as(frag).to(frag.device)
            for k, v in scalars.items():
                if k == "step" and isinstance(st.get("step"), torch.Tensor):
                    st["step"].fill_(float(v))
                elif k not in st:
                    st[k] = v.to(frag.device) if isinstance(v, torch.Tensor) else v
        if hasattr(self.inner, "_plans"):
            self.inner._plans.clear()
        if hasattr(self.inner, "_step_t") and "step" in scalars:
            for t in self.inner._step_t.values():
                t.fill_(float(scalars["step"]))

    def state_dict(self) -> Dict[str, Any]:  # type: ignore[override]
        return self.shard_state_dict()

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:  # type: ignore[override]
        self.load_shard_states([state_dict])


def _optimizer_factory(cfg_opt: Optional[Dict[str, Any]], client: Optional[torch.optim.Optimizer],
                       master_weights: bool, on_gpu: bool
                       ) -> Tuple[Dict[str, Any], Callable[[List[Dict[str, Any]]], torch.optim.Optimizer]]:
    from determined_amd.ops import FusedAdamW, FusedSGD

    if client is not None:
        cls = type(client)
        defaults = dict(client.defaults)
        if isinstance(client, (FusedAdamW, FusedSGD)):
            mw = master_weights or bool(getattr(client, "master_weights", False))

            def make(groups: List[Dict[str, Any]]) -> torch.optim.Optimizer:
                o = cls(groups, **defaults, master_weights=mw)
                o.set_grad_clipping(client.max_grad_norm)
                return o

            return defaults, make
        if on_gpu and isinstance(client, torch.optim.AdamW):
            d = {"lr": defaults["lr"], "betas": defaults["betas"], "eps": defaults["eps"],
                 "weight_decay": defaults["weight_decay"], "adam_w_mode": True}
            return d, lambda groups: FusedAdamW(groups, **d, master_weights=master_weights)
        if on_gpu and type(client) is torch.optim.Adam:
            d = {"lr": defaults["lr"], "betas": defaults["betas"], "eps": defaults["eps"],
                 "weight_decay": defaults["weight_decay"], "adam_w_mode": False}
            return d, lambda groups: FusedAdamW(groups, **d, master_weights=master_weights)
        return defaults, lambda groups: cls(groups, **defaults)
    if cfg_opt is None:
        raise DeepSpeedConfigError("no optimizer: pass one to initialize() or set 'optimizer' in the config")
    typ = str(cfg_opt.get("type", "")).lower()
    params = dict(cfg_opt.get("params") or {})
    if typ in ("adam", "adamw", "fusedadam"):
        adam_w_mode = bool(params.pop("adam_w_mode", True)) if typ != "adamw" else True
        if typ == "adam" and "torch_adam" in params:
            params.pop("torch_adam")
        d = {"lr": float(params.pop("lr", 1e-3)), "betas": tuple(params.pop("betas", (0.9, 0.999))),
             "eps": float(params.pop("eps", 1e-8)), "weight_decay": float(params.pop("weight_decay", 0.0)),
             "adam_w_mode": adam_w_mode}
        params.pop("bias_correction", None)
        if params:
            logger.warning("ignoring unsupported Adam params %s", sorted(params))
        return d, lambda groups: FusedAdamW(groups, **d, master_weights=master_weights)
    if typ == "sgd":
        d = {"lr": float(params.pop("lr", 1e-3)), "momentum": float(params.pop("momentum", 0.0)),
             "dampening": float(params.pop("dampening", 0.0)),
             "weight_decay": float(params.pop("weight_decay", 0.0)), "nesterov": bool(params.pop("nesterov", False))}
        return d, lambda groups: FusedSGD(groups, **d, master_weights=master_weights)
    raise DeepSpeedConfigError(f"unsupported optimizer type {cfg_opt.get('type')!r} (Adam, AdamW, SGD)")


# ---------------------------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------------------------
class ZeroEngine(nn.Module):
    """DeepSpeed-engine-like wrapper: ``loss = engine(batch); engine.backward(loss); engine.step()``."""

    def __init__(self, model: nn.Module, config: DeepSpeedConfig, optimizer: Optional[torch.optim.Optimizer] = None,
                 model_parameters: Optional[Iterable] = None, lr_scheduler: Any = None,
                 process_group: Optional[dist.ProcessGroup] = None, mpu: Any = None) -> None:
        super().__init__()
        self.config = config
        if mpu is not None and hasattr(mpu, "get_data_parallel_group"):
            process_group = mpu.get_data_parallel_group()
        self.process_group = process_group
        # tensor/model parallelism: gradients are reduced over the data-parallel group only;
        # the clipping norm additionally sums over the model-parallel group
        self.mp_group = mpu.get_model_parallel_group() if mpu is not None and \
            hasattr(mpu, "get_model_parallel_group") else None
        self.mp_size = int(mpu.get_model_parallel_world_size()) if mpu is not None and \
            hasattr(mpu, "get_model_parallel_world_size") else 1
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world_size = dist.get_world_size(process_group) if self.distributed else 1
        self.global_rank = dist.get_rank() if self.distributed else 0
        self.dp_rank = dist.get_rank(process_group) if self.distributed else 0
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        backend = dist.get_backend(process_group) if self.distributed else "none"
        self._use_avg = backend == "nccl"
        if torch.cuda.is_available():
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        self.stage = config.zero_stage
        self._shard_world = self.world_size if self.stage >= 1 else 1
        self._shard_rank = self.dp_rank if self.stage >= 1 else 0
        model = model.to(self.device)
        if config.bf16:
            model = model.to(torch.bfloat16)
        self.module = model
        self.micro_steps = 0
        self.global_steps = 0
        self.global_samples = 0
        self.skipped_steps = 0
        self._grad_norm: Optional[torch.Tensor] = None
        self._sync_enabled = True
        self._boundary_now = False

        # -- parameters & groups -----------------------------------------------------------
        if optimizer is not None:
            user_groups = [dict(g) for g in optimizer.param_groups]
        elif model_parameters is not None:
            mp = list(model_parameters)
            user_groups = [dict(g) for g in mp] if mp and isinstance(mp[0], dict) else [{"params": mp}]
        else:
            user_groups = [{"params": [p for p in model.parameters() if p.requires_grad]}]
        module_ids = {id(p) for p in model.parameters()}
        seen = set()
        for g in user_groups:
            ps = []
            for p in g["params"]:
                if id(p) in module_ids and id(p) not in seen and p.requires_grad:
                    ps.append(p)
                    seen.add(id(p))
            g["params"] = ps
        self._params: List[nn.Parameter] = [p for g in user_groups for p in g["params"]]
        self._group_of = {id(p): gi for gi, g in enumerate(user_groups) for p in g["params"]}
        self._pindex = {id(p): i for i, p in enumerate(self._params)}
        self._broadcast_module()

        # -- flat spaces -------------------------------------------------------------------
        self._build_spaces()

        # -- optimizer over fragments ------------------------------------------------------
        master = config.bf16 or any(p.dtype == torch.bfloat16 for p in self._params)
        defaults, factory = _optimizer_factory(config.optimizer if optimizer is None else None, optimizer,
                                               master, self.device.type == "cuda")
        opt_groups = []
        for g in user_groups:
            d = dict(defaults)
            d.update({k: v for k, v in g.items() if k != "params"})
            d["params"] = g["params"]
            opt_groups.append(d)
        self.optimizer = ZeroOptimizer(opt_groups, defaults, factory)
        # fragment = (param ∩ this rank's chunk of a bucket); P-view as the param, shard-view as grad
        frag_groups: List[List[nn.Parameter]] = [[] for _ in opt_groups]
        info_groups: List[List[Tuple[int, int, int]]] = [[] for _ in opt_groups]
        for sp in self.spaces:
            for b in sp.buckets:
                for li, s, e, boff in b.fragments(self._shard_rank):
                    p = b.params[li]
                    pv, gv = self._fragment_views(sp, b, boff, e - s)
                    frag = nn.Parameter(pv, requires_grad=False)
                    if gv.dtype != pv.dtype and hasattr(frag, "grad_dtype"):
                        frag.grad_dtype = None  # fp32-accumulated grads on bf16 weights
                    frag.grad = gv
                    gi = self._group_of[id(p)]
                    frag_groups[gi].append(frag)
                    info_groups[gi].append((self._pindex[id(p)], s, e))
        self.optimizer._bind(frag_groups, [fi for grp in info_groups for fi in grp])
        if self.optimizer.inner is not None and hasattr(self.optimizer.inner, "_partial_reducer"):
            inner = self.optimizer.inner
            inner._partial_reducer = self._allreduce_norm if (self._shard_world > 1 or self.mp_size > 1) else None
            if self.mp_size > 1:
                # each TP rank holds different shards of sharded params but a full copy of
                # replicated ones: count the latter 1/tp per rank so the TP sum counts them once
                wmap = {}
                for frag, (pi, _, _) in zip(self.optimizer._inner_params(), self.optimizer.frag_info):
                    sharded = bool(getattr(self._params[pi], "tensor_model_parallel", False))
                    wmap[id(frag)] = 1.0 if sharded else 1.0 / self.mp_size
                inner._norm_weight = lambda t, _w=wmap: _w.get(id(t), 1.0)
        if config.gradient_clipping > 0 and self.optimizer.inner is not None:
            if hasattr(self.optimizer.inner, "set_grad_clipping"):
                self.optimizer.inner.set_grad_clipping(config.gradient_clipping)
        self._clip_fallback = config.gradient_clipping > 0 and not hasattr(self.optimizer.inner, "set_grad_clipping")

        # -- scheduler -----------------------------------------------------------------------
        if lr_scheduler is not None and callable(lr_scheduler) and not hasattr(lr_scheduler, "step"):
            lr_scheduler = lr_scheduler(self.optimizer)
        if lr_scheduler is None and config.scheduler is not None:
            lr_scheduler = build_scheduler(config.scheduler, self.optimizer)
        self.lr_scheduler = lr_scheduler

        self._install_hooks()

    # -- setup helpers ------------------------------------------------------------------------
    def _build_spaces(self) -> None:
        """One flat parameter/gradient space per parameter dtype, cut into reduce buckets."""
        config = self.config
        by_dtype: Dict[torch.dtype, List[nn.Parameter]] = {}
        for p in self._params:
            by_dtype.setdefault(p.dtype, []).append(p)
        self.spaces: List[_FlatSpace] = []
        for dt, ps in by_dtype.items():
            gdt = config.grad_accum_dtype or config.communication_dtype or \
                (torch.float32 if config.gas > 1 else dt)
            self.spaces.append(_FlatSpace(ps, dt, gdt, self._shard_world, self._shard_rank,
                                          config.reduce_bucket_elems, self.device, self._pindex))
        self._space_of: Dict[int, _FlatSpace] = {}
        for sp in self.spaces:
            for b in sp.buckets:
                for p in b.params:
                    self._space_of[id(p)] = sp
            if self.stage == 2:
                sp.GS = torch.zeros(sp.shard_numel, dtype=sp.grad_dtype, device=self.device)

    def _fragment_views(self, sp: "_FlatSpace", b: "_Bucket", boff: int, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """(parameter view, gradient view) of ``n`` elements at bucket offset ``boff`` of this rank."""
        pv = sp.P.narrow(0, b.start + boff, n)
        if self.stage == 2:
            assert sp.GS is not None
            return pv, sp.GS.narrow(0, b.shard_off + (boff - self._shard_rank * b.chunk), n)
        return pv, sp.G.narrow(0, b.start + boff, n)

    def _install_hooks(self) -> None:
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(p)) for p in self._params]

    def _broadcast_module(self) -> None:
        if self.world_size <= 1:
            return
        src = dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0
        ts = [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]
        by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
        for t in ts:
            by_dtype.setdefault(t.dtype, []).append(t)
        with torch.no_grad():
            for group in by_dtype.values():
                flat = torch.cat([t.reshape(-1) for t in group])
                dist.broadcast(flat, src=src, group=self.process_group)
                off = 0
                for t in group:
                    t.copy_(flat[off : off + t.numel()].view_as(t))
                    off += t.numel()

    def _allreduce_norm(self, sumsq: torch.Tensor) -> None:
        if self._shard_world > 1:
            dist.all_reduce(sumsq, group=self.process_group)
        if self.mp_size > 1:
            dist.all_reduce(sumsq, group=self.mp_group)

    # -- gradient hooks -------------------------------------------------------------------------
    def _make_hook(self, p: nn.Parameter) -> Callable[[torch.Tensor], None]:
        def hook(_: torch.Tensor) -> None:
            self._on_grad(p)

        return hook

    def _on_grad(self, p: nn.Parameter) -> None:
        sp = self._space_of[id(p)]
        b, i = sp.slot[id(p)]
        g = p.grad
        if g is None:
            return
        v = sp.gviews[id(p)]
        if b.touched[i]:  # already holds this window's earlier micro-batches
            b.add_dst.append(v)
            b.add_src.append(g)
        else:
            b.copy_dst.append(v)
            b.copy_src.append(g)
            b.touched[i] = True
        p.grad = None
        if not b.arrived[i]:
            b.arrived[i] = True
            b.pending -= 1
        if b.pending == 0:
            self._complete(sp, b)

    def _flush(self, b: _Bucket) -> None:
        if b.copy_dst:
            torch._foreach_copy_(b.copy_dst, b.copy_src)
        if b.add_dst:
            torch._foreach_add_(b.add_dst, b.add_src)
        b.copy_dst, b.copy_src, b.add_dst, b.add_src = [], [], [], []

    def _complete(self, sp: _FlatSpace, b: _Bucket) -> None:
        self._flush(b)
        if self._boundary_now and self._sync_enabled and b.work is None:
            b.work = self._reduce(sp, b)

    def _reduce(self, sp: _FlatSpace, b: _Bucket) -> Any:
        if self.world_size <= 1:
            if self.stage == 2:
                assert sp.GS is not None
                sp.GS.narrow(0, b.shard_off, b.chunk).copy_(sp.bucket_slice(sp.G, b))
            return None
        op = dist.ReduceOp.AVG if self._use_avg else dist.ReduceOp.SUM
        src = sp.bucket_slice(sp.G, b)
        if self.stage == 2:
            assert sp.GS is not None
            out = sp.GS.narrow(0, b.shard_off, b.chunk)
            return dist.reduce_scatter_tensor(out, src, op=op, group=self.process_group, async_op=True)
        return dist.all_reduce(src, op=op, group=self.process_group, async_op=True)

    def _end_backward(self) -> None:
        """After one micro-batch's backward: fill gradients that never arrived, mark touched."""
        for sp in self.spaces:
            for b in sp.buckets:
                if self._boundary_now:
                    if b.pending > 0:
                        for i, p in enumerate(b.params):
                            if not b.touched[i]:  # no gradient in the whole window
                                sp.gviews[id(p)].zero_()
                                b.touched[i] = True
                        self._complete(sp, b)
                else:
                    self._flush(b)
                b.arrived = [False] * len(b.params)
                b.pending = len(b.params)

    # -- public API (DeepSpeed engine surface) ---------------------------------------------------
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        self._wait_gather()
        return self.module(*args, **kwargs)

    def is_gradient_accumulation_boundary(self) -> bool:
        return (self.micro_steps + 1) % self.config.gas == 0

    def backward(self, loss: torch.Tensor, retain_graph: bool = False, scale_wrt_gas: bool = True) -> torch.Tensor:
        self.begin_micro_backward()
        if scale_wrt_gas and self.config.gas > 1:
            loss = loss / self.config.gas
        loss.backward(retain_graph=retain_graph)
        self._end_backward()
        return loss

    def begin_micro_backward(self) -> None:
        """Bracket a micro-batch backward that is not driven through ``backward(loss)`` (the
        pipeline engine back-propagates a received output gradient): call this before, and
        ``_end_backward()`` after, ``torch.autograd.backward``."""
        self._wait_gather()
        self._boundary_now = self.is_gradient_accumulation_boundary()
        if self.micro_steps % self.config.gas == 0:  # first micro-batch of a window: overwrite G
            for sp in self.spaces:
                for b in sp.buckets:
                    b.touched = [False] * len(b.params)

    @contextlib.contextmanager
    def no_sync(self) -> Iterator[None]:
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def _finish_reduce(self) -> None:
        for sp in self.spaces:
            for b in sp.buckets:
                if b.work is not None:
                    b.work.wait()
                    b.work = None
                    if not self._use_avg and self.world_size > 1:
                        if self.stage == 2:
                            assert sp.GS is not None
                            sp.GS.narrow(0, b.shard_off, b.chunk).div_(self.world_size)
                        else:
                            sp.bucket_slice(sp.G, b).div_(self.world_size)

    def _gather(self) -> None:
        if self._shard_world <= 1:
            return
        for sp in self.spaces:
            for b in sp.buckets:
                full = sp.bucket_slice(sp.P, b)
                mine = sp.chunk_slice(sp.P, b)
                if not self._use_avg:  # gloo: no in-place aliasing of input and output
                    mine = mine.clone()
                b.gather_work = dist.all_gather_into_tensor(full, mine, group=self.process_group, async_op=True)

    def _wait_gather(self) -> None:
        for sp in self.spaces:
            for b in sp.buckets:
                if b.gather_work is not None:
                    b.gather_work.wait()
                    b.gather_work = None

    def step(self, lr_kwargs: Optional[Dict[str, Any]] = None) -> None:
        """Call once per micro-batch; the update happens on the accumulation boundary."""
        boundary = self.is_gradient_accumulation_boundary()
        self.micro_steps += 1
        self.global_samples += self.config.micro_batch * self.world_size
        if not boundary:
            return
        self._finish_reduce()
        self.optimizer._sync_hyper()
        inner = self.optimizer.inner
        if inner is not None:
            if self._clip_fallback:
                self._clip_generic(inner)
            inner.step()
            self._grad_norm = getattr(inner, "last_grad_norm", None)
        elif self.config.gradient_clipping > 0 and (self._shard_world > 1 or self.mp_size > 1):
            self._allreduce_norm(torch.zeros(1, dtype=torch.float32, device=self.device))
        self._gather()
        # Stream-level wait (RCCL): later kernels on the compute stream see the gathered
        # params while the host runs ahead; direct users of ``engine.module`` stay correct.
        self._wait_gather()
        self.global_steps += 1
        if self.lr_scheduler is not None:
            self.lr_scheduler.step(**(lr_kwargs or {}))

    def _clip_generic(self, inner: torch.optim.Optimizer) -> None:
        grads = [p.grad for g in inner.param_groups for p in g["params"] if p.grad is not None]
        sq = torch.zeros(1, dtype=torch.float32, device=self.device)
        for g in grads:
            sq += g.float().pow(2).sum()
        if self._shard_world > 1:
            self._allreduce_norm(sq)
        norm = sq.sqrt()
        self._grad_norm = norm
        coef = (self.config.gradient_clipping / (norm + 1e-6)).clamp(max=1.0)
        for g in grads:
            g.mul_(coef.to(g.dtype))

    # -- info --------------------------------------------------------------------------------
    def train_batch_size(self) -> int:
        return self.config.train_batch_size

    def train_micro_batch_size_per_gpu(self) -> int:
        return self.config.micro_batch

    def gradient_accumulation_steps(self) -> int:
        return self.config.gas

    def zero_optimization_stage(self) -> int:
        return self.stage

    def bfloat16_enabled(self) -> bool:
        return self.config.bf16

    def fp16_enabled(self) -> bool:
        return False

    def get_lr(self) -> List[float]:
        return [g["lr"] for g in self.optimizer.param_groups]

    def get_global_grad_norm(self) -> Optional[float]:
        return None if self._grad_norm is None else float(self._grad_norm.reshape(-1)[0].item())

    def was_step_applied(self) -> bool:
        return True

    def to(self, *args: Any, **kwargs: Any) -> "ZeroEngine":  # type: ignore[override]
        # parameters are views into the engine's flat buffers; moving them would break that.
        return self

    def parameters(self, recurse: bool = True) -> Iterator[nn.Parameter]:  # type: ignore[override]
        return self.module.parameters(recurse)

    def state_dict(self, *args: Any, **kwargs: Any) -> Dict[str, Any]:  # type: ignore[override]
        self._wait_gather()
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, sd: Dict[str, Any], strict: bool = True) -> Any:  # type: ignore[override]
        self._wait_gather()
        with torch.no_grad():
            res = self.module.load_state_dict(sd, strict=strict)
        self._refresh_master()
        return res

    def _refresh_master(self) -> None:
        inner = self.optimizer.inner
        if inner is None:
            return
        with torch.no_grad():
            for g in inner.param_groups:
                for frag in g["params"]:
                    st = inner.state.get(frag)
                    if st and "master" in st:
                        st["master"].copy_(frag.detach().float())

    # -- checkpointing ----------------------------------------------------------------------
    def save_checkpoint(self, save_dir: Union[str, os.PathLike], tag: Optional[str] = None,
                        client_state: Optional[Dict[str, Any]] = None, save_latest: bool = True) -> bool:
        """``{save_dir}/{tag}/mp_rank_00_model_states.pt`` (rank 0: weights, scheduler, counters)
        + ``zero_pp_rank_{r}_mp_rank_00_optim_states.pt`` (every rank: its optimizer shard)."""
        self._wait_gather()
        tag = tag or f"global_step{self.global_steps}"
        d = os.path.join(os.fspath(save_dir), str(tag))
        os.makedirs(d, exist_ok=True)
        # stage 3 gathers the partitioned weights with collectives: every rank takes part
        full_sd = self.state_dict() if self.stage == 3 else None
        if self.global_rank == 0 or (self.dp_rank == 0 and self.process_group is not None):
            sd = {k: v.detach().to("cpu", copy=True) for k, v in (full_sd or self.state_dict()).items()}
            torch.save({
                "module": sd,
                "lr_scheduler": self.lr_scheduler.state_dict() if self.lr_scheduler is not None and
                hasattr(self.lr_scheduler, "state_dict") else None,
                "global_steps": self.global_steps, "global_samples": self.global_samples,
                "micro_steps": self.micro_steps, "skipped_steps": self.skipped_steps,
                "dp_world_size": self.world_size, "zero_stage": self.stage,
                "client_state": client_state or {}, "ds_config": json.dumps(self.config.raw, default=str),
            }, os.path.join(d, "mp_rank_00_model_states.pt"))
        if self._shard_world > 1 or self.dp_rank == 0:
            torch.save({"optimizer": self.optimizer.shard_state_dict(), "shard_world": self._shard_world,
                        "shard_rank": self._shard_rank, "zero_stage": self.stage},
                       os.path.join(d, f"zero_pp_rank_{self._shard_rank}_mp_rank_00_optim_states.pt"))
        if save_latest and self.global_rank == 0:
            with open(os.path.join(os.fspath(save_dir), "latest"), "w") as f:
                f.write(str(tag))
        return True

    def load_checkpoint(self, load_dir: Union[str, os.PathLike], tag: Optional[str] = None,
                        load_module_strict: bool = True, load_optimizer_states: bool = True,
                        load_lr_scheduler_states: bool = True, load_module_only: bool = False
                        ) -> Tuple[Optional[str], Optional[Dict[str, Any]]]:
        load_dir = os.fspath(load_dir)
        if tag is None:
            latest = os.path.join(load_dir, "latest")
            if not os.path.exists(latest):
                logger.warning("no 'latest' file in %s and no tag given", load_dir)
                return None, None
            tag = open(latest).read().strip()
        d = os.path.join(load_dir, str(tag))
        ms = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
        self.load_state_dict(ms["module"], strict=load_module_strict)
        if load_module_only:
            return d, ms.get("client_state", {})
        if load_optimizer_states:
            files = sorted(f for f in os.listdir(d) if f.startswith("zero_pp_rank_") and f.endswith("_optim_states.pt"))
            if not files:
                raise FileNotFoundError(f"no optimizer shards in {d}")
            mine = f"zero_pp_rank_{self._shard_rank}_mp_rank_00_optim_states.pt"
            shards = []
            for f in files:
                sh = torch.load(os.path.join(d, f), map_location="cpu", weights_only=True, mmap=True)
                if sh.get("shard_world") == self._shard_world and f == mine:
                    shards = [sh["optimizer"]]
                    break
                shards.append(sh["optimizer"])
            self.optimizer.load_shard_states(shards)
            self._refresh_master_if_missing(shards)
        if load_lr_scheduler_states and self.lr_scheduler is not None and ms.get("lr_scheduler") is not None:
            self.lr_scheduler.load_state_dict(ms["lr_scheduler"])
        self.global_steps = int(ms.get("global_steps", 0))
        self.global_samples = int(ms.get("global_samples", 0))
        self.micro_steps = int(ms.get("micro_steps", self.global_steps * self.config.gas))
        self.skipped_steps = int(ms.get("skipped_steps", 0))
        return d, ms.get("client_state", {})

    def _refresh_master_if_missing(self, shards: List[Dict[str, Any]]) -> None:
        if not any("master" in ent for sh in shards for ent in sh["pieces"]):
            self._refresh_master()


def initialize(args: Any = None, model: Optional[nn.Module] = None, optimizer: Any = None,
               model_parameters: Optional[Iterable] = None, training_data: Any = None, lr_scheduler: Any = None,
               mpu: Any = None, dist_init_required: Optional[bool] = None, collate_fn: Any = None,
               config: Union[None, str, Dict[str, Any]] = None, config_params: Optional[Dict[str, Any]] = None
               ) -> Tuple[ZeroEngine, ZeroOptimizer, Any, Any]:
    """``deepspeed.initialize``-compatible entry point: returns (engine, optimizer, loader, sched)."""
    if model is None:
        raise ValueError("initialize() requires a model")
    if config is None:
        config = config_params
    if config is None and args is not None:
        config = getattr(args, "deepspeed_config", None) or getattr(args, "deepspeed", None)
        if isinstance(config, bool):
            config = None
    if config is None:
        raise DeepSpeedConfigError("initialize() requires a DeepSpeed config (config=dict or path)")
    group = mpu.get_data_parallel_group() if mpu is not None and hasattr(mpu, "get_data_parallel_group") else None
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    from determined_amd.parallel.pipeline import PipelineEngine, PipelineModule

    if isinstance(model, PipelineModule):
        world = max(1, world // model.num_stages)  # batch sizes count data-parallel replicas only
    cfg = DeepSpeedConfig(config, world)
    if isinstance(optimizer, dict):
        cfg.optimizer, optimizer = optimizer, None
    opt_obj = optimizer if isinstance(optimizer, torch.optim.Optimizer) else None
    if optimizer is not None and opt_obj is None and callable(optimizer):
        params = list(model_parameters) if model_parameters is not None else list(model.parameters())
        opt_obj = optimizer(params)
    if isinstance(model, PipelineModule):
        pe = PipelineEngine(model, cfg, optimizer=opt_obj, model_parameters=model_parameters,
                            lr_scheduler=lr_scheduler)
        return pe, pe.optimizer, None, pe.lr_scheduler
    engine_cls: Any = ZeroEngine
    if cfg.zero_stage == 3:
        from determined_amd.parallel.zero3 import Zero3Engine

        engine_cls = Zero3Engine
    engine = engine_cls(model, cfg, optimizer=opt_obj, model_parameters=model_parameters, lr_scheduler=lr_scheduler,
                        process_group=group, mpu=mpu)
    loader = None
    if training_data is not None:
        from torch.utils.data import DataLoader, DistributedSampler

        sampler = DistributedSampler(training_data, num_replicas=engine.world_size, rank=engine.dp_rank) \
            if engine.world_size > 1 else None
        loader = DataLoader(training_data, batch_size=cfg.micro_batch, sampler=sampler, collate_fn=collate_fn,
                            drop_last=True)
    return engine, engine.optimizer, loader, engine.lr_scheduler
