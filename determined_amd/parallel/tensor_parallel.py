"""Megatron-style tensor parallelism over RCCL (reference: the model-parallel unit that
DeepSpeedTrial consumes, ``harness/determined/pytorch/deepspeed/_mpu.py``; the layers
themselves come from Megatron in the reference's GPT-NeoX example).

Topology: ``initialize_model_parallel(tp)`` splits the world into tensor-parallel groups of
``tp`` CONSECUTIVE ranks (on an 8-GPU node TP peers are xGMI neighbours; with tp <= 4 the
remaining ranks form the data-parallel groups, strided by ``tp``).  ``get_mpu()`` returns an
object with the DeepSpeed/Megatron mpu method names, so ``zero.initialize(..., mpu=mpu)``
reduces gradients over the data-parallel group only.

Layers (weights sharded along one dimension, activations replicated between blocks):

* ``ColumnParallelLinear``: W split by output rows; input identity forward / all-reduce
  backward; output left sharded (``gather_output=False``) for a following row-parallel layer;
* ``RowParallelLinear``: W split by input columns; partial products all-reduced forward
  (one collective per block half), identity backward; bias added once after the reduce;
* ``VocabParallelEmbedding`` and ``vocab_parallel_cross_entropy``: vocabulary sharded, the
  softmax statistics (max, sum-exp, target logit) combined with three small all-reduces, so
  the full [tokens, vocab] logits never exist on one GPU.

Parameters that are sharded carry ``p.tensor_model_parallel = True``; replicated ones do
not (used to count each gradient exactly once in global-norm clipping).
"""

import math
from typing import Any, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

_TP_GROUP: Optional[dist.ProcessGroup] = None
_DP_GROUP: Optional[dist.ProcessGroup] = None
_TP_SIZE = 1
_TP_RANK = 0
_DP_SIZE = 1
_DP_RANK = 0


def initialize_model_parallel(tensor_model_parallel_size: int = 1) -> None:
    global _TP_GROUP, _DP_GROUP, _TP_SIZE, _TP_RANK, _DP_SIZE, _DP_RANK
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    tp = int(tensor_model_parallel_size)
    if world % tp:
        raise ValueError(f"world size {world} is not divisible by tensor-parallel size {tp}")
    _TP_SIZE, _TP_RANK = tp, rank % tp
    _DP_SIZE, _DP_RANK = world // tp, rank // tp
    if not dist.is_initialized():
        return
    for start in range(0, world, tp):  # every rank must create every group (collective call)
        g = dist.new_group(list(range(start, start + tp)))
        if start <= rank < start + tp:
            _TP_GROUP = g
    for off in range(tp):
        g = dist.new_group(list(range(off, world, tp)))
        if rank % tp == off:
            _DP_GROUP = g


def destroy_model_parallel() -> None:
    global _TP_GROUP, _DP_GROUP, _TP_SIZE, _TP_RANK, _DP_SIZE, _DP_RANK
    _TP_GROUP = _DP_GROUP = None
    _TP_SIZE, _TP_RANK, _DP_SIZE, _DP_RANK = 1, 0, 1, 0


def get_tensor_model_parallel_group() -> Optional[dist.ProcessGroup]:
    return _TP_GROUP


def get_tensor_model_parallel_world_size() -> int:
    return _TP_SIZE


def get_tensor_model_parallel_rank() -> int:
    return _TP_RANK


def get_data_parallel_group() -> Optional[dist.ProcessGroup]:
    return _DP_GROUP


class ModelParallelUnit:
    """mpu object with the names DeepSpeed / Megatron engines call."""

    def get_model_parallel_group(self) -> Optional[dist.ProcessGroup]:
        return _TP_GROUP

    def get_model_parallel_world_size(self) -> int:
        return _TP_SIZE

    def get_model_parallel_rank(self) -> int:
        return _TP_RANK

    get_tensor_model_parallel_group = get_model_parallel_group
    get_tensor_model_parallel_world_size = get_model_parallel_world_size
    get_tensor_model_parallel_rank = get_model_parallel_rank

    def get_data_parallel_group(self) -> Optional[dist.ProcessGroup]:
        return _DP_GROUP

    def get_data_parallel_world_size(self) -> int:
        return _DP_SIZE

    def get_data_parallel_rank(self) -> int:
        return _DP_RANK


def get_mpu() -> ModelParallelUnit:
    return ModelParallelUnit()


# ---------------------------------------------------------------------------------------------
# autograd collectives
# ---------------------------------------------------------------------------------------------
def _all_reduce(x: torch.Tensor) -> torch.Tensor:
    if _TP_SIZE > 1:
        dist.all_reduce(x, group=_TP_GROUP)
    return x


class _CopyToTP(torch.autograd.Function):
    """identity forward, all-reduce backward (input of a column-parallel layer)."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        return _all_reduce(g.contiguous().clone())


class _ReduceFromTP(torch.autograd.Function):
    """all-reduce forward, identity backward (output of a row-parallel layer)."""

    @staticmethod
    def forward(ctx, x):
        return _all_reduce(x.contiguous().clone())

    @staticmethod
    def backward(ctx, g):
        return g


class _GatherFromTP(torch.autograd.Function):
    """all-gather along the last dim forward, take own slice backward."""

    @staticmethod
    def forward(ctx, x):
        if _TP_SIZE == 1:
            return x
        parts = [torch.empty_like(x) for _ in range(_TP_SIZE)]
        dist.all_gather(parts, x.contiguous(), group=_TP_GROUP)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        if _TP_SIZE == 1:
            return g
        n = g.shape[-1] // _TP_SIZE
        return g[..., _TP_RANK * n : (_TP_RANK + 1) * n].contiguous()


copy_to_tensor_model_parallel_region = _CopyToTP.apply
reduce_from_tensor_model_parallel_region = _ReduceFromTP.apply
gather_from_tensor_model_parallel_region = _GatherFromTP.apply


# ---------------------------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------------------------
def _shard(full: torch.Tensor, dim: int) -> torch.Tensor:
    n = full.shape[dim] // _TP_SIZE
    return full.narrow(dim, _TP_RANK * n, n).clone()


class ColumnParallelLinear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, gather_output: bool = False,
                 init_method: Any = None, stride: int = 1) -> None:
        super().__init__()
        if out_features % (_TP_SIZE * stride):
            raise ValueError(f"out_features {out_features} not divisible by tp {_TP_SIZE} x stride {stride}")
        self.in_features, self.out_features = in_features, out_features
        self.gather_output = gather_output
        self.stride = stride
        full = torch.empty(out_features, in_features)
        (init_method or (lambda w: nn.init.kaiming_uniform_(w, a=math.sqrt(5))))(full)
        # with stride s (e.g. fused QKV: s=3) every one of the s blocks is split separately
        self.weight = nn.Parameter(self._split_rows(full))
        self.weight.tensor_model_parallel = True
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_features // _TP_SIZE))
            self.bias.tensor_model_parallel = True
        else:
            self.register_parameter("bias", None)

    def _split_rows(self, full: torch.Tensor) -> torch.Tensor:
        if _TP_SIZE == 1:
            return full
        blocks = full.chunk(self.stride, dim=0)
        return torch.cat([_shard(b, 0) for b in blocks], dim=0)

    def load_full(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> None:
        with torch.no_grad():
            self.weight.copy_(self._split_rows(weight))
            if bias is not None and self.bias is not None:
                self.bias.copy_(self._split_rows(bias[:, None])[:, 0])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = F.linear(copy_to_tensor_model_parallel_region(x), self.weight, self.bias)
        return gather_from_tensor_model_parallel_region(y) if self.gather_output else y


class RowParallelLinear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, input_is_parallel: bool = True,
                 init_method: Any = None) -> None:
        super().__init__()
        if in_features % _TP_SIZE:
            raise ValueError(f"in_features {in_features} not divisible by tp {_TP_SIZE}")
        self.in_features, self.out_features = in_features, out_features
        self.input_is_parallel = input_is_parallel
        full = torch.empty(out_features, in_features)
        (init_method or (lambda w: nn.init.kaiming_uniform_(w, a=math.sqrt(5))))(full)
        self.weight = nn.Parameter(_shard(full, 1) if _TP_SIZE > 1 else full)
        self.weight.tensor_model_parallel = True
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None  # replicated

    def load_full(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> None:
        with torch.no_grad():
            self.weight.copy_(_shard(weight, 1) if _TP_SIZE > 1 else weight)
            if bias is not None and self.bias is not None:
                self.bias.copy_(bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.input_is_parallel and _TP_SIZE > 1:
            n = x.shape[-1] // _TP_SIZE
            x = x[..., _TP_RANK * n : (_TP_RANK + 1) * n]
        y = reduce_from_tensor_model_parallel_region(F.linear(x, self.weight))
        return y + self.bias if self.bias is not None else y


class VocabParallelEmbedding(nn.Module):
    def __init__(self, num_embeddings: int, embedding_dim: int, init_method: Any = None) -> None:
        super().__init__()
        if num_embeddings % _TP_SIZE:
            raise ValueError(f"vocabulary {num_embeddings} not divisible by tp {_TP_SIZE}")
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.per_rank = num_embeddings // _TP_SIZE
        self.start = _TP_RANK * self.per_rank
        full = torch.empty(num_embeddings, embedding_dim)
        (init_method or nn.init.normal_)(full)
        self.weight = nn.Parameter(_shard(full, 0) if _TP_SIZE > 1 else full)
        self.weight.tensor_model_parallel = True

    def load_full(self, weight: torch.Tensor) -> None:
        with torch.no_grad():
            self.weight.copy_(_shard(weight, 0) if _TP_SIZE > 1 else weight)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if _TP_SIZE == 1:
            return F.embedding(ids, self.weight)
        local = ids - self.start
        outside = (local < 0) | (local >= self.per_rank)
        out = F.embedding(local.masked_fill(outside, 0), self.weight)
        out = out.masked_fill(outside.unsqueeze(-1), 0.0)
        return reduce_from_tensor_model_parallel_region(out)


class _VocabParallelCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, vocab_start, ignore_index, vocab_size):
        lg = logits.float()
        if vocab_size is not None and vocab_start + lg.shape[-1] > vocab_size:  # padded columns
            lg = lg.clone()
            lg[..., max(0, vocab_size - vocab_start):] = float("-inf")
        mx = lg.max(dim=-1).values
        if _TP_SIZE > 1:
            dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=_TP_GROUP)
        lg = lg - mx.unsqueeze(-1)
        V = lg.shape[-1]
        local = target - vocab_start
        outside = (local < 0) | (local >= V) | (target == ignore_index)
        idx = local.masked_fill(outside, 0)
        tgt_logit = lg.gather(-1, idx.unsqueeze(-1)).squeeze(-1).masked_fill(outside, 0.0)
        ex = lg.exp()
        se = ex.sum(-1)
        if _TP_SIZE > 1:
            dist.all_reduce(tgt_logit, group=_TP_GROUP)
            dist.all_reduce(se, group=_TP_GROUP)
        loss = se.log() - tgt_logit
        valid = target != ignore_index
        loss = loss.masked_fill(~valid, 0.0)
        sm = ex / se.unsqueeze(-1)
        ctx.save_for_backward(sm, idx, (~outside), valid)
        return loss

    @staticmethod
    def backward(ctx, g):
        sm, idx, inside, valid = ctx.saved_tensors
        grad = sm
        rows = inside.nonzero(as_tuple=True)
        grad[rows + (idx[rows],)] -= 1.0
        grad = grad * (g * valid).unsqueeze(-1)
        return grad, None, None, None, None


def vocab_parallel_cross_entropy(logits: torch.Tensor, target: torch.Tensor, vocab_start: int = 0,
                                 ignore_index: int = -100, vocab_size: Optional[int] = None) -> torch.Tensor:
    """Per-token loss for vocabulary-sharded logits ``[..., V/tp]`` (rank r holds columns
    ``[r*V/tp, (r+1)*V/tp)``); global columns >= ``vocab_size`` (padding) are excluded."""
    return _VocabParallelCE.apply(logits, target, vocab_start, ignore_index, vocab_size)
