"""DistributedContext: ranks and Python-object collectives for the Core API.

Reference: ``harness/determined/core/_distributed.py`` (ZMQ pub/sub between a chief and
workers).  Here object collectives ride on ``torch.distributed`` over a dedicated **gloo**
(CPU/TCP) group, so they never occupy RCCL streams or GPU memory; tensor traffic (gradients)
uses the default RCCL group created by the launcher.
"""

import logging
import os
from typing import Any, List, Optional

logger = logging.getLogger("determined_amd.core")


class DistributedContext:
    def __init__(
        self,
        *,
        rank: int,
        size: int,
        local_rank: int,
        local_size: int,
        cross_rank: int,
        cross_size: int,
        chief_ip: Optional[str] = None,
        _group: Any = None,
        _local_group: Any = None,
        _owns_pg: bool = False,
    ) -> None:
        self.rank = rank
        self.size = size
        self.local_rank = local_rank
        self.local_size = local_size
        self.cross_rank = cross_rank
        self.cross_size = cross_size
        self._chief_ip = chief_ip
        self._group = _group
        self._local_group = _local_group
        self._owns_pg = _owns_pg
        if size > 1 and _group is None:
            self._init_groups()

    # -- construction ------------------------------------------------------------------------
    def _init_groups(self) -> None:
        import torch.distributed as dist

        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", self._chief_ip or "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", os.environ.get("DET_C10D_PORT", "29400"))
            dist.init_process_group("gloo", rank=self.rank, world_size=self.size)
            self._owns_pg = True
        self._group = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
        # node-local groups: every rank must take part in creating every group
        self._local_group = None
        for node in range(self.cross_size):
            ranks = list(range(node * self.local_size, (node + 1) * self.local_size))
            g = dist.new_group(ranks=ranks, backend="gloo")
            if node == self.cross_rank:
                self._local_group = g

    @classmethod
    def from_torch_distributed(cls, chief_ip: Optional[str] = None) -> "DistributedContext":
        """Build from the env that ``torch.distributed.run`` sets (RANK, LOCAL_RANK, ...)."""
        rank = int(os.environ.get("RANK", "0"))
        size = int(os.environ.get("WORLD_SIZE", "1"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        local_size = int(os.environ.get("LOCAL_WORLD_SIZE", str(size)))
        cross_rank = int(os.environ.get("GROUP_RANK", str(rank // max(local_size, 1))))
        cross_size = max(size // max(local_size, 1), 1)
        return cls(rank=rank, size=size, local_rank=local_rank, local_size=local_size, cross_rank=cross_rank,
                   cross_size=cross_size, chief_ip=chief_ip or os.environ.get("DET_CHIEF_IP"))

    @classmethod
    def from_deepspeed(cls, chief_ip: Optional[str] = None) -> "DistributedContext":
        """Build from the deepspeed launcher's env (RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_SIZE,
        CROSS_RANK, CROSS_SIZE; reference ``_distributed.py:from_deepspeed``), falling back to the
        torchrun names where a variable is missing."""
        if "LOCAL_SIZE" not in os.environ and "CROSS_SIZE" not in os.environ:
            return cls.from_torch_distributed(chief_ip)
        size = int(os.environ["WORLD_SIZE"])
        local_size = int(os.environ.get("LOCAL_SIZE", os.environ.get("LOCAL_WORLD_SIZE", str(size))))
        return cls(rank=int(os.environ["RANK"]), size=size, local_rank=int(os.environ["LOCAL_RANK"]),
                   local_size=local_size, cross_rank=int(os.environ.get("CROSS_RANK", "0")),
                   cross_size=int(os.environ.get("CROSS_SIZE", str(max(size // max(local_size, 1), 1)))),
                   chief_ip=chief_ip or os.environ.get("DET_CHIEF_IP"))

    @classmethod
    def from_horovod(cls, hvd: Any = None, chief_ip: Optional[str] = None) -> "DistributedContext":
        raise RuntimeError("Horovod is replaced by the native RCCL launcher; use from_torch_distributed()")

    def close(self) -> None:
        if self._owns_pg:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
            self._owns_pg = False

    # -- accessors (reference API) -------------------------------------------------------------
    def get_rank(self) -> int:
        return self.rank

    def get_local_rank(self) -> int:
        return self.local_rank

    def get_size(self) -> int:
        return self.size

    def get_local_size(self) -> int:
        return self.local_size

    def get_cross_rank(self) -> int:
        return self.cross_rank

    def get_cross_size(self) -> int:
        return self.cross_size

    def get_num_agents(self) -> int:
        return self.cross_size

    # -- collectives -------------------------------------------------------------------------
    def allgather(self, stuff: Any) -> List[Any]:
        if self.size == 1:
            return [stuff]
        import torch.distributed as dist

        out: List[Any] = [None] * self.size
        dist.all_gather_object(out, stuff, group=self._group)
        return out

    def gather(self, stuff: Any) -> Optional[List[Any]]:
        if self.size == 1:
            return [stuff]
        import torch.distributed as dist

        out: Optional[List[Any]] = [None] * self.size if self.rank == 0 else None
        dist.gather_object(stuff, out, dst=self._global(0, self._group), group=self._group)
        return out

    def broadcast(self, stuff: Any) -> Any:
        if self.size == 1:
            return stuff
        import torch.distributed as dist

        buf = [stuff if self.rank == 0 else None]
        dist.broadcast_object_list(buf, src=self._global(0, self._group), group=self._group)
        return buf[0]

    def allgather_local(self, stuff: Any) -> List[Any]:
        if self.local_size == 1:
            return [stuff]
        import torch.distributed as dist

        out: List[Any] = [None] * self.local_size
        dist.all_gather_object(out, stuff, group=self._local_group)
        return out

    def gather_local(self, stuff: Any) -> Optional[List[Any]]:
        if self.local_size == 1:
            return [stuff]
        import torch.distributed as dist

        out = [None] * self.local_size if self.local_rank == 0 else None
        dist.gather_object(stuff, out, dst=self.cross_rank * self.local_size, group=self._local_group)
        return out

    def broadcast_local(self, stuff: Any = None) -> Any:
        if self.local_size == 1:
            return stuff
        import torch.distributed as dist

        buf = [stuff if self.local_rank == 0 else None]
        dist.broadcast_object_list(buf, src=self.cross_rank * self.local_size, group=self._local_group)
        return buf[0]

    @staticmethod
    def _global(group_rank: int, group: Any) -> int:
        import torch.distributed as dist

        try:
            return dist.get_global_rank(group, group_rank)
        except Exception:
            return group_rank


class DummyDistributedContext(DistributedContext):
    def __init__(self) -> None:
        super().__init__(rank=0, size=1, local_rank=0, local_size=1, cross_rank=0, cross_size=1)


def _run_on_rank_0_and_broadcast(fn, dist_ctx: DistributedContext, *args: Any, **kwargs: Any) -> Any:
    out = None
    err = None
    if dist_ctx.rank == 0:
        try:
            out = fn(*args, **kwargs)
        except Exception as e:  # propagate to every rank
            err = e
    out, err = dist_ctx.broadcast((out, err))
    if err is not None:
        raise err
    return out
