"""core.Context and core.init() (reference: ``harness/determined/core/_context.py``)."""

import logging
import os
import pathlib
import signal
import sys
import threading
import traceback
import types
from typing import Any, Dict, Optional, Union

from determined_amd import storage
from determined_amd._info import get_cluster_info
from determined_amd.core._checkpoint import CheckpointContext, DummyCheckpointContext
from determined_amd.core._distributed import DistributedContext, DummyDistributedContext
from determined_amd.core._experimental import DummyExperimentalCoreContext, ExperimentalCoreContext
from determined_amd.core._preempt import DummyPreemptContext, PreemptContext, PreemptMode
from determined_amd.core._profiler import DummyProfilerContext, ProfilerContext
from determined_amd.core._searcher import DummySearcherContext, SearcherContext, _parse_searcher_units
from determined_amd.core._train import DummyTrainContext, EarlyExitReason, TrainContext

logger = logging.getLogger("determined_amd.core")


class InvalidHP(Exception):
    """Raise from trial code to report that a hyperparameter configuration is invalid."""


class Context:
    def __init__(self, checkpoint: CheckpointContext, distributed: Optional[DistributedContext] = None,
                 preempt: Optional[PreemptContext] = None, train: Optional[TrainContext] = None,
                 searcher: Optional[SearcherContext] = None, info: Any = None,
                 profiler: Optional[ProfilerContext] = None, _log_shipper: Any = None,
                 _tensorboard_manager: Any = None, experimental: Optional[ExperimentalCoreContext] = None,
                 _heartbeat: Any = None) -> None:
        self.checkpoint = checkpoint
        self.distributed = distributed or DummyDistributedContext()
        self.preempt = preempt or DummyPreemptContext(self.distributed)
        self.train = train or DummyTrainContext()
        self.searcher = searcher or DummySearcherContext(self.distributed)
        self.info = info
        self.profiler = profiler or DummyProfilerContext()
        self.experimental = experimental or DummyExperimentalCoreContext()
        self._log_shipper = _log_shipper
        self._tensorboard_manager = _tensorboard_manager
        self._heartbeat = _heartbeat

    def start(self) -> None:
        self.preempt.start()
        if self._log_shipper is not None:
            self._log_shipper.start()
        if self._heartbeat is not None:
            self._heartbeat.start()

    def __enter__(self) -> "Context":
        self.start()
        return self

    def close(self, exc_type=None, exc_val=None, exc_tb=None) -> None:
        if self._heartbeat is not None:
            self._heartbeat.close(exc_type, exc_val, exc_tb)
        self.preempt.close()
        self.profiler._close()
        self.distributed.close()
        if self._tensorboard_manager is not None:
            self._tensorboard_manager.close()
        if self._log_shipper is not None:
            self._log_shipper.close()

    def __exit__(self, exc_type: Optional[type], exc_val: Optional[BaseException],
                 exc_tb: Optional[types.TracebackType]) -> None:
        self.close(exc_type, exc_val, exc_tb)
        if isinstance(exc_val, InvalidHP):
            self.train.report_early_exit(EarlyExitReason.INVALID_HP)
            logger.info("InvalidHP detected, converting to exit(0)")
            sys.exit(0)


def _install_stacktrace_on_sigusr1() -> None:
    if not hasattr(signal, "SIGUSR1") or threading.current_thread() is not threading.main_thread():
        return
    old = None

    def handler(signum: int, frame: Any) -> None:
        traceback.print_stack(frame, file=sys.stderr)
        if callable(old):
            old(signum, frame)

    old = signal.signal(signal.SIGUSR1, handler)


def _get_storage_manager(checkpoint_storage: Optional[Union[str, Dict[str, Any]]]) -> Optional[storage.StorageManager]:
    if checkpoint_storage is None:
        return None
    if isinstance(checkpoint_storage, str):
        return storage.from_string(checkpoint_storage)
    return storage.build(checkpoint_storage)


def _default_local_storage() -> storage.StorageManager:
    base = os.environ.get("DET_LOCAL_CHECKPOINT_DIR", os.path.expanduser("~/.local/share/determined_amd"))
    logger.info(f"no checkpoint storage provided; storing checkpoints in {base}")
    return storage.SharedFSStorageManager(base)


def _dummy_init(*, distributed: Optional[DistributedContext] = None,
                checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None,
                tensorboard_path: Optional[pathlib.Path] = None,
                preempt_mode: PreemptMode = PreemptMode.WorkersAskChief,
                searcher_length: int = 1) -> Context:
    distributed = distributed or DummyDistributedContext()
    sm = _get_storage_manager(checkpoint_storage) or _default_local_storage()
    _install_stacktrace_on_sigusr1()
    return Context(
        distributed=distributed,
        checkpoint=DummyCheckpointContext(distributed, sm),
        preempt=DummyPreemptContext(distributed, preempt_mode),
        train=DummyTrainContext(tensorboard_path),
        searcher=DummySearcherContext(distributed, searcher_length),
        profiler=DummyProfilerContext(),
    )


def init(*, distributed: Optional[DistributedContext] = None,
         checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None,
         preempt_mode: PreemptMode = PreemptMode.WorkersAskChief,
         tensorboard_mode: Any = None, _info: Any = None, _unmanaged: bool = False,
         _heartbeat_interval: float = 60.0) -> Context:
    """Build a core.Context; on-cluster it talks to the master, off-cluster it runs locally.

    ``_info``/``_unmanaged`` are used by ``experimental.core_v2`` for unmanaged trials: the
    process runs outside the cluster but reports metrics and checkpoints to the master (and, on the
    chief, its RUNNING / COMPLETED / ERROR state plus periodic heartbeats: ``core/_heartbeat.py``).

    ``tensorboard_mode`` (``TensorboardMode`` or "AUTO" / "MANUAL", default AUTO): in AUTO the chief
    writes reported metrics as TensorBoard scalars and uploads its TensorBoard directory when the
    context closes; in MANUAL nothing is written or uploaded automatically."""
    from determined_amd.core._tensorboard_mode import TensorboardMode

    tb_mode = TensorboardMode.parse(tensorboard_mode)
    info = _info if _info is not None else get_cluster_info()
    if info is None:
        return _dummy_init(distributed=distributed, checkpoint_storage=checkpoint_storage,
                           preempt_mode=preempt_mode)
    from determined_amd.common.api import Session
    from determined_amd.core._log_shipper import maybe_log_shipper

    session = Session(info.master_url, token=info.session_token)
    if distributed is None and (len(info.container_addrs) > 1 or len(info.slot_ids) > 1) and \
            int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise ValueError("you must provide a valid DistributedContext for a multi-slot task")
    distributed = distributed or DummyDistributedContext()
    sm = _get_storage_manager(checkpoint_storage)
    if info.task_type == "TRIAL":
        cfg = info.trial._config
        if sm is None:
            sm = storage.build(cfg["checkpoint_storage"])
        tb = None
        tbd_writer = None
        try:
            from determined_amd.tensorboard import build_manager

            auto_chief = tb_mode == TensorboardMode.AUTO and distributed.rank == 0
            tb, tbd_writer = build_manager(cfg, info, distributed, sync_on_close=auto_chief, write_metrics=auto_chief)
        except Exception as e:  # tensorboard is best effort
            logger.debug(f"tensorboard disabled: {e}")
        train = TrainContext(session, info.trial.trial_id, info.trial._trial_run_id, info.trial.experiment_id,
                             distributed, tb, tbd_writer)
        if _unmanaged:
            checkpoint = CheckpointContext(distributed, sm, session, info.task_id, info.allocation_id,
                                           info.trial.trial_id, tb)
            _install_stacktrace_on_sigusr1()
            from determined_amd.core._heartbeat import UnmanagedTrialHeartbeat

            hb = UnmanagedTrialHeartbeat(session, info.trial.trial_id, _heartbeat_interval) \
                if distributed.rank == 0 else None
            return Context(checkpoint=checkpoint, distributed=distributed,
                           preempt=DummyPreemptContext(distributed, preempt_mode), train=train,
                           searcher=DummySearcherContext(distributed, 10**9), info=info, _tensorboard_manager=tb,
                           experimental=ExperimentalCoreContext(session, info.trial.trial_id), _heartbeat=hb)
        searcher = SearcherContext(session, distributed, info.trial.trial_id, info.trial._trial_run_id,
                                   info.allocation_id, _parse_searcher_units(cfg))
        checkpoint = CheckpointContext(distributed, sm, session, info.task_id, info.allocation_id,
                                       info.trial.trial_id, tb)
        preempt = PreemptContext(session, info.allocation_id, distributed, preempt_mode)
        profiler = ProfilerContext(session, info.agent_id, info.trial.trial_id, info.trial._trial_run_id,
                                   distributed)
        _install_stacktrace_on_sigusr1()
        return Context(checkpoint=checkpoint, distributed=distributed, preempt=preempt, train=train,
                       searcher=searcher, info=info, profiler=profiler,
                       _log_shipper=maybe_log_shipper(session, info, distributed), _tensorboard_manager=tb,
                       experimental=ExperimentalCoreContext(session, info.trial.trial_id))
    sm = sm or _default_local_storage()
    _install_stacktrace_on_sigusr1()
    return Context(checkpoint=DummyCheckpointContext(distributed, sm), distributed=distributed,
                   preempt=PreemptContext(session, info.allocation_id, distributed, preempt_mode), info=info)
