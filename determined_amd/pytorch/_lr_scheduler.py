"""LRScheduler wrapper (reference: ``harness/determined/pytorch/_lr_scheduler.py``)."""

import enum
from typing import Any, Dict, List


class LRScheduler:
    class StepMode(enum.Enum):
        STEP_EVERY_EPOCH = 1
        STEP_EVERY_BATCH = 2
        MANUAL_STEP = 3
        STEP_EVERY_OPTIMIZER_STEP = 4

    def __init__(self, scheduler: Any, step_mode: "LRScheduler.StepMode", frequency: int = 1) -> None:
        if not isinstance(step_mode, LRScheduler.StepMode):
            raise TypeError("step_mode must be an LRScheduler.StepMode")
        if frequency < 1:
            raise ValueError("frequency must be >= 1")
        self._scheduler = scheduler
        self._step_mode = step_mode
        self._frequency = frequency

    def step(self, *args: Any, **kwargs: Any) -> None:
        self._scheduler.step(*args, **kwargs)

    def get_last_lr(self) -> List[float]:
        return self._scheduler.get_last_lr()

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self._scheduler.load_state_dict(state_dict)

    def state_dict(self) -> Dict[str, Any]:
        return self._scheduler.state_dict()

    def __getattr__(self, name: str) -> Any:
        return getattr(self._scheduler, name)
