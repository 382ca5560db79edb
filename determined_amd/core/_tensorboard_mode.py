"""How a trial's TensorBoard artifacts are produced (reference ``core/_tensorboard_mode.py``).

AUTO   -- the chief writes every reported training / validation metric as TensorBoard scalars into
          ``TrainContext.get_tensorboard_path()`` and uploads its TensorBoard directory to checkpoint
          (or tensorboard) storage when the context closes; other ranks' files are not uploaded.
MANUAL -- nothing is written or uploaded automatically: the user writes what they want under the
          TensorBoard path and calls ``TrainContext.upload_tensorboard_files()``.
"""

import enum
from typing import Any


class TensorboardMode(enum.Enum):
    AUTO = "AUTO"
    MANUAL = "MANUAL"

    @classmethod
    def parse(cls, v: Any) -> "TensorboardMode":
        if v is None:
            return cls.AUTO
        if isinstance(v, cls):
            return v
        try:
            return cls(str(v).upper())
        except ValueError:
            raise ValueError(f"tensorboard_mode must be AUTO or MANUAL, got {v!r}") from None
