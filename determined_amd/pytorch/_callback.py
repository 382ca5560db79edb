"""PyTorchCallback hooks (reference: ``harness/determined/pytorch/_callback.py``)."""

from typing import Any, Dict, List, Optional


class PyTorchCallback:
    def on_trial_startup(self, first_batch_idx: int, checkpoint_uuid: Optional[str]) -> None:
        pass

    def on_trial_shutdown(self) -> None:
        pass

    def on_validation_start(self) -> None:
        pass

    def on_validation_end(self, metrics: Dict[str, Any]) -> None:
        pass

    def on_checkpoint_load_start(self, checkpoint: Dict[str, Any]) -> None:
        pass

    def on_checkpoint_save_start(self, checkpoint: Dict[str, Any]) -> None:
        pass

    def on_checkpoint_end(self, checkpoint_dir: str) -> None:
        pass

    def on_checkpoint_write_end(self, checkpoint_dir: str) -> None:
        pass

    def on_checkpoint_upload_end(self, uuid: str) -> None:
        pass

    def state_dict(self) -> Dict[str, Any]:
        return {}

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        pass

    def on_training_start(self) -> None:
        pass

    def on_training_epoch_start(self, epoch_idx: int) -> None:
        pass

    def on_training_epoch_end(self, epoch_idx: int) -> None:
        pass

    def on_training_workload_end(self, avg_metrics: Dict[str, Any], batch_metrics: List[Dict[str, Any]]) -> None:
        pass

    def on_validation_epoch_start(self) -> None:
        pass

    def on_validation_epoch_end(self, outputs: List[Any]) -> None:
        pass
