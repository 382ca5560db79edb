"""Helpers shared by model-hub trials (reference: ``model_hub/model_hub/utils.py``)."""

import os
from typing import Any, Dict, List, Union

import numpy as np
import torch


def expand_like(arrays: List[np.ndarray], fill: float = -100) -> np.ndarray:
    """Concatenate along dim 0, padding dim 1 to the longest array with ``fill``."""
    if arrays[0].ndim == 1:
        return np.concatenate(arrays)
    rows = sum(a.shape[0] for a in arrays)
    width = max(a.shape[1] for a in arrays)
    out = np.full((rows, width, *arrays[0].shape[2:]), fill, dtype=np.result_type(*arrays, np.asarray(fill)))
    r = 0
    for a in arrays:
        out[r : r + a.shape[0], : a.shape[1]] = a
        r += a.shape[0]
    return out


def numpify(x: Union[List, np.ndarray, torch.Tensor]) -> np.ndarray:
    if isinstance(x, np.ndarray):
        return x
    if isinstance(x, list):
        return np.array(x)
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    raise TypeError("Expected input of type List, np.ndarray, or torch.Tensor.")


def download_url(download_directory: str, url: str) -> str:
    """Return the cached copy of ``url`` in ``download_directory``; fetching is unavailable offline."""
    name = url.rstrip("/").rsplit("/", 1)[-1]
    path = os.path.join(download_directory, name)
    if os.path.exists(path):
        return path
    raise RuntimeError(f"{url} is not cached at {path} and this environment has no network access")


def compute_num_training_steps(experiment_config: Dict[str, Any], global_batch_size: int) -> int:
    (unit, length), = experiment_config["searcher"]["max_length"].items()
    if unit == "batches":
        return int(length)
    if unit == "epochs":
        if "records_per_epoch" not in experiment_config:
            raise ValueError("set hyperparameter num_training_steps (or records_per_epoch) to size the LR schedule")
        return int(length) * int(experiment_config["records_per_epoch"] / global_batch_size)
    return int(length / global_batch_size)


class AttrDict(dict):
    """dict with attribute access, converting nested dicts recursively."""

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            if isinstance(v, dict) and not isinstance(v, AttrDict):
                self[k] = AttrDict(v)

    def __getattr__(self, item: str) -> Any:
        try:
            return self[item]
        except KeyError as e:
            raise AttributeError(item) from e

    def __setattr__(self, item: str, value: Any) -> None:
        self[item] = value
