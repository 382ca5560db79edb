"""Load a trained PyTorchTrial back from a checkpoint directory
(reference: ``harness/determined/pytorch/_load.py``)."""

import importlib
import json
import pathlib
import sys
from typing import Any, Dict, Optional

import torch

from determined_amd import core
from determined_amd.pytorch._context import PyTorchTrialContext


class CheckpointLoadContext(PyTorchTrialContext):
    """A PyTorchTrialContext that only builds models (no training, no master)."""

    def __init__(self, hparams: Dict[str, Any], exp_conf: Optional[Dict[str, Any]], device: torch.device) -> None:
        core_ctx = core._dummy_init()
        super().__init__(core_context=core_ctx, trial_seed=0, hparams=hparams, slots_per_trial=1,
                         num_gpus=1 if device.type == "cuda" else 0, exp_conf=exp_conf, aggregation_frequency=1,
                         steps_completed=0, managed_training=False, debug_enabled=False)
        self.device = device

    def wrap_model(self, model: torch.nn.Module) -> torch.nn.Module:
        model = model.to(self.device)
        self.models.append(model)
        return model


def _import_trial_class(spec: str, code_dir: pathlib.Path) -> Any:
    module, _, qual = spec.partition(":")
    if code_dir.exists() and str(code_dir) not in sys.path:
        sys.path.insert(0, str(code_dir))
    mod = importlib.import_module(module)
    obj = mod
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


def load_trial_from_checkpoint_path(path: str, trial_class: Optional[type] = None,
                                    trial_kwargs: Optional[Dict[str, Any]] = None,
                                    torch_load_kwargs: Optional[Dict[str, Any]] = None,
                                    map_location: Any = None) -> Any:
    """Rebuild the trial (models with weights loaded) from a checkpoint directory."""
    p = pathlib.Path(path)
    load_data = json.loads((p / "load_data.json").read_text())
    cls = trial_class or _import_trial_class(load_data["trial_cls_spec"], p / "code")
    device = torch.device("cuda" if torch.cuda.is_available() and map_location != "cpu" else "cpu")
    ctx = CheckpointLoadContext(load_data.get("hparams") or {}, load_data.get("experiment_config"), device)
    trial = cls(ctx, **(trial_kwargs or {}))
    kw = {"map_location": map_location or device, "weights_only": True}
    kw.update(torch_load_kwargs or {})
    ckpt = torch.load(str(p / "state_dict.pth"), **kw)
    for model, sd in zip(ctx.models, ckpt["models_state_dict"]):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
        model.load_state_dict(sd)
    return trial
