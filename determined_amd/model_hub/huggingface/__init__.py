"""PyTorchTrial building blocks for HuggingFace models (reference:
``model_hub/model_hub/huggingface``): hparam -> kwargs parsing, Auto-class model building,
default optimizer / LR schedule, dataset loading, and ``BaseTransformerTrial``.

MI355X-native differences: the default optimizer is the fused single-launch AdamW (with bf16
master weights when the model is bf16) and gradient clipping is fused into its step instead
of a separate ``clip_grad_norm_`` pass; models can be built from a config alone
(``use_pretrained_weights: false``) since nothing can be downloaded here.
"""

import dataclasses
import logging
from typing import Any, Dict, List, Optional, Tuple, Union

import torch

from determined_amd import pytorch as det_torch
from determined_amd.model_hub.utils import AttrDict, compute_num_training_steps

logger = logging.getLogger("determined_amd.model_hub.huggingface")


# ---------------------------------------------------------------------------------------------
# kwargs parsing
# ---------------------------------------------------------------------------------------------
class _Partial:
    """Dataclass mix-in: fields without defaults are only set when provided."""

    def __init__(self, **kwargs: Any) -> None:
        names = {f.name for f in dataclasses.fields(self)}  # type: ignore[arg-type]
        for k, v in kwargs.items():
            if k in names:
                object.__setattr__(self, k, v)
        for f in dataclasses.fields(self):  # type: ignore[arg-type]
            if not hasattr(self, f.name) and f.default is not dataclasses.MISSING:
                object.__setattr__(self, f.name, f.default)

    def as_dict(self) -> Dict[str, Any]:
        return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)  # type: ignore[arg-type]
                if hasattr(self, f.name)}

    def __repr__(self) -> str:
        return f"{type(self).__qualname__}({', '.join(f'{k}={v!r}' for k, v in self.as_dict().items())})"


@dataclasses.dataclass(init=False, repr=False)
class DatasetKwargs(_Partial):
    dataset_name: Optional[str] = None
    dataset_config_name: Optional[str] = None
    validation_split_percentage: Optional[float] = None
    train_file: Optional[str] = None
    validation_file: Optional[str] = None


@dataclasses.dataclass(init=False, repr=False)
class ConfigKwargs(_Partial):
    num_labels: Optional[int] = dataclasses.field()
    finetuning_task: Optional[str] = dataclasses.field()
    pretrained_model_name_or_path: Optional[str] = None
    cache_dir: Optional[str] = None
    revision: Optional[str] = "main"
    use_auth_token: Optional[bool] = False


@dataclasses.dataclass(init=False, repr=False)
class TokenizerKwargs(_Partial):
    do_lower_case: Optional[bool] = dataclasses.field()
    pretrained_model_name_or_path: Optional[str] = None
    cache_dir: Optional[str] = None
    revision: Optional[str] = "main"
    use_auth_token: Optional[bool] = False
    use_fast: Optional[bool] = True


@dataclasses.dataclass(init=False, repr=False)
class ModelKwargs(_Partial):
    pretrained_model_name_or_path: str = dataclasses.field()
    cache_dir: Optional[str] = None
    revision: Optional[str] = "main"
    use_auth_token: Optional[bool] = False


@dataclasses.dataclass
class OptimizerKwargs:
    weight_decay: Optional[float] = 0
    adafactor: Optional[bool] = False
    learning_rate: Optional[float] = 5e-5
    max_grad_norm: Optional[float] = 1.0
    adam_beta1: Optional[float] = 0.9
    adam_beta2: Optional[float] = 0.999
    adam_epsilon: Optional[float] = 1e-8
    scale_parameter: Optional[bool] = False
    relative_step: Optional[bool] = False


@dataclasses.dataclass
class LRSchedulerKwargs:
    num_training_steps: int
    lr_scheduler_type: Optional[str] = "linear"
    num_warmup_steps: Optional[int] = 0


def parse_dict_to_dataclasses(dataclass_types: Tuple[Any, ...], args: Dict[str, Any],
                              as_dict: bool = False) -> Tuple[Any, ...]:
    """Fill each dataclass from the keys of ``args`` it declares (one key may feed several)."""
    out = []
    for dt in dataclass_types:
        keys = {f.name for f in dataclasses.fields(dt) if f.init}
        obj = dt(**{k: v for k, v in args.items() if k in keys})
        if as_dict:
            obj = AttrDict(obj.as_dict() if hasattr(obj, "as_dict") else dataclasses.asdict(obj))
        out.append(obj)
    return tuple(out)


def default_parse_config_tokenizer_model_kwargs(hparams: Dict[str, Any]) -> Tuple[AttrDict, AttrDict, AttrDict]:
    hp = hparams if isinstance(hparams, AttrDict) else AttrDict(hparams)
    cfg, tok, model = parse_dict_to_dataclasses((ConfigKwargs, TokenizerKwargs, ModelKwargs), hp, as_dict=True)
    for key, target in (("config_name", cfg), ("tokenizer_name", tok), ("model_name", model)):
        if key in hp:
            target["pretrained_model_name_or_path"] = hp[key]
    for t in (cfg, tok):  # config / tokenizer default to the model's name or path
        if t.get("pretrained_model_name_or_path") is None:
            t["pretrained_model_name_or_path"] = model.get("pretrained_model_name_or_path")
    if "model_type" in hp:  # offline: build the config from its type + overrides
        cfg["model_type"] = hp["model_type"]
        cfg.update(hp.get("config_overrides", {}) or {})
    if any(t.get("pretrained_model_name_or_path") is None for t in (cfg, tok, model)):
        raise ValueError("set model_name (and optionally config_name / tokenizer_name) in hyperparameters")
    return cfg, tok, model


def default_parse_optimizer_lr_scheduler_kwargs(hparams: Dict[str, Any]) -> Tuple[OptimizerKwargs,
                                                                                  LRSchedulerKwargs]:
    return parse_dict_to_dataclasses((OptimizerKwargs, LRSchedulerKwargs), hparams)  # type: ignore[return-value]


# ---------------------------------------------------------------------------------------------
# builders
# ---------------------------------------------------------------------------------------------
def _model_modes() -> Dict[str, Any]:
    import transformers as tf

    return {"base": tf.AutoModel, "pretraining": tf.AutoModelForPreTraining, "causal-lm": tf.AutoModelForCausalLM,
            "masked-lm": tf.AutoModelForMaskedLM, "seq2seq-lm": tf.AutoModelForSeq2SeqLM,
            "sequence-classification": tf.AutoModelForSequenceClassification,
            "multiple-choice": tf.AutoModelForMultipleChoice,
            "next-sentence": tf.AutoModelForNextSentencePrediction,
            "token-classification": tf.AutoModelForTokenClassification,
            "question-answering": tf.AutoModelForQuestionAnswering}


def build_using_auto(config_kwargs: Dict[str, Any], tokenizer_kwargs: Dict[str, Any], model_mode: str,
                     model_kwargs: Union[Dict[str, Any], ModelKwargs], use_pretrained_weights: bool = True
                     ) -> Tuple[Any, Any, Any]:
    """Config, tokenizer and model via the Auto classes.  ``config_kwargs`` may instead carry
    ``model_type`` (+ config overrides) to build a randomly initialised model offline; the
    tokenizer is ``None`` when it cannot be loaded locally."""
    import transformers as tf

    ck = dict(config_kwargs)
    if "model_type" in ck:
        mt = ck.pop("model_type")
        for k in ("pretrained_model_name_or_path", "cache_dir", "revision", "use_auth_token"):
            ck.pop(k, None)
        config = tf.AutoConfig.for_model(mt, **ck)
    else:
        ck.pop("use_auth_token", None)
        config = tf.AutoConfig.from_pretrained(**ck)
    tokenizer = None
    try:
        tk = {k: v for k, v in dict(tokenizer_kwargs).items() if k != "use_auth_token"}
        tokenizer = tf.AutoTokenizer.from_pretrained(**tk)
    except Exception as e:  # offline without a local tokenizer
        logger.warning("tokenizer unavailable (%s); continuing without one", type(e).__name__)
    builder = _model_modes()[model_mode]
    mk = dataclasses.asdict(model_kwargs) if isinstance(model_kwargs, ModelKwargs) else dict(model_kwargs)
    mk.pop("use_auth_token", None)
    if use_pretrained_weights:
        model = builder.from_pretrained(config=config, **mk)
    else:
        model = builder.from_config(config)
    return config, tokenizer, model


def group_parameters_for_optimizer(model: torch.nn.Module, weight_decay: Optional[float] = 0,
                                   no_decay: Tuple[str, ...] = ("bias", "LayerNorm.weight")) -> List[Dict[str, Any]]:
    decay, nodecay = [], []
    for n, p in model.named_parameters():
        (nodecay if any(nd in n for nd in no_decay) else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": nodecay, "weight_decay": 0.0}]


def build_default_optimizer(model: torch.nn.Module, optimizer_kwargs: OptimizerKwargs) -> torch.optim.Optimizer:
    groups = group_parameters_for_optimizer(model, optimizer_kwargs.weight_decay)
    if optimizer_kwargs.adafactor:
        from transformers.optimization import Adafactor

        return Adafactor(groups, lr=optimizer_kwargs.learning_rate, scale_parameter=optimizer_kwargs.scale_parameter,
                         relative_step=optimizer_kwargs.relative_step)
    from determined_amd.ops import FusedAdamW

    opt = FusedAdamW(groups, lr=optimizer_kwargs.learning_rate,
                     betas=(optimizer_kwargs.adam_beta1, optimizer_kwargs.adam_beta2), eps=optimizer_kwargs.adam_epsilon,
                     master_weights=any(p.dtype == torch.bfloat16 for p in model.parameters()))
    if optimizer_kwargs.max_grad_norm and optimizer_kwargs.max_grad_norm > 0:
        opt.set_grad_clipping(optimizer_kwargs.max_grad_norm)  # fused into step()
    return opt


def build_default_lr_scheduler(optimizer: torch.optim.Optimizer, scheduler_kwargs: LRSchedulerKwargs) -> Any:
    from transformers.optimization import get_scheduler

    return get_scheduler(scheduler_kwargs.lr_scheduler_type, optimizer, num_warmup_steps=scheduler_kwargs.num_warmup_steps,
                         num_training_steps=scheduler_kwargs.num_training_steps)


def default_load_dataset(data_config_input: Dict[str, Any]) -> Any:
    """``datasets.load_dataset`` by name (local cache only, no network) or from train/validation files."""
    import datasets as hf_datasets

    (dc,) = parse_dict_to_dataclasses((DatasetKwargs,), data_config_input)
    if dc.dataset_name is not None:
        ds = hf_datasets.load_dataset(dc.dataset_name, dc.dataset_config_name)
        if "validation" not in ds:
            if dc.validation_split_percentage is None:
                raise ValueError("dataset has no validation split; set validation_split_percentage")
            p = dc.validation_split_percentage
            ds["validation"] = hf_datasets.load_dataset(dc.dataset_name, dc.dataset_config_name, split=f"train[:{p}%]")
            ds["train"] = hf_datasets.load_dataset(dc.dataset_name, dc.dataset_config_name, split=f"train[{p}%:]")
        return ds
    files = {k: v for k, v in (("train", dc.train_file), ("validation", dc.validation_file)) if v is not None}
    if not files:
        raise ValueError("provide dataset_name or train_file/validation_file")
    ext = next(iter(files.values())).rsplit(".", 1)[-1]
    return hf_datasets.load_dataset("text" if ext == "txt" else ext, data_files=files)


def remove_unused_columns(model: torch.nn.Module, dataset: Any) -> None:
    """Drop dataset columns the model's ``forward`` does not accept (in place)."""
    import inspect

    accepted = set(inspect.signature(model.forward).parameters) | {"label", "label_ids"}
    drop = [c for c in dataset.column_names if c not in accepted]
    if drop:
        dataset.set_format(type=dataset.format["type"], columns=[c for c in dataset.column_names if c not in drop])


class BaseTransformerTrial(det_torch.PyTorchTrial):
    """PyTorchTrial over an HF Auto model: builds config/tokenizer/model from hparams, wraps the
    fused AdamW + HF LR schedule, and trains on ``model(**batch).loss``.  Subclasses provide the
    data loaders and ``evaluate_batch``."""

    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        if not hasattr(self, "hparams"):
            self.hparams = AttrDict(context.get_hparams())
        if not hasattr(self, "data_config"):
            self.data_config = AttrDict(context.get_data_config())
        if not hasattr(self, "exp_config"):
            self.exp_config = AttrDict(context.get_experiment_config())
        self.check_hparams()
        self.config_kwargs, self.tokenizer_kwargs, self.model_kwargs = \
            default_parse_config_tokenizer_model_kwargs(self.hparams)
        opt_kwargs, sched_kwargs = default_parse_optimizer_lr_scheduler_kwargs(self.hparams)
        self.config, self.tokenizer, model = build_using_auto(
            self.config_kwargs, self.tokenizer_kwargs, self.hparams.model_mode, self.model_kwargs,
            use_pretrained_weights=self.hparams.use_pretrained_weights)
        if self.hparams.get("bf16", False):
            model = model.to(torch.bfloat16)
        self.model = self.context.wrap_model(model.to(context.device))
        self.optimizer = self.context.wrap_optimizer(build_default_optimizer(model, opt_kwargs))
        self.lr_scheduler = self.context.wrap_lr_scheduler(build_default_lr_scheduler(self.optimizer, sched_kwargs),
                                                           det_torch.LRScheduler.StepMode.STEP_EVERY_BATCH)

    def check_hparams(self) -> None:
        if not isinstance(self.hparams, AttrDict):
            self.hparams = AttrDict(self.hparams)
        if "num_training_steps" not in self.hparams:
            self.hparams.num_training_steps = compute_num_training_steps(self.context.get_experiment_config(),
                                                                         self.context.get_global_batch_size())
        if "use_pretrained_weights" not in self.hparams:
            logger.warning("using pretrained weights by default; set use_pretrained_weights: false to train "
                           "from scratch")
            self.hparams.use_pretrained_weights = True
        self.hparams.setdefault("use_apex_amp", False)
        if self.hparams.use_apex_amp:
            raise ValueError("apex AMP does not exist on ROCm; set bf16: true instead")
        for hp in ("model_mode", "num_training_steps"):
            if hp not in self.hparams:
                raise ValueError(f"{hp} is a required hyperparameter for BaseTransformerTrial")

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Any:
        out = self.model(**batch)
        loss = out["loss"] if isinstance(out, dict) else out[0]
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer)
        return loss
