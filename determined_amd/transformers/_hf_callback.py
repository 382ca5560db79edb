"""HuggingFace ``transformers.Trainer`` integration (reference:
``harness/determined/transformers/_hf_callback.py``).

``DetCallback`` connects an HF Trainer run to the Core API:

* ``on_log``: metrics whose keys start with ``eval_`` are reported as validation metrics,
  step-progress logs (``loss``, ``learning_rate``, ``grad_norm``...) as training metrics; the
  same step is never reported twice (HF re-logs the last step after training/evaluation);
* ``on_save``: the freshly written ``checkpoint-{step}/`` (plus ``runs/`` tensorboard files)
  is uploaded as a sharded Determined checkpoint (every rank contributes; ranks sharing a
  directory upload each file once) with ``steps_completed`` metadata;
* searcher: progress is reported per step (``max_length.batches``) or per epoch
  (``max_length.epochs``); when an operation's length is reached the callback makes the
  Trainer log + evaluate + save, reports the searcher metric (falling back to
  ``state.best_metric``) and moves to the next operation or stops training;
* preemption (pause/kill from the master) forces a save, then exits after the upload;
* ``load_last_checkpoint``: on a restarted trial the latest checkpoint is downloaded into
  ``output_dir`` and ``args.resume_from_checkpoint`` points at it.

Off-cluster (no ``DET_*`` environment) the callback runs one local searcher operation sized
from ``TrainingArguments`` so the same script works under ``core.init()`` on a laptop.
"""

import json
import logging
import os
from typing import Any, Dict, Iterator, List, Optional, Tuple

import transformers
from transformers import trainer_utils

from determined_amd._info import get_cluster_info
from determined_amd.core._searcher import DummySearcherOperation

logger = logging.getLogger("determined_amd.transformers")

EVAL = "eval_"
TEST = "test_"
TRAIN_AVG = "train_"
TRAIN = "train_progress"


def get_metric_type(d: Dict[str, Any]) -> str:
    """Classify an HF log dict by its first key's prefix."""
    for k in d:
        if k.startswith(EVAL):
            return EVAL
        if k.startswith(TEST):
            return TEST
        if k.startswith(TRAIN_AVG):
            return TRAIN_AVG
        return TRAIN
    return TRAIN


def get_ds_config_path_from_args(args: List[str]) -> Optional[str]:
    for i, a in enumerate(args[:-1]):
        if a == "--deepspeed":
            return args[i + 1]
    return None


class DetCallback(transformers.TrainerCallback):  # type: ignore[misc]
    def __init__(self, core_context: Any, args: transformers.TrainingArguments,
                 filter_metrics: Optional[List[str]] = None, user_data: Optional[Dict[str, Any]] = None) -> None:
        super().__init__()
        self.core_context = core_context
        self.filter_metrics = filter_metrics
        self.user_data = user_data
        self._info = get_cluster_info()
        self.load_last_checkpoint(args)
        self.last_metrics: Dict[str, Any] = {"train_step": -1, "eval_step": -1}
        self.updating_searcher = False
        if self._info is not None and self._info.trial is not None:
            searcher_config = self._info.trial._config["searcher"]
            self.searcher_ops: Iterator[Any] = self.core_context.searcher.operations()
        else:
            length_key, length = ("batches", args.max_steps) if args.max_steps > 0 else \
                ("epochs", int(args.num_train_epochs))
            searcher_config = {"name": "single", "metric": args.metric_for_best_model or "eval_loss",
                               "max_length": {length_key: length}}
            self.searcher_ops = iter([DummySearcherOperation(length, core_context.distributed.rank == 0)])
        self.current_op = next(self.searcher_ops)
        self.searcher_metric = searcher_config["metric"]
        if searcher_config["name"] == "custom":
            self.searcher_unit = "batches"
            self.searcher_max_length = self.current_op.length
        else:
            self.searcher_unit = list(searcher_config["max_length"].keys())[0]
            self.searcher_max_length = list(searcher_config["max_length"].values())[0]
            self._check_searcher_compatibility(args)

    # -- metrics -----------------------------------------------------------------------------
    def _get_metrics(self, logs: Dict[str, Any]) -> Tuple[Dict[str, Any], str]:
        kind = get_metric_type(logs)
        if not self.filter_metrics:
            return dict(logs), kind
        return {k: v for k, v in logs.items() if any(m in k for m in self.filter_metrics)}, kind

    def on_log(self, args: transformers.TrainingArguments, state: transformers.TrainerState,
               control: transformers.TrainerControl, logs: Optional[Dict[str, Any]] = None, **kw: Any) -> None:
        if logs is None:
            logger.warning("on_log called with empty logs")
            return
        metrics, kind = self._get_metrics(logs)
        if kind == TRAIN:
            if self.last_metrics["train_step"] != state.global_step:
                if state.is_world_process_zero:
                    self.core_context.train.report_training_metrics(steps_completed=state.global_step,
                                                                    metrics=metrics)
                metrics["train_step"] = state.global_step
        elif kind == EVAL:
            if self.last_metrics["eval_step"] != state.global_step:
                if state.is_world_process_zero:
                    self.core_context.train.report_validation_metrics(steps_completed=state.global_step,
                                                                      metrics=metrics)
                metrics["eval_step"] = state.global_step
        else:
            logger.debug("metrics of type %s not reported: %s", kind, sorted(metrics))
        self.last_metrics.update(metrics)
        if self.updating_searcher:
            self._update_searcher(state, control)
        if not self.updating_searcher and self.core_context.preempt.should_preempt():
            control.should_save = True

    # -- checkpoints --------------------------------------------------------------------------
    def on_save(self, args: transformers.TrainingArguments, state: transformers.TrainerState,
                control: transformers.TrainerControl, **kw: Any) -> None:
        local_path = os.path.join(args.output_dir, f"checkpoint-{state.global_step}")
        if state.is_world_process_zero and self.user_data is not None:
            self._on_save_user_data(local_path)
        md: Dict[str, Any] = {"steps_completed": state.global_step}
        if self._info is not None and self._info.trial is not None:
            md["trial_id"] = self._info.trial.trial_id
        prefix = (f"checkpoint-{state.global_step}/", "runs/")
        self.core_context.checkpoint.upload(args.output_dir, metadata=md, shard=True,
                                            selector=lambda p: p.startswith(prefix))
        if self.core_context.preempt.should_preempt():
            raise SystemExit("preempted after checkpoint upload")

    def _on_save_user_data(self, save_path: str) -> None:
        os.makedirs(save_path, exist_ok=True)
        with open(os.path.join(save_path, "my_data.json"), "w") as f:
            json.dump(self.user_data, f)

    def load_last_checkpoint(self, args: transformers.TrainingArguments) -> None:
        latest = self._info.latest_checkpoint if self._info is not None else None
        if latest is None:
            return
        if args.overwrite_output_dir:
            logger.info("Skip downloading last checkpoint from Determined due to overwrite_output_dir=True.")
            return
        # every file: resuming DeepSpeed-style runs needs all shards on every node
        self.core_context.checkpoint.download(latest, args.output_dir)
        path = trainer_utils.get_last_checkpoint(args.output_dir)
        args.resume_from_checkpoint = path
        logger.info("Latest checkpoint downloaded to %s.", path)

    # -- searcher -----------------------------------------------------------------------------
    def on_step_end(self, args: transformers.TrainingArguments, state: transformers.TrainerState,
                    control: transformers.TrainerControl, **kw: Any) -> None:
        if state.epoch and self.searcher_unit == "batches":
            if state.is_world_process_zero:
                self.current_op.report_progress(state.global_step)
            if state.global_step >= self.current_op.length:
                logger.info("searcher operation length %d reached; updating searcher", self.current_op.length)
                self._update_searcher(state, control)

    def on_epoch_end(self, args: transformers.TrainingArguments, state: transformers.TrainerState,
                     control: transformers.TrainerControl, **kw: Any) -> None:
        if state.epoch and self.searcher_unit == "epochs":
            if state.is_world_process_zero:
                self.current_op.report_progress(state.epoch)
            if state.epoch >= self.current_op.length:
                logger.info("searcher operation length %s epochs reached; updating searcher", state.epoch)
                self._update_searcher(state, control)

    def _metrics_reported(self, step: int) -> bool:
        return self.last_metrics["eval_step"] == step and self.last_metrics["train_step"] == step

    def _update_searcher(self, state: transformers.TrainerState, control: transformers.TrainerControl) -> None:
        if not self._metrics_reported(state.global_step):
            # have the Trainer log, evaluate and save first; we come back from on_log
            control.should_log = True
            control.should_evaluate = True
            control.should_save = True
            self.updating_searcher = True
            return
        if state.is_world_process_zero:
            if self.searcher_metric in self.last_metrics:
                metric = self.last_metrics[self.searcher_metric]
            else:
                logger.warning("Searcher metric %s not among recorded metrics %s; reporting "
                               "trainer_state.best_metric.", self.searcher_metric, sorted(self.last_metrics))
                metric = state.best_metric
            logger.info("Metric reported to searcher: %s", metric)
            self.current_op.report_completed(metric)
        self.updating_searcher = False
        try:
            self.current_op = next(self.searcher_ops)
        except StopIteration:
            control.should_training_stop = True

    def _check_searcher_compatibility(self, args: transformers.TrainingArguments) -> None:
        if self.searcher_unit == "batches":
            if args.max_steps == -1:
                self._log_config_mismatch("epochs", args.num_train_epochs)
            elif args.max_steps != self.searcher_max_length:
                self._log_config_mismatch("batches", args.max_steps)
        elif self.searcher_unit == "epochs":
            if args.max_steps != -1:
                self._log_config_mismatch("batches", args.max_steps)
            elif args.num_train_epochs != self.searcher_max_length:
                self._log_config_mismatch("epochs", args.num_train_epochs)

    def _log_config_mismatch(self, trainer_units: str, trainer_len: float) -> None:
        logger.warning("Searcher configuration does not match HF Trainer configuration: searcher uses %s=%s, "
                       "HF Trainer uses %s=%s. Use (--num_train_epochs and searcher.max_length.epochs) OR "
                       "(--max_steps and searcher.max_length.batches).", self.searcher_unit,
                       self.searcher_max_length, trainer_units, trainer_len)
