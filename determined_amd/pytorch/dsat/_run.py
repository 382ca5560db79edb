"""Driving an autotuning search (reference: ``dsat/_run_dsat.py``, ``dsat/_utils.py``)."""

import argparse
import copy
import json
import logging
import os
import pathlib
from typing import Any, Dict, List, Optional

import yaml

from determined_amd.pytorch.dsat import defaults
from determined_amd.pytorch.dsat._search import METHODS, BaseDSATSearchMethod

logger = logging.getLogger("determined_amd.pytorch.dsat")


def get_ds_config_from_hparams(hparams: Dict[str, Any], base_dir: str = ".") -> Dict[str, Any]:
    """The DeepSpeed config a trial should use: ``hparams["deepspeed_config"]`` (a path relative
    to the model directory, or a dict) with ``hparams["overwrite_deepspeed_args"]`` merged in."""
    from determined_amd.pytorch.deepspeed import overwrite_deepspeed_config

    base = hparams.get(defaults.CONFIG_KEY, {})
    if isinstance(base, str):
        base = os.path.join(base_dir, base)
    return overwrite_deepspeed_config(base, hparams.get(defaults.OVERWRITE_KEY) or {})


def build_search_method(name: str, exp_config: Dict[str, Any], **kw: Any) -> BaseDSATSearchMethod:
    if name not in METHODS:
        raise ValueError(f"unknown dsat search method {name!r}; choose from {sorted(METHODS)}")
    opts = dict(defaults.AUTOTUNING_ARG_DEFAULTS)
    opts.update({k: v for k, v in kw.items() if v is not None})
    hp = exp_config.get("hyperparameters") or {}
    # experiment-config hyperparameters are {name: {type: const, val: ...}} or plain values
    plain = {k: (v["val"] if isinstance(v, dict) and v.get("type") == "const" else v) for k, v in hp.items()}
    return METHODS[name](plain, opts["zero_stages"], opts["max_trials"], opts["max_concurrent_trials"],
                         opts["start_profile_step"], opts["end_profile_step"], opts["metric"],
                         opts["min_mbs"], opts["max_mbs"], opts["random_seed"])


def search_experiment_config(exp_config: Dict[str, Any], method: BaseDSATSearchMethod) -> Dict[str, Any]:
    cfg = copy.deepcopy(exp_config)
    cfg["name"] = f"{cfg.get('name', 'experiment')} (dsat)"
    cfg["searcher"] = {"name": "custom", "metric": method.metric_name,
                       "smaller_is_better": method.smaller_is_better,
                       "max_length": {"batches": method.end}}
    cfg["checkpoint_policy"] = "none"
    cfg["max_restarts"] = 0
    cfg["min_validation_period"] = {"batches": method.end}
    return cfg


def run_autotuning(name: str, config_path: str, model_dir: str, session: Any = None,
                   searcher_dir: Optional[str] = None, **kw: Any) -> Dict[str, Any]:
    """Run the search from this process (LocalSearchRunner); returns the summary."""
    from determined_amd.searcher import LocalSearchRunner

    with open(config_path) as f:
        exp_config = yaml.safe_load(f)
    run_full = bool(kw.pop("run_full_experiment", False))
    method = build_search_method(name, exp_config, **kw)
    runner = LocalSearchRunner(method, pathlib.Path(searcher_dir or "./dsat_searcher_state"), session=session)
    exp_id = runner.run(search_experiment_config(exp_config, method), model_dir=model_dir)
    summary = method.summary()
    summary["search_experiment_id"] = exp_id
    best = method.best()
    if best is not None:
        hp = copy.deepcopy(exp_config.get("hyperparameters") or {})
        ow = dict((hp.get(defaults.OVERWRITE_KEY) or {}))
        if isinstance(ow, dict) and ow.get("type") == "const":
            ow = dict(ow["val"])
        ow["train_micro_batch_size_per_gpu"] = best.mbs
        ow.pop("train_batch_size", None)
        ow["zero_optimization"] = dict(ow.get("zero_optimization") or {}, stage=best.stage)
        hp[defaults.OVERWRITE_KEY] = ow
        summary["best_hyperparameters"] = hp
        if run_full:
            from determined_amd.searcher._custom import _tar_dir

            cfg = dict(exp_config, hyperparameters=hp, name=f"{exp_config.get('name', 'experiment')} (dsat best)")
            r = runner._session.post("/api/v1/experiments", {"config": cfg, "model_def": _tar_dir(model_dir)})
            summary["full_experiment_id"] = r["experiment"]["id"]
    out = pathlib.Path(searcher_dir or "./dsat_searcher_state") / "dsat_summary.json"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(summary, indent=2))
    return summary


def get_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m determined_amd.pytorch.dsat",
                                description="Autotune ZeRO stage and micro-batch size of a DeepSpeedTrial")
    p.add_argument("search_method", choices=sorted(METHODS))
    p.add_argument("config_path")
    p.add_argument("model_dir")
    p.add_argument("-m", "--master", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    p.add_argument("--max-trials", type=int)
    p.add_argument("--max-concurrent-trials", type=int)
    p.add_argument("--zero-stages", type=int, nargs="+", choices=[0, 1, 2, 3])
    p.add_argument("--start-profile-step", type=int)
    p.add_argument("--end-profile-step", type=int)
    p.add_argument("--metric", choices=defaults.SMALLER_IS_BETTER_METRICS + defaults.LARGER_IS_BETTER_METRICS)
    p.add_argument("--min-mbs", type=int)
    p.add_argument("--max-mbs", type=int)
    p.add_argument("--random-seed", type=int)
    p.add_argument("--run-full-experiment", action="store_true")
    p.add_argument("--searcher-dir", default=None)
    return p


def main(argv: Optional[List[str]] = None) -> int:
    a = get_parser().parse_args(argv)
    from determined_amd.common.api import Session

    logging.basicConfig(level=logging.INFO, format="%(levelname)s: %(message)s")
    kw = {k: getattr(a, k) for k in ("max_trials", "max_concurrent_trials", "zero_stages", "start_profile_step",
                                     "end_profile_step", "metric", "min_mbs", "max_mbs", "random_seed")}
    summary = run_autotuning(a.search_method, a.config_path, a.model_dir, session=Session(a.master),
                             searcher_dir=a.searcher_dir, run_full_experiment=a.run_full_experiment, **kw)
    print(json.dumps(summary, indent=2))
    return 0
