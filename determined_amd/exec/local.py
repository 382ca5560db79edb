"""Run an experiment's trial locally without a master (``det experiment create --local``)."""

import json
import os
import sys


def main(entrypoint: str) -> int:
    from determined_amd import pytorch
    from determined_amd.exec.harness import load_trial_class
    from determined_amd.pytorch._trainer import _period

    hp = json.loads(os.environ["DET_LOCAL_HPARAMS"])
    cfg = json.loads(os.environ["DET_LOCAL_CONFIG"])
    cls = load_trial_class(entrypoint)
    from determined_amd import config as expconf

    ml = expconf.Length.parse(cfg["searcher"]["max_length"])
    with pytorch.init(hparams=hp, exp_conf=cfg) as ctx:
        trial = cls(ctx)
        unit = {None: "batches", expconf.Unit.BATCHES: "batches", expconf.Unit.EPOCHS: "epochs",
                expconf.Unit.RECORDS: "records"}[ml.unit]
        pytorch.Trainer(trial, ctx).fit(max_length=_period({unit: ml.units}, hp.get("global_batch_size")),
                                        validation_period=_period(cfg.get("min_validation_period"),
                                                                  hp.get("global_batch_size")),
                                        searcher_metric_name=cfg["searcher"]["metric"])
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
