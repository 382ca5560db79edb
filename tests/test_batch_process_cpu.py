"""torch_batch_process on CPU: sharding across 2 gloo ranks, checkpointed progress, reducers,
per-rank outputs through upload_path."""

import json
import pathlib
import tempfile

import torch

from tests.dist_utils import run_distributed


class _Squares(torch.utils.data.Dataset):
    def __len__(self):
        return 21

    def __getitem__(self, i):
        return torch.tensor([float(i)])


def _worker(rank, world, store):
    from determined_amd import core, pytorch
    from determined_amd.pytorch.experimental import TorchBatchProcessor, torch_batch_process

    class SumReducer(pytorch.MetricReducer):
        def __init__(self):
            self.reset()

        def reset(self):
            self.total = 0.0

        def update(self, v):
            self.total += v

        def per_slot_reduce(self):
            return self.total

        def cross_slot_reduce(self, per_slot):
            return sum(per_slot)

    seen = []

    class P(TorchBatchProcessor):
        def __init__(self, context):
            self.context = context
            self.model = context.prepare_model_for_inference(torch.nn.Identity())
            self.red = context.wrap_reducer(SumReducer(), name="sum_of_squares")
            self.out = []

        def process_batch(self, batch, batch_idx):
            x = self.model(self.context.to_device(batch))
            seen.extend(int(v) for v in x.flatten())
            self.red.update(float((x ** 2).sum()))
            self.out.append(x)

        def on_checkpoint_start(self):
            with self.context.upload_path() as p:
                torch.save(torch.cat(self.out), p / f"part{len(list(p.iterdir()))}.pt")
            self.out = []

    dist_ctx = core.DistributedContext.from_torch_distributed()
    torch_batch_process(P, _Squares(), batch_size=2, checkpoint_interval=2, distributed_context=dist_ctx,
                        checkpoint_storage=store)
    return seen


def test_torch_batch_process_two_ranks():
    with tempfile.TemporaryDirectory() as store:
        res = run_distributed(_worker, 2, args=(store,))
        allseen = sorted(res[0] + res[1])
        assert allseen == list(range(21))  # every sample exactly once across ranks
        assert not set(res[0]) & set(res[1])
        ckpts = [p for p in pathlib.Path(store).iterdir() if (p / "batch_completed.json").exists()]
        done = sorted(json.loads((p / "batch_completed.json").read_text())["batch_completed"] for p in ckpts)
        assert done[-1] == 6  # ceil(21 / 2 / 2) batches per rank
        outs = [p for p in pathlib.Path(store).rglob("part*.pt")]
        assert {p.parent.name for p in outs} == {"rank_0", "rank_1"}
