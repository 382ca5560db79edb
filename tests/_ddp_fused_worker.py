"""One rank of tests/test_ddp_fused_gpu.py (run as a child process, RANK/WORLD_SIZE/MASTER_* in env).

Each rank builds the same fused bf16 ResNet-50, computes the single-process gradients of BOTH
ranks' half batches (the reference), then runs its own half through the repo DDP (bucketed
all-reduce hooks over gloo) and compares the averaged gradients with the mean of the two
single-process gradients.  Writes a JSON report to argv[1]."""

import json
import os
import sys

import torch
import torch.distributed as dist
import torch.nn.functional as F


def main(out_path: str) -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import determined_amd.ops as ops
    from determined_amd.models.resnet import resnet50
    from determined_amd.ops import conv as conv_ops
    from determined_amd.parallel.ddp import DistributedDataParallel

    ops.ext()
    torch.manual_seed(0)
    model = resnet50(num_classes=100).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    halves = []
    for r in range(world):
        g = torch.Generator(device="cuda")
        g.manual_seed(100 + r)
        x = torch.randn(8, 3, 128, 128, generator=g, device="cuda").to(torch.bfloat16)
        halves.append((x.contiguous(memory_format=torch.channels_last),
                       torch.randint(0, 100, (8,), generator=g, device="cuda")))

    def grads(m, x, y):
        F.cross_entropy(m(x).float(), y).backward()
        out = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
        model.zero_grad(set_to_none=True)
        return out

    with conv_ops.agree_across_ranks():  # both ranks pick the same kernels (identical call sequence)
        per_half = [grads(model, x, y) for x, y in halves]
        ref = {n: sum(h[n] for h in per_half) / world for n in per_half[0]}
        ddp = DistributedDataParallel(model)
        x, y = halves[rank]
        F.cross_entropy(ddp(x).float(), y).backward()
        ddp.finish()
    worst, worst_name, missing = 0.0, "", []
    flat = []
    for n, p in model.named_parameters():
        if p.grad is None:
            missing.append(n)
            continue
        g = p.grad.float()
        flat.append(g.reshape(-1))
        den = ref[n].norm().item()
        err = (g - ref[n]).norm().item() / max(den, 1e-6)
        if den > 1e-6 and err > worst:
            worst, worst_name = err, n
    flat_t = torch.cat(flat).cpu()
    other = flat_t.clone()
    dist.broadcast(other, src=0)
    rep = {"rank": rank, "worst_rel_err": worst, "worst_param": worst_name, "missing": missing,
           "n_params": len(flat), "same_as_rank0": bool(torch.equal(other, flat_t)),
           "grad_norm": float(flat_t.norm())}
    with open(out_path, "w") as f:
        json.dump(rep, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
