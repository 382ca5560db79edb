"""Diagnostic: ResNet-50 bf16 gradients with the compact shortcut gradient on vs off."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import determined_amd.ops as ops
from determined_amd.models.resnet import resnet50
from determined_amd.ops import conv as C

torch.manual_seed(0)
model = resnet50(num_classes=10, zero_init_residual=False).cuda().to(memory_format=torch.channels_last)
state = {k: v.clone() for k, v in model.state_dict().items()}
x = torch.randn(16, 3, 96, 96, device="cuda").contiguous(memory_format=torch.channels_last)
orig = C._StridedGrad.take.__func__
log = []
def take(cls, g):
    got = orig(cls, g)
    log.append((None if g is None else tuple(g.shape), got is not None))
    return got
C._StridedGrad.take = classmethod(take)

def grads(dtype, disabled):
    ops._DISABLED = frozenset(disabled)
    model.load_state_dict(state)
    model.to(dtype)
    model.zero_grad()
    model(x.to(dtype)).float().square().mean().backward()
    out = {n: p.grad.float().clone() for n, p in model.named_parameters()}
    model.float()
    return out

allf = {"stem_conv", "stem_stats", "split_grad", "avgpool", "igemm_conv", "conv_stats", "bn_conv", "bn_prologue",
        "bn_lazy_bwd", "compact_shortcut_grad"}
ref = grads(torch.float32, allf)
sets = [set(a.split("+")) - {""} for a in sys.argv[1:]] or [set()]
for dis in sets:
    for rep in range(2):
        log.clear()
        g = grads(torch.bfloat16, dis)
        errs = {n: ((g[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-12)).item() for n in ref}
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
        print("disabled", sorted(dis), "takes", sum(1 for l in log if l[1]), "stem err %.4f" % errs["conv1.weight"],
              "worst", [(n, round(e, 3)) for n, e in worst], flush=True)
