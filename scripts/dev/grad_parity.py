"""Per-parameter gradient cosines of the bf16 ResNet-50: fused vs all-fusions-off vs an fp32
reference, for a residual-BN init scale (RES_W, default 0: torchvision's zero init) -- shows how
well-conditioned the comparison is before a test relies on it."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import torch.nn.functional as F
import determined_amd.ops as ops
from determined_amd.models.resnet import resnet50

ALL = frozenset({"stem_conv", "stem_stats", "split_grad", "avgpool", "igemm_conv", "conv_stats", "bn_conv",
                 "bn_prologue", "bn_lazy_bwd", "compact_shortcut_grad", "bn_residual_fold"})
res_w = float(os.environ.get("RES_W", "0"))
torch.manual_seed(0)
m = resnet50(num_classes=100)
for b in [b for l in (m.layer1, m.layer2, m.layer3, m.layer4) for b in l]:
    torch.nn.init.constant_(b.bn3.weight, res_w)
sd = {k: v.clone() for k, v in m.state_dict().items()}
g = torch.Generator().manual_seed(3)
x = torch.randn(16, 3, 128, 128, generator=g)
t = torch.randint(0, 100, (16,), generator=g)


def run(dtype, disabled):
    ops._DISABLED = disabled
    mm = resnet50(num_classes=100)
    mm.load_state_dict(sd)
    mm = mm.cuda().to(dtype).to(memory_format=torch.channels_last)
    xx = x.cuda().to(dtype).contiguous(memory_format=torch.channels_last)
    F.cross_entropy(mm(xx).float(), t.cuda()).backward()
    return {n: p.grad.float() for n, p in mm.named_parameters()}


ref = run(torch.float32, ALL)
fused = run(torch.bfloat16, frozenset())
plain = run(torch.bfloat16, ALL)
cos = lambda a, b: F.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()  # noqa: E731
rows = [(n, cos(fused[n], ref[n]), cos(plain[n], ref[n]), cos(fused[n], plain[n])) for n in ref]
print(f"RES_W={res_w}: min cos fused/ref {min(r[1] for r in rows):.4f} plain/ref {min(r[2] for r in rows):.4f} "
      f"fused/plain {min(r[3] for r in rows):.4f}")
for r in sorted(rows, key=lambda r: r[1])[:6]:
    print(f"   {r[0]:40s} fused/ref {r[1]:.4f} plain/ref {r[2]:.4f} fused/plain {r[3]:.4f}")
