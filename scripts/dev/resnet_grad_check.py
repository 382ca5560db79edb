"""Per-parameter gradient agreement of the bf16 ResNet-50 (current kernel set) against an fp32
composition of the same weights; prints the worst parameters.  DAMD_DISABLE_FUSIONS selects the
path under test."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch.nn.functional as F
from determined_amd.models.resnet import resnet50, Bottleneck

torch.manual_seed(0)
m = resnet50(num_classes=100)
for mod in m.modules():
    if isinstance(mod, torch.nn.BatchNorm2d):
        torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
x = torch.randn(int(os.environ.get("B", "8")), 3, 96, 96)
t = torch.randint(0, 100, (x.shape[0],))
sd = {k: v.clone() for k, v in m.state_dict().items()}

def run(dtype, cl):
    mm = resnet50(num_classes=100)
    mm.load_state_dict(sd)
    mm = mm.cuda().to(dtype)
    xx = x.cuda().to(dtype)
    if cl:
        mm = mm.to(memory_format=torch.channels_last)
        xx = xx.contiguous(memory_format=torch.channels_last)
    F.cross_entropy(mm(xx).float(), t.cuda()).backward()
    return {n: p.grad.float().cpu() for n, p in mm.named_parameters()}

ref = run(torch.float32, False)
if os.environ.get("PERTURB"):
    x = x * (1 + 1e-3 * torch.randn_like(x))  # fp32 vs fp32 with a 1e-3 input perturbation
    got = run(torch.float32, False)
else:
    got = run(torch.bfloat16, True)
rows = sorted(((((got[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-12)).item(), n) for n in ref), reverse=True)
print(os.environ.get("DAMD_DISABLE_FUSIONS", ""), "worst:", [(n, round(r, 4)) for r, n in rows[:8]])
print("median rel", rows[len(rows) // 2][0])
