"""Debug: per-parameter gradient differences, fused vs unfused BN backward vs fp32 oracle."""
import copy
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
from imagent_amd.models import resnet
from imagent_amd.models.native import bind_native

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
torch.manual_seed(3)
base = resnet.build(arch, num_classes=1000)
g = torch.Generator(device=DEV).manual_seed(5)
x = torch.randn(8, 48, 48, 4, device=DEV, generator=g).to(torch.bfloat16)
x[..., 3] = 0
lab = torch.randint(0, 1000, (8,), device=DEV, generator=g)
grads = []
for fuse in (False, True):
    model = copy.deepcopy(base)
    st = bind_native(model, DEV)
    for b in model.blocks():
        b._fuse_bnb = fuse
    model.train()
    st.arena.zero_grad()
    F.cross_entropy(model(x), lab).backward()
    torch.cuda.synchronize()
    grads.append({n: p.grad.float().clone() for n, p in model.named_parameters()})
ref = copy.deepcopy(base).to(DEV)
with torch.no_grad():
    for p in ref.parameters():
        p.copy_(p.to(torch.bfloat16).float())
ref.train()
xr = x[..., :3].float().permute(0, 3, 1, 2).contiguous()
F.cross_entropy(ref(xr), lab).backward()
for n, p in ref.named_parameters():
    print(f"{n:40s} unfused {rel(grads[0][n], p.grad):.4f} fused {rel(grads[1][n], p.grad):.4f} "
          f"f-vs-u {rel(grads[1][n], grads[0][n]):.4f}")
