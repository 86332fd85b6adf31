import os, sys
sys.path.insert(0, os.getcwd())
import torch, torch.nn.functional as F
from imagent_amd.models import native, resnet
from imagent_amd.models.native import bind_native
from imagent_amd.ops.misc import normalize_u8
DEV = "cuda"
torch.manual_seed(5)
model = resnet.build("resnet50", num_classes=1000)
st = bind_native(model, DEV)
img = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=DEV)
lab = torch.randint(0, 1000, (8,), device=DEV)
model.train()
def run(fused):
    native._FUSED_STEM = fused
    st.arena.zero_grad()
    x = normalize_u8(img, (64, 64), 4, (0.5,) * 3, (0.5,) * 3)
    F.cross_entropy(model(x), lab).backward()
    torch.cuda.synchronize()
    return {n: p.grad.float().clone() for n, p in model.named_parameters()}
def rel(a, b): return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
u1 = run(False); u2 = run(False); f1 = run(True); f2 = run(True); u3 = run(False)
for n in ["conv1.weight", "bn1.weight", "bn1.bias", "layer1.0.conv1.weight", "fc.weight"]:
    print(n, "u1-u2", rel(u2[n], u1[n]), "f1-u1", rel(f1[n], u1[n]), "f2-f1", rel(f2[n], f1[n]), "u3-u1", rel(u3[n], u1[n]))
