"""Debug: per-conv fp8 output vs fake-quant emulation inside the R18 fp8 forward."""
import math
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
from imagent_amd.models import resnet
from imagent_amd.models.native import bind_native
import imagent_amd.ops.block as blk

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def fq(t, e):
    return (t * 2.0 ** -e).clamp(-448, 448).to(torch.float8_e4m3fn).float() * 2.0 ** e


orig = blk._fwd8


def wrapped(conv, h, h8, bn):
    y = orig(conv, h, h8, bn)
    if h8 is not None:
        ex = int(h8[1].item())
        ew = int(conv.w8_exp.item())
        xin = h.float().permute(0, 3, 1, 2)
        w = conv.weight.detach().float()
        ref = F.conv2d(fq(xin, ex), fq(w, ew), None, conv.stride, conv.padding)
        # also: what the kernel was given
        x8 = h8[0].view(torch.float8_e4m3fn).float() * 2.0 ** ex
        w8 = conv.w8.view(torch.float8_e4m3fn).float().permute(0, 3, 1, 2) * 2.0 ** ew
        ref2 = F.conv2d(x8.permute(0, 3, 1, 2), w8, None, conv.stride, conv.padding)
        print(f"conv {tuple(conv.weight.shape)} s{conv.stride}: vs emul {rel(y.permute(0,3,1,2), ref):.4f} "
              f"vs given-operands {rel(y.permute(0,3,1,2), ref2):.4f}  x8-vs-fq(h) {rel(x8.permute(0,3,1,2), fq(xin, ex)):.4f} "
              f"w8-vs-fq(w) {rel(w8, fq(w, ew)):.4f} ex {ex} ew {ew}")
    return y


blk._fwd8 = wrapped
torch.manual_seed(11)
m = resnet.build(sys.argv[1] if len(sys.argv) > 1 else "resnet18", num_classes=1000)
st = bind_native(m, DEV, fp8=True)
g = torch.Generator(device=DEV).manual_seed(12)
x = (torch.rand(16, 64, 64, 4, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
x[..., 3] = 0
m.train()
logits = m(x)
torch.cuda.synchronize()
print("done")
