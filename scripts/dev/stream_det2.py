import os, sys
sys.path.insert(0, os.getcwd())
import torch
from imagent_amd.ops.conv import igemm_fwd
DEV = "cuda"
torch.manual_seed(0)
cases = [("stem", (8, 64, 64, 4), (64, 7, 32), 2, 3, 7, True), ("ds64", (8, 16, 16, 64), (128, 1, 1, 64), 2, 0, 1, False),
         ("ds128", (8, 8, 8, 128), (256, 1, 1, 128), 2, 0, 1, False), ("exp", (8, 16, 16, 64), (256, 1, 1, 64), 1, 0, 1, False),
         ("exp128", (8, 8, 8, 128), (512, 1, 1, 128), 1, 0, 1, False)]
side = torch.cuda.Stream()
A = torch.randn(4096, 4096, device=DEV)
for name, xs, ws, s, p, k, stem in cases:
    x = torch.randn(*xs, device=DEV).to(torch.bfloat16)
    if stem:
        x[..., 3] = 0
    w = (torch.randn(*ws, device=DEV) * 0.05).to(torch.bfloat16)
    Co = ws[0]
    slab0 = torch.zeros(32, 2, Co, device=DEV)
    y0 = igemm_fwd(x, w, s, p, k, k, stats=slab0, stem=stem)
    torch.cuda.synchronize()
    bad = 0
    worst = 0.0
    for r in range(300):
        if r % 3 == 0:
            with torch.cuda.stream(side):
                A @ A
        slab = torch.zeros(32, 2, Co, device=DEV)
        y = igemm_fwd(x, w, s, p, k, k, stats=slab, stem=stem)
        if not torch.equal(y, y0):
            bad += 1
        e = ((slab.sum(0) - slab0.sum(0)).norm() / slab0.sum(0).norm()).item()
        worst = max(worst, e)
    torch.cuda.synchronize()
    print(name, "output mismatches", bad, "/300, worst stats rel", worst, flush=True)
