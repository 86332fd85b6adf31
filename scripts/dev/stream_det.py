import os, sys
sys.path.insert(0, os.getcwd())
import torch
from imagent_amd.ops.conv import igemm_fwd
DEV = "cuda"
torch.manual_seed(0)
cases = [("stem", (64, 224, 224, 4), (64, 7, 32), 2, 3, 7, True), ("ds64", (64, 56, 56, 64), (128, 1, 1, 64), 2, 0, 1, False),
         ("ds128", (64, 28, 28, 128), (256, 1, 1, 128), 2, 0, 1, False), ("exp", (64, 56, 56, 64), (256, 1, 1, 64), 1, 0, 1, False)]
for name, xs, ws, s, p, k, stem in cases:
    x = torch.randn(*xs, device=DEV).to(torch.bfloat16)
    if stem:
        x[..., 3] = 0
    w = (torch.randn(*ws, device=DEV) * 0.05).to(torch.bfloat16)
    Co = ws[0]
    slab0 = torch.zeros(32, 2, Co, device=DEV)
    y0 = igemm_fwd(x, w, s, p, k, k, stats=slab0, stem=stem)
    bad = 0
    worst = 0.0
    for r in range(200):
        slab = torch.zeros(32, 2, Co, device=DEV)
        y = igemm_fwd(x, w, s, p, k, k, stats=slab, stem=stem)
        if not torch.equal(y, y0):
            bad += 1
        e = ((slab.sum(0) - slab0.sum(0)).norm() / slab0.sum(0).norm()).item()
        worst = max(worst, e)
    torch.cuda.synchronize()
    print(name, "output mismatches", bad, "/200, worst stats rel", worst, flush=True)
