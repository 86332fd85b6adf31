"""Repeat one eager training step from a fixed state and report the spread of
parameter updates (split-K atomics give ~1e-6; a race shows as outliers)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def run(tag, reps=12, overlap=True, bnb=True, arch="resnet18", B=8, H=64):
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.parallel.comm import LocalCommunicator
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.train.engine import StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD
    torch.manual_seed(21)
    model = resnet.build(arch, num_classes=1000)
    st = bind_native(model, DEV, bnb_fusion=bnb, wgrad_overlap=overlap)
    ddp = DataParallel(model, st.arena, LocalCommunicator(), rebuild_buckets=False)
    opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
    runner = StepRunner(ddp, opt, DeviceMetrics(DEV), "hip")
    tf = InputTransform("hip", (H, H), cpad=resnet.ResNet.STEM_CPAD)
    model.train()
    g = torch.Generator(device=DEV).manual_seed(22)
    imgs = torch.randint(0, 256, (4, B, H, H, 3), dtype=torch.uint8, device=DEV, generator=g)
    labs = torch.randint(0, 1000, (4, B), device=DEV, generator=g)
    for i in range(3):
        runner.train_step([(tf(imgs[i]), labs[i])])
    torch.cuda.synchronize()
    state = [t.clone() for t in (st.arena.P, opt.buf)] + [b.clone() for b in model.buffers()]

    def restore():
        for dst, src in zip([st.arena.P, opt.buf] + list(model.buffers()), state):
            dst.copy_(src)
        st.refresh_shadows(full=True)
    ups = []
    poison = os.environ.get("POISON") == "1"
    for r in range(reps):
        restore()
        runner.train_step([(tf(imgs[3]), labs[3])])
        torch.cuda.synchronize()
        ups.append((st.arena.P - state[0]).clone())
    nan = sum(int(not torch.isfinite(u).all()) for u in ups)
    if nan:
        print(f"{tag}: {nan} of {len(ups)} updates non-finite", flush=True)
        ups = [u.nan_to_num() for u in ups]
    if os.environ.get("PERPARAM") == "1":
        names = [n for n, _ in model.named_parameters()]
        d0 = ups[0] - ups[1]
        rows = []
        for i, (n, p_) in enumerate(model.named_parameters()):
            rows.append((rel(st.arena.flat_slice(ups[0], i), st.arena.flat_slice(ups[1], i)), n))
        rows.sort(reverse=True)
        print(tag, "per-param rep0 vs rep1:", [(n, f"{e:.1e}") for e, n in rows[:8]], flush=True)
    errs = sorted(rel(u, ups[0]) for u in ups[1:])
    print(f"{tag:40s} max {errs[-1]:.2e} median {errs[len(errs)//2]:.2e}", flush=True)


if __name__ == "__main__":
    run("B8 H64", reps=6)
    run("B32 H64", reps=6, B=32)
