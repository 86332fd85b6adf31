"""Which PyTorch (ATen / library) device launches remain in the HIP training step, and where from.

python scripts/aten_audit.py [--arch resnet50] [--batch 256] [--steps 2] [--out profiles/aten_audit.md]

Builds the step exactly as bench.py does (bind_native -> DataParallel over the own RCCL communicator -> FlatSGD ->
StepRunner, GPU-normalised synthetic uint8 input), warms it up, then runs ``--steps`` steps under torch.profiler with
Python stacks. Every ``aten::`` operator that launched a device kernel is listed with its launches per step and the
innermost in-repo source lines of its call stack. The own kernels are ctypes launches, invisible to the profiler's
operator view, so a clean step prints an empty table (the rocprofv3 kernel table says the same from the device side:
no ``at::native`` / ``Cijk_`` rows).
"""

import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def build_step(arch: str, batch: int, size: int):
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.data.synthetic import SyntheticImageNet
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.parallel import launcher
    from imagent_amd.parallel.comm import make_communicator
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.parallel.dist import init_distributed
    from imagent_amd.train.engine import StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD
    ctx = init_distributed(launcher.discover("auto"), "nccl", 600.0, verbose=False)
    dev = ctx.device
    torch.manual_seed(0)
    model = resnet.build(arch)
    order = list(reversed(range(len(list(model.parameters())))))
    native = bind_native(model, dev, order)
    comm = make_communicator(ctx, "rccl")
    ddp = DataParallel(model, native.arena, comm, rebuild_buckets=False)
    native.refresh_shadows(full=True)
    opt = FlatSGD(native.arena, lr=0.1, momentum=0.9, weight_decay=1e-4, after_step=native.refresh_shadows)
    runner = StepRunner(ddp, opt, DeviceMetrics(dev), "hip", 0.0, None)
    src = SyntheticImageNet(batch * 2, size, 1000, batch, dev, seed=0, rank=0)
    tf = InputTransform("hip", (size, size), cpad=resnet.ResNet.STEM_CPAD)
    model.train()

    def steps(n):
        for u8, y in src.batches(n):
            runner.train_step([(tf(u8), y)])

    return steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    steps = build_step(a.arch, a.batch, a.size)
    steps(3)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        steps(a.steps)
        torch.cuda.synchronize()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = collections.Counter()
    kern = collections.defaultdict(set)
    for e in prof.events():
        if not e.name.startswith("aten::") or not e.kernels:
            continue
        if e.cpu_parent is not None and e.cpu_parent.name.startswith("aten::") and e.cpu_parent.kernels:
            continue  # counted at the outermost aten op that launched
        frames = [f for f in (e.stack or []) if repo in f and "torch/" not in f][:3]
        where = " <- ".join(f.replace(repo + "/", "") for f in frames) or "(no in-repo frame)"
        rows[(e.name, where)] += len(e.kernels)
        for k in e.kernels:
            kern[(e.name, where)].add(k.name[:60])
    lines = [f"# ATen / library device launches in the HIP training step ({a.arch}, {a.batch} img, "
             f"{a.steps} profiled steps)", "",
             "`python scripts/aten_audit.py` (torch.profiler over the bench.py step; own kernels are ctypes launches "
             "and do not appear).", "",
             "| launches/step | aten op | kernels | call site (innermost in-repo frames) |", "|---:|---|---|---|"]
    for (name, where), n in sorted(rows.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {n / a.steps:g} | `{name}` | {', '.join(sorted(kern[(name, where)]))} | {where} |")
    if not rows:
        lines.append("| 0 | (none) | | |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
