"""Two-stream HIP-graph capture of a whole training step (GraphedStep(two_stream=True)): does it capture, replay and
match eager? Rounds 1 and 5 saw ``hipStreamEndCapture`` segfault on ResNet-18 in the deterministic mode with the
weight-gradient side stream captured. This runs that configuration (and R50) with Python's faulthandler plus a native
SIGSEGV backtrace (scripts/segv_bt.c), so a crash names the native frames.

    python -X faulthandler scripts/graph_capture_repro.py --arch resnet18 --deterministic 1 --batch 64
"""
import argparse
import ctypes
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--deterministic", type=int, default=1)
    ap.add_argument("--two-stream", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--comm", default="rccl", help="rccl (the bench's path, self-collectives at N = 1) or local")
    a = ap.parse_args()
    faulthandler.enable()
    lib = os.path.join(ROOT, "scripts", "bin", "libsegv_bt.so")
    if os.path.exists(lib):
        ctypes.CDLL(lib).install()
    import torch
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.data.synthetic import SyntheticImageNet
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.ops import streams
    from imagent_amd.parallel.comm import make_communicator
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.parallel.dist import init_distributed
    from imagent_amd.parallel import launcher
    from imagent_amd.train.engine import GraphedStep, StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD

    ctx = init_distributed(launcher.discover("single"), "nccl", 600.0, verbose=False)
    dev = ctx.device

    def build():
        torch.manual_seed(0)
        m = resnet.build(a.arch)
        order = list(reversed(range(len(list(m.parameters())))))
        if a.deterministic:
            from imagent_amd.ops.conv import set_deterministic
            set_deterministic(True)
        st = bind_native(m, dev, order)
        comm = make_communicator(ctx, a.comm)
        ddp = DataParallel(m, st.arena, comm, rebuild_buckets=False)
        st.refresh_shadows(full=True)
        opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
        met = DeviceMetrics(dev)
        m.train()
        return m, st, StepRunner(ddp, opt, met, "hip"), opt, met

    src = SyntheticImageNet(a.batch * 4, a.size, 1000, a.batch, dev, seed=0)
    tf = InputTransform("hip", (a.size, a.size), cpad=resnet.ResNet.STEM_CPAD)
    batches = list(src.batches(a.steps))
    print(f"[repro] {a.arch} batch {a.batch} deterministic {a.deterministic} two_stream {a.two_stream} "
          f"side stream {streams.overlap_enabled()}", flush=True)
    # eager reference
    m, st, run, opt, met = build()
    for u8, y in batches:
        run.train_step([(tf(u8), y)])
    torch.cuda.synchronize()
    p_eager = st.arena.P.clone()
    loss_eager = met.reduced()[0]
    # graphed
    m, st, run, opt, met = build()
    print(f"[repro] side stream enabled: {streams.overlap_enabled()}", flush=True)
    g = GraphedStep(lambda x, y: run.train_step([(x, y)]), warmup=2, key_fn=lambda: opt.lr,
                    two_stream=bool(a.two_stream))
    for i, (u8, y) in enumerate(batches):
        print(f"[repro] step {i} ({'eager' if g.graph is None and g.eager_calls < g.warmup else 'capture/replay'})",
              flush=True)
        g(tf(u8), y)
    torch.cuda.synchronize()
    rel = ((st.arena.P - p_eager).norm() / p_eager.norm()).item()
    print(f"[repro] captured={g.graph is not None} replays={g.replays} loss eager {loss_eager:.5f} graphed "
          f"{met.reduced()[0]:.5f} | params rel diff graphed vs eager {rel:.3e}", flush=True)
    ctx.shutdown()


if __name__ == "__main__":
    main()
