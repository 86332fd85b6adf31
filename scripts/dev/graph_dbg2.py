import os, sys
sys.path.insert(0, os.getcwd())
import torch
DEV = "cuda"
def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()
def main():
    """Whole-step HIP-graph capture/replay (engine.GraphedStep): from the same
    state and batch, one replayed step updates the parameters like one eager
    step (up to split-K atomic ordering)."""
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.parallel.comm import LocalCommunicator
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.train.engine import GraphedStep, StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD
    torch.manual_seed(21)
    model = resnet.build("resnet18", num_classes=1000)
    st = bind_native(model, DEV)
    ddp = DataParallel(model, st.arena, LocalCommunicator(), rebuild_buckets=False)
    opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
    runner = StepRunner(ddp, opt, DeviceMetrics(DEV), "hip")
    tf = InputTransform("hip", (64, 64), cpad=resnet.ResNet.STEM_CPAD)
    model.train()
    g = torch.Generator(device=DEV).manual_seed(22)
    imgs = torch.randint(0, 256, (4, 8, 64, 64, 3), dtype=torch.uint8, device=DEV, generator=g)
    labs = torch.randint(0, 1000, (4, 8), device=DEV, generator=g)

    def one(u8, y):
        runner.train_step([(tf(u8), y)])
    step = GraphedStep(one, warmup=2, key_fn=lambda: opt.lr)
    for i in range(3):  # 2 eager warm-up steps, then capture (+ replay)
        step(imgs[i], labs[i])
    assert step.graph is not None and step.replays == 1
    state = [t.clone() for t in (st.arena.P, opt.buf)] + [b.clone() for b in model.buffers()]

    def restore():
        for dst, src in zip([st.arena.P, opt.buf] + list(model.buffers()), state):
            dst.copy_(src)
        st.refresh_shadows(full=True)
    one(imgs[3], labs[3])  # eager
    upd_eager = st.arena.P - state[0]
    restore()
    one(imgs[3], labs[3])  # eager again
    upd_eager2 = st.arena.P - state[0]
    print("eager vs eager", rel(upd_eager2, upd_eager))
    restore()
    step(imgs[3], labs[3])  # replay
    torch.cuda.synchronize()
    assert step.replays == 2
    upd_graph = st.arena.P - state[0]
    print('graph vs eager', rel(upd_graph, upd_eager))


main()
