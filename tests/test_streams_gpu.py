"""Weight-gradient side stream vs no overlap.

Side-stream operands are held until the end-of-backward join (ops/streams.py
``protect``). The run must give the update of a run with the side stream off,
and the held list must be empty after every step (round-1 advice).

Two steps from the same initial state and batches per mode (the second one
exercises the steady state: buffers recycled from the first step); the
first-step updates are compared by projection ratio, as in test_model_gpu.py's graph-vs-eager test:
BN statistics are fp32 atomic sums, so two runs of the SAME mode already
differ by ulp flips that the random-init network amplifies; a freed-too-early
operand or a missing join moves the update by O(1).
"""

import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DEV = torch.device("cuda:0")


def _run(overlap):
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.ops import streams
    from imagent_amd.parallel.comm import LocalCommunicator
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.train.engine import StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD
    torch.manual_seed(5)
    model = resnet.build("resnet18", num_classes=1000)
    order = list(reversed(range(len(list(model.parameters())))))
    st = bind_native(model, DEV, order, wgrad_overlap=overlap)
    assert streams.overlap_enabled() == overlap
    ddp = DataParallel(model, st.arena, LocalCommunicator(), rebuild_buckets=False)
    opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
    runner = StepRunner(ddp, opt, DeviceMetrics(DEV), "hip")
    tf = InputTransform("hip", (64, 64), cpad=resnet.ResNet.STEM_CPAD)
    model.train()
    g = torch.Generator(device=DEV).manual_seed(6)
    imgs = torch.randint(0, 256, (2, 32, 64, 64, 3), dtype=torch.uint8, device=DEV, generator=g)
    labs = torch.randint(0, 1000, (2, 32), device=DEV, generator=g)
    p0 = st.arena.P.clone()
    upd = None
    for i in range(2):
        runner.train_step([(tf(imgs[i]), labs[i])])
        torch.cuda.synchronize()
        assert streams.held() == 0, "side-stream operands still held after the step"
        assert streams.deferred() == 0, "deferred weight-gradient launches left queued"
        if i == 0:  # compare the first update: the second one also carries the first one's
            upd = st.arena.P - p0  # atomic-order differences, amplified by the random-init BNs
    assert bool(torch.isfinite(st.arena.P).all())
    params = list(model.parameters())
    slices = {kind: torch.cat([st.arena.flat_slice(upd, i) for i, p in enumerate(params) if (p.dim() > 1) == kind])
              for kind in (True, False)}
    streams.set_wgrad_overlap(False)
    return slices


def _ratio(a, b):
    return (a * b).sum().item() / (b * b).sum().item()


def test_side_stream_matches_no_overlap():
    ref = _run(False)
    got = _run(True)
    for kind in (True, False):
        r = _ratio(got[kind], ref[kind])
        print(f"weights={kind}: projection ratio {r:.5f}")
        assert abs(r - 1.0) < 0.1, (kind, r)
        assert got[kind].abs().max() > 0
