"""The native RCCL communicator really runs on one MI355X.

At world size 1 the communicator still hands every collective to RCCL (a
one-rank communicator, ``IMAGENT_RCCL_SELF`` default on), so the comm-stream
ordering, event joins and buffer lifetimes of the multi-GPU data-parallel
step (imagenet.py:316 DDP, :128 backward all-reduce) execute here exactly as
they do at N = 8.

The data-parallel test runs three native R18 steps with the weight-gradient
side stream on, the iteration-1 bucket rebuild on, and the ordering probe
(``DataParallel.verify_order``): each bucket is checksummed ON the comm stream
right after its all-reduce and must equal the finished gradient bit for bit.
A negative control removes the comm stream's wait on the side stream and
delays the side stream: the probe must then catch stale buckets.
"""

import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _comm():
    from imagent_amd.parallel.comm import RcclCommunicator
    return RcclCommunicator(0, 1, torch.device("cuda:0"), None, self_collectives=True)


def test_rccl_self_collectives_execute():
    c = _comm()
    try:
        assert c.active and c.nranks == 1
        t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
        want = t.clone()
        c.allreduce_(t, "avg")
        c.join()
        torch.cuda.synchronize()
        assert torch.equal(t, want)
        b = torch.arange(1000, device="cuda", dtype=torch.int64)
        c.broadcast_(b, 0)
        g = c.allgather(torch.ones(5, device="cuda", dtype=torch.bfloat16))
        torch.cuda.synchronize()
        assert g.shape == (1, 5) and bool((g == 1).all())
        assert torch.equal(b, torch.arange(1000, device="cuda"))
        assert c.collectives == 3
        assert c.healthy()
    finally:
        c.close()


def _setup(rebuild=True):
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.train.engine import StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = resnet.build("resnet18", num_classes=1000)
    order = list(reversed(range(len(list(model.parameters())))))
    st = bind_native(model, dev, order, wgrad_overlap=True)
    comm = _comm()
    ddp = DataParallel(model, st.arena, comm, bucket_cap_mb=2.0, first_bucket_mb=0.5,
                       rebuild_buckets=rebuild, probe_order=True)
    st.refresh_shadows(full=True)
    opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
    runner = StepRunner(ddp, opt, DeviceMetrics(dev), "hip")
    model.train()
    return st, comm, ddp, opt, runner


def _batch(step):
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    g = torch.Generator(device="cuda").manual_seed(11 + step)
    u8 = torch.randint(0, 256, (32, 96, 96, 3), dtype=torch.uint8, device="cuda", generator=g)
    y = torch.randint(0, 1000, (32,), device="cuda", generator=g)
    return InputTransform("hip", (96, 96), cpad=resnet.ResNet.STEM_CPAD)(u8), y


def test_ddp_step_over_rccl_orders_buckets_after_wgrad():
    from imagent_amd.ops import streams
    st, comm, ddp, opt, runner = _setup(rebuild=True)
    try:
        n0 = comm.collectives
        for step in range(3):
            runner.train_step([_batch(step)])
            torch.cuda.synchronize()
            assert streams.held() == 0, "side-stream operands not released at the end-of-backward join"
            assert len(runner._inflight) <= runner.max_inflight  # run-ahead limit (blocking events)
            bad = ddp.verify_order()  # before the relayout below moves the buckets
            assert bad == [], f"step {step}: buckets {bad} all-reduced before their producers finished"
            # iteration-1 relayout, as Trainer.train_epoch does it
            if getattr(ddp, "pending_relayout", None) is not None:
                assert step == 0
                opt.set_flats(ddp.apply_pending_relayout(opt.flats()))
                st.rebind()
        nb = len(ddp.buckets)
        assert nb > 4
        # every bucket of every step went through RCCL
        assert comm.collectives - n0 >= 3 * nb - 2 * 2, (comm.collectives - n0, nb)
        assert ddp.iteration == 3
        assert bool(torch.isfinite(st.arena.P).all())
    finally:
        comm.close()


def test_ordering_probe_catches_missing_side_stream_dependency():
    """Negative control: without the comm stream's wait on the wgrad side
    stream (and with that stream held back by a sleep kernel), buckets whose
    last producer was a side-stream wgrad get reduced too early."""
    from imagent_amd.ops import streams
    st, comm, ddp, opt, runner = _setup(rebuild=False)
    try:
        runner.train_step([_batch(0)])  # warm-up: kernel variants, momentum buffers
        torch.cuda.synchronize()
        assert ddp.verify_order() == []
        comm.depend_on = lambda stream: None          # the bug under test
        cur = comm._cur
        comm._cur = lambda: torch.cuda.default_stream(comm.device).cuda_stream  # issue from the main stream
        # a side stream on a hardware queue of its own (full-CU-mask stream): a stream that
        # happens to share a queue with the comm stream would serialise the two in hardware
        # and hide the missing dependency
        import ctypes as C
        from imagent_amd.ops import _lib
        h = C.c_void_p()
        assert _lib.comm().imc_stream_create(0, 2, C.byref(h)) == 0
        side = torch.cuda.ExternalStream(h.value, device=torch.device("cuda:0"))
        streams._streams[0] = side
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            torch.cuda._sleep(200_000_000)  # hold every wgrad of this step back
        runner.train_step([_batch(1)])
        torch.cuda.synchronize()
        bad = ddp.verify_order()
        comm._cur = cur
        assert len(bad) > 0, "ordering probe did not detect buckets reduced before their wgrad kernels"
    finally:
        streams._streams.pop(0, None)
        comm.close()
