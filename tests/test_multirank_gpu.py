"""Two ranks on ONE MI355X: the data-parallel step with the native HIP kernels.

The 8-GPU scaling run is the driver's, not ours, and RCCL refuses two ranks on
one device. This rehearses everything around the collective on the real
kernels instead: two processes share cuda:0 and talk through gloo (which
handles device tensors), each runs the HIP forward / hand-scheduled backward
whose weight-gradient kernels release buckets through ``notify_ready`` (on
the wgrad side stream), the bucketed reducer averages the flat gradient
arena, and the fused SGD steps the masters (imagenet.py:316 DDP, :128
backward, :131 step).

Checked per rank: the averaged arena gradient equals the mean of the two
ranks' LOCAL gradients (each rank recomputes its own with communication
disabled, and the two are all-gathered), and after three SGD steps every
rank holds bit-identical parameters (``DataParallel.check_consistency``).
"""

import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, det=False):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", IMAGENT_DETERMINISTIC="1" if det else "0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.parallel.comm import TorchCommunicator
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.train.engine import StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD

    dev = torch.device("cuda:0")
    torch.manual_seed(100 + rank)  # DIFFERENT init per rank: the rank-0 broadcast must fix it
    model = resnet.build("resnet18", num_classes=1000)
    order = list(reversed(range(len(list(model.parameters())))))
    st = bind_native(model, dev, order)
    comm = TorchCommunicator()
    ddp = DataParallel(model, st.arena, comm, bucket_cap_mb=4.0, first_bucket_mb=1.0, rebuild_buckets=False)
    st.refresh_shadows(full=True)
    opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
    runner = StepRunner(ddp, opt, DeviceMetrics(dev), "hip")
    tf = InputTransform("hip", (64, 64), cpad=resnet.ResNet.STEM_CPAD)
    model.train()
    g = torch.Generator(device=dev).manual_seed(7 + rank)  # different data per rank
    worst = worst_vec = 0.0
    for _ in range(3):
        u8 = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=dev, generator=g)
        y = torch.randint(0, 1000, (8,), device=dev, generator=g)
        x = tf(u8)
        # this rank's local gradient, no communication (both passes from the same BN statistics shift:
        # st.save_ws, every BN's last batch mean / rstd, is written by each training forward)
        shift = st.save_ws.clone()
        st.arena.zero_grad()
        with ddp.no_sync():
            runner.loss(model(x), y).backward()
        torch.cuda.synchronize()
        want = comm.allgather(st.arena.G.clone()).mean(0)
        # the real data-parallel step: averaged gradient, then SGD
        st.save_ws.copy_(shift)
        opt.zero_grad()
        runner.loss(model(x), y).backward()
        torch.cuda.synchronize()
        # matrices (conv / fc weights) tightly; vectors (BatchNorm affine, fc
        # bias) loosely: BN affine gradients are small differences of large sums
        # and two forward+backward passes differ in fp32 atomic order (see
        # test_model_gpu.test_graphed_step_matches_eager)
        # Per bucket: the averaged gradient must be the mean of the local ones --
        # projection ratio 1 (a bucket reduced before it was complete, twice, or
        # not at all gives 0.5 / 2 / 0). The two backward passes themselves
        # differ: BN statistics are fp32 atomic sums, an order change now and
        # then moves a bf16 activation by one ulp, and a random-init network at
        # batch 8 amplifies that towards the stem (measured up to ~0.2
        # relative on the stem-side buckets, projection ratio >= 0.97; the
        # session-start code shows the same).
        for lo, hi, _ in ddp.buckets:
            gb, wb = st.arena.G[lo:hi], want[lo:hi]
            ratio = (gb * wb).sum().item() / max((wb * wb).sum().item(), 1e-30)
            worst = max(worst, abs(ratio - 1.0))
            worst_vec = max(worst_vec, ((gb - wb).norm() / wb.norm().clamp_min(1e-12)).item())
        opt.step()
    torch.cuda.synchronize()
    same = ddp.check_consistency(raise_on_mismatch=False)
    with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
        f.write(f"{worst} {worst_vec} {int(same)} {len(ddp.buckets)} {ddp.iteration}\n")
    dist.destroy_process_group()


@pytest.mark.parametrize("det", [False, True])
def test_two_ranks_one_gpu_native_step(det):
    """det: the deterministic mode (IMAGENT_DETERMINISTIC=1: fixed-order BatchNorm statistics and reductions),
    in which the two backward passes agree up to the weight gradients' split-K atomic order: tolerances 1e-3."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, det), nprocs=world, start_method="spawn",
                           join=True)
        for r in range(world):
            err, err_vec, same, nb, it = open(os.path.join(d, f"r{r}.txt")).read().split()
            tol, tol_vec = (1e-3, 1e-3) if det else (0.1, 0.5)
            assert float(err) < tol, err              # |projection ratio - 1| per bucket
            assert float(err_vec) < tol_vec, err_vec  # relative difference per bucket
            assert same == "1"
            assert int(nb) > 1 and int(it) == 3
