"""Headline benchmark: ResNet-50 224x224 bf16 DDP training throughput.

BASELINE.json metric: "images/sec (whole node) ResNet-50 224x224 DDP at
1/2/4/8 MI355X"; baseline = the reference's FLOP-normalised headline,
4,337 R50@224-equivalent img/s for its whole 16-GPU job.

    python bench.py --gpus N --steps K --warmup W
    (N > 1: one rank per GPU. Under torch.distributed.run the ranks read
    RANK/WORLD_SIZE/MASTER_*; run bare, bench.py starts torch.distributed.run
    itself as a child process and forwards its output and exit code.)

Each timed step is a complete training step on the hand-written MI355X
path: GPU normalisation of synthetic uint8 images -> HIP forward (MFMA
implicit-GEMM convs, fused BN/ReLU/add) -> fused softmax-xent -> HIP backward
with bucketed RCCL all-reduce of fp32 gradients overlapped on a side stream ->
fused SGD (momentum 0.9, wd 1e-4) + bf16 shadow refresh. Random-init weights,
synthetic data (no network), per-GPU batch fixed (weak scaling). The K steps
are bracketed by barrier + device synchronize on both sides; the reported time
is the max over ranks.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_IMG_S = 4337.0  # R50@224-equivalent, whole reference job
# the reference job's throughput, FLOP-normalised per (arch, image size);
# resnet18@448 is the reference's own measured config (fp32, 16 GPUs)
BASELINES = {("resnet50", 224): BASELINE_IMG_S, ("resnet18", 224): 9776.0, ("resnet152", 224): 1540.0,
             ("resnet18", 448): 2444.0}
_NAMES = {"resnet18": "ResNet-18", "resnet34": "ResNet-34", "resnet50": "ResNet-50", "resnet101": "ResNet-101",
          "resnet152": "ResNet-152"}


def _self_launch(argv) -> int:
    """``python bench.py --gpus N`` outside a launcher: run ``torch.distributed.run
    --nproc-per-node N bench.py ...`` as a CHILD (this process never touched the
    GPU, and is not replaced) and return its exit code. Rank 0's JSON line
    reaches stdout through the child's inherited stdout (imagenet.sh:26 starts
    one task per GPU with srun; this is the single-node equivalent)."""
    import socket
    import subprocess
    a = [x for x in (argv if argv is not None else sys.argv[1:])]
    n = None
    for i, x in enumerate(a):
        if x == "--gpus":
            n = int(a[i + 1])
        elif x.startswith("--gpus="):
            n = int(x.split("=", 1)[1])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + a
    print("bench: launching " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--arch", default="resnet50")
    # 4096/GPU: the per-GPU batch sized for 288 GB of HBM (142.5 GiB peak, 186 GiB reserved: ~0.0455 GiB per image).
    # It fills the chip on the 7x7/14x14 stages and shrinks the all-reduce's and the per-step fixed costs' share
    # (round 5: 2048 16,498 / 16,522 img/s vs 1024 16,087 / 16,094; round 6, two boxes, alternating: 4096 17,610 /
    # 17,558 vs 2048 17,424 / 17,469, and 17,511 / 17,487 vs 17,354 / 17,390). The stem output and the layer-1
    # tensors hold 3.3 G elements (6.6 GB) at this batch: every kernel's buffer descriptors are tile / split / band
    # based and a duplicated-batch training step matches bit for bit per half
    # (tests/test_large_tensors_gpu.py::test_train_step_4096_duplicated_halves)
    ap.add_argument("--batch-size", type=int, default=None,
                    help="per GPU (default 4096; halved down to 256 when the device has too little free HBM)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--kernels", default="hip", choices=["hip", "torch"])
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--first-bucket-mb", type=float, default=2.0)
    ap.add_argument("--grad-allreduce-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: all-reduce bf16 copies of the gradient buckets (half the xGMI bytes; fp32 "
                         "masters and SGD unchanged)")
    ap.add_argument("--rccl-min-channels", type=int, default=None,
                    help="NCCL_MIN_NCHANNELS for the RCCL communicator (default: RCCL's choice)")
    ap.add_argument("--rccl-max-channels", type=int, default=None,
                    help="NCCL_MAX_NCHANNELS: caps the CUs RCCL's collectives take from the overlapped backward")
    ap.add_argument("--bn-fusion", type=int, default=1, help="0: separate BN-backward reduce pass")
    ap.add_argument("--wgrad-overlap", type=int, default=1, help="0: weight gradients on the main stream")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: capture the whole step in a HIP graph and replay it (1 GPU; launch-bound small batches); "
                         "2: also capture the weight-gradient side stream")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "lars"],
                    help="lars: layer-wise adaptive rates for the large-batch (8192) configuration")
    ap.add_argument("--eval", type=int, default=0,
                    help="N > 0: after the timed training steps, also time N validation steps (the folded-BN eval "
                         "forward + loss + top-k counters, imagenet.py:166-210) and report val_img_s")
    ap.add_argument("--fp32-split", type=int, default=0,
                    help="with --dtype fp32 --kernels hip: convs as 3 x bf16 split products (~2^-16 relative per "
                         "product, within 1e-4 of fp32 convs) instead of the exact f32 MFMA")
    ap.add_argument("--deterministic", type=int, default=0,
                    help="1: BatchNorm statistics without float atomics (fixed-order passes; ops/conv.py)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"],
                    help="fp8: e4m3 forward convs (block-scaled MFMA), bf16 backward; fp32: the reference's own "
                         "precision (imagenet.py:312 trains fp32): exact-f32 MFMA kernels with --kernels hip "
                         "(models/native_f32.py), PyTorch/MIOpen with --kernels torch")
    a = ap.parse_args(argv)
    f32_hip = a.dtype == "fp32" and a.kernels == "hip"
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and "SLURM_PROCID" not in os.environ:
        raise SystemExit(_self_launch(argv))

    from imagent_amd.data.loader import InputTransform
    from imagent_amd.data.synthetic import SyntheticImageNet
    from imagent_amd.models import resnet
    from imagent_amd.models.arena import ParamArena
    from imagent_amd.parallel import launcher
    from imagent_amd.parallel.comm import make_communicator, rccl_communicators
    from imagent_amd.parallel.ddp import DataParallel
    from imagent_amd.parallel.dist import init_distributed
    from imagent_amd.train.engine import StepRunner
    from imagent_amd.train.meters import DeviceMetrics
    from imagent_amd.train.optim import FlatSGD

    topo = launcher.discover("auto")
    if topo.world_size != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but the launcher reports world size {topo.world_size}")
    ctx = init_distributed(topo, "nccl", 600.0, verbose=False)
    on_gpu = ctx.device.type == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize(ctx.device)

    if os.environ.get("IMAGENT_MEM_FRACTION") and ctx.device.type == "cuda":  # cap this process's share of HBM
        torch.cuda.set_per_process_memory_fraction(float(os.environ["IMAGENT_MEM_FRACTION"]), ctx.device)
    auto_reduced = False
    if a.batch_size is None:
        a.batch_size = 4096
        if ctx.device.type == "cuda" and ctx.world_size == 1:
            # a GPU shared with another job (seen on the dev pool: a neighbour holding up
            # to 283 of the 288 GB) cannot fit the default: the allocator reserves ~0.0455 GiB
            # per image (186 GiB at 4096, 93.4 at 2048) + 15 % headroom, and below that it
            # thrashes (hipMalloc retries every step). Multi-rank runs keep the default on every rank.
            free = torch.cuda.mem_get_info(ctx.device)[0] / 2**30
            frac = os.environ.get("IMAGENT_MEM_FRACTION")
            if frac:
                free = min(free, float(frac) * torch.cuda.get_device_properties(ctx.device).total_memory / 2**30)
            while a.batch_size > 256 and 0.0525 * a.batch_size > free:
                a.batch_size //= 2
            if a.batch_size != 4096:
                auto_reduced = True
                print(f"bench: {free:.1f} GiB of HBM free, running {a.batch_size} img/GPU", file=sys.stderr,
                      flush=True)

    def max_over_ranks(seconds: float) -> float:
        # the c10d default group is CPU-side gloo for nccl jobs (parallel/dist.py): reduce a host tensor
        t = torch.tensor([seconds], dtype=torch.float64)
        if ctx.world_size > 1:
            if ctx.c10d_backend == "nccl":
                t = t.to(ctx.device)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t.item())

    def run():
        dev = ctx.device
        torch.manual_seed(0)
        model = resnet.build(a.arch)
        order = list(reversed(range(len(list(model.parameters())))))
        native = None
        if f32_hip:
            from imagent_amd.models.native_f32 import bind_native_f32
            native = bind_native_f32(model, dev, order)
            if a.fp32_split:
                from imagent_amd.ops.f32 import set_split
                set_split(True)
            arena = native.arena
        elif a.kernels == "hip":
            from imagent_amd.models.native import bind_native
            if a.deterministic:
                from imagent_amd.ops.conv import set_deterministic
                set_deterministic(True)
            native = bind_native(model, dev, order, bnb_fusion=bool(a.bn_fusion), fp8=a.dtype == "fp8",
                                 wgrad_overlap=bool(a.wgrad_overlap))
            arena = native.arena
        else:
            model.to(dev)
            arena = ParamArena(list(model.named_parameters()), dev, order=order)
        # RCCL reads its channel limits when the communicator is created
        if a.rccl_min_channels is not None:
            os.environ["NCCL_MIN_NCHANNELS"] = str(a.rccl_min_channels)
        if a.rccl_max_channels is not None:
            os.environ["NCCL_MAX_NCHANNELS"] = str(a.rccl_max_channels)
        comm = make_communicator(ctx, "rccl" if a.kernels == "hip" else "torch" if ctx.world_size > 1 else "local")
        ddp = DataParallel(model, arena, comm, bucket_cap_mb=a.bucket_mb, first_bucket_mb=a.first_bucket_mb,
                           rebuild_buckets=False, grad_reduce_dtype=a.grad_allreduce_dtype)
        if native is not None:  # compute shadows of the rank-0-broadcast masters
            native.refresh_shadows(full=True)
        after = native.refresh_shadows if native else None
        if a.optimizer == "lars":
            from imagent_amd.train.optim import FlatLARS
            opt = FlatLARS(arena, lr=0.1 * a.batch_size * a.gpus / 256, momentum=0.9, weight_decay=5e-5, eta=1e-3,
                           after_step=after)
        else:
            opt = FlatSGD(arena, lr=0.1, momentum=0.9, weight_decay=1e-4, after_step=after)
        metrics = DeviceMetrics(dev)
        runner = StepRunner(ddp, opt, metrics, "hip_f32" if f32_hip else a.kernels, 0.0,
                            torch.bfloat16 if (a.kernels == "torch" and a.dtype == "bf16") else None)
        if a.kernels == "torch":
            model.to(memory_format=torch.channels_last)
        src = SyntheticImageNet(a.batch_size * 4, a.image_size, 1000, a.batch_size, dev, seed=0,
                                rank=ctx.rank)
        tf = InputTransform("hip_f32" if f32_hip else a.kernels, (a.image_size, a.image_size),
                            cpad=resnet.ResNet.STEM_CPAD)
        model.train()

        def one(u8, y):
            runner.train_step([(tf(u8), y)])

        if a.graph:
            if ctx.world_size > 1:
                raise SystemExit("--graph is validated for one GPU only")
            from imagent_amd.train.engine import GraphedStep
            one = GraphedStep(one, warmup=2, key_fn=lambda: opt.lr, two_stream=a.graph == 2)

        def steps(n):
            for u8, y in src.batches(n):
                one(u8, y)

        steps(a.warmup)
        ctx.barrier()
        sync()
        c0 = comm.collectives
        t0 = time.perf_counter()
        steps(a.steps)
        sync()
        ctx.barrier()
        t1 = time.perf_counter()
        coll_per_step = (comm.collectives - c0) / max(1, a.steps)
        T = max_over_ranks(t1 - t0)
        # the mean loss of the warm-up + timed steps only (read before the instrumented steps below)
        loss, _, _, _ = metrics.reduced(comm if ctx.world_size > 1 else None)
        # after the timed region: two more steps with the bucket timeline recorded (parallel/ddp.py CommTimeline:
        # exposed communication after the last backward kernel, per-bucket issue offsets, comm-stream busy time)
        overlap = None
        if not a.graph:
            ddp.comm_timeline(True)
            steps(2)
            sync()
            overlap = ddp.timeline.stats()
            ddp.comm_timeline(False)
        n_rccl = rccl_communicators()  # counted while the training communicator is open
        val = None
        if a.eval > 0:  # validation throughput (Trainer.validate's step): eval-mode forward under no_grad
            model.eval()
            vsrc = src.batches(a.eval + 2)
            for _ in range(2):
                u8, y = next(vsrc)
                runner.eval_step(tf(u8), y)
            ctx.barrier()
            sync()
            v0 = time.perf_counter()
            for u8, y in vsrc:
                runner.eval_step(tf(u8), y)
            sync()
            ctx.barrier()
            Tv = max_over_ranks(time.perf_counter() - v0)
            val = dict(val_img_s=round(a.gpus * a.batch_size * a.eval / Tv, 2), val_steps=a.eval,
                       val_ms_per_step=round(1000.0 * Tv / a.eval, 3))
            model.train()
        value = a.gpus * a.batch_size * a.steps / T
        base = BASELINES.get((a.arch, a.image_size))
        if ctx.rank == 0:
            out = {
                "metric": f"images/sec (whole node) {_NAMES.get(a.arch, a.arch)} {a.image_size}x{a.image_size} DDP",
                "value": round(value, 2),
                "unit": "images/s",
                "n_gpus": a.gpus,
                "steps": a.steps,
                "warmup": a.warmup,
                "ms_per_step": round(1000.0 * T / a.steps, 3),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": round(value / base, 3) if base else None,
                "dtype": ("fp32" if (not on_gpu or a.dtype == "fp32") else "bf16" if a.dtype == "bf16" else
                          "fp8 (e4m3 forward convs, bf16 backward)"),
                "fp32_kernels": (("own kernels: convs as 3 x bf16 split products (~2^-16 per product)"
                                  if a.fp32_split else "own exact-f32 MFMA kernels") if f32_hip else "PyTorch/MIOpen")
                if a.dtype == "fp32" else None,
                "data": f"synthetic (uint8 3x{a.image_size}x{a.image_size} on device, GPU-normalised; "
                        "random-init weights)",
                "config": {
                    "model": a.arch,
                    "global_batch": a.batch_size * a.gpus,
                    "per_gpu_batch": a.batch_size,
                    "image_size": a.image_size,
                    "seq_len": None,
                    "parallelism": f"dp{a.gpus}",
                    "kernels": a.kernels,
                    "hip_graph": bool(a.graph),
                    "optimizer": "sgd(momentum=0.9, wd=1e-4)" if a.optimizer == "sgd" else
                                 "lars(momentum=0.9, wd=5e-5, eta=1e-3)",
                    "grad_allreduce": (f"{a.grad_allreduce_dtype} bucketed {comm.name} avg on the comm stream, "
                                       f"{coll_per_step:g} collectives/step" if coll_per_step > 0 else
                                       "none (world of one, collectives skipped)"),
                    "grad_allreduce_dtype": a.grad_allreduce_dtype,
                    "bucket_plan_mb": [round(v, 2) for v in ddp.bucket_sizes_mb()],
                    "rccl_env": {k: os.environ[k] for k in ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS",
                                                            "NCCL_P2P_DISABLE", "NCCL_ALGO", "NCCL_PROTO")
                                 if k in os.environ},
                    "comm": comm.name,
                    "rccl_communicators_per_process": n_rccl,
                    "c10d_backend": ctx.c10d_backend,
                    "world_size": ctx.world_size,
                    "comm_nranks": getattr(comm, "nranks", comm.world_size),
                    "collectives_per_step": coll_per_step,
                    "comm_overlap": overlap,
                    "comm_overlap_source": "2 instrumented steps after the timed region (not the timed steps)"
                    if overlap is not None else None,
                    "wgrad_side_stream": bool(a.wgrad_overlap) and a.kernels == "hip" and not f32_hip,
                    "auto_batch_reduced": auto_reduced,
                    "bucket_mb": a.bucket_mb,
                    "deterministic": bool(a.deterministic),
                    "mean_train_loss": round(loss, 4),
                    "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if dev.type == "cuda" else None,
                    "reserved_hbm_gib": round(torch.cuda.max_memory_reserved(dev) / 2**30, 1)
                    if dev.type == "cuda" else None,
                    "alloc_retries": int(torch.cuda.memory_stats(dev).get("num_alloc_retries", 0))
                    if dev.type == "cuda" else None,
                },
            }
            if val:
                out.update(val)
            print(json.dumps(out), flush=True)
        comm.close()

    # IMAGENT_MAIN_PRIO=1 (A/B): the whole step on a high-priority stream, so that the critical-path kernels'
    # workgroups are dispatched ahead of the weight-gradient side stream's as CU slots free up. Measured slower
    # (4096 img 17,639 / 17,712 -> 16,981 / 16,962 img/s, 256 img 13,547 -> 9,328: profiles/ab/prio_r6.txt)
    if on_gpu and os.environ.get("IMAGENT_MAIN_PRIO", "0") == "1":
        hp = torch.cuda.Stream(device=ctx.device, priority=min(torch.cuda.Stream.priority_range()))
        with torch.cuda.stream(hp):
            run()
    else:
        run()
    ctx.shutdown()


if __name__ == "__main__":
    main()
