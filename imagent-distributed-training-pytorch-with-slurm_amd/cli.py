"""Command line: a superset of the reference's flags.

The six reference flags keep their names and defaults (``imagenet.py:435-450``):
``--seed 0 --backend nccl --batch-size 128 (per GPU) --epochs 100 --lr 0.1
--save-model``. The reference's hard-coded choices become flags with the
reference values as defaults (ResNet-18, 448x448, Normalize 0.5/0.5, momentum
0.9, wd 1e-4, step decay 0.1 every 30 epochs, 10 workers, ``../data/imagenet``,
TensorBoard dir ``imagenet_FR``).

Usage::

    python -m imagent_amd.cli --arch resnet50 --image-size 224 --data synthetic
    srun python imagenet.py --backend=nccl          # Slurm, like imagenet.sh
    torchrun --nproc-per-node 8 imagenet.py ...     # single node
"""

from __future__ import annotations

import argparse
import sys


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Imagenet Pytorch (MI355X-native)")
    # --- reference flags (same names, same defaults) ---
    p.add_argument("--seed", default=0, type=int, help="seed for initializing training. ")
    p.add_argument("--backend", type=str, default="nccl", help="c10d backend (nccl == RCCL on ROCm, or gloo)")
    p.add_argument("--batch-size", type=int, default=128, metavar="N", help="input batch size per GPU")
    p.add_argument("--epochs", type=int, default=100, metavar="N")
    p.add_argument("--lr", type=float, default=0.1, metavar="LR")
    p.add_argument("--save-model", action="store_true", default=False, help="save the best model")
    # --- model / data ---
    p.add_argument("--arch", default="resnet18", choices=["resnet18", "resnet34", "resnet50", "resnet101",
                                                           "resnet152"])
    p.add_argument("--image-size", type=int, default=448)
    p.add_argument("--deterministic", action="store_true",
                   help="BatchNorm statistics without float atomics (fixed-order reduction passes): two runs "
                        "from the same state give bit-identical statistics (HIP kernels)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"],
                   help="compute dtype. HIP kernels: bf16 (fp32 masters/accumulation), fp8 = e4m3 forward "
                        "convs on the block-scaled MFMA with bf16 backward, fp32 = the reference's precision "
                        "(imagenet.py:312) on the own exact-f32 MFMA kernels (models/native_f32.py; every ResNet "
                        "depth, BatchNorm widths up to 2048 channels). --kernels torch: PyTorch ops (oracle)")
    p.add_argument("--data", default="imagenet", choices=["imagenet", "records", "synthetic"],
                   help="imagenet: JPEG folders decoded by worker processes; records: train.imrec / val.imrec "
                        "(python -m imagent_amd.data.records) gathered by the native thread pool")
    p.add_argument("--data-root", default=None, help="default: <cwd>/../data/imagenet (imagenet.py:287)")
    p.add_argument("--workers", type=int, default=10, help="decode processes (imagenet) / gather threads (records)")
    p.add_argument("--num-classes", type=int, default=1000, help="synthetic data only")
    p.add_argument("--synthetic-train-size", type=int, default=1281167)
    p.add_argument("--synthetic-val-size", type=int, default=50000)
    p.add_argument("--synthetic-task", default="random", choices=["random", "colour", "mix"],
                   help="random: uniform noise + labels (throughput); colour: learnable class-coloured images; "
                        "mix: overlapping class Gaussians over smooth random bases (Bayes top-1 ~85 %% at 100 classes)")
    p.add_argument("--flip", action="store_true", help="random horizontal flip (reference: none)")
    p.add_argument("--record-resize", action="store_true",
                   help="records stored at another size than --image-size are bilinearly resampled on the GPU "
                        "(fused into the normalise kernel) instead of cropped: e.g. 320^2 records for 448^2 "
                        "training halve the host gather bytes (profiles/loader_throughput.md)")
    # --- optimisation ---
    p.add_argument("--optimizer", default="sgd",
                   choices=["sgd", "lars", "adam", "adamw", "adagrad", "rmsprop", "adadelta", "asgd", "nadam"])
    p.add_argument("--lars-eta", type=float, default=1e-3, help="LARS trust coefficient")
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--wd", "--weight-decay", dest="wd", type=float, default=1e-4)
    p.add_argument("--nesterov", action="store_true")
    p.add_argument("--schedule-decay", type=float, default=4e-3, help="Nadam (Keras) schedule decay")
    p.add_argument("--lr-schedule", default="step", choices=["step", "cosine"])
    p.add_argument("--lr-step", type=int, default=30)
    p.add_argument("--lr-gamma", type=float, default=0.1)
    p.add_argument("--warmup-epochs", type=float, default=0.0)
    p.add_argument("--scale-lr", action="store_true", help="lr *= global_batch / 256")
    p.add_argument("--label-smoothing", type=float, default=0.0)
    p.add_argument("--accum-steps", type=int, default=1, help="gradient accumulation micro-batches")
    # --- parallelism / runtime ---
    p.add_argument("--launcher", default="auto", choices=["auto", "slurm", "torchrun", "single"])
    p.add_argument("--kernels", default="auto", choices=["auto", "hip", "torch"],
                   help="hip = hand-written MI355X kernels; torch = PyTorch ops (oracle / CPU)")
    p.add_argument("--comm", default="auto", choices=["auto", "rccl", "torch", "local"])
    p.add_argument("--device", default=None)
    p.add_argument("--bucket-mb", type=float, default=16.0)
    p.add_argument("--first-bucket-mb", type=float, default=2.0)
    p.add_argument("--grad-allreduce-dtype", default="fp32", choices=["fp32", "bf16"],
                   help="bf16: all-reduce bf16 copies of the gradient buckets (half the xGMI bytes)")
    p.add_argument("--broadcast-buffers", default="eval", choices=["eval", "always", "never"])
    p.add_argument("--no-rebuild-buckets", dest="rebuild_buckets", action="store_false")
    p.add_argument("--pg-timeout", type=float, default=1800.0)
    p.add_argument("--hip-graph", action="store_true",
                   help="capture each training step in a HIP graph and replay it (1 GPU, step LR schedule)")
    p.add_argument("--step-timeout", type=float, default=0.0,
                   help="hang watchdog: if no training / validation step completes for this many seconds, "
                        "dump all stacks, abort the communicators and exit with status 75")
    p.add_argument("--check-consistency", type=int, default=0,
                   help="every N steps verify parameters are bit-identical across ranks")
    # --- logging / checkpoint ---
    p.add_argument("--log-interval", type=int, default=50)
    p.add_argument("--tb-dir", default="imagenet_FR")
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--resume", default=None)
    p.add_argument("--max-steps", type=int, default=0, help="cap train steps per epoch (0 = full)")
    p.add_argument("--max-val-steps", type=int, default=0)
    p.add_argument("--quiet-banner", action="store_true")
    p.add_argument("--profile", default=None, help="write a torch.profiler trace to this dir")
    return p


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    from .train.engine import Trainer
    tr = Trainer(args)
    try:
        if args.profile:
            from .utils.profiling import profiled
            with profiled(args.profile):
                tr.run()
        else:
            tr.run()
    finally:
        tr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
