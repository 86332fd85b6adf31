"""Convergence comparison: the bf16 HIP path vs the fp32 PyTorch path on a learnable task.

ImageNet is not available on the build / GPU boxes, so the reference's published 100-epoch
curve (/root/reference/imagent_sgd.out) cannot be reproduced; this runs the training CLI
(imagenet.py:371-429 semantics) on the ``--synthetic-task colour`` data (one mean colour +
stripe orientation per class, per-pixel noise; train / val from different seeds) for both
``--kernels hip`` (bf16, hand-written kernels, RCCL self-collectives, wgrad side stream) and
``--kernels torch --dtype fp32`` (the PyTorch oracle) with the same seed, and writes the
per-epoch curves side by side as a markdown table.

    python scripts/convergence.py --arch resnet50 --classes 100 --epochs 4 --out profiles/convergence_r50.md

``--task mix`` (default) is the task that can fail: overlapping class Gaussians whose Bayes-optimal top-1 is
~85 % (data/synthetic.py), so the oracle's curve ends below 100 % and every other path is compared with it
point for point (the summary line gives each path's last-epoch top-1 minus the oracle's).
"""

import argparse
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, timeout, extra_env=None):
    env = dict(os.environ, PYTHONPATH=ROOT, **(extra_env or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    t0 = time.time()
    # the child's log is echoed as it arrives (a long run shows progress) and kept for parsing
    p = subprocess.Popen([sys.executable, "-u", "-m", "imagent_amd.cli"] + args, cwd=ROOT, env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    lines = []
    for line in p.stdout:
        lines.append(line)
        sys.stdout.write("    " + line)
        sys.stdout.flush()
        if time.time() - t0 > timeout:
            p.kill()
            break
    rc = p.wait()
    out = "".join(lines)
    if rc != 0:
        sys.stderr.write(out[-4000:])
        raise SystemExit(f"training run failed ({rc}): {' '.join(args)}")
    return out, time.time() - t0


def curve(out):
    first = [float(m) for m in re.findall(r"iter \d+/\d+ loss ([0-9.naninf]+)", out)]
    summ = [(float(a), float(b)) for a, b in re.findall(r"Train loss: ([0-9.e+-]+) ; Test loss: ([0-9.e+-]+)", out)]
    top1 = [float(v) for v in re.findall(r"; Test top1 accuracy: ([0-9.e+-]+)", out)]
    return first, summ, top1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--image-size", type=int, default=64)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--steps-per-epoch", type=int, default=200)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variant", action="append", default=None,
                    help="extra run 'label|cli args|ENV=V,ENV2=V' (diagnostics), compared with the oracle")
    ap.add_argument("--warmup-epochs", type=float, default=0.0)
    ap.add_argument("--task", default="mix", choices=["mix", "colour"],
                    help="mix: overlapping class Gaussians (Bayes top-1 ~85 %% at 100 classes; can tell numerics "
                         "apart); colour: the easy task every path saturates")
    ap.add_argument("--paths", default="gram,pergemm,fp8",
                    help="HIP runs besides 'hip bf16' and the oracle: gram (every bottleneck in the Gram form, "
                         "IMAGENT_GRAM_MIN_ROWS=0), pergemm (IMAGENT_BN_GRAM=0), fp8 (--dtype fp8, Gram form)")
    a = ap.parse_args()
    base = ["--arch", a.arch, "--image-size", str(a.image_size), "--data", "synthetic", "--synthetic-task", a.task,
            "--num-classes", str(a.classes), "--batch-size", str(a.batch_size),
            "--synthetic-train-size", str(a.batch_size * a.steps_per_epoch), "--synthetic-val-size", "2048",
            "--lr", str(a.lr), "--epochs", str(a.epochs), "--log-interval", "20", "--quiet-banner", "--tb-dir", "",
            "--warmup-epochs", str(a.warmup_epochs)]
    rows = {}
    runs = [("hip bf16", ["--kernels", "hip"], {}), ("torch fp32", ["--kernels", "torch", "--dtype", "fp32"], {})]
    named = {"gram": ("hip bf16, every bottleneck Gram-form", ["--kernels", "hip"], {"IMAGENT_GRAM_MIN_ROWS": "0"}),
             "pergemm": ("hip bf16, per-op bn3 (IMAGENT_BN_GRAM=0)", ["--kernels", "hip"], {"IMAGENT_BN_GRAM": "0"}),
             "fp8": ("hip fp8, every bottleneck Gram-form", ["--kernels", "hip", "--dtype", "fp8"],
                     {"IMAGENT_GRAM_MIN_ROWS": "0"})}
    for k in [p for p in a.paths.split(",") if p]:
        runs.append(named[k])
    for v in a.variant or []:
        label, cli, envs = (v.split("|") + ["", ""])[:3]
        runs.append((label, cli.split(), dict(e.split("=", 1) for e in envs.split(",") if e)))
    for name, extra, env in runs:
        out, secs = run(base + extra, a.timeout, env)
        rows[name] = curve(out) + (secs,)
        print(f"{name}: {secs:.0f} s, first {rows[name][0][:3]}, epochs {rows[name][1]}, top1 {rows[name][2]}",
              flush=True)
    lines = [f"# Convergence: {a.arch}, bf16 HIP path vs fp32 PyTorch path (learnable synthetic task)", "",
             f"`python scripts/convergence.py --arch {a.arch} --classes {a.classes} --epochs {a.epochs} "
             f"--batch-size {a.batch_size} --steps-per-epoch {a.steps_per_epoch} --image-size {a.image_size} "
             f"--lr {a.lr}` on 1x MI355X: the training CLI, same seed and data for both paths "
             f"(`--synthetic-task {a.task}`, {a.classes} classes, {a.image_size}x{a.image_size}, "
             f"{a.steps_per_epoch} steps of {a.batch_size} per epoch, 2048 validation images from another seed). "
             "ImageNet parity with the reference's 100-epoch curve stays unpinned (no dataset here).", "",
             "| epoch | hip bf16 train loss | hip val loss | hip val top1 % | torch fp32 train loss | torch val loss "
             "| torch val top1 % |", "|---:|---:|---:|---:|---:|---:|---:|"]
    h, t = rows["hip bf16"], rows["torch fp32"]
    lines.append(f"| 0 (first logged interval) | {h[0][0]:.4f} | | | {t[0][0]:.4f} | | |")
    for e in range(min(len(h[1]), len(t[1]))):
        lines.append(f"| {e + 1} | {h[1][e][0]:.4f} | {h[1][e][1]:.4f} | {h[2][e]:.2f} | {t[1][e][0]:.4f} | "
                     f"{t[1][e][1]:.4f} | {t[2][e]:.2f} |")
    lines += ["", f"Wall time of the whole run (incl. start-up and validation): hip {h[3]:.0f} s, torch {t[3]:.0f} s.", ""]
    if len(runs) > 2:
        lines += ["Further runs (validation top1 % per epoch; train loss of the last epoch):", "",
                  "| run | first interval loss | val top1 per epoch | last train loss |", "|---|---:|---|---:|"]
        for name, _, _ in runs:
            f, sm, t1, _ = rows[name]
            lines.append(f"| {name} | {f[0]:.3f} | {' / '.join(f'{v:.1f}' for v in t1)} | {sm[-1][0]:.4f} |")
        lines.append("")
    o1 = t[2][-1] if t[2] else float("nan")
    lines += [f"Last-epoch val top-1 minus the fp32 oracle's ({o1:.2f} %):", ""]
    for name, _, _ in runs:
        if name != "torch fp32" and rows[name][2]:
            lines.append(f"* {name}: {rows[name][2][-1] - o1:+.2f} points")
    lines.append("")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
