"""Seed sweep of the trainer-test configuration: HIP bf16 vs the PyTorch fp32 oracle vs PyTorch bf16 autocast.

One CLI run per (path, seed) on the same task (R18, 64 px, synthetic 'colour', batch 32 by default); per run the
logged-interval losses, the per-epoch train / validation means and top-1 are collected, and the table reports,
per path, how often a run passes through a loss spike (an interval loss above ln 10 after the first
logged interval: worse than chance) and the distribution of the last-epoch numbers. This tells a numerics
defect (one path spiking far more often than the others) from the task's own chaotic early phase (all paths
alike). Reference hot loop: /root/reference/imagenet.py:113-131.

    python scripts/seed_sweep.py --seeds 0-5 --out gpurun_out/sweep -- --lr 0.05
"""

from __future__ import annotations

import argparse
import json
import math
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = ["--arch", "resnet18", "--image-size", "64", "--data", "synthetic", "--synthetic-task", "colour",
        "--num-classes", "10", "--batch-size", "32", "--synthetic-train-size", str(32 * 150),
        "--synthetic-val-size", "1024", "--lr", "0.05", "--log-interval", "10", "--quiet-banner", "--tb-dir", "",
        "--warmup-epochs", "0.5", "--epochs", "2"]
PATHS = {"hip_bf16": ["--kernels", "hip"], "torch_fp32": ["--kernels", "torch", "--dtype", "fp32"],
         "torch_bf16": ["--kernels", "torch", "--dtype", "bf16"],
         # the HIP path with a device synchronise after every step (no CPU run-ahead) / weight gradients on the main
         # stream: A/B arms for cross-step and cross-stream ordering
         "hip_sync": ["--kernels", "hip"], "hip_nowgs": ["--kernels", "hip"]}
PATH_ENV = {"hip_sync": {"IMAGENT_STEP_SYNC": "1"}, "hip_nowgs": {"IMAGENT_WGRAD_OVERLAP": "0"}}


def parse(out: str):
    iters = [float(m) for m in re.findall(r"iter \d+/\d+ loss ([0-9.naninf]+)", out)]
    summ = [(float(a), float(b)) for a, b in re.findall(r"Train loss: ([0-9.e+-]+|nan|inf) ; Test loss: ([0-9.e+-]+|nan|inf)", out)]
    top1 = [float(v) for v in re.findall(r"; Test top1 accuracy: ([0-9.e+-]+)", out)]
    return iters, summ, top1


def seeds_of(s: str):
    if "-" in s:
        a, b = s.split("-")
        return list(range(int(a), int(b) + 1))
    return [int(v) for v in s.split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0-5")
    ap.add_argument("--paths", default="hip_bf16,torch_fp32,torch_bf16")
    ap.add_argument("--out", required=True)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    os.makedirs(a.out, exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    rows = []
    for seed in seeds_of(a.seeds):
        for path in a.paths.split(","):
            args = BASE + PATHS[path] + ["--seed", str(seed)] + rest
            r = subprocess.run([sys.executable, "-u", "-m", "imagent_amd.cli"] + args, cwd=a.out,
                               env=dict(env, **PATH_ENV.get(path, {})),
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=a.timeout)
            with open(os.path.join(a.out, f"{path}_s{seed}.log"), "w") as f:
                f.write(r.stdout)
            if r.returncode != 0:
                raise SystemExit(f"{path} seed {seed} failed:\n{r.stdout[-3000:]}")
            iters, summ, top1 = parse(r.stdout)
            spike = max(iters[1:]) if len(iters) > 1 else float("nan")
            row = dict(path=path, seed=seed, iters=iters, epochs=summ, top1=top1, max_interval_after_first=spike,
                       spiked=bool(spike > math.log(10)))
            rows.append(row)
            print(f"[sweep] {path:10s} seed {seed}: epochs {summ} top1 {top1} max interval {spike:.3f}", flush=True)
    with open(os.path.join(a.out, "sweep.json"), "w") as f:
        json.dump(dict(args=BASE + rest, rows=rows), f)
    print("\n| path | runs | runs with a spike > ln 10 | last-epoch train mean > 0.6 | last-epoch train mean (median, max) | "
          "epoch-1 val loss (median, max) | last-epoch val top-1 (min) |")
    print("|---|---|---|---|---|---|---|")
    for path in a.paths.split(","):
        rs = [r for r in rows if r["path"] == path]
        last = [r["epochs"][-1][0] for r in rs]
        v1 = [r["epochs"][0][1] for r in rs]
        t1 = [r["top1"][-1] for r in rs]
        print(f"| {path} | {len(rs)} | {sum(r['spiked'] for r in rs)} | {sum(v > 0.6 for v in last)} | "
              f"{statistics.median(last):.3f}, "
              f"{max(last):.3f} | {statistics.median(v1):.3g}, {max(v1):.3g} | {min(t1):.1f} |")


if __name__ == "__main__":
    main()
