"""Summarise a rocprofv3 ``--kernel-trace`` run as a per-step markdown table.

Accepts the SQLite database rocprofv3 writes by default (``*_results.db``) or a
``--stats`` ``kernel_stats.csv``. With the database, training steps are
delimited by a marker kernel (default: the fused SGD update, one launch per
step); the first ``--skip`` steps are dropped and the table reports per-step
kernel time, wall time between markers and GPU busy time (union of kernel
intervals) -- busy == wall means the step is GPU-bound, not launch-bound.

    python scripts/prof_summary.py gpurun_out/prof/run_results.db --title "..." \
        > profiles/r50_b256_v3_kernel_stats.md
"""

from __future__ import annotations

import argparse
import collections
import csv
import glob
import sqlite3


def _short(name: str, n: int = 100) -> str:
    return name if len(name) <= n else name[:n] + "..."


def from_db(path: str, marker: str, skip: int):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [r[2] for r in rows if marker in r[0]]
    if len(marks) < skip + 2:
        raise SystemExit(f"need >= {skip + 2} '{marker}' launches, found {len(marks)}")
    marks = marks[skip:]
    t0, t1 = marks[0], marks[-1]
    ks = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    nsteps = len(marks) - 1
    busy, cs, ce = 0, None, None
    for _, s, e in ks:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e in ks:
        agg[n][0] += 1
        agg[n][1] += e - s
    table = [(n, cnt, tot) for n, (cnt, tot) in agg.items()]
    head = (f"{nsteps} steps after {skip} skipped: wall {(t1 - t0) / nsteps / 1e6:.2f} ms/step, GPU busy "
            f"{busy / nsteps / 1e6:.2f} ms/step, kernel sum {sum(t for _, _, t in table) / nsteps / 1e6:.2f} "
            f"ms/step, {len(ks) / nsteps:.0f} launches/step")
    return table, nsteps, head


def from_csv(path: str, steps: float):
    rows = list(csv.DictReader(open(path)))
    table = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in rows]
    return table, steps, f"{steps:g} profiled steps (counts include warmup)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="rocprofv3 *_results.db or kernel_stats.csv (glob ok)")
    ap.add_argument("--steps", type=float, default=0, help="csv only: steps the counts cover")
    ap.add_argument("--marker", default="sgd_kernel", help="db only: one launch per step")
    ap.add_argument("--skip", type=int, default=3, help="db only: warmup steps to drop")
    ap.add_argument("--title", default="rocprofv3 --kernel-trace")
    ap.add_argument("--note", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    paths = glob.glob(a.path, recursive=True)
    if not paths:
        raise SystemExit(f"no file matches {a.path}")
    if paths[0].endswith(".db"):
        table, nsteps, head = from_db(paths[0], a.marker, a.skip)
    else:
        table, nsteps, head = from_csv(paths[0], a.steps)
    tot = sum(t for _, _, t in table)
    print(f"# {a.title}\n")
    if a.note:
        print(a.note + "\n")
    print(head + "\n")
    print("| ms/step | % | calls/step | avg us | kernel |\n|---:|---:|---:|---:|---|")
    table.sort(key=lambda r: -r[2])
    for name, cnt, t in table[: a.top]:
        print(f"| {t / nsteps / 1e6:.3f} | {100 * t / tot:.2f} | {cnt / nsteps:g} | {t / cnt / 1e3:.1f} | "
              f"`{_short(name)}` |")


if __name__ == "__main__":
    main()
