"""Per-kernel HBM bytes per training step from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB per
dispatch), e.g. scripts/_r8p.sh's output:

python scripts/pmc_bytes_table.py FETCH.csv WRITE.csv [--top 40]

Steps are counted by the optimizer kernel (one `sgd_kernel` launch per step); every dispatch in the file is
averaged over them. Times are the PMC runs' own (dispatches serialised by the profiler, so no stream overlap):
bytes / time is a kernel's stand-alone HBM rate.
"""

import argparse
import collections
import csv


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


# FETCH_SIZE counts half of the bytes read on MI355X / ROCm 7 (profiles/hbm_roof.md: calibrated on kernels that move a
# known 1 GiB: FETCH_SIZE 524,305 for 1,048,576 KiB read; WRITE_SIZE exact in KiB)
FETCH_UNIT = 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    fr, wr = load(a.fetch), load(a.write)
    steps = sum(1 for n, _, _ in fr if short(n) == "sgd_kernel") or 1
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0])
    for n, v, t in fr:
        g = agg[short(n)]
        g[0] += 1
        g[1] += v * FETCH_UNIT
        g[3] += t
    for n, v, _ in wr:
        agg[short(n)][2] += v * 1024
    tot_f = sum(g[1] for g in agg.values()) / steps
    tot_w = sum(g[2] for g in agg.values()) / steps
    tot_t = sum(g[3] for g in agg.values()) / steps
    print(f"{steps} steps; per step: fetched {tot_f / 1e9:.1f} GB, written {tot_w / 1e9:.1f} GB, "
          f"kernel time (serialised) {tot_t / 1e6:.1f} ms -> {(tot_f + tot_w) / tot_t / 1e3:.2f} TB/s average\n")
    print("| GB/step (read + write) | read | write | calls/step | ms/step (serialised) | TB/s | kernel |")
    print("|---:|---:|---:|---:|---:|---:|---|")
    for n, g in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:a.top]:
        c, f, w, t = g[0] / steps, g[1] / steps, g[2] / steps, g[3] / steps
        print(f"| {(f + w) / 1e9:.2f} | {f / 1e9:.2f} | {w / 1e9:.2f} | {c:.1f} | {t / 1e6:.3f} | "
              f"{(f + w) / max(t, 1) / 1e3:.2f} | `{n}` |")


if __name__ == "__main__":
    main()
