"""Per-call roofline table of every conv kernel call in a training step.

Joins the conv call log that ``IMAGENT_CONV_LOG=<path>`` makes ops/conv.py write (one JSON line
per conv call: op, GEMM shape, flags, how many conv kernels it dispatched) with a rocprofv3
``--kernel-trace`` database of the SAME run: conv dispatches in dispatch order are assigned to
the logged calls in call order (every call's kernels are launched from the one host thread, so
dispatch ids follow the call order), steps are delimited by the fused SGD kernel.

Floors per call (the verdict's definitions): FLOP floor at the dense bf16 MFMA peak
(2.5 PFLOP/s), byte floor at 8 TB/s over the operand bytes the call must move at least once
(gathered input, weights, output; + the fused epilogue's operands: BN-backward x / y-mask bits / x2, the
accumulated old output). "roof" = max of the two, "of roof" = roof / achieved, "above roof" =
achieved - roof, the table is ranked by it (where the time is).

    IMAGENT_CONV_LOG=gpurun_out/convlog.jsonl rocprofv3 --kernel-trace -d gpurun_out/prof -o run \\
        --output-format rocpd -- python3 bench.py --steps 3 --warmup 2
    python scripts/conv_roofline.py gpurun_out/convlog.jsonl gpurun_out/prof/run_results.db > profiles/x.md
"""

from __future__ import annotations

import argparse
import collections
import json
import sqlite3

PEAK_FLOPS = 2.5e15
PEAK_BYTES = 8e12
CONV_KERNELS = ("igemm_", "conv_stream_kernel", "halo3x3_kernel", "wgrad_")


def flops_bytes(r):
    if r["op"].startswith("conv wgrad"):
        k = r["KH"] * r["KW"] * r["C"]
        fl = 2.0 * r["M"] * r["Co"] * k
        by = r["M"] * r["Co"] * 2 + r["N"] * r["H"] * r["W"] * r["C"] * 2 + r["Co"] * k * 4 * 2
        return fl, by
    k = r["taps"] * r["C"]
    fl = 2.0 * r["M"] * r["Nout"] * k
    xb = r["N"] * r["H"] * r["W"] * r["C"] * 2
    if r.get("sY", 1) > 1:  # one parity class of a strided dgrad: its share of the gathered input
        xb /= r["sY"] * r["sY"]
    yb = r["M"] * r["Nout"] * (4 if r["flags"] & 1 else 2)
    by = xb + r["Nout"] * k * 2 + yb
    if r["flags"] & 8:  # accumulate: the old output is read
        by += yb
    if r.get("bnb"):  # BN-backward epilogue reads x (+ the output's ReLU mask bits, + x2 of the second branch)
        by += yb * (1 + r.get("y2", False) / 16 + r.get("x2", False))
    return fl, by


def shape_str(r):
    if r["op"].startswith("conv wgrad"):
        return f"{r['C']}->{r['Co']} {r['KH']}x{r['KW']}/s{r['stride']} @{r['H']}"
    s = f"K {r['taps']}x{r['C']} -> {r['Nout']}, M {r['M']} ({r['OH']}x{r['OW']})"
    tags = [t for t, on in (("stats", r.get("stats")), ("bnb", r.get("bnb")), ("acc", r["flags"] & 8),
                            ("xbn", r.get("xbn")), ("par", r.get("sY", 1) > 1)) if on]
    return s + (" [" + ",".join(tags) + "]" if tags else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=2, help="steps to drop (warm-up)")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--title", default="per-call conv roofline")
    a = ap.parse_args()
    recs = [json.loads(l) for l in open(a.log)]
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, dispatch_id, start, end, stream_id from kernels order by dispatch_id").fetchall()
    conv = [r for r in rows if any(k in r[0] for k in CONV_KERNELS) and "fixup" not in r[0]]
    need = sum(r["kernels"] for r in recs)
    if need != len(conv):
        raise SystemExit(f"log has {need} conv dispatches, trace {len(conv)}: not the same run?")
    marks = [r[1] for r in rows if a.marker in r[0]]
    # assign dispatches to calls
    calls = []
    i = 0
    for r in recs:
        ks = conv[i:i + r["kernels"]]
        i += r["kernels"]
        if not ks:
            continue
        step = sum(1 for m in marks if m < ks[0][1])
        calls.append((step, r, ks))
    by_step = collections.defaultdict(list)
    for st, r, ks in calls:
        by_step[st].append((r, ks))
    steps = [s for s in sorted(by_step) if s >= a.skip and s < len(marks)]
    if not steps:
        raise SystemExit("no complete step after --skip")
    n = len(by_step[steps[0]])
    agg = []
    for j in range(n):
        r, ks = by_step[steps[0]][j]
        us = sum(sum((k[3] - k[2]) for k in by_step[s][j][1]) for s in steps if len(by_step[s]) == n) / len(steps) / 1e3
        fl, by = flops_bytes(r)
        tf, tb = fl / PEAK_FLOPS * 1e6, by / PEAK_BYTES * 1e6
        roof = max(tf, tb)
        names = sorted({k[0].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0] for k in ks})
        agg.append(dict(j=j, op=r["op"].replace("conv ", ""), shape=shape_str(r), kern=" + ".join(names), us=us,
                        tflop=fl / us / 1e6 if us else 0, flop_us=tf, byte_us=tb, roof=roof,
                        frac=roof / us if us else 0, excess=us - roof, side=r["stream"]))
    tot = sum(x["us"] for x in agg)
    tot_roof = sum(x["roof"] for x in agg)
    print(f"# {a.title}\n")
    print(f"{len(steps)} steps averaged; {n} conv calls per step; kernel time {tot / 1e3:.2f} ms/step, "
          f"sum of per-call roofs {tot_roof / 1e3:.2f} ms/step ({100 * tot_roof / tot:.0f} % of roof overall). "
          f"Floors: {PEAK_FLOPS / 1e15:.1f} PFLOP/s dense bf16, {PEAK_BYTES / 1e12:.0f} TB/s HBM. Times are in-step "
          "kernel durations (the weight-gradient stream overlaps the main one, so concurrent kernels share "
          "the chip).\n")
    print("| # | op | GEMM shape | kernel | us | TFLOP/s | FLOP floor us | byte floor us | of roof | above roof us |")
    print("|---:|---|---|---|---:|---:|---:|---:|---:|---:|")
    for x in sorted(agg, key=lambda x: -x["excess"]):
        print(f"| {x['j']} | {x['op']} | {x['shape']} | `{x['kern']}` | {x['us']:.1f} | {x['tflop']:.0f} | "
              f"{x['flop_us']:.1f} | {x['byte_us']:.1f} | {100 * x['frac']:.0f} % | {x['excess']:.1f} |")
    # per-kernel rollup
    kk = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for x in agg:
        kk[x["kern"]][0] += x["us"]
        kk[x["kern"]][1] += x["roof"]
        kk[x["kern"]][2] += 1
    print("\n| kernel | calls | ms/step | roof ms | of roof |")
    print("|---|---:|---:|---:|---:|")
    for k, (u, rf, cnt) in sorted(kk.items(), key=lambda t: -t[1][0]):
        print(f"| `{k}` | {cnt} | {u / 1e3:.2f} | {rf / 1e3:.2f} | {100 * rf / u:.0f} % |")


if __name__ == "__main__":
    main()
