"""Per-step kernel table of the validation forward in a ``bench.py --eval N`` rocprofv3 --kernel-trace run:
the validation steps are the kernels after the last training step's SGD launch, split at the cross-entropy
forward launches (one per validation step).

    python scripts/eval_prof_summary.py gpurun_out/prof_eval/ev_results.db [--skip 2] > profiles/...md
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--title", default="ResNet-50 validation forward")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    last_sgd = max(i for i, r in enumerate(rows) if "sgd_kernel" in r[0])
    ev = rows[last_sgd + 1:]
    cuts = [i for i, r in enumerate(ev) if "xent_fwd" in r[0]]
    steps = []
    lo = 0
    for cix in cuts:
        steps.append(ev[lo:cix + 1])
        lo = cix + 1
    steps = steps[a.skip:]
    n = len(steps)
    agg = collections.defaultdict(lambda: [0, 0])
    wall = 0
    for st in steps:
        wall += st[-1][2] - st[0][1]
        for nm, s, e in st:
            k = nm.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:110]
            agg[k][0] += e - s
            agg[k][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"# {a.title}\n")
    print(f"{n} validation steps (after {a.skip} skipped): wall {wall / n / 1e6:.2f} ms/step, kernel sum "
          f"{tot / n / 1e6:.2f} ms/step, {sum(v[1] for v in agg.values()) // n} launches/step, "
          f"{sum(v[1] for k, v in agg.items() if 'at::native' in k) // max(n, 1)} ATen launches/step\n")
    print("| ms/step | calls/step | avg us | kernel |\n|---:|---:|---:|---|")
    for k, (t, cnt) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"| {t / n / 1e6:.3f} | {cnt / n:.1f} | {t / cnt / 1e3:.1f} | `{k}` |")


if __name__ == "__main__":
    main()
