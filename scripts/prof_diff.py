"""Per-kernel ms/step difference between two rocprofv3 --kernel-trace databases
(steps delimited by the SGD kernel, first --skip dropped).

    python scripts/prof_diff.py A/run_results.db B/run_results.db [--top 15]
"""
import argparse
import collections
import sqlite3


def load(p, skip):
    c = sqlite3.connect(p)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [r[2] for r in rows if "sgd_kernel" in r[0]]
    lo, hi = marks[skip - 1], marks[-1]
    n = len(marks) - skip
    d = collections.defaultdict(float)
    for nm, s, e in rows:
        if lo < s and e <= hi:
            d[nm[:110]] += (e - s) / n / 1e6
    return d, (hi - lo) / n / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--top", type=int, default=15)
    x = ap.parse_args()
    a, wa = load(x.a, x.skip)
    b, wb = load(x.b, x.skip)
    print(f"wall ms/step {wa:.2f} -> {wb:.2f}; kernel sum {sum(a.values()):.2f} -> {sum(b.values()):.2f}")
    for k in sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, 0) - a.get(k, 0)))[:x.top]:
        print(f"{a.get(k, 0):8.3f} -> {b.get(k, 0):8.3f}  {k}")


if __name__ == "__main__":
    main()
