"""Per-queue / per-stream view of a rocprofv3 --kernel-trace database: which
hardware queue each stream's kernels ran on, busy time per stream per step,
and how much of the weight-gradient stream's time overlapped the main stream.

    python scripts/stream_timeline.py gpurun_out/prof/run_results.db [--marker sgd_kernel] [--skip 3] [--kernels 30]

``--kernels N``: also a per-stream kernel table (the N largest kernels of each stream by in-step time), so the
main stream's critical-path ranking is not mixed with the side-stream weight gradients.
"""
import argparse
import collections
import sqlite3


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def inter(a, b):
    return union(a) + union(b) - union(a + b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--kernels", type=int, default=0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    marks = [r[2] for r in rows if a.marker in r[0]]
    lo, hi = marks[a.skip - 1], marks[-1]
    nsteps = len(marks) - a.skip
    rows = [r for r in rows if lo < r[1] and r[2] <= hi]
    by = collections.defaultdict(list)
    sq = collections.defaultdict(set)
    names = collections.defaultdict(collections.Counter)
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0]))
    for n, s, e, st, q in rows:
        k = per[st][n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:100]]
        k[0] += e - s
        k[1] += 1
        by[st].append((s, e))
        sq[st].add(q)
        names[st][n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]] += 1
    wall = (hi - lo) / nsteps / 1e6
    print(f"{nsteps} steps, wall {wall:.2f} ms/step")
    main_st = max(by, key=lambda k: len(by[k]))
    for st, iv in sorted(by.items(), key=lambda kv: -len(kv[1])):
        top = ", ".join(f"{k} x{v // nsteps}" for k, v in names[st].most_common(3))
        ov = inter(iv, by[main_st]) / nsteps / 1e6 if st != main_st else float("nan")
        print(f"stream {st} queues {sorted(sq[st])}: {len(iv) // nsteps} kernels/step, busy "
              f"{union(iv) / nsteps / 1e6:.2f} ms/step, overlapped with main {ov:.2f} ms/step | {top}")
    allv = [x for v in by.values() for x in v]
    print(f"GPU busy (any stream) {union(allv) / nsteps / 1e6:.2f} ms/step")
    if a.kernels:
        for st, iv in sorted(by.items(), key=lambda kv: -len(kv[1])):
            tot = sum(v[0] for v in per[st].values()) / nsteps / 1e6
            print(f"\nstream {st}: kernel sum {tot:.2f} ms/step\n\n| ms/step | calls/step | avg us | kernel |\n|---:|---:|---:|---|")
            for k, (t, cnt) in sorted(per[st].items(), key=lambda kv: -kv[1][0])[: a.kernels]:
                print(f"| {t / nsteps / 1e6:.3f} | {cnt // nsteps} | {t / cnt / 1e3:.1f} | `{k}` |")


if __name__ == "__main__":
    main()
