"""Per-step wall times and the largest idle gaps between kernels in a
rocprofv3 kernel-trace database (step marker: the fused SGD kernel)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
ends = [i for i, r in enumerate(rows) if "sgd_kernel" in r[0]]
print("step walls (ms):", [round((rows[ends[k]][2] - rows[ends[k - 1]][2]) / 1e6, 2) for k in range(1, len(ends))])
s = rows[ends[-2] + 1:ends[-1] + 1]
busy_end = s[0][2]
gaps = []
for b in s[1:]:
    g = (b[1] - busy_end) / 1e3
    if g > 100:
        gaps.append((round(g), b[0][:60]))
    busy_end = max(busy_end, b[2])
print("idle gaps > 100 us before:", sorted(gaps, reverse=True)[:12])
