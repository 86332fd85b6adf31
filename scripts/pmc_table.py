"""Per-kernel hardware-counter table from single-purpose rocprofv3 --pmc passes.

python scripts/pmc_table.py OUT.md DIR  (DIR/p0..p4/*.db as scripts/_r5e.sh collects them:
p0 GRBM_GUI_ACTIVE, p1 TCC_HIT_sum TCC_MISS_sum, p2 FETCH_SIZE, p3 WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES,
p4 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS)

Counter passes serialise dispatches: times are stand-alone kernel times (mean over passes). Derived columns:
L2 hit % = TCC_HIT / (TCC_HIT + TCC_MISS); HBM GB/s = (2 x FETCH_SIZE + WRITE_SIZE) / time (on gfx950
FETCH_SIZE reports half the bytes of a wide streaming read, MI355X_MICROARCH.md §HBM); MFMA % = MFMA busy cycles
per SIMD over GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) x 1024 SIMDs; LDS confl/inst; BF16 TFLOP/s.
"""
import collections
import glob
import os
import sqlite3
import sys


def main(out, d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for i in range(5):
        dbs = glob.glob(os.path.join(d, f"p{i}", "*.db"))
        if not dbs:
            continue
        con = sqlite3.connect(dbs[0])
        seen = set()
        for kn, did, cn, v, dur in con.execute(
                "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
            m = agg[kn]
            m[cn] += v
            if did not in seen:
                seen.add(did)
                m[f"dur{i}"] += dur
                m[f"n{i}"] += 1
    rows = []
    for kn, m in agg.items():
        runs = [i for i in range(5) if m[f"n{i}"]]
        dur = sum(m[f"dur{i}"] for i in runs) / len(runs)
        n = sum(m[f"n{i}"] for i in runs) / len(runs)
        r = dict(name=kn.replace("(anonymous namespace)::", "").replace("void ", ""), n=n, dur=dur)
        h, ms = m["TCC_HIT_sum"], m["TCC_MISS_sum"]
        if h + ms:
            r["l2"] = 100.0 * h / (h + ms)
        if m["n2"] and m["n3"]:
            r["hbm"] = 2 * m["FETCH_SIZE"] * 1024 / max(m["dur2"], 1) + m["WRITE_SIZE"] * 1024 / max(m["dur3"], 1)
        if m["GRBM_GUI_ACTIVE"] and m["n3"]:
            r["mfma"] = 100.0 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024) * m["n0"] / m["n3"]
        if m["SQ_INSTS_LDS"]:
            r["lds"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
        if m["SQ_INSTS_VALU_MFMA_MOPS_BF16"] and m["n4"]:
            r["tf"] = m["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / max(m["dur4"], 1) / 1e3
        rows.append(r)
    rows.sort(key=lambda r: -r["dur"])
    tot = sum(r["dur"] for r in rows)
    steps = max((r["n"] for r in rows if "sgd_kernel" in r["name"]), default=1)

    def f(v, fmt):
        return (fmt % v) if v is not None else ""

    lines = [f"Stand-alone kernel times over {steps:g} steps (counter passes serialise dispatches); "
             f"sum {tot / 1e6 / steps:.2f} ms/step.", "",
             "| ms/step | calls/step | avg us | L2 hit % | HBM GB/s | MFMA % | LDS confl/inst | BF16 TF/s | kernel |",
             "|---:|---:|---:|---:|---:|---:|---:|---:|---|"]
    for r in rows[:45]:
        nm = r["name"].split("(")[0][:80]
        lines.append("| %.3f | %.1f | %.1f | %s | %s | %s | %s | %s | `%s` |" % (
            r["dur"] / 1e6 / steps, r["n"] / steps, r["dur"] / r["n"] / 1e3, f(r.get("l2"), "%.0f"),
            f(r.get("hbm"), "%.0f"), f(r.get("mfma"), "%.1f"), f(r.get("lds"), "%.2f"), f(r.get("tf"), "%.0f"), nm))
    text = "\n".join(lines) + "\n"
    with open(out, "w") as fh:
        fh.write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
