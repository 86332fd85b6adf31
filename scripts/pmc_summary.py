"""Summarise rocprofv3 ``--pmc`` SQLite databases into one per-kernel markdown table.

Usage: python scripts/pmc_summary.py OUT.md FETCH.db WRITE_MFMA.db LDS.db

The three databases are three rocprofv3 --pmc passes (see scripts/pmc_passes.sh; rocprofv3 cannot
collect all counters in one pass).  Counters are joined on kernel name and summed
over dispatches.  Derived columns (MI355X: 8 XCDs, 256 CUs x 4 SIMDs):

  HBM GB/s   = FETCH_SIZE KiB / time(pass 1) + WRITE_SIZE KiB / time(pass 2)
  MFMA util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
               (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy counts per SIMD)
  LDS confl  = SQ_LDS_BANK_CONFLICT extra cycles per LDS instruction (SQ_INSTS_LDS)
  BF16 TF    = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 FLOP / time(pass 3)

Kernel times under --pmc are serialised dispatches (no overlap between the
compute and weight-gradient streams), so they read as stand-alone kernel times.
"""
import collections
import sqlite3
import sys


def load(path, idx, agg):
    con = sqlite3.connect(path)
    seen = set()
    for kn, did, cn, v, dur in con.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        m = agg[kn]
        m[cn] += v
        if did not in seen:
            seen.add(did)
            m["dur%d" % idx] += dur
            m["n%d" % idx] += 1


def main(out, paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for i, p in enumerate(paths):
        load(p, i, agg)
    rows = []
    for kn, m in agg.items():
        runs = [i for i in range(len(paths)) if m["n%d" % i]]
        dur = sum(m["dur%d" % i] for i in runs) / len(runs)  # ns, mean over passes
        n = sum(m["n%d" % i] for i in runs) / len(runs)
        r = {"name": kn, "n": n, "dur": dur}
        if m["n0"] and m["n1"]:
            r["hbm"] = (m["FETCH_SIZE"] * 1024 / max(m["dur0"], 1)
                        + m["WRITE_SIZE"] * 1024 / max(m["dur1"], 1))  # bytes/ns = GB/s
        if m["GRBM_GUI_ACTIVE"]:
            r["mfma"] = 100.0 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if m["SQ_INSTS_LDS"]:
            r["lds"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
        if m["SQ_INSTS_VALU_MFMA_MOPS_BF16"] and m["n2"]:
            r["tf"] = m["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / max(m["dur2"], 1) / 1e3
        rows.append(r)
    rows.sort(key=lambda r: -r["dur"])
    tot = sum(r["dur"] for r in rows)

    def f(v, fmt):
        return (fmt % v) if v is not None else ""

    lines = [
        "| total ms | % | calls | avg us | HBM GB/s | MFMA util % | LDS confl/inst | BF16 TFLOP/s | kernel |",
        "|---:|---:|---:|---:|---:|---:|---:|---:|---|",
    ]
    for r in rows[:40]:
        name = r["name"].replace("(anonymous namespace)::", "")
        name = name[:90] + ("..." if len(name) > 90 else "")
        lines.append("| %.3f | %.1f | %d | %.1f | %s | %s | %s | %s | `%s` |" % (
            r["dur"] / 1e6, 100 * r["dur"] / tot, r["n"], r["dur"] / r["n"] / 1e3,
            f(r.get("hbm"), "%.0f"), f(r.get("mfma"), "%.1f"), f(r.get("lds"), "%.2f"),
            f(r.get("tf"), "%.0f"), name))
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines[:32]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
