"""Per-kernel PMC counter sums (and derived ratios) from rocprofv3 --pmc databases.

    python scripts/pmc_kernels.py gpurun_out/pmcA/run_results.db [more.db ...] [--grep igemm]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in a.dbs:
        con = sqlite3.connect(p)
        seen = set()
        for kn, did, cn, v, dur in con.execute(
                "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
            if a.grep not in kn:
                continue
            kn = kn.replace("(anonymous namespace)::", "").replace("void ", "")[:90]
            agg[kn][cn] += v
            if (p, did) not in seen:
                seen.add((p, did))
                agg[kn]["_dur_ns"] += dur
                agg[kn]["_n"] += 1
    for kn, m in agg.items():
        print(f"== {kn}  (dispatches {m['_n']:.0f}, mean {m['_dur_ns'] / max(m['_n'], 1) / 1e3:.1f} us)")
        w = m.get("SQ_WAVE_CYCLES")
        for cn in sorted(m):
            if cn.startswith("_"):
                continue
            extra = f"  ({100 * m[cn] / w:.1f} % of wave cycles)" if w and cn.startswith("SQ_WAIT") or (
                w and cn.startswith("SQ_ACTIVE")) else ""
            print(f"   {cn:28s} {m[cn]:.4g}{extra}")
        if m.get("GRBM_GUI_ACTIVE") and m.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            print(f"   MFMA util {100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.1f} %")
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
            t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            print(f"   L2 hit rate {100 * m['TCC_HIT_sum'] / max(t, 1):.1f} %")


if __name__ == "__main__":
    main()
