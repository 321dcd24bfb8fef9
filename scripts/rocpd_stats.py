"""Per-kernel statistics from a rocprofv3 rocpd database (run_results.db): the
--kernel-trace --stats summary as CSV (name, calls, total/avg/min/max ns, VGPR,
SGPR, LDS, scratch), sorted by total time.
Usage: python scripts/rocpd_stats.py <run_results.db> [out.csv]"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", name)  # drop the argument list


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: {"calls": 0, "total": 0, "min": None, "max": 0})
    res = {}
    for name, dur, vgpr, agpr, sgpr, lds, scratch in c.execute(
            "select name, duration, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, scratch_size from kernels"):
        k = short(name)
        a = agg[k]
        a["calls"] += 1
        a["total"] += dur
        a["min"] = dur if a["min"] is None else min(a["min"], dur)
        a["max"] = max(a["max"], dur)
        res[k] = (vgpr, agpr, sgpr, lds, scratch)
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["total"])
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "vgpr", "agpr", "sgpr", "lds_bytes",
                "scratch_bytes"])
    for k, a in rows:
        w.writerow([k, a["calls"], a["total"], round(a["total"] / a["calls"]), a["min"], a["max"], *res[k]])


if __name__ == "__main__":
    main()
