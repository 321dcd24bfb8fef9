"""Per-kernel times of one encode per shape from a rocprofv3 run_results.db of
scripts/bench_nested_shapes.py (diagnostic)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, grid_x / workgroup_x, (end - start) / 1e3 from kernels order by start"))
short = lambda n: n.split("(anonymous namespace)::")[-1].split("(")[0][:34]
idx = [i for i, r in enumerate(rows) if "tc_write_fields_kernel<true>" in r[0] or "tc_write_coll" in r[0]]
for k in idx[5::6]:  # the last encode of each shape
    s = k
    while s > 0 and any(t in rows[s - 1][0] for t in ("tc_", "scan", "copyBuffer")):
        s -= 1
    e = k
    while e + 1 < len(rows) and "tc_write" in rows[e + 1][0]:
        e += 1
    tot = 0.0
    for r in rows[s:e + 1]:
        print(f"  {short(r[0]):36s} {r[1]:8d} {r[2]:9.1f}")
        tot += r[2]
    print(f"  total {tot:.1f} us\n")
