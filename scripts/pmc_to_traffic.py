"""profiles/pmc_latest.json from a scripts/profile.sh summary: per-launch HBM bytes of the
bench's encode and decode kernels = FETCH_SIZE*1024*2 (gfx950 half-count correction,
MI355X_MICROARCH.md §HBM; calibrated here: it equals the algorithmic read bytes exactly)
+ WRITE_SIZE*1024, and the kernel trace's average launch duration of the same kernels
(trace_ms). Usage: python scripts/pmc_to_traffic.py SUMMARY KEY [OUT [TRACE_SOURCE]]
Each entry is stamped with lib_sha16 (the profiled libfory_rowfmt.so): bench.py reports
the traffic only when the running build has the same hash."""
import hashlib
import json
import os
import sys

summ = json.load(open(sys.argv[1]))
key = sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_latest.json"
try:
    cur = json.load(open(out))
except (OSError, ValueError):
    cur = {}
ent = {}
for name, e in summ["pmc"].items():
    if "<spill>" in name:
        continue
    role = "encode" if name.startswith("encode") or name.startswith("var_encode") else \
        "decode" if name.startswith("decode") or name.startswith("var_decode_kernelILb1") or \
        name == "var_decode_flat_kernel<pass2>" else None
    if role and "fetch_bytes_x2" in e and "write_bytes" in e:
        ent[role] = int(e["fetch_bytes_x2"] + e["write_bytes"])
        ent[role + "_kernel"] = name
        ent[role + "_fetch_bytes_x2"] = int(e["fetch_bytes_x2"])
        ent[role + "_write_bytes"] = int(e["write_bytes"])
# the kernel trace of the same command (profile.sh's first pass): average launch duration
# of each role's kernel, read by bench.py's roofline "trace" (trace_frac)
kern = summ.get("kernels", {})
tr = {}
for role in ("encode", "decode"):
    k = ent.get(role + "_kernel")
    if k and k in kern:
        tr[role] = round(kern[k]["avg_ns"] / 1e6, 4)
if tr:
    ent["trace_ms"] = tr
    ent["trace_source"] = sys.argv[4] if len(sys.argv) > 4 else os.path.dirname(sys.argv[1])
lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fury_amd", "lib", "libfory_rowfmt.so")
ent["lib_sha16"] = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
cur[key] = ent
json.dump(cur, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps(ent))
