"""Summarise a scripts/profile.sh run: per-kernel avg duration (kernel trace) and
per-launch counter values (PMC passes). HBM bytes follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE/WRITE_SIZE are in KB; gfx950 FETCH_SIZE reads 1/2 of a 16-B/lane
streaming read (x2 applied as 'fetch_bytes_x2'; other widths uncalibrated)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]


def rows(pattern):
    for f in glob.glob(os.path.join(root, pattern), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def short(name):
    import re
    m = re.search(r"(encode_fixed_\w*?kernel|decode_fixed_\w*?kernel|var_encode_kernel|var_decode_kernelILb[01]|"
                  r"var_encode_tile_kernel|var_decode_tile_kernelILb[01]|var_encode_flat\d?_lean_kernel|var_encode_flat\d?_kernel|"
                  r"var_decode_flat_kernel|"
                  r"var_sizes_kernel|scan_\w+?_kernel|fill_offsets_kernel|frame_\w+?_kernel|flat_tile_bases_kernel|"
                  r"gen_\w+?_kernel)", name)
    if m:
        k = m.group(1)
        t = re.search(r"var_(?:en|de)code_flat_(?:lean_)?kernel<([^>]*)>", name)  # (v7 / v9 have no spill form)
        if t and t.group(1).split(",")[-1].strip() == "true":
            k += "<spill>"  # the small big-image launch: kept apart from the main launch's averages
            if k.startswith("var_decode_flat_kernel"):
                k = "var_decode_flat_kernel<spill>"
            return k
        if k.startswith("var_decode") and not k.endswith(("0", "1")):
            if k == "var_decode_flat_kernel":
                m2 = re.search(r"var_decode_flat_kernel<(\d+|true|false), (true|false)", name)
                k += "<pass2>" if (m2 and m2.group(2) == "true") else "<pass1>"
            else:
                k += "ILb1" if "<true>" in name else ("ILb0" if "<false>" in name else "")
        return k
    return name[:60]


out = {"kernels": {}, "pmc": {}}
stats = [r for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)
         if "pmc_" not in os.path.relpath(f, root) for r in csv.DictReader(open(f))]
for r in stats:
    out["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                        "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
# per-kernel resources from the kernel trace (VGPR / AGPR / SGPR, LDS, scratch, workgroup)
out["resources"] = {}
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    if "pmc_" in os.path.relpath(f, root):
        continue
    for r in csv.DictReader(open(f)):
        k = short(r.get("Kernel_Name", ""))
        if k in out["resources"]:
            continue
        out["resources"][k] = {c: r[c] for c in r
                               if any(t in c for t in ("VGPR", "SGPR", "LDS", "Scratch", "Segment", "Workgroup_Size"))}
acc = defaultdict(lambda: defaultdict(list))
for d in glob.glob(os.path.join(root, "pmc_*")):
    if not os.path.isdir(d):
        continue
    for r in rows(os.path.relpath(d, root) + "/**/*counter_collection.csv"):
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    e = {c: sum(v) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in e:
        e["fetch_bytes"] = e["FETCH_SIZE"] * 1024
        e["fetch_bytes_x2"] = e["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in e:
        e["write_bytes"] = e["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in e and e["SQ_WAVE_CYCLES"] > 0:  # where the waves' time goes (quad-cycles)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in e:
                e[c + "_frac"] = e[c] / e["SQ_WAVE_CYCLES"]
    if "SQ_LDS_IDX_ACTIVE" in e and e["SQ_LDS_IDX_ACTIVE"] > 0 and "SQ_LDS_BANK_CONFLICT" in e:
        e["lds_bank_conflict_frac"] = e["SQ_LDS_BANK_CONFLICT"] / e["SQ_LDS_IDX_ACTIVE"]
    out["pmc"][k] = e
print(json.dumps(out, indent=1))
