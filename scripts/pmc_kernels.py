"""Per-kernel means of rocprofv3 --pmc counters (csv output, one or more pass dirs):
{kernel: {counter: mean per dispatch, "dispatches": n}}, plus derived ratios when the
SQ wave-time counters are present (WAIT_ANY / WAVE_CYCLES, ACTIVE_INST_ANY / WAVE_CYCLES)
and HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, KB -> bytes; MI355X_MICROARCH.md §HBM).
Usage: python scripts/pmc_kernels.py <dir> [<dir> ...] > summary.json"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("fory_amd::", "")
    return re.sub(r"\(.*\)$", "", name)


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = short(r.get("Kernel_Name", ""))
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = max(len(v) for v in cs.values())
        wc = row.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in row:
                    row[c + "/WAVE_CYCLES"] = round(row[c] / wc, 3)
        if "FETCH_SIZE" in row or "WRITE_SIZE" in row:
            row["hbm_bytes"] = 2 * 1024 * row.get("FETCH_SIZE", 0) + 1024 * row.get("WRITE_SIZE", 0)
        out[k] = row
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
