"""Per-box summary of scripts/r06/gpu_box.sh probes: enc_ab times per variant and the PMC
pass's per-launch averages of the encode / decode v5 kernels (write requests, write stalls
at the memory side, wave-wait cycles). Usage: python scripts/r06/box_summary.py DIR..."""
import collections
import csv
import json
import os
import sys

for d in sys.argv[1:]:
    runs = [json.loads(l) for l in open(os.path.join(d, "enc_ab.jsonl")) if l.startswith("{")]
    bus = runs[0]["bus"] if runs else "?"
    print(f"== {d} (bus {bus})")
    for r in runs:
        print(f"   {r['variant']:45s} {r['ms']:8.3f} ms")
    f = os.path.join(d, "counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "_v5_kernel" not in name:
            continue
        agg[name.replace("void fory_amd::(anonymous namespace)::", "").split("(")[0]][r["Counter_Name"]].append(
            float(r["Counter_Value"]))
    for k, c in sorted(agg.items()):
        m = {n: sum(v) / len(v) for n, v in c.items()}
        wr = m.get("TCC_EA0_WRREQ_sum", 0)
        st = m.get("TCC_EA0_WRREQ_STALL_sum", 0)
        wa, wc = m.get("SQ_WAIT_ANY", 0), m.get("SQ_WAVE_CYCLES", 0)
        print(f"   {k:60s} wrreq {wr / 1e6:7.1f} M  wr_stall {st / 1e6:7.1f} M ({st / max(wr, 1):.3f}/req)  "
              f"wait_any/wave_cycles {wa / max(wc, 1):.3f}")
