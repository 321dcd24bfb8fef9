#!/usr/bin/env python3
"""bench.py — device-resident row-format encode+decode throughput on MI355X.

Metric (BASELINE.json): "row-format encode+decode GiB/s (device-resident),
64M Struct(100 prim) rows" = (row bytes written by encode + row bytes read by
decode) / (t_encode + t_decode) / 2^30, summed over all ranks.

One step = encode the whole per-GPU batch (columns -> rows, RAW rows =
BinaryRow.toBytes of each object; --frame for the Encoder.encode(MemoryBuffer,T)
frame stream) + decode it back (rows -> columns), inputs resident in HBM.
Multi-GPU: one process per GPU (torchrun), each encodes/decodes its own shard
of records (weak scaling: rows per GPU fixed); no data-path collective — only a
barrier and a MAX of the elapsed time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config struct104|mixed40|nested]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="struct104", choices=["struct104", "mixed40", "mixed40_long", "nested"])
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (default: config size)")
    ap.add_argument("--frame", action="store_true", help="frame-stream mode instead of raw rows")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16, help="host threads of the CPU baseline")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_latest.json"),
                    help="per-launch HBM traffic from a rocprofv3 PMC run of this command")
    return ap.parse_args()


DEFAULT_ROWS = {"struct104": 64 * 1024 * 1024, "mixed40": 16 * 1024 * 1024, "nested": 8 * 1024 * 1024,
                "mixed40_long": 8 * 1024 * 1024}  # mixed40_long: strings 0..128 B (robustness, not a BASELINE config)


def setup_dist(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dist, world, rank, local


def barrier(dist):
    import torch
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()


def make_batch(config, n, row0, device):
    """Device columns + algorithmic byte counts for the config."""
    import torch
    from fury_amd import workloads as W
    from fury_amd.format.columns import to_device
    from fury_amd.format.native import DeviceColumn
    if config == "struct104":
        schema = W.struct_schema()
        vals = W.gen_struct_device(n, seed_base=17 + row0, device=device)
        cols = [DeviceColumn(v, None, None, n) for v in vals]
        col_bytes = sum(v.numel() * v.element_size() for v in vals)
    else:
        mixed = config.startswith("mixed40")
        mk = W.mixed_host_columns if mixed else W.nested_host_columns
        seed = (23 if mixed else 29) + row0
        host = mk(n, seed=seed, max_len=128) if config == "mixed40_long" else mk(n, seed=seed)
        cols = to_device(host, device)
        col_bytes = 0
        for c in host:
            for a in (c.values, c.offsets, c.validity):
                if a is not None:
                    col_bytes += a.nbytes
        # string/item value buffers carry 8 bytes of generator padding: not algorithmic
    torch.cuda.synchronize()
    return schema if config == "struct104" else (W.mixed_schema() if config.startswith("mixed40")
                                                 else W.nested_schema()), cols, col_bytes


def cpu_baseline(config, frame, seconds, threads=1):
    """The oracle (scalar C port of the Java writer/reader) on a bounded sample of the
    workload: `threads` host threads, each with its own encoder state and buffers,
    running encode+decode round trips of the same 200K-record sample (the oracle's C
    calls release the GIL), as the JVM path would run one Encoders.bean encoder per
    core thread."""
    import threading
    from oracle import oracle
    from fury_amd import workloads as W
    if config == "struct104":
        schema = W.struct_schema()
        n = 200_000
        cols = W.struct_host_columns(n)
    elif config.startswith("mixed40"):
        schema, n = W.mixed_schema(), 200_000
        cols = W.mixed_host_columns(n, max_len=128 if config == "mixed40_long" else 32)
    else:
        schema, n = W.nested_schema(), 200_000
        cols = W.nested_host_columns(n)
    oracle.load()
    tallies = [[0, 0] for _ in range(threads)]  # [reps, row bytes] per thread
    t0 = time.perf_counter()

    def worker(k):
        while True:
            buf, offs = oracle.encode(schema, cols, n, 1 if frame else 0)
            oracle.decode(schema, buf, offs, n, 1 if frame else 0)
            tallies[k][0] += 1
            tallies[k][1] += 2 * int(offs[-1])
            if time.perf_counter() - t0 >= seconds:
                break

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    reps = sum(t[0] for t in tallies)
    row_bytes = sum(t[1] for t in tallies)
    return {"value": row_bytes / el / 2**30, "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x (encode+decode) of {n} {config} rows "
                      f"({'frame' if frame else 'raw'}) on {threads} thread(s), "
                      f"oracle/rowfmt_oracle.c scalar per thread, {el:.1f} s",
            "rows_per_s": reps * n / el}


def main():
    args = parse()
    import torch
    dist, world, rank, local = setup_dist(args)
    device = torch.device("cuda", local)
    from fury_amd.format.encoder import RowEncoder
    from fury_amd.format import native

    config = args.config
    n = args.rows or DEFAULT_ROWS[config]
    frame = 1 if args.frame else 0
    schema, cols, col_bytes = make_batch(config, n, rank * n, device)
    enc = RowEncoder(schema, device=device)
    plan = enc.plan
    ws = enc.workspace(n)
    arr = native.column_array(cols)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream

    # output rows (sized once; varlen sizes via the device scan)
    if plan.fixed_width:
        total = n * plan.stride(frame)
        offs = None
    else:
        offs = torch.empty(n + 1, dtype=torch.int64, device=device)
        native.encoded_size(plan, arr, n, frame, offs, ws, stream)
        total = int(offs[n].item())
    out = torch.empty(max(16, total), dtype=torch.uint8, device=device)
    # decode targets
    if plan.fixed_width:
        dcols = enc.alloc_fixed_outputs(n)
    else:
        native.encode(plan, arr, n, frame, offs, out, status, ws, stream)
        dcols = enc.decode(out[:total], n, frame, offs)
    darr = native.column_array(dcols)

    def step(ev=None):
        # events: 0 | encoded_size | 3 | encode | 1 | decode_sizes | 4 | decode | 2
        if ev:
            ev[0].record()
        if not plan.fixed_width:
            native.encoded_size(plan, arr, n, frame, offs, ws, stream)
        if ev:
            ev[3].record()
        native.encode(plan, arr, n, frame, offs, out, status, ws, stream)
        if ev:
            ev[1].record()
        if not plan.fixed_width:
            native.decode_sizes(plan, out, offs, n, frame, darr, status, ws, stream)
        if ev:
            ev[4].record()
        native.decode(plan, out, offs, n, frame, darr, status, ws, stream)
        if ev:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    native.read_status(status, stream)
    # correctness guard on the measured data: decode(encode(x)) == x (fixed-width configs)
    if plan.fixed_width:
        for a, b in zip(dcols, cols):
            if not torch.equal(a.values[:n].view(torch.uint8), b.values.view(torch.uint8)):
                raise SystemExit("round-trip mismatch on the benchmark batch")

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    barrier(dist)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    barrier(dist)
    el = time.perf_counter() - t0
    native.read_status(status, stream)
    t = torch.tensor([el], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    enc_ms = sorted(e[0].elapsed_time(e[1]) for e in evs)
    dec_ms = sorted(e[1].elapsed_time(e[2]) for e in evs)
    enc_avg = sum(enc_ms) / len(enc_ms)
    dec_avg = sum(dec_ms) / len(dec_ms)
    # the encode / decode calls alone (varlen plans: without their sizing passes)
    enc_k = sum(e[3].elapsed_time(e[1]) for e in evs) / len(evs)
    dec_k = sum(e[4].elapsed_time(e[2]) for e in evs) / len(evs)

    row_bytes = total  # per GPU per direction
    value = world * 2 * row_bytes * args.steps / el / 2**30
    # roofline of the dominant kernel: algorithmic bytes (columns + rows) / its avg duration
    algo = col_bytes + row_bytes
    dom, dom_ms = ("encode", enc_k) if enc_k >= dec_k else ("decode", dec_k)
    achieved = algo / (dom_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.pmc) as fh:
            pmc = json.load(fh)
        key = f"{config}:{n}:{frame}"
        if key in pmc:
            traffic = pmc[key].get(dom)
    except (OSError, ValueError):
        pass
    res = {
        "metric": "row-format encode+decode GiB/s (device-resident), 64M Struct(100 prim) rows",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el * 1000 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (java.util.Random per record, as Struct.createPOJO)" if config == "struct104"
                else "synthetic (numpy seeded)",
        "config": {"workload": f"{config} {'frame-stream' if frame else 'raw rows'}, {n} rows per GPU",
                   "rows_per_gpu": n, "row_bytes_total_per_gpu": row_bytes,
                   "column_bytes_per_gpu": col_bytes, "frame_mode": "stream" if frame else "raw",
                   "schema_hash": plan.schema_hash, "parallelism": f"record-sharded x{world}, no collective"},
        "kernels_ms": {"encode_avg": round(enc_avg, 4), "decode_avg": round(dec_avg, 4),
                       "encode_min": round(enc_ms[0], 4), "decode_min": round(dec_ms[0], 4),
                       "encode_call_avg": round(enc_k, 4), "decode_call_avg": round(dec_k, 4)},
        "roofline": {"bound": "hbm", "kernel": dom if plan.fixed_width else dom + " call (sizing pass excluded)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": algo},
        "step_hbm_frac": round(2 * algo / ((enc_avg + dec_avg) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # all host cores of this GPU's share (the box allots 16 per GPU), then one core
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        res["cpu_baseline"] = cpu_baseline(config, frame, args.cpu_seconds, threads)
        single = cpu_baseline(config, frame, args.cpu_seconds / 2, 1)
        res["cpu_baseline"]["single_core"] = {"value": single["value"], "unit": "GiB/s",
                                              "rows_per_s": single["rows_per_s"], "sample": single["sample"]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
