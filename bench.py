#!/usr/bin/env python3
"""bench.py — device-resident row-format encode+decode throughput on MI355X.

Metric (BASELINE.json): "row-format encode+decode GiB/s (device-resident),
64M Struct(100 prim) rows" = (row bytes written by encode + row bytes read by
decode) / (t_encode + t_decode) / 2^30, summed over all ranks.

One step = encode every record of the job (columns -> rows; RAW rows =
BinaryRow.toBytes of each object, --frame for the Encoder.encode(MemoryBuffer,T)
frame stream) + decode it back (rows -> columns), inputs resident in HBM.

Struct104 (default): BASELINE config C4 — a FIXED total of 256Mi records
(strong scaling), split into contiguous per-rank ranges (fury_amd.shard), no
data-path collective. A rank processes its range in resident windows of at most
64Mi records (the 64M-row headline batch; 256Mi rows' columns + rows + decoded
columns would need 565 GB, a window needs 141 GB of the 288 GB HBM), so at N=1
a step is 4 windows of the headline batch, at N=4 one, at N=8 one 32Mi window.
Every window is a full encode + decode of 64Mi (32Mi) records; a rank's windows
reuse one set of resident columns (the byte shuffle's memory traffic does not
depend on the values of a fixed-width schema). A second timed loop reports the
weak-scaling extra (64Mi records per rank, one window) under "weak".

Multi-GPU: `python bench.py --gpus N` starts `torch.distributed.run` with N
ranks as a child process (before anything touches the GPU) and exits with its
code; under torchrun (WORLD_SIZE set) each rank takes cuda:LOCAL_RANK. Fewer
visible GPUs than N is an error, never a silent 1-GPU run. Timing: barrier +
synchronize on both sides, MAX of the elapsed time over ranks.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
                       [--config struct104|mixed40|mixed40_long|nested] [--frame]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MI = 1024 * 1024


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="struct104", choices=["struct104", "mixed40", "mixed40_long", "nested"])
    ap.add_argument("--total-rows", type=int, default=0,
                    help="records of the whole job, split over the ranks (default: C4 256Mi for struct104, "
                         "the config size for the varlen configs)")
    ap.add_argument("--rows", type=int, default=0, help="(compat) records per GPU: total = rows x gpus")
    ap.add_argument("--window-rows", type=int, default=64 * MI, help="max resident records per rank window")
    ap.add_argument("--weak-rows", type=int, default=64 * MI,
                    help="records per rank of the weak-scaling extra (struct104; 0 = skip)")
    ap.add_argument("--frame", action="store_true", help="frame-stream mode instead of raw rows")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group backend (gloo: rehearsal of the multi-rank path)")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow more ranks than visible GPUs (rank -> cuda:(local_rank %% count)); rehearsal only")
    ap.add_argument("--init-dist", action="store_true",
                    help="initialise the process group even for one rank (rehearses the RCCL branch on a 1-GPU box)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extras", type=int, default=-1,
                    help="struct104: also time BASELINE C2/C3 (Mixed 16Mi, Nested 8Mi; raw + frame) in the same run "
                         "(-1 = at N=1 only, 0 = off, 1 = on)")
    ap.add_argument("--extra-steps", type=int, default=5)
    ap.add_argument("--extra-warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16, help="host threads of the CPU baseline")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_latest.json"),
                    help="per-launch HBM traffic from a rocprofv3 PMC run of this command")
    return ap.parse_args()


DEFAULT_TOTAL = {"struct104": 256 * MI, "mixed40": 16 * MI, "nested": 8 * MI,
                 "mixed40_long": 8 * MI}  # mixed40_long: strings 0..128 B (robustness, not a BASELINE config)


_LINE_OUT = sys.stdout


def launch_ranks(args) -> int:
    """Parent of an N-rank run: torchrun as a child process (no GPU touched here;
    device_count() does not initialise the GPU)."""
    import socket
    import torch
    have = torch.cuda.device_count()
    if have < args.gpus and not args.oversubscribe:
        print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible; refusing to measure fewer ranks",
              file=sys.stderr)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def setup_dist(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    have = torch.cuda.device_count()
    if have < world and not args.oversubscribe:
        raise SystemExit(f"bench.py: {world} ranks but only {have} GPU(s) visible")
    dev = local % max(1, have)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1 or args.init_dist:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
        # n_gpus = ranks that actually initialised
        one = torch.ones(1, dtype=torch.int64, device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(one)
        if int(one.item()) != world:
            raise SystemExit("bench.py: not every rank initialised")
    return dist, world, rank, dev


def device_identity(dev: int) -> dict:
    """This rank's device: ordinal and PCI bus id (hipDeviceGetPCIBusId), so that a
    multi-GPU line proves its ranks ran on distinct GPUs."""
    import ctypes
    import torch
    ident = {"ordinal": dev, "pci_bus_id": None}
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, dev) == 0:
            ident["pci_bus_id"] = buf.value.decode()
    except OSError:
        pass
    props = torch.cuda.get_device_properties(dev)
    ident["name"] = props.name
    uuid = getattr(props, "uuid", None)
    if uuid is not None:
        ident["uuid"] = str(uuid)
    return ident


def check_devices(devices, oversubscribe: bool):
    """A multi-rank line must come from distinct GPUs: two ranks on one device (same
    PCI bus id, or the same ordinal when no id is known) is an error unless the run is
    an explicit --oversubscribe rehearsal. Returns an error string or None."""
    keys = [d.get("pci_bus_id") or f"ordinal:{d.get('ordinal')}" for d in devices]
    if len(set(keys)) < len(keys) and not oversubscribe:
        return f"{len(keys)} ranks ran on {len(set(keys))} distinct device(s): {keys}"
    return None


def gather_devices(dist, ident, world):
    if dist is None:
        return [ident]
    out = [None] * world
    dist.all_gather_object(out, ident)
    return out


def barrier(dist):
    import torch
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(dist, x: float, backend: str) -> float:
    import torch
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_batch(config, n, row0, device):
    """Device columns + algorithmic column byte count for the config."""
    import torch
    from fury_amd import workloads as W
    from fury_amd.format.columns import to_device
    from fury_amd.format.native import DeviceColumn
    if config == "struct104":
        schema = W.struct_schema()
        vals = W.gen_struct_device(n, seed_base=17 + row0, device=device)
        cols = [DeviceColumn(v, None, None, n) for v in vals]
        col_bytes = sum(v.numel() * v.element_size() for v in vals)
        torch.cuda.synchronize()
        return schema, cols, col_bytes
    mixed = config.startswith("mixed40")
    seed = (23 if mixed else 29) + row0
    if mixed:
        cols = W.mixed_device_columns(n, seed=seed, device=device, max_len=128 if config == "mixed40_long" else 32)
    else:
        cols = W.nested_device_columns(n, seed=seed, device=device)
    col_bytes = 0
    for c in cols:
        for a in (c.offsets, c.validity):
            if a is not None:
                col_bytes += a.numel() * a.element_size()
        if c.values is not None:
            col_bytes += c.values.numel() * c.values.element_size()
            if c.offsets is not None:  # string bytes: 8 bytes of generator padding are not algorithmic
                col_bytes -= 8
    torch.cuda.synchronize()
    return (W.mixed_schema() if mixed else W.nested_schema()), cols, col_bytes


def prefix_cols(cols, n):
    """The first n records of fixed-width device columns (views, no copy)."""
    from fury_amd.format.native import DeviceColumn
    return [DeviceColumn(c.values[:n], None, None if c.validity is None else c.validity, n) for c in cols]


def check_round_trip(plan, cols, dcols, n):
    """decode(encode(x)) == x on the measured batch: values, offsets, validity of every column."""
    import torch
    from fury_amd.format.types import ArrowType
    for i, (a, b) in enumerate(zip(cols, dcols)):
        f = plan.fields[i]
        k = a.length
        if b.length != k:
            return f"column {i}: length {b.length} != {k}"
        if a.offsets is not None:
            if not torch.equal(a.offsets[:k + 1].to(torch.int64), b.offsets[:k + 1].to(torch.int64)):
                return f"column {i}: offsets differ"
        if a.values is not None and f.type.id != ArrowType.STRUCT:
            if f.type.id in (ArrowType.STRING, ArrowType.BINARY):
                nb = int(a.offsets[k].item()) if k > 0 else 0
            else:
                nb = k * a.values.element_size()
            va = a.values.view(torch.uint8)[:nb]
            vb = b.values.view(torch.uint8)[:nb]
            if f.nullable and a.validity is not None and f.type.id not in (ArrowType.STRING, ArrowType.BINARY):
                # null slots decode to 0; compare valid slots only
                w = a.values.element_size()
                bits = torch.arange(k, device=a.values.device)
                valid = ((a.validity[bits // 8] >> (bits % 8).to(torch.uint8)) & 1).bool()
                mask = valid.repeat_interleave(w)
                va, vb = va[mask], vb[mask]
            if not torch.equal(va, vb):
                return f"column {i}: values differ"
        if f.nullable and a.validity is not None and k > 0:
            bits = torch.arange(k, device=a.validity.device)
            ga = (a.validity[bits // 8] >> (bits % 8).to(torch.uint8)) & 1
            gb = (b.validity[bits // 8] >> (bits % 8).to(torch.uint8)) & 1
            if not torch.equal(ga, gb):
                return f"column {i}: validity differs"
    return None


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


def jdk_probe():
    """The reference's own CPU path needs a JVM (java/fory-format); record what the box has."""
    java = shutil.which("java")
    out = {"java": java, "javac": shutil.which("javac")}
    if java:
        try:
            r = subprocess.run([java, "-version"], capture_output=True, text=True, timeout=20)
            out["version"] = (r.stderr or r.stdout).strip().splitlines()[0] if (r.stderr or r.stdout) else ""
        except (OSError, subprocess.SubprocessError) as e:
            out["version"] = f"probe failed: {e}"
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.init_dist):
        sys.exit(launch_ranks(args))
    # the JSON line is the only thing on stdout: RCCL's init banner and gloo's connection
    # notices are written to fd 1 by native code, so fd 1 is pointed at stderr for the run
    # and the line goes to a saved copy of the original stdout
    global _LINE_OUT
    sys.stdout.flush()
    _LINE_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    dist, world, rank, dev = setup_dist(args)
    device = torch.device("cuda", dev)
    devices = gather_devices(dist, device_identity(dev), world)
    bad_devices = check_devices(devices, args.oversubscribe)
    if bad_devices:
        raise SystemExit(f"bench.py: {bad_devices}; refusing to report a multi-GPU line")
    from fury_amd.format.encoder import RowEncoder
    from fury_amd.format import native
    from fury_amd.shard import shard_range

    config = args.config
    frame = 1 if args.frame else 0
    total_rows = args.total_rows or (args.rows * world if args.rows else DEFAULT_TOTAL[config])
    b, e = shard_range(total_rows, world, rank)
    share = e - b
    fixed = config == "struct104"
    window = min(args.window_rows, share) if fixed else share
    nwin = (share + window - 1) // window if window > 0 else 0
    weak_rows = args.weak_rows if fixed else 0
    alloc = max(window, weak_rows)
    schema, cols_all, col_bytes_all = make_batch(config, alloc, b, device)
    enc = RowEncoder(schema, device=device)
    plan = enc.plan
    ws = enc.workspace(alloc)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream

    # ------------------------------------------------------------------ fixed width
    if plan.fixed_width:
        stride = plan.stride(frame)
        out = torch.empty(max(16, alloc * stride), dtype=torch.uint8, device=device)
        dcols_all = enc.alloc_fixed_outputs(alloc)
        col_row = col_bytes_all // alloc  # column bytes per record (624 for Struct104)
        # windows of this rank's share: (records, input cols, output cols)
        wins = []
        left = share
        while left > 0:
            m = min(window, left)
            wins.append(m)
            left -= m
        arrs = {}

        def arrays(m):
            if m not in arrs:
                arrs[m] = (native.column_array(prefix_cols(cols_all, m)), native.column_array(prefix_cols(dcols_all, m)))
            return arrs[m]

        def step(evs=None):
            for j, m in enumerate(wins):
                a_in, a_out = arrays(m)
                ev = evs[j] if evs is not None else None
                if ev:
                    ev[0].record()
                native.encode(plan, a_in, m, frame, None, out, status, ws, stream)
                if ev:
                    ev[1].record()
                native.decode(plan, out, None, m, frame, a_out, status, ws, stream)
                if ev:
                    ev[2].record()

        for _ in range(args.warmup):
            step()
        native.read_status(status, stream)
        if wins:
            bad = check_round_trip(plan, prefix_cols(cols_all, wins[0]), prefix_cols(dcols_all, wins[0]), wins[0])
            if bad:
                raise SystemExit(f"round-trip mismatch on the benchmark batch: {bad}")
        evs = [[[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in wins] for _ in range(args.steps)]
        recs = [(m, ev) for step_evs in evs for m, ev in zip(wins, step_evs)]
        barrier(dist)
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(evs[k])
        barrier(dist)
        el = max_over_ranks(dist, time.perf_counter() - t0, args.backend)
        native.read_status(status, stream)
        enc_ms = [ev[0].elapsed_time(ev[1]) for _, ev in recs]
        dec_ms = [ev[1].elapsed_time(ev[2]) for _, ev in recs]
        # dominant kernel: per-launch algorithmic bytes / average launch time (full windows)
        wmax = max(wins) if wins else 0
        full = [i for i, (m, _) in enumerate(recs) if m == wmax]
        enc_avg = sum(enc_ms[i] for i in full) / max(1, len(full))
        dec_avg = sum(dec_ms[i] for i in full) / max(1, len(full))
        algo = wmax * (col_row + stride)
        dom, dom_ms = ("encode", enc_avg) if enc_avg >= dec_avg else ("decode", dec_avg)
        achieved = algo / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        value = 2 * total_rows * stride * args.steps / el / 2**30
        res_weak = None
        if weak_rows > 0:  # weak-scaling extra: weak_rows records per rank, one window
            a_in, a_out = arrays(weak_rows)
            for _ in range(max(1, args.warmup // 2)):
                native.encode(plan, a_in, weak_rows, frame, None, out, status, ws, stream)
                native.decode(plan, out, None, weak_rows, frame, a_out, status, ws, stream)
            barrier(dist)
            t1 = time.perf_counter()
            for _ in range(args.steps):
                native.encode(plan, a_in, weak_rows, frame, None, out, status, ws, stream)
                native.decode(plan, out, None, weak_rows, frame, a_out, status, ws, stream)
            barrier(dist)
            elw = max_over_ranks(dist, time.perf_counter() - t1, args.backend)
            native.read_status(status, stream)
            res_weak = {"value": round(world * 2 * weak_rows * stride * args.steps / elw / 2**30, 3),
                        "unit": "GiB/s", "scaling": "weak", "rows_per_gpu": weak_rows,
                        "ms_per_step": round(elw * 1000 / args.steps, 4)}
        row_bytes_step = total_rows * stride
        res = {
            "metric": "row-format encode+decode GiB/s (device-resident), 64M Struct(100 prim) rows",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1000 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (java.util.Random per record, as Struct.createPOJO)",
            "config": {"workload": f"struct104 {'frame-stream' if frame else 'raw rows'}: BASELINE C4, "
                                   f"{total_rows} records split over {world} rank(s), windows of <= "
                                   f"{args.window_rows} records (the 64M-row headline batch); each rank generates "
                                   f"one window of {wmax} records and encodes + decodes it {len(wins)} time(s) "
                                   f"per step (its share), the columns resident in HBM",
                       "total_rows": total_rows, "rows_per_gpu": share, "windows_per_gpu": len(wins),
                       "window_rows": wmax, "row_bytes_total": row_bytes_step,
                       "column_bytes_per_record": col_row, "frame_mode": "stream" if frame else "raw",
                       "schema_hash": plan.schema_hash,
                       "parallelism": f"record-sharded x{world} (contiguous ranges), no collective"},
            "kernels_ms": {"encode_avg": round(enc_avg, 4), "decode_avg": round(dec_avg, 4),
                           "encode_min": round(min(enc_ms), 4) if enc_ms else None,
                           "decode_min": round(min(dec_ms), 4) if dec_ms else None},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "frac_basis": "hipEvent time of the launch (average over the timed windows)",
                         "trace": trace_frac(args.pmc, config, wmax, frame, dom, algo),
                         "traffic": pmc_traffic(args.pmc, config, wmax, frame, dom),
                         "traffic_source": "profiles/pmc_latest.json (rocprofv3 --pmc pass of this command, "
                                           "same lib_sha16; null when the build differs)",
                         "algorithmic_bytes_per_launch": algo},
            "lib_sha16": lib_sha16(),
            "step_hbm_frac": round(2 * algo / ((enc_avg + dec_avg) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if enc_avg + dec_avg > 0 else None,
        }
        if res_weak:
            res["weak"] = res_weak
    # ------------------------------------------------------------------ varlen
    else:
        res = measure_varlen(args, config, frame, total_rows, dist, world, device, args.steps, args.warmup,
                             batch=(schema, cols_all, col_bytes_all, enc, ws, status, stream))
        res = {"metric": METRIC, **res}
    if plan.fixed_width and config == "struct104" and extras_on(args, world):
        # BASELINE C2 / C3 (Mixed 16Mi, Nested 8Mi), raw rows and frame streams decoded from the
        # stream alone: timed in the same default run, so the driver observes them too; the
        # headline line above is unchanged by them (measured before, in its own batch)
        del cols_all, dcols_all, out, arrs
        torch.cuda.empty_cache()
        res["extra_configs"] = []
        for cfg in ("mixed40", "nested"):
            for fr in (0, 1):
                x = measure_varlen(args, cfg, fr, DEFAULT_TOTAL[cfg], dist, world, device, args.extra_steps,
                                   args.extra_warmup)
                res["extra_configs"].append(x)
                torch.cuda.empty_cache()
    res["devices"] = devices
    if args.oversubscribe:
        res["oversubscribed"] = True
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # all host cores of this GPU's share (the box allots 16 per GPU), then one core
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        res["cpu_baseline"] = cpu_baseline(config, frame, args.cpu_seconds, threads)
        single = cpu_baseline(config, frame, args.cpu_seconds / 2, 1)
        res["cpu_baseline"]["single_core"] = {"value": single["value"], "unit": "GiB/s",
                                              "rows_per_s": single["rows_per_s"], "sample": single["sample"]}
        res["cpu_baseline"]["reference_jvm"] = jdk_probe()
    if rank == 0:
        print(json.dumps(res), file=_LINE_OUT, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


METRIC = "row-format encode+decode GiB/s (device-resident), 64M Struct(100 prim) rows"


def extras_on(args, world) -> bool:
    """C2 / C3 lines beside the headline: on by default at N = 1 (the driver's BENCH run);
    --extras 1 forces them on multi-GPU runs too, --extras 0 off."""
    return args.extras == 1 or (args.extras < 0 and world == 1)


def measure_varlen(args, config, frame, total_rows, dist, world, device, steps, warmup, batch=None):
    """One varlen config (Mixed / Nested): every timed step = encoded_size + encode, then
    [frame index +] decode_sizes + decode of this rank's share, inputs resident in HBM;
    HIP events on the launch stream around each call. Returns the line's fields."""
    import torch
    from fury_amd.format.encoder import RowEncoder
    from fury_amd.format import native
    from fury_amd.shard import shard_range
    rank = dist.get_rank() if dist is not None else 0
    b, e = shard_range(total_rows, world, rank)
    n = e - b
    if batch is None:
        schema, cols, col_bytes = make_batch(config, n, b, device)
        enc = RowEncoder(schema, device=device)
        ws = enc.workspace(n)
        status = torch.zeros(1, dtype=torch.int32, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
    else:
        schema, cols, col_bytes, enc, ws, status, stream = batch
    plan = enc.plan
    arr = native.column_array(cols)
    offs = torch.empty(n + 1, dtype=torch.int64, device=device)
    native.encoded_size(plan, arr, n, frame, offs, ws, stream)
    total = int(offs[n].item())
    out = torch.empty(max(16, total), dtype=torch.uint8, device=device)
    native.encode(plan, arr, n, frame, offs, out, status, ws, stream)
    dcols = enc.decode(out[:total], n, frame, offs)
    darr = native.column_array(dcols)

    # frame streams decode from the stream alone (a receiver has no row offsets):
    # the device frame index (fory_rowfmt_index_frames) runs inside the decode
    ioffs, iws = offs, None
    if frame:
        ioffs = torch.empty(n + 1, dtype=torch.int64, device=device)
        iws = torch.empty(max(256, native.index_workspace_bytes(plan, n, total)), dtype=torch.uint8,
                          device=device)

    def step(ev=None):
        # events: 0 | encoded_size | 3 | encode | 1 | index_frames | 5 | decode_sizes | 4 | decode | 2
        if ev:
            ev[0].record()
        native.encoded_size(plan, arr, n, frame, offs, ws, stream)
        if ev:
            ev[3].record()
        native.encode(plan, arr, n, frame, offs, out, status, ws, stream)
        if ev:
            ev[1].record()
        if frame:
            native.index_frames(plan, out, total, n, frame, ioffs, status, iws, stream)
        if ev:
            ev[5].record()
        native.decode_sizes(plan, out, ioffs, n, frame, darr, status, ws, stream)
        if ev:
            ev[4].record()
        native.decode(plan, out, ioffs, n, frame, darr, status, ws, stream)
        if ev:
            ev[2].record()

    for _ in range(warmup):
        step()
    native.read_status(status, stream)
    bad = check_round_trip(plan, cols, dcols, n)
    if bad:
        raise SystemExit(f"round-trip mismatch on the benchmark batch: {bad}")
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(steps)]
    barrier(dist)
    t0 = time.perf_counter()
    for k in range(steps):
        step(evs[k])
    barrier(dist)
    el = max_over_ranks(dist, time.perf_counter() - t0, args.backend)
    native.read_status(status, stream)
    enc_avg = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs)  # sizes + scan + encode
    dec_avg = sum(e[1].elapsed_time(e[2]) for e in evs) / len(evs)  # [index] + decode_sizes + decode
    idx_avg = sum(e[1].elapsed_time(e[5]) for e in evs) / len(evs)  # frame index (stream mode)
    enc_k = sum(e[3].elapsed_time(e[1]) for e in evs) / len(evs)    # encode call alone
    dec_k = sum(e[4].elapsed_time(e[2]) for e in evs) / len(evs)    # decode call alone
    algo = col_bytes + total
    dom, dom_ms = ("encode", enc_avg) if enc_avg >= dec_avg else ("decode", dec_avg)
    achieved = algo / (dom_ms * 1e-3) / 1e9
    row_bytes_all = total
    if dist is not None:
        t = torch.tensor([float(total)], dtype=torch.float64,
                         device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(t)
        row_bytes_all = int(t.item())
    value = 2 * row_bytes_all * steps / el / 2**30
    res = {
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(el * 1000 / steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch generator on the device, seeded; uniform string / list lengths as the config)",
        "config": {"workload": f"{config} {'frame-stream (decoded from the stream alone)' if frame else 'raw rows'}, "
                               f"{total_rows} records split over {world} rank(s)",
                   "total_rows": total_rows, "rows_per_gpu": n, "row_bytes_total_per_gpu": total,
                   "column_bytes_per_gpu": col_bytes, "frame_mode": "stream" if frame else "raw",
                   "schema_hash": plan.schema_hash,
                   "parallelism": f"record-sharded x{world} (contiguous ranges), no collective"},
        "kernels_ms": {"encode_avg": round(enc_avg, 4), "decode_avg": round(dec_avg, 4),
                       "encode_call_avg": round(enc_k, 4), "decode_call_avg": round(dec_k, 4),
                       "frame_index_avg": round(idx_avg, 4) if frame else None},
        "roofline": {"bound": "hbm", "kernel": dom + " (sizing passes included)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "call_frac": {"encode": round(algo / (enc_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "decode": round(algo / (dec_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                     "frac_basis": "hipEvent time of the calls incl. sizing passes (call_frac: the call alone)",
                     "trace": trace_frac(args.pmc, config, n, frame, "encode" if enc_k >= dec_k else "decode", algo),
                     "traffic": pmc_traffic(args.pmc, config, n, frame, dom),
                     "traffic_source": "profiles/pmc_latest.json (rocprofv3 --pmc pass of this command, "
                                       "same lib_sha16; null when the build differs)",
                     "algorithmic_bytes_per_launch": algo},
        "lib_sha16": lib_sha16(),
        "step_hbm_frac": round(2 * algo / ((enc_avg + dec_avg) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
    }
    return res


def lib_sha16() -> str:
    """Identity of the product library build that runs (sha256 of libfory_rowfmt.so)."""
    import hashlib
    from fury_amd import _lib
    try:
        with open(_lib.LIB_PATH, "rb") as fh:
            return hashlib.sha256(fh.read()).hexdigest()[:16]
    except OSError:
        return ""


def pmc_traffic(path, config, n, frame, dom):
    """Per-launch HBM bytes of the dominant kernel from a stored rocprofv3 PMC pass —
    only when that pass measured THIS library build (entry's lib_sha16); else null."""
    try:
        with open(path) as fh:
            pmc = json.load(fh)
        key = f"{config}:{n}:{frame}"
        ent = pmc.get(key)
        if ent and ent.get("lib_sha16") and ent.get("lib_sha16") == lib_sha16():
            return ent.get(dom)
    except (OSError, ValueError):
        pass
    return None


def trace_frac(path, config, n, frame, kern, algo):
    """The same fraction from the rocprofv3 kernel trace of this command (average launch
    duration of the call's main kernel, profiles/*/rocprof_kernel_stats.csv) when that
    trace measured THIS library build; else null. The stamped entry names the kernel."""
    try:
        with open(path) as fh:
            ent = json.load(fh).get(f"{config}:{n}:{frame}")
        if not ent or ent.get("lib_sha16") != lib_sha16():
            return None
        ms = (ent.get("trace_ms") or {}).get(kern)
        if not ms:
            return None
        return {"kernel": ent.get(kern + "_kernel"), "avg_ms": ms,
                "frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "source": ent.get("trace_source")}
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    main()
