"""Schemas and synthetic inputs of the BASELINE.json configs.

S  Struct104: java/benchmark/.../data/Struct.java:136-175 —
   Struct.createStructClass(100, false) declares numFields/4+1 = 26 groups of
   {int, long, float, double} named f0..f103; values per record come from
   java.util.Random drawn in declaration order (Struct.createPOJO :112-134),
   here seeded per record with seed_base + row (seed_base 17 as in the reference).
M  Mixed: 32 fixed (11 int, 11 long, 10 double) + 8 String fields f{5k}.
N  Nested: Outer{a: long, b: double, c: Inner}, Inner{x: int, y: long, z: List<Long>}.
Schema order is the Java one: fields sorted by name (Descriptor.java:415-423).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from .format.columns import HostColumn, pack_validity
from .format.infer import _java_compare_key
from .format.types import ArrowType, DataType, DataTypes, Field, Schema

_STRUCT_KINDS = [ArrowType.INT32, ArrowType.INT64, ArrowType.FLOAT, ArrowType.DOUBLE]
_NP = {ArrowType.INT32: np.int32, ArrowType.INT64: np.int64, ArrowType.FLOAT: np.float32,
       ArrowType.DOUBLE: np.float64}


def sorted_names(names: Sequence[str]) -> List[str]:
    return sorted(names, key=_java_compare_key)


# ---------------------------------------------------------------------------
# S: the benchmark Struct
# ---------------------------------------------------------------------------
def struct_decl(num_fields: int = 100):
    """Declared (name, type_id) list of Struct.createStructClass(numFields, false)."""
    out = []
    for i in range(num_fields // 4 + 1):
        for k in range(4):
            out.append((f"f{i * 4 + k}", _STRUCT_KINDS[k]))
    return out


def struct_schema(num_fields: int = 100, boxed: bool = False) -> Schema:
    decl = dict(struct_decl(num_fields))
    return Schema([Field(n, DataType(decl[n]), boxed) for n in sorted_names(decl)])


def struct_schema_order(num_fields: int = 100) -> List[int]:
    """schema position -> declared index."""
    decl = [n for n, _ in struct_decl(num_fields)]
    pos = {n: i for i, n in enumerate(decl)}
    return [pos[n] for n in sorted_names(decl)]


_MULT = np.uint64(0x5DEECE66D)
_ADD = np.uint64(0xB)
_MASK = np.uint64((1 << 48) - 1)


def _jr_next(seed: np.ndarray, bits: int):
    seed = (seed * _MULT + _ADD) & _MASK
    v = (seed >> np.uint64(48 - bits)).astype(np.int64)
    if bits == 32:
        v = v.astype(np.uint32).view(np.int32).astype(np.int64)
    return seed, v


def gen_struct_host(n: int, num_fields: int = 100, seed_base: int = 17, row0: int = 0) -> List[np.ndarray]:
    """Declared-order columns, java.util.Random(seed_base + row) per record (numpy, vectorised)."""
    rows = np.arange(row0, row0 + n, dtype=np.int64) + seed_base
    seed = (rows.astype(np.uint64) ^ _MULT) & _MASK
    out = []
    with np.errstate(over="ignore"):
        for _, kind in struct_decl(num_fields):
            if kind == ArrowType.INT32:  # nextInt = next(32)
                seed, v = _jr_next(seed, 32)
                out.append(v.astype(np.int32))
            elif kind == ArrowType.INT64:  # nextLong = ((long)next(32) << 32) + next(32)
                seed, hi = _jr_next(seed, 32)
                seed, lo = _jr_next(seed, 32)
                out.append(((hi.astype(np.uint64) << np.uint64(32)) + lo.astype(np.uint64)).view(np.int64))
            elif kind == ArrowType.FLOAT:  # nextFloat = next(24) / (1 << 24)
                seed, v = _jr_next(seed, 24)
                out.append((v.astype(np.float32) / np.float32(1 << 24)).astype(np.float32))
            else:  # nextDouble = ((long)next(26) << 27) + next(27)) * 0x1.0p-53
                seed, a = _jr_next(seed, 26)
                seed, b = _jr_next(seed, 27)
                out.append(((a << 27) + b).astype(np.float64) * (1.0 / (1 << 53)))
    return out


def struct_host_columns(n: int, num_fields: int = 100, seed_base: int = 17, row0: int = 0) -> List[HostColumn]:
    decl = gen_struct_host(n, num_fields, seed_base, row0)
    return [HostColumn(decl[j], None, None, n) for j in struct_schema_order(num_fields)]


def gen_struct_device(n: int, num_fields: int = 100, seed_base: int = 17, device="cuda"):
    """Same values as gen_struct_host, generated on the device with torch int64 ops
    (java.util.Random's 48-bit LCG; int64 multiply wraps, the mask restores mod 2^48)."""
    import torch
    mult, add, mask = 0x5DEECE66D, 0xB, (1 << 48) - 1
    seed = (torch.arange(n, dtype=torch.int64, device=device) + seed_base) ^ mult
    seed &= mask

    def nxt(seed, bits):
        seed = (seed * mult + add) & mask
        return seed, seed >> (48 - bits)

    def as_i32(v):  # (int) of a 32-bit value
        return torch.where(v >= (1 << 31), v - (1 << 32), v)

    cols = []
    for _, kind in struct_decl(num_fields):
        if kind == ArrowType.INT32:
            seed, v = nxt(seed, 32)
            cols.append(as_i32(v).to(torch.int32))
        elif kind == ArrowType.INT64:
            seed, hi = nxt(seed, 32)
            seed, lo = nxt(seed, 32)
            cols.append((as_i32(hi) << 32) + as_i32(lo))
        elif kind == ArrowType.FLOAT:
            seed, v = nxt(seed, 24)
            cols.append(v.to(torch.float32) / float(1 << 24))
        else:
            seed, a = nxt(seed, 26)
            seed, b = nxt(seed, 27)
            cols.append(((a << 27) + b).to(torch.float64) * (1.0 / (1 << 53)))
    return [cols[j] for j in struct_schema_order(num_fields)]


# ---------------------------------------------------------------------------
# M: mixed fixed + utf8
# ---------------------------------------------------------------------------
def mixed_decl():
    out = []
    j = 0
    for i in range(40):
        if i % 5 == 0:
            out.append((f"f{i}", ArrowType.STRING))
        else:
            out.append((f"f{i}", [ArrowType.INT32, ArrowType.INT64, ArrowType.DOUBLE][j % 3]))
            j += 1
    return out


def mixed_schema() -> Schema:
    decl = dict(mixed_decl())
    return Schema([Field(n, DataType(decl[n]), decl[n] == ArrowType.STRING) for n in sorted_names(decl)])


def mixed_host_columns(n: int, seed: int = 23, max_len: int = 32, null_rate: float = 0.0) -> List[HostColumn]:
    rng = np.random.default_rng(seed)
    schema = mixed_schema()
    cols = []
    for f in schema.fields:
        t = f.type.id
        if t == ArrowType.STRING:
            lens = rng.integers(0, max_len + 1, size=n, dtype=np.int64)
            valid = rng.random(n) >= null_rate if null_rate > 0 else np.ones(n, bool)
            lens = np.where(valid, lens, 0)
            offs = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(lens, out=offs[1:])
            data = rng.integers(32, 127, size=int(offs[-1]) + 8, dtype=np.uint8)  # printable ASCII
            cols.append(HostColumn(data, offs.astype(np.int32), pack_validity(valid), n))
        else:
            if t == ArrowType.DOUBLE:
                v = rng.standard_normal(n)
            else:
                v = rng.integers(np.iinfo(_NP[t]).min, np.iinfo(_NP[t]).max, size=n, dtype=_NP[t])
            cols.append(HostColumn(np.ascontiguousarray(v, dtype=_NP[t]), None, None, n))
    return cols


# ---------------------------------------------------------------------------
# N: nested struct + list<int64>
# ---------------------------------------------------------------------------
def nested_schema() -> Schema:
    inner = DataTypes.struct_field("c", True, [
        Field("x", DataType(ArrowType.INT32), False),
        Field("y", DataType(ArrowType.INT64), False),
        DataTypes.array_field("z", Field("item", DataType(ArrowType.INT64), True)),
    ])
    return Schema([
        Field("a", DataType(ArrowType.INT64), False),
        Field("b", DataType(ArrowType.DOUBLE), False),
        inner,
    ])


def nested_host_columns(n: int, seed: int = 29, max_len: int = 16, null_rate: float = 0.0) -> List[HostColumn]:
    """Pre-order columns: a, b, c(struct), x, y, z(list), item."""
    rng = np.random.default_rng(seed)
    a = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    b = rng.standard_normal(n)
    x = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int32)
    y = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    lens = rng.integers(0, max_len + 1, size=n, dtype=np.int64)
    if null_rate > 0:
        c_valid = rng.random(n) >= null_rate
        z_valid = rng.random(n) >= null_rate
    else:
        c_valid = np.ones(n, bool)
        z_valid = np.ones(n, bool)
    lens = np.where(c_valid & z_valid, lens, 0)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    m = int(offs[-1])
    items = rng.integers(-2**63, 2**63 - 1, size=max(1, m), dtype=np.int64)
    item_valid = rng.random(m) >= null_rate if null_rate > 0 else np.ones(m, bool)
    return [
        HostColumn(a, None, None, n),
        HostColumn(b, None, None, n),
        HostColumn(None, None, pack_validity(c_valid), n),
        HostColumn(x, None, None, n),
        HostColumn(y, None, None, n),
        HostColumn(None, offs.astype(np.int32), pack_validity(z_valid), n),
        HostColumn(items, None, pack_validity(item_valid), m),
    ]


def row_bytes_fixed(schema: Schema) -> int:
    n = len(schema.fields)
    return ((n + 63) // 64) * 8 + 8 * n


def column_bytes(schema: Schema) -> int:
    return sum(f.type.width for f in schema.fields)


# ---------------------------------------------------------------------------
# Device-side generators of M and N for bench.py (the same shapes and length
# distributions as the host generators above, drawn with torch on the device so a
# 16M-record batch is ready in milliseconds; values differ, the bytes moved do not).
# ---------------------------------------------------------------------------
def _dev_validity(valid, device):
    """Arrow validity (LSB-first) of a bool tensor, padded to 4 bytes."""
    import torch
    n = valid.numel()
    nb = max(4, ((n + 7) // 8 + 3) // 4 * 4)
    bits = torch.zeros(nb * 8, dtype=torch.uint8, device=device)
    bits[:n] = valid.to(torch.uint8)
    w = (1 << torch.arange(8, device=device, dtype=torch.int32)).to(torch.uint8)
    return (bits.view(nb, 8) * w).sum(dim=1, dtype=torch.int32).to(torch.uint8)


def _dev_strings(n, max_len, gen, device):
    import torch
    lens = torch.randint(0, max_len + 1, (n,), generator=gen, device=device, dtype=torch.int64)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[n].item())
    if total > 0x7FFFFFFF:
        raise ValueError("string column beyond int32 Arrow offsets")
    data = torch.randint(32, 127, (total + 8,), generator=gen, device=device, dtype=torch.uint8)
    return data, offs.to(torch.int32)


def mixed_device_columns(n: int, seed: int = 23, device="cuda", max_len: int = 32):
    """M on the device: DeviceColumns in schema order (strings nullable, all valid)."""
    import torch
    from .format.native import DeviceColumn
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    cols = []
    for f in mixed_schema().fields:
        t = f.type.id
        if t == ArrowType.STRING:
            data, offs = _dev_strings(n, max_len, gen, device)
            valid = _dev_validity(torch.ones(n, dtype=torch.bool, device=device), device)
            cols.append(DeviceColumn(data, offs, valid, n))
        elif t == ArrowType.DOUBLE:
            cols.append(DeviceColumn(torch.randn(n, generator=gen, device=device, dtype=torch.float64), None, None, n))
        else:
            dt = torch.int32 if t == ArrowType.INT32 else torch.int64
            lo, hi = (-2**31, 2**31 - 1) if dt == torch.int32 else (-2**63, 2**63 - 1)
            cols.append(DeviceColumn(torch.randint(lo, hi, (n,), generator=gen, device=device, dtype=dt), None, None, n))
    return cols


def nested_device_columns(n: int, seed: int = 29, device="cuda", max_len: int = 16):
    """N on the device, pre-order: a, b, c(struct), x, y, z(list), item (no nulls)."""
    import torch
    from .format.native import DeviceColumn
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    i64 = (-2**63, 2**63 - 1)
    a = torch.randint(*i64, (n,), generator=gen, device=device, dtype=torch.int64)
    b = torch.randn(n, generator=gen, device=device, dtype=torch.float64)
    x = torch.randint(-2**31, 2**31 - 1, (n,), generator=gen, device=device, dtype=torch.int32)
    y = torch.randint(*i64, (n,), generator=gen, device=device, dtype=torch.int64)
    lens = torch.randint(0, max_len + 1, (n,), generator=gen, device=device, dtype=torch.int64)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=offs[1:])
    m = int(offs[n].item())
    items = torch.randint(*i64, (max(1, m),), generator=gen, device=device, dtype=torch.int64)
    ones = torch.ones(n, dtype=torch.bool, device=device)
    return [
        DeviceColumn(a, None, None, n),
        DeviceColumn(b, None, None, n),
        DeviceColumn(None, None, _dev_validity(ones, device), n),
        DeviceColumn(x, None, None, n),
        DeviceColumn(y, None, None, n),
        DeviceColumn(None, offs.to(torch.int32), _dev_validity(ones, device), n),
        DeviceColumn(items, None, _dev_validity(torch.ones(m, dtype=torch.bool, device=device), device), m),
    ]
