"""Host-side column batches (numpy) and their device (torch) counterparts.

A batch of N bean objects is handed to the device path as Arrow-style columns,
one per pre-order schema node (the layout the C-ABI's ``fory_column`` takes):
fixed-width values, int32 offsets for utf8/binary/list, Arrow validity
bitmaps (1 = valid) for nullable fields. This is the same columnar view the
reference builds in ArrowWriter (java/fory-format/.../vectorized/ArrowWriter.java:55-99),
used here as the batch input instead of N Java objects.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from .types import ArrowType, Field, Schema

NP_DTYPE = {
    ArrowType.BOOL: np.uint8,
    ArrowType.INT8: np.int8,
    ArrowType.INT16: np.int16,
    ArrowType.INT32: np.int32,
    ArrowType.INT64: np.int64,
    ArrowType.FLOAT: np.float32,
    ArrowType.DOUBLE: np.float64,
    ArrowType.DATE32: np.int32,
    ArrowType.TIMESTAMP: np.int64,
}


@dataclass
class HostColumn:
    values: Optional[np.ndarray] = None
    offsets: Optional[np.ndarray] = None
    validity: Optional[np.ndarray] = None
    length: int = 0


def pack_validity(valid: np.ndarray) -> np.ndarray:
    """Arrow validity bitmap (LSB-first, 1 = valid), padded to a multiple of 4 bytes."""
    valid = np.asarray(valid, dtype=bool)
    bits = np.packbits(valid, bitorder="little")
    pad = (-len(bits)) % 4
    if pad or len(bits) == 0:
        bits = np.concatenate([bits, np.zeros(pad if len(bits) else 4, np.uint8)])
    return bits


def unpack_validity(bitmap: Optional[np.ndarray], n: int) -> np.ndarray:
    if bitmap is None:
        return np.ones(n, dtype=bool)
    return np.unpackbits(np.asarray(bitmap, np.uint8), bitorder="little")[:n].astype(bool)


def validity_bytes(n: int) -> int:
    return max(4, ((n + 7) // 8 + 3) // 4 * 4)


def _build(f: Field, vals: Sequence[Any], out: List[HostColumn], absent: Optional[np.ndarray] = None):
    """Appends the pre-order columns of field f for python values `vals`
    (`absent`: slots under a null parent struct, where a not-null field may be None)."""
    n = len(vals)
    valid = np.array([v is not None for v in vals], dtype=bool)
    col = HostColumn(length=n)
    col.validity = pack_validity(valid) if f.nullable else None
    bad = ~valid if absent is None else (~valid & ~absent)
    if not f.nullable and bad.any():
        raise ValueError(f"null value for not-null field {f.name}")
    t = f.type.id
    out.append(col)
    if t in NP_DTYPE:
        dt = NP_DTYPE[t]
        arr = np.zeros(n, dtype=dt)
        for i, v in enumerate(vals):
            if v is not None:
                arr[i] = (1 if v else 0) if t == ArrowType.BOOL else v
        col.values = arr
    elif t == ArrowType.DECIMAL128:
        arr = np.zeros((n, 2), dtype=np.int64)
        for i, v in enumerate(vals):
            if v is not None:
                arr[i] = decimal_words(v, f.type.scale)
        col.values = arr
    elif t in (ArrowType.STRING, ArrowType.BINARY):
        parts = []
        offs = np.zeros(n + 1, dtype=np.int32)
        pos = 0
        for i, v in enumerate(vals):
            if v is not None:
                b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
                parts.append(b)
                pos += len(b)
            offs[i + 1] = pos
        col.offsets = offs
        col.values = np.frombuffer(b"".join(parts) + b"\0" * 8, dtype=np.uint8).copy()
    elif t == ArrowType.LIST:
        offs = np.zeros(n + 1, dtype=np.int32)
        items: List[Any] = []
        for i, v in enumerate(vals):
            if v is not None:
                items.extend(v)
            offs[i + 1] = len(items)
        col.offsets = offs
        _build(f.children[0], items, out)
    elif t == ArrowType.MAP:  # Arrow map: entry offsets + key / value columns (entries struct elided)
        offs = np.zeros(n + 1, dtype=np.int32)
        keys: List[Any] = []
        vals_: List[Any] = []
        for i, v in enumerate(vals):
            if v is not None:
                pairs = list(v.items()) if isinstance(v, dict) else list(v)
                keys.extend(k for k, _ in pairs)
                vals_.extend(x for _, x in pairs)
            offs[i + 1] = len(keys)
        col.offsets = offs
        _build(f.children[0], keys, out)
        _build(f.children[1], vals_, out)
    elif t == ArrowType.STRUCT:
        gone = ~valid if absent is None else (~valid | absent)
        for c in f.children:
            _build(c, [None if v is None else v[c.name] for v in vals], out, gone)
    else:
        raise NotImplementedError(f"type {f.type} not supported")


def decimal_words(v, scale: int):
    """An Arrow decimal128 value: the unscaled integer at `scale` (a decimal.Decimal, or an
    int taken as already unscaled), as (lo, hi) little-endian two's complement int64 words.
    A Decimal whose scale differs is an error, as DecimalUtility.checkPrecisionAndScale's."""
    import decimal
    if isinstance(v, decimal.Decimal):
        sign, digits, exp = v.as_tuple()
        if -exp != scale:
            raise ValueError(f"BigDecimal scale must equal the field's: {-exp} != {scale}")
        u = int("".join(map(str, digits)) or "0")
        u = -u if sign else u
    else:
        u = int(v)
    if not -(1 << 127) <= u < (1 << 127):
        raise ValueError("decimal value exceeds 128 bits")
    u &= (1 << 128) - 1
    lo, hi = u & ((1 << 64) - 1), u >> 64
    return np.array([lo, hi], dtype=np.uint64).view(np.int64)


def decimal_value(words, scale: int):
    """decimal.Decimal of one (lo, hi) decimal128 element."""
    import decimal
    lo, hi = (int(x) for x in np.asarray(words, dtype=np.int64).view(np.uint64))
    u = lo | (hi << 64)
    if u >= 1 << 127:
        u -= 1 << 128
    return decimal.Decimal(u).scaleb(-scale, context=decimal.Context(prec=80))


def alloc_values(type_id: int, k: int):
    """Zeroed values of k elements of a fixed-width or decimal column (None otherwise)."""
    if type_id in NP_DTYPE:
        return np.zeros(max(1, k), NP_DTYPE[type_id])
    if type_id == ArrowType.DECIMAL128:
        return np.zeros((max(1, k), 2), np.int64)
    return None


def build_columns(schema: Schema, rows: Sequence[Dict[str, Any]]) -> List[HostColumn]:
    """Python row dicts (schema field name -> value, None = null) -> pre-order columns."""
    out: List[HostColumn] = []
    for f in schema.fields:
        _build(f, [r[f.name] for r in rows], out)
    return out


def to_device(cols: List[HostColumn], device="cuda"):
    import torch
    from .native import DeviceColumn

    def t(a):
        if a is None:
            return None
        return torch.from_numpy(np.ascontiguousarray(a)).to(device)

    return [DeviceColumn(t(c.values), t(c.offsets), t(c.validity), c.length) for c in cols]


def to_host(cols) -> List[HostColumn]:
    def h(a):
        return None if a is None else a.detach().cpu().numpy()
    return [HostColumn(h(c.values), h(c.offsets), h(c.validity), c.length) for c in cols]
