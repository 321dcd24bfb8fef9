"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (rowfmt_oracle.c).

The oracle is a scalar C restatement of java/fory-format's row writer/reader
(citations in rowfmt_oracle.c). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product path
(fury_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: a prebuilt variant (the `make asan` build) instead of _build/liboracle.so
LIB = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")
SRC = os.path.join(_HERE, "rowfmt_oracle.c")


class _Desc(ctypes.Structure):
    _fields_ = [("type_id", ctypes.c_int32), ("nullable", ctypes.c_int32),
                ("num_children", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class _Col(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("validity", ctypes.c_void_p), ("length", ctypes.c_int64),
                ("capacity", ctypes.c_int64)]


_lib = None


def build() -> str:
    if os.environ.get("ORACLE_LIB"):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-o", LIB, SRC])
    return LIB


def load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(LIB)
        lib.oracle_schema_hash.restype = ctypes.c_int64
        lib.oracle_schema_hash.argtypes = [ctypes.POINTER(_Desc), ctypes.c_int]
        lib.oracle_encode.restype = ctypes.c_int64
        lib.oracle_encode.argtypes = [ctypes.POINTER(_Desc), ctypes.c_int, ctypes.POINTER(_Col),
                                      ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_void_p]
        lib.oracle_decode.restype = ctypes.c_int
        lib.oracle_decode.argtypes = [ctypes.POINTER(_Desc), ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                      ctypes.POINTER(_Col), ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
        lib.oracle_gen_struct.restype = None
        lib.oracle_gen_struct.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]
        _lib = lib
    return _lib


def _desc(schema):
    out = []

    def visit(f):
        # a decimal's descriptor carries its precision (0 = 38), or FORY_DECIMAL_BIGINTEGER for a
        # BigInteger field; the scale is the column's
        res = 0
        if f.type.id == _DECIMAL:
            res = _BIGINTEGER if getattr(f.type, "big_integer", False) else (getattr(f.type, "precision", 0) or 38)
        out.append((f.type.id, 1 if f.nullable else 0, len(f.children), res))
        for c in f.children:
            visit(c)

    for f in schema.fields:
        visit(f)
    arr = (_Desc * max(1, len(out)))()
    for i, (t, n, k, r) in enumerate(out):
        arr[i].type_id, arr[i].nullable, arr[i].num_children, arr[i].reserved = t, n, k, r
    return arr, len(out)


_DECIMAL = 23  # ArrowType.DECIMAL (DECIMAL128's id)
_BIGINTEGER = 0x100  # FORY_DECIMAL_BIGINTEGER (include/fory_rowfmt.h)


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def _cols(cols) -> ctypes.Array:
    arr = (_Col * max(1, len(cols)))()
    for i, c in enumerate(cols):
        arr[i].values = _p(c.values)
        arr[i].offsets = _p(c.offsets)
        arr[i].validity = _p(c.validity)
        arr[i].length = c.length
        arr[i].capacity = 0 if c.values is None else c.values.nbytes
    return arr


def schema_hash(schema) -> int:
    d, n = _desc(schema)
    return int(load().oracle_schema_hash(d, n))


def encode(schema, cols, n: int, frame_mode: int) -> Tuple[np.ndarray, np.ndarray]:
    """Returns (bytes uint8, offsets int64[n+1])."""
    lib = load()
    d, nd = _desc(schema)
    ca = _cols(cols)
    offs = np.zeros(n + 1, dtype=np.int64)
    total = lib.oracle_encode(d, nd, ca, n, frame_mode, None, 0, offs.ctypes.data)
    if total == -3:
        raise OracleUnsupported("decimal precision exceeds the field's (DecimalUtility.checkPrecisionAndScale)")
    if total < 0:
        raise RuntimeError(f"oracle_encode sizing failed: {total}")
    out = np.zeros(max(1, total), dtype=np.uint8)
    got = lib.oracle_encode(d, nd, ca, n, frame_mode, out.ctypes.data, out.nbytes, offs.ctypes.data)
    if got != total:
        raise RuntimeError(f"oracle_encode failed: {got}")
    return out[:total], offs


class OracleUnsupported(RuntimeError):
    """The reference's UnsupportedOperationException on encode (decimal precision)."""


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__(f"oracle_decode status {code}")
        self.code = code


def decode(schema, buf: np.ndarray, offsets: Optional[np.ndarray], n: int, frame_mode: int):
    """Returns pre-order host columns (fury_amd.format.columns.HostColumn)."""
    from fury_amd.format.columns import HostColumn, NP_DTYPE, validity_bytes
    from fury_amd.format.types import ArrowType, preorder

    lib = load()
    d, nd = _desc(schema)
    fields = preorder(schema)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    nc = max(1, len(fields))
    slots = np.zeros(nc, dtype=np.int64)
    nbytes = np.zeros(nc, dtype=np.int64)
    rc = lib.oracle_decode(d, nd, buf.ctypes.data, buf.nbytes, _p(offsets), n, frame_mode,
                           _cols([]), 1, slots.ctypes.data, nbytes.ctypes.data)
    if rc:
        raise OracleError(rc)
    cols = []
    for i, f in enumerate(fields):
        ln = n if i < len(fields) and _is_top(schema, i) else int(slots[i])
        c = HostColumn(length=ln)
        t = f.type.id
        if t in NP_DTYPE:
            c.values = np.zeros(max(1, ln), dtype=NP_DTYPE[t])
        elif t == ArrowType.DECIMAL128:  # decimal128: (lo, hi) little-endian int64 words
            c.values = np.zeros((max(1, ln), 2), dtype=np.int64)
        elif t in (ArrowType.STRING, ArrowType.BINARY):
            c.offsets = np.zeros(ln + 1, dtype=np.int32)
            c.values = np.zeros(max(1, int(nbytes[i])), dtype=np.uint8)
        elif t in (ArrowType.LIST, ArrowType.MAP):
            c.offsets = np.zeros(ln + 1, dtype=np.int32)
        if f.nullable:
            c.validity = np.zeros(validity_bytes(ln), dtype=np.uint8)
        cols.append(c)
    rc = lib.oracle_decode(d, nd, buf.ctypes.data, buf.nbytes, _p(offsets), n, frame_mode,
                           _cols(cols), 0, None, None)
    if rc:
        raise OracleError(rc)
    return cols


def _is_top(schema, idx: int) -> bool:
    at = 0
    for f in schema.fields:
        if at == idx:
            return True
        at += _subtree_size(f)
    return False


def _subtree_size(f) -> int:
    return 1 + sum(_subtree_size(c) for c in f.children)


def gen_struct_columns(num_decl_fields: int, n: int, seed_base: int = 17, row0: int = 0) -> List[np.ndarray]:
    """java.util.Random(seed_base + row) values of the benchmark Struct, declared order."""
    lib = load()
    kinds = [np.int32, np.int64, np.float32, np.float64]
    arrs = [np.zeros(n, dtype=kinds[k % 4]) for k in range(num_decl_fields)]
    ptrs = (ctypes.c_void_p * num_decl_fields)(*[a.ctypes.data for a in arrs])
    lib.oracle_gen_struct(num_decl_fields, seed_base, row0, n, ptrs)
    return arrs
