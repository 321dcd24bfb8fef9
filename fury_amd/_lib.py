"""ctypes binding of the C-ABI in include/fory_rowfmt.h (libfory_rowfmt.so).

The library is built in-tree (``make``; ``__graft_entry__.build()``) into
``fury_amd/lib/libfory_rowfmt.so``. There is no fallback: if the library is
missing, importing the device path raises ``RuntimeError`` loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FORY_ROWFMT_LIB: another build of the same library (A/B of two builds on one box)
LIB_PATH = os.environ.get("FORY_ROWFMT_LIB") or os.path.join(_HERE, "lib", "libfory_rowfmt.so")

# fory_status (include/fory_rowfmt.h)
FORY_OK = 0
FORY_ERR_INVALID_ARGUMENT = 1
FORY_ERR_UNSUPPORTED = 2
FORY_ERR_CAPACITY = 3
FORY_ERR_SCHEMA_MISMATCH = 4
FORY_ERR_CORRUPT = 5
FORY_ERR_DEVICE = 6
FORY_ERR_ENCODER = 7

FRAME_RAW = 0
FRAME_STREAM = 1
FRAME_COLLECTION = 2
FRAME_HASHED = 3  # Encoder.encode(T) -> [i64 schemaHash][row] (Encoders.java:203-210)


class FieldDesc(ctypes.Structure):
    _fields_ = [
        ("type_id", ctypes.c_int32),
        ("nullable", ctypes.c_int32),
        ("num_children", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class Column(ctypes.Structure):
    _fields_ = [
        ("values", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("validity", ctypes.c_void_p),
        ("length", ctypes.c_int64),
        ("capacity", ctypes.c_int64),
    ]


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("schema_hash", ctypes.c_int64),
        ("num_fields", ctypes.c_int32),
        ("num_columns", ctypes.c_int32),
        ("bitmap_bytes", ctypes.c_int32),
        ("fixed_size", ctypes.c_int32),
        ("fixed_width", ctypes.c_int32),
        ("row_size", ctypes.c_int32),
    ]


# Every exported symbol and its prototype (checked by tests/test_capi_symbols.py).
PROTOTYPES = {
    "fory_rowfmt_abi_version": (ctypes.c_int32, []),
    "fory_rowfmt_last_error": (ctypes.c_char_p, []),
    "fory_rowfmt_plan_create": (
        ctypes.c_int,
        [ctypes.POINTER(FieldDesc), ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)],
    ),
    "fory_rowfmt_plan_destroy": (None, [ctypes.c_void_p]),
    "fory_rowfmt_plan_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(PlanInfo)]),
    "fory_rowfmt_workspace_bytes": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64]),
    "fory_rowfmt_encode_workspace_bytes": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "fory_rowfmt_decode_workspace_bytes": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "fory_rowfmt_encoded_size": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(Column), ctypes.c_int64, ctypes.c_int32,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p],
    ),
    "fory_rowfmt_encode": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(Column), ctypes.c_int64, ctypes.c_int32,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p],
    ),
    "fory_rowfmt_decode_sizes": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
         ctypes.POINTER(Column), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_void_p],
    ),
    "fory_rowfmt_decode": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
         ctypes.POINTER(Column), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_void_p],
    ),
    "fory_rowfmt_read_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "fory_rowfmt_index_workspace_bytes": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]),
    "fory_rowfmt_index_frames": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "fory_rowfmt_split_windows": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
         ctypes.POINTER(ctypes.c_int32)]),
    "fory_rowfmt_host_encode_windows": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(Column), ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "fory_rowfmt_host_ctx_create": (
        ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "fory_rowfmt_host_ctx_destroy": (None, [ctypes.c_void_p]),
    "fory_rowfmt_host_encode": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(Column), ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
         ctypes.c_int64]),
    "fory_rowfmt_host_decode": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
         ctypes.POINTER(Column)]),
    "fory_rowfmt_host_encode_var": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(Column), ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "fory_rowfmt_host_decode_var_sizes": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
         ctypes.c_void_p]),
    "fory_rowfmt_host_decode_stream_sizes": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.POINTER(ctypes.c_int64)]),
    "fory_rowfmt_host_decode_var": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Column)]),
    "fory_rowfmt_host_decode_var_into": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(Column),
         ctypes.c_void_p, ctypes.c_void_p]),
    "fory_rowfmt_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "fory_rowfmt_host_unregister": (ctypes.c_int, [ctypes.c_void_p]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Loads libfory_rowfmt.so (raises RuntimeError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: build the HIP extension first (`make` or "
            "`python -c 'import __graft_entry__; __graft_entry__.build()'`). "
            "There is no CPU fallback for the device path.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fory_rowfmt_abi_version() != 1:
        raise RuntimeError("libfory_rowfmt ABI version mismatch")
    _lib = lib
    return lib


def last_error() -> str:
    return load().fory_rowfmt_last_error().decode("utf-8", "replace")
