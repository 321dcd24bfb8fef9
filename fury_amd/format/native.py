"""Device path: thin wrappers over the C-ABI (libfory_rowfmt.so).

Device memory and streams come from torch (plumbing only); all compute is in
the HIP kernels behind the C-ABI. Nothing here falls back to the CPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional

from .. import _lib
from .errors import raise_for
from .types import ArrowType, Schema, flatten, preorder


def frame_header_bytes(frame_mode: int) -> int:
    """Bytes before each row: STREAM [i32 size][i64 hash], HASHED [i64 hash],
    COLLECTION [i32 size] (the payload replaces the row), RAW none."""
    return {_lib.FRAME_STREAM: 12, _lib.FRAME_HASHED: 8, _lib.FRAME_COLLECTION: 4}.get(frame_mode, 0)


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


class NativePlan:
    """fory_rowfmt_plan_create: layout + schema hash of a schema."""

    def __init__(self, schema: Schema):
        lib = _lib.load()
        self.schema = schema
        self._desc, self._ndesc = flatten(schema)
        h = ctypes.c_void_p()
        rc = lib.fory_rowfmt_plan_create(self._desc, self._ndesc, ctypes.byref(h))
        if rc:
            raise_for(rc, _lib.last_error())
        self.handle = h
        info = _lib.PlanInfo()
        rc = lib.fory_rowfmt_plan_info(h, ctypes.byref(info))
        if rc:
            raise_for(rc, _lib.last_error())
        self.schema_hash = int(info.schema_hash)
        self.num_fields = int(info.num_fields)
        self.num_columns = int(info.num_columns)
        self.bitmap_bytes = int(info.bitmap_bytes)
        self.fixed_size = int(info.fixed_size)
        self.fixed_width = bool(info.fixed_width)
        self.row_size = int(info.row_size)
        self.fields = preorder(schema)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.load().fory_rowfmt_plan_destroy(self.handle)
                self.handle = None
        except Exception:
            pass

    def stride(self, frame_mode: int) -> int:
        assert self.fixed_width
        return self.fixed_size + frame_header_bytes(frame_mode)

    def workspace_bytes(self, num_rows: int) -> int:
        return int(_lib.load().fory_rowfmt_workspace_bytes(self.handle, num_rows))

    def encode_workspace_bytes(self, cols, num_rows: int) -> int:
        """Workspace for encode through the columnar tree engine (cols: column_array)."""
        return int(_lib.load().fory_rowfmt_encode_workspace_bytes(self.handle, cols, num_rows))

    def decode_workspace_bytes(self, out_cols, num_rows: int) -> int:
        """Workspace for the columnar decode given the levels allocated in out_cols (column_array)."""
        return int(_lib.load().fory_rowfmt_decode_workspace_bytes(self.handle, out_cols, num_rows))


@dataclass
class DeviceColumn:
    """One pre-order column on the device (torch tensors, contiguous)."""
    values: object = None     # tensor (any dtype, viewed as bytes)
    offsets: object = None    # int32 tensor [length+1]
    validity: object = None   # uint8 tensor [ceil(length/8)] (rounded up to 4 bytes)
    length: int = 0


def column_array(cols: List[DeviceColumn]):
    arr = (_lib.Column * max(1, len(cols)))()
    for i, c in enumerate(cols):
        arr[i].values = _ptr(c.values)
        arr[i].offsets = _ptr(c.offsets)
        arr[i].validity = _ptr(c.validity)
        arr[i].length = c.length
        arr[i].capacity = 0 if c.values is None else c.values.numel() * c.values.element_size()
    return arr


def _check(rc: int):
    if rc:
        raise_for(rc, _lib.last_error())


def encoded_size(plan: NativePlan, cols_arr, n: int, frame: int, d_offsets, ws, stream=None):
    lib = _lib.load()
    s = stream if stream is not None else _stream_handle()
    _check(lib.fory_rowfmt_encoded_size(plan.handle, cols_arr, n, frame, _ptr(d_offsets),
                                        _ptr(ws), ws.numel(), s))


def encode(plan: NativePlan, cols_arr, n: int, frame: int, d_offsets, out, status, ws,
           stream=None, capacity: Optional[int] = None):
    lib = _lib.load()
    s = stream if stream is not None else _stream_handle()
    cap = out.numel() if capacity is None else capacity
    _check(lib.fory_rowfmt_encode(plan.handle, cols_arr, n, frame, _ptr(d_offsets), _ptr(out), cap,
                                  _ptr(status), _ptr(ws), ws.numel(), s))


def decode_sizes(plan: NativePlan, rows, d_offsets, n: int, frame: int, cols_arr, status, ws,
                 stream=None):
    lib = _lib.load()
    s = stream if stream is not None else _stream_handle()
    _check(lib.fory_rowfmt_decode_sizes(plan.handle, _ptr(rows), _ptr(d_offsets), n, frame, cols_arr,
                                        _ptr(status), _ptr(ws), ws.numel(), s))


def decode(plan: NativePlan, rows, d_offsets, n: int, frame: int, cols_arr, status, ws, stream=None):
    lib = _lib.load()
    s = stream if stream is not None else _stream_handle()
    _check(lib.fory_rowfmt_decode(plan.handle, _ptr(rows), _ptr(d_offsets), n, frame, cols_arr,
                                  _ptr(status), _ptr(ws), ws.numel(), s))


def index_workspace_bytes(plan: NativePlan, n: int, rows_bytes: int) -> int:
    return int(_lib.load().fory_rowfmt_index_workspace_bytes(plan.handle, n, rows_bytes))


def index_frames(plan: NativePlan, rows, rows_bytes: int, n: int, frame: int, d_offsets, status, ws, stream=None):
    """fory_rowfmt_index_frames: frame starts of a STREAM batch from the stream alone."""
    lib = _lib.load()
    s = stream if stream is not None else _stream_handle()
    _check(lib.fory_rowfmt_index_frames(plan.handle, _ptr(rows), rows_bytes, n, frame, _ptr(d_offsets),
                                        _ptr(status), _ptr(ws), 0 if ws is None else ws.numel(), s))


def read_status(status, stream=None):
    lib = _lib.load()
    s = stream if stream is not None else _stream_handle()
    _check(lib.fory_rowfmt_read_status(_ptr(status), s))


def is_varlen(f) -> bool:
    return f.type.id in (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST)


def _np_ptr(a) -> Optional[int]:
    return None if a is None else a.ctypes.data


class HostPipeline:
    """fory_rowfmt_host_*: host-memory batches (numpy arrays, e.g. the Arrow view of
    off-heap MemoryBuffers) through the device kernels: the C++ chunk pipeline for
    fixed-width plans (encode/decode), whole batches for varlen plans (encode_var /
    decode_var)."""

    def __init__(self, plan: NativePlan, chunk_rows: int = 1 << 20, device: int = 0):
        lib = _lib.load()
        self.plan = plan
        h = ctypes.c_void_p()
        _check(lib.fory_rowfmt_host_ctx_create(plan.handle, device, chunk_rows, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            _lib.load().fory_rowfmt_host_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _host_array(cols):
        arr = (_lib.Column * max(1, len(cols)))()
        for i, c in enumerate(cols):
            arr[i].values = _np_ptr(c.values)
            arr[i].offsets = _np_ptr(c.offsets)
            arr[i].validity = _np_ptr(c.validity)
            arr[i].length = c.length
            arr[i].capacity = 0 if c.values is None else c.values.nbytes
        return arr

    def encode(self, host_cols, n: int, frame: int, out) -> None:
        """host_cols: HostColumn list (numpy); out: uint8 numpy array of >= n*stride bytes."""
        _check(_lib.load().fory_rowfmt_host_encode(self.handle, self._host_array(host_cols), n, frame,
                                                   _np_ptr(out), out.nbytes))

    def encode_windows(self, host_cols, n: int, frame: int, windows):
        """fory_rowfmt_host_encode_windows: whole rows/frames into a list of uint8 numpy
        windows (greedy); returns (rows per window, bytes per window)."""
        import numpy as np
        nw = len(windows)
        ptrs = (ctypes.c_void_p * nw)(*[w.ctypes.data for w in windows])
        caps = np.array([w.nbytes for w in windows], np.int64)
        rows = np.zeros(nw, np.int64)
        nbytes = np.zeros(nw, np.int64)
        _check(_lib.load().fory_rowfmt_host_encode_windows(self.handle, self._host_array(host_cols), n, frame,
                                                           ctypes.cast(ptrs, ctypes.c_void_p), _np_ptr(caps), nw,
                                                           _np_ptr(rows), _np_ptr(nbytes)))
        return rows, nbytes

    def decode(self, rows, n: int, frame: int, host_out_cols) -> None:
        _check(_lib.load().fory_rowfmt_host_decode(self.handle, _np_ptr(rows), rows.nbytes, n, frame,
                                                   self._host_array(host_out_cols)))

    # -- varlen plans: whole batch per call --------------------------------
    def encode_var(self, host_cols, n: int, frame: int, out=None):
        """Returns (rows uint8 array, row offsets int64[n+1]); grows `out` on capacity errors."""
        import numpy as np
        lib = _lib.load()
        arr = self._host_array(host_cols)
        offs = np.zeros(n + 1, np.int64)
        total = ctypes.c_int64(0)
        if out is None:
            out = np.zeros(1, np.uint8)
        rc = lib.fory_rowfmt_host_encode_var(self.handle, arr, n, frame, _np_ptr(out), out.nbytes,
                                             _np_ptr(offs), ctypes.byref(total))
        if rc == _lib.FORY_ERR_CAPACITY and total.value > out.nbytes:  # MemoryBuffer grows and retries
            out = np.zeros(total.value, np.uint8)
            rc = lib.fory_rowfmt_host_encode_var(self.handle, arr, n, frame, _np_ptr(out), out.nbytes,
                                                 _np_ptr(offs), ctypes.byref(total))
        _check(rc)
        return out[:total.value], offs

    def decode_var(self, rows, offsets, n: int, frame: int):
        """Host rows -> host columns (HostColumn list, pre-order)."""
        counts, nbytes = self.decode_var_sizes(rows, offsets, n, frame)
        return self.decode_var_finish(counts, nbytes)

    def decode_var_sizes(self, rows, offsets, n: int, frame: int):
        """fory_rowfmt_host_decode_var_sizes: stages the rows, returns per-column
        (element counts, value bytes)."""
        import numpy as np
        from .types import preorder
        fields = preorder(self.plan.schema)
        counts = np.zeros(max(1, len(fields)), np.int64)
        nbytes = np.zeros(max(1, len(fields)), np.int64)
        offs = np.ascontiguousarray(offsets, dtype=np.int64)
        _check(_lib.load().fory_rowfmt_host_decode_var_sizes(self.handle, _np_ptr(rows), _np_ptr(offs), n, frame,
                                                             _np_ptr(counts), _np_ptr(nbytes)))
        return counts, nbytes

    def decode_stream(self, rows, n: int):
        """N x Encoder.decode(MemoryBuffer) over host frames alone (no row offsets):
        returns (columns, bytes consumed)."""
        import numpy as np
        from .types import preorder
        fields = preorder(self.plan.schema)
        counts = np.zeros(max(1, len(fields)), np.int64)
        nbytes = np.zeros(max(1, len(fields)), np.int64)
        used = ctypes.c_int64(0)
        _check(_lib.load().fory_rowfmt_host_decode_stream_sizes(self.handle, _np_ptr(rows), rows.nbytes, n,
                                                                _np_ptr(counts), _np_ptr(nbytes),
                                                                ctypes.byref(used)))
        return self.decode_var_finish(counts, nbytes), used.value

    def decode_var_into(self, rows, offsets, n: int, frame: int, cols=None):
        """fory_rowfmt_host_decode_var_into: one pipelined call into caller-sized host
        columns (HostColumn list, `length` = element capacity, as a receiver keeps its
        buffers across batches); on FORY_ERR_CAPACITY the columns are sized from the
        reported totals and the call repeats. Returns the columns, trimmed to the batch."""
        import numpy as np
        from .types import preorder
        lib = _lib.load()
        fields = preorder(self.plan.schema)
        counts = np.zeros(max(1, len(fields)), np.int64)
        nbytes = np.zeros(max(1, len(fields)), np.int64)
        offs = np.ascontiguousarray(offsets, dtype=np.int64)
        if cols is None:
            cols = self.alloc_columns(np.zeros_like(counts), np.zeros_like(nbytes))
        rc = lib.fory_rowfmt_host_decode_var_into(self.handle, _np_ptr(rows), _np_ptr(offs), n, frame,
                                                  self._host_array(cols), _np_ptr(counts), _np_ptr(nbytes))
        if rc == _lib.FORY_ERR_CAPACITY:
            cols = self.alloc_columns(counts, nbytes)
            rc = lib.fory_rowfmt_host_decode_var_into(self.handle, _np_ptr(rows), _np_ptr(offs), n, frame,
                                                      self._host_array(cols), _np_ptr(counts), _np_ptr(nbytes))
        _check(rc)
        return self.trim_columns(cols, counts, nbytes)

    def trim_columns(self, cols, counts, nbytes):
        """Views of the first counts[i] elements (nbytes[i] string bytes) of each column."""
        from .columns import HostColumn, validity_bytes
        out = []
        for i, c in enumerate(cols):
            k = int(counts[i])
            t = HostColumn(length=k)
            if c.values is not None:
                t.values = c.values[:max(1, int(nbytes[i]))] if c.values.dtype.itemsize == 1 and c.offsets is not None \
                    else c.values[:max(1, k)]
            if c.offsets is not None:
                t.offsets = c.offsets[:k + 1]
            if c.validity is not None:
                t.validity = c.validity[:validity_bytes(k)]
            out.append(t)
        return out

    def alloc_columns(self, counts, nbytes):
        """Zeroed host columns for per-column element counts / string bytes (length = count)."""
        import numpy as np
        from .columns import HostColumn, NP_DTYPE, alloc_values, validity_bytes
        from .types import ArrowType, preorder
        fields = preorder(self.plan.schema)
        cols = []
        for i, f in enumerate(fields):
            k, t = int(counts[i]), f.type.id
            c = HostColumn(length=k)
            if t in (ArrowType.STRING, ArrowType.BINARY):
                c.values = np.zeros(max(1, int(nbytes[i])), np.uint8)
            elif t in NP_DTYPE or t == ArrowType.DECIMAL128:
                c.values = alloc_values(t, k)
            if t in (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST, ArrowType.MAP):
                c.offsets = np.zeros(k + 1, np.int32)
            if f.nullable:
                c.validity = np.zeros(validity_bytes(k), np.uint8)
            cols.append(c)
        return cols

    def decode_var_finish(self, counts, nbytes):
        """fory_rowfmt_host_decode_var: the staged batch into freshly sized host columns."""
        import numpy as np
        from .columns import HostColumn, NP_DTYPE, alloc_values, validity_bytes
        from .types import ArrowType, preorder
        fields = preorder(self.plan.schema)
        cols = []
        for i, f in enumerate(fields):
            k, t = int(counts[i]), f.type.id
            c = HostColumn(length=k)
            if t in (ArrowType.STRING, ArrowType.BINARY):
                c.values = np.zeros(max(1, int(nbytes[i])), np.uint8)
            elif t in NP_DTYPE or t == ArrowType.DECIMAL128:
                c.values = alloc_values(t, k)
            if t in (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST, ArrowType.MAP):
                c.offsets = np.zeros(k + 1, np.int32)
            if f.nullable:
                c.validity = np.zeros(validity_bytes(k), np.uint8)
            cols.append(c)
        _check(_lib.load().fory_rowfmt_host_decode_var(self.handle, self._host_array(cols)))
        return cols


def split_windows(row_offsets, n: int, max_window_bytes: int = (1 << 31) - 1, stride: int = 0):
    """fory_rowfmt_split_windows: rows [first[w], first[w+1]) per <= max_window_bytes window
    (host numpy offsets, or row i at i * stride)."""
    import numpy as np
    offs = None if row_offsets is None else np.ascontiguousarray(row_offsets, dtype=np.int64)
    total = int(offs[n]) if offs is not None else n * stride
    # each window holds >= 1 row, and two consecutive windows hold > max_window_bytes
    cap = max(1, min(n, 2 * total // max(1, max_window_bytes) + 2))
    first = np.zeros(cap + 1, np.int64)
    nw = ctypes.c_int32(0)
    _check(_lib.load().fory_rowfmt_split_windows(_np_ptr(offs), stride, n, max_window_bytes, cap, _np_ptr(first),
                                                 ctypes.byref(nw)))
    return first[:nw.value + 1]


def host_register(a) -> None:
    """Pins a numpy array's memory in place (hipHostRegister)."""
    _check(_lib.load().fory_rowfmt_host_register(a.ctypes.data, a.nbytes))


def host_unregister(a) -> None:
    _check(_lib.load().fory_rowfmt_host_unregister(a.ctypes.data))
