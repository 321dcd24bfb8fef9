"""Encoders / RowEncoder — batch mirror of the reference's row-format API.

Reference API (java/fory-format/src/main/java/org/apache/fory/format/encoder):
  Encoders.bean(Class[, initialBufferSize])  -> RowEncoder   Encoders.java:63-231
  RowEncoder.schema() / toRow(T) / fromRow(BinaryRow)          RowEncoder.java:26-32
  Encoder.encode(T) / encode(MemoryBuffer, T) / decode(...)    Encoder.java:27-40

Here the unit of work is a batch of N objects held as device columns:
  encode(columns, n, frame_mode=FRAME_STREAM)  == N x encode(MemoryBuffer, obj)
                                                  into one fresh buffer
  encode(columns, n, frame_mode=FRAME_RAW)     == N x toRow(obj).toBytes()
  decode(rows, frame_mode=...)                 == N x decode(buffer) / fromRow(row)
  encode(columns, n, frame_mode=FRAME_HASHED)  == N x encode(obj) -> byte[] ([i64 hash][row]),
                                                  back to back with row offsets
  Encoders.array_encoder / map_encoder         == N x ArrayEncoder / MapEncoder
                                                  .encode(MemoryBuffer, collection)
Same bytes, same schema hash, same exceptions (errors.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Union

from .. import _lib
from . import native
from .infer import infer_schema
from .native import DeviceColumn, NativePlan
from .types import ArrowType, Schema

FRAME_RAW = _lib.FRAME_RAW
FRAME_STREAM = _lib.FRAME_STREAM
FRAME_COLLECTION = _lib.FRAME_COLLECTION
FRAME_HASHED = _lib.FRAME_HASHED


def _torch_dtype(type_id):
    import torch
    return {
        ArrowType.BOOL: torch.uint8, ArrowType.INT8: torch.int8, ArrowType.INT16: torch.int16,
        ArrowType.INT32: torch.int32, ArrowType.INT64: torch.int64, ArrowType.FLOAT: torch.float32,
        ArrowType.DOUBLE: torch.float64, ArrowType.DATE32: torch.int32,
        ArrowType.TIMESTAMP: torch.int64,
    }[type_id]


@dataclass
class EncodedRows:
    """Rows (RAW) or frames (STREAM) of a batch, back to back in one device buffer."""
    buffer: object                 # uint8 tensor, exactly total bytes
    offsets: Optional[object]      # int64 tensor [n+1] (None for fixed-width: i*stride)
    num_rows: int
    frame_mode: int
    stride: int = -1               # fixed-width plans: bytes per row/frame


class RowEncoder:
    def __init__(self, schema: Schema, bean_class=None, device="cuda"):
        self._schema = schema
        self.bean_class = bean_class
        self.device = device
        self.plan = NativePlan(schema)
        self._ws = None

    # -- RowEncoder.schema() ------------------------------------------------
    def schema(self) -> Schema:
        return self._schema

    @property
    def schema_hash(self) -> int:
        return self.plan.schema_hash

    def workspace(self, n: int, cols=None, decode: bool = False):
        import torch
        if cols is None:
            need = self.plan.workspace_bytes(n)
        elif decode:
            need = self.plan.decode_workspace_bytes(cols, n)
        else:
            need = self.plan.encode_workspace_bytes(cols, n)
        need = max(256, need)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    # -- encode ---------------------------------------------------------------
    def encode(self, columns: List[DeviceColumn], num_rows: int,
               frame_mode: int = FRAME_STREAM) -> EncodedRows:
        import torch
        p = self.plan
        arr = native.column_array(columns)
        ws = self.workspace(num_rows, arr)
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        if p.fixed_width:
            stride = p.stride(frame_mode)
            total = num_rows * stride
            out = torch.empty(max(16, total), dtype=torch.uint8, device=self.device)
            native.encode(p, arr, num_rows, frame_mode, None, out, status, ws)
            native.read_status(status)
            return EncodedRows(out[:total], None, num_rows, frame_mode, stride)
        offs = torch.empty(num_rows + 1, dtype=torch.int64, device=self.device)
        native.encoded_size(p, arr, num_rows, frame_mode, offs, ws)
        total = int(offs[num_rows].item())
        out = torch.empty(max(16, total), dtype=torch.uint8, device=self.device)
        native.encode(p, arr, num_rows, frame_mode, offs, out, status, ws)
        native.read_status(status)
        return EncodedRows(out[:total], offs, num_rows, frame_mode)

    def to_rows(self, columns: List[DeviceColumn], num_rows: int) -> EncodedRows:
        return self.encode(columns, num_rows, FRAME_RAW)

    # -- decode ---------------------------------------------------------------
    def alloc_fixed_outputs(self, num_rows: int) -> List[DeviceColumn]:
        import torch
        cols = []
        for f in self.plan.fields:
            vals = torch.empty(max(1, num_rows), dtype=_torch_dtype(f.type.id), device=self.device)
            val = None
            if f.nullable:
                val = torch.zeros(_validity_bytes(num_rows), dtype=torch.uint8, device=self.device)
            cols.append(DeviceColumn(vals, None, val, num_rows))
        return cols

    def decode(self, rows: Union[EncodedRows, object], num_rows: Optional[int] = None,
               frame_mode: Optional[int] = None, offsets=None) -> List[DeviceColumn]:
        import torch
        if isinstance(rows, EncodedRows):
            buf, num_rows, frame_mode, offsets = rows.buffer, rows.num_rows, rows.frame_mode, rows.offsets
        else:
            buf = rows
        if frame_mode is None:
            frame_mode = FRAME_STREAM
        p = self.plan
        ws = self.workspace(num_rows)
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        if p.fixed_width:
            if buf.numel() < num_rows * p.stride(frame_mode):
                from .errors import IndexOutOfBoundsException
                raise IndexOutOfBoundsException("row buffer shorter than num_rows * row size")
            cols = self.alloc_fixed_outputs(num_rows)
            native.decode(p, buf, None, num_rows, frame_mode, native.column_array(cols), status, ws)
            native.read_status(status)
            return cols
        # varlen: columns are sized level by level. Level L = the columns under L
        # lists / maps; their positions are the element totals of the level above.
        # decode_sizes fills the Arrow offsets of every level whose columns are
        # allocated; each round allocates the next level from the totals.
        n = num_rows
        fields = p.fields
        container, cdepth = _containers(p.schema)
        cols = [DeviceColumn(length=0) for _ in fields]
        var_kinds = (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST, ArrowType.MAP)
        totals = {}

        def alloc(level):
            for i, f in enumerate(fields):
                if cdepth[i] != level:
                    continue
                npos = n if container[i] < 0 else int(totals[container[i]])
                c = DeviceColumn(length=npos)
                t = f.type.id
                if t in var_kinds:
                    c.offsets = torch.zeros(npos + 1, dtype=torch.int32, device=self.device)
                elif t == ArrowType.DECIMAL128:  # decimal128: (lo, hi) int64 words per element
                    c.values = torch.empty((max(1, npos), 2), dtype=torch.int64, device=self.device)
                elif t != ArrowType.STRUCT:
                    c.values = torch.empty(max(1, npos), dtype=_torch_dtype(t), device=self.device)
                if f.nullable:
                    c.validity = torch.zeros(_validity_bytes(npos), dtype=torch.uint8, device=self.device)
                cols[i] = c

        if offsets is None:
            if frame_mode != FRAME_STREAM:
                raise ValueError("raw rows / collection frames are not self-delimiting: row offsets are required")
            offsets = self.index_frames(buf, n)
        alloc(0)
        for level in range(max(cdepth) + 1):
            var_idx = [i for i, f in enumerate(fields) if cdepth[i] == level and f.type.id in var_kinds]
            if not var_idx:
                break
            arr = native.column_array(cols)
            ws = self.workspace(n, arr, decode=True)
            native.decode_sizes(p, buf, offsets, n, frame_mode, arr, status, ws)
            last = torch.stack([cols[i].offsets[cols[i].length] for i in var_idx]).cpu().tolist()
            native.read_status(status)
            totals.update(zip(var_idx, last))
            for i in var_idx:  # string / binary bytes of this level
                if fields[i].type.id in (ArrowType.STRING, ArrowType.BINARY):
                    cols[i].values = torch.empty(max(1, int(totals[i])), dtype=torch.uint8, device=self.device)
            alloc(level + 1)
        arr = native.column_array(cols)
        ws = self.workspace(n, arr, decode=True)
        native.decode(p, buf, offsets, n, frame_mode, arr, status, ws)
        native.read_status(status)
        return cols

    def index_frames(self, buf, num_rows: int):
        """Frame starts of the first num_rows frames of a STREAM buffer, found on the device
        (Encoder.decode(MemoryBuffer) x N walks [i32 size][i64 hash] frames, Encoders.java:176-193).
        Returns the int64 offsets tensor [n+1]; offsets[n] = bytes consumed."""
        import torch
        p = self.plan
        offs = torch.empty(num_rows + 1, dtype=torch.int64, device=self.device)
        need = max(256, native.index_workspace_bytes(p, num_rows, buf.numel()))
        iws = torch.empty(need, dtype=torch.uint8, device=self.device)
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        native.index_frames(p, buf, buf.numel(), num_rows, FRAME_STREAM, offs, status, iws)
        native.read_status(status)
        return offs

    def from_rows(self, rows: EncodedRows) -> List[DeviceColumn]:
        return self.decode(rows)


def _subtree_size(f) -> int:
    return 1 + sum(_subtree_size(c) for c in f.children)


def _containers(schema):
    """Per pre-order column: the nearest list / map ancestor (-1: none) and the
    number of list / map ancestors (the decode_sizes level that positions it)."""
    container, cdepth = [], []

    def walk(f, anc, depth):
        container.append(anc)
        cdepth.append(depth)
        me = len(container) - 1
        inner = f.type.id in (ArrowType.LIST, ArrowType.MAP)
        for c in f.children:
            walk(c, me if inner else anc, depth + (1 if inner else 0))

    for f in schema.fields:
        walk(f, -1, 0)
    return container, cdepth


def _validity_bytes(n: int) -> int:
    return max(4, ((n + 7) // 8 + 3) // 4 * 4)


class CollectionEncoder(RowEncoder):
    """ArrayEncoder / MapEncoder mirror (Encoders.java:276-580): a batch of N collections
    held as a one-field schema (the collection column); encode/decode default to the
    collection frames [i32 size][BinaryArray | BinaryMap] (FRAME_COLLECTION)."""

    def field(self):
        return self.plan.schema.fields[0]

    def encode(self, columns, num_rows, frame_mode=FRAME_COLLECTION):
        return super().encode(columns, num_rows, frame_mode)

    def decode(self, rows, num_rows=None, frame_mode=None, offsets=None):
        if not isinstance(rows, EncodedRows) and frame_mode is None:
            frame_mode = FRAME_COLLECTION
        return super().decode(rows, num_rows, frame_mode, offsets)


class Encoders:
    """Factory mirror of Encoders (Encoders.java:63-231)."""

    @staticmethod
    def array_encoder(element_field, device="cuda") -> CollectionEncoder:
        """Encoders.arrayEncoder (Encoders.java:276-330,357-432) for Collection<element>."""
        from .types import DataTypes
        return CollectionEncoder(Schema([DataTypes.array_field("", element_field)]), None, device)

    @staticmethod
    def map_encoder(key_field, value_field, device="cuda") -> CollectionEncoder:
        """Encoders.mapEncoder (Encoders.java:434-580) for Map<key, value>."""
        from .types import DataTypes
        return CollectionEncoder(Schema([DataTypes.map_field("", key_field, value_field)]), None, device)

    @staticmethod
    def bean(bean_class_or_schema, initial_buffer_size: int = 16, device="cuda") -> RowEncoder:
        del initial_buffer_size  # device buffers are sized exactly per batch
        if isinstance(bean_class_or_schema, Schema):
            return RowEncoder(bean_class_or_schema, None, device)
        try:
            schema = infer_schema(bean_class_or_schema)
        except Exception as e:  # Encoders.java:227-230
            from .errors import EncoderException
            raise EncoderException(f"Create encoder failed, \nbeanClass: {bean_class_or_schema}") from e
        return RowEncoder(schema, bean_class_or_schema, device)
