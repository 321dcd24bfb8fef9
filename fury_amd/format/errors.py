"""Exceptions mirroring the reference's error behaviour on this path.

  EncoderException            java/fory-format/.../encoder/EncoderException.java
                              (thrown by Encoders.bean, Encoders.java:227-230)
  ClassNotCompatibleException schema-hash mismatch in decode (Encoders.java:182-190)
  IndexOutOfBoundsException   MemoryBuffer bounds checks (MemoryBuffer.java:303-309)
  UnsupportedOperationException DataTypes.unsupported / BinaryArrayWriter.java:99-101
  IllegalArgumentException    Preconditions.checkArgument
"""
from __future__ import annotations

from .. import _lib


class EncoderException(RuntimeError):
    pass


class ClassNotCompatibleException(RuntimeError):
    pass


class IndexOutOfBoundsException(IndexError):
    pass


class UnsupportedOperationException(NotImplementedError):
    pass


class IllegalArgumentException(ValueError):
    pass


class CorruptRowException(RuntimeError):
    """A row or frame whose size field is out of range."""


class DeviceException(RuntimeError):
    pass


_MAP = {
    _lib.FORY_ERR_INVALID_ARGUMENT: IllegalArgumentException,
    _lib.FORY_ERR_UNSUPPORTED: UnsupportedOperationException,
    _lib.FORY_ERR_CAPACITY: IndexOutOfBoundsException,
    _lib.FORY_ERR_SCHEMA_MISMATCH: ClassNotCompatibleException,
    _lib.FORY_ERR_CORRUPT: CorruptRowException,
    _lib.FORY_ERR_DEVICE: DeviceException,
    _lib.FORY_ERR_ENCODER: EncoderException,
}


def raise_for(code: int, message: str):
    raise _MAP.get(code, RuntimeError)(f"[fory_status {code}] {message}")
