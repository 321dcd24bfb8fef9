"""fury_amd.format — MI355X batch path for Fory's row format (java/fory-format)."""
from .types import ArrowType, DataType, DataTypes, Field, Schema, flatten, preorder  # noqa: F401
from .infer import infer_schema, lower_camel_to_lower_underscore  # noqa: F401
from .errors import (  # noqa: F401
    ClassNotCompatibleException, CorruptRowException, DeviceException, EncoderException,
    IllegalArgumentException, IndexOutOfBoundsException, UnsupportedOperationException)
from .columns import HostColumn, build_columns, pack_validity, unpack_validity  # noqa: F401


def __getattr__(name):
    # The device path (Encoders/RowEncoder) imports torch lazily.
    if name in ("Encoders", "RowEncoder", "CollectionEncoder", "EncodedRows", "FRAME_RAW", "FRAME_STREAM",
                "FRAME_COLLECTION", "FRAME_HASHED"):
        from . import encoder
        return getattr(encoder, name)
    raise AttributeError(name)
