"""CPU: decimal fields in the oracle (oracle/rowfmt_oracle.c, w_write_decimal / the
DECIMAL read), restated from the reference:
  BinaryWriter.writeDecimal (BinaryWriter.java:214-230): checkPrecisionAndScale, then
  DecimalUtility.writeBigDecimalToArrowBuf(value, buf, 0, DECIMAL_BYTE_LENGTH = 32)
  (DecimalUtils.java:23): the unscaled value's little-endian two's complement,
  sign-extended to 32 bytes, behind an (offset, 32) slot;
  UnsafeTrait.getDecimal (UnsafeTrait.java:139-150) reads the 32 bytes back.
The byte images below are worked by hand from that algorithm (Arrow-Java 15's
DecimalUtility is not in the reference tree); the schema hashes of decimal schemas are
pinned by the reference's own infer.py (tests/golden/schema_hashes.json)."""
import decimal

import numpy as np
import pytest

from oracle import oracle
from fury_amd.format.columns import build_columns, decimal_value, decimal_words
from fury_amd.format.types import DataTypes, Field, Schema


def one(scale=18, precision=38):
    return Schema([Field("d", DataTypes.decimal(precision, scale), True)])


def row_of(schema, value):
    cols = build_columns(schema, [{"d": value}])
    buf, offs = oracle.encode(schema, cols, 1, 0)
    return buf.tobytes(), cols


def test_decimal_row_layout():
    # 1.5 at scale 18 -> unscaled 1_500_000_000_000_000_000 = 0x14D1120D7B160000
    b, _ = row_of(one(), decimal.Decimal("1.500000000000000000"))
    assert len(b) == 8 + 8 + 32  # bitmap, one slot, 32 bytes out of line
    assert b[:8] == bytes(8)
    assert b[8:16] == (16 << 32 | 32).to_bytes(8, "little")  # (offset 16 from the row start, size 32)
    assert b[16:32] == (0x14D1120D7B160000).to_bytes(16, "little")
    assert b[32:48] == bytes(16)  # sign extension of a positive value


def test_negative_decimal_is_sign_extended():
    b, _ = row_of(one(scale=0), -1)
    assert b[16:48] == b"\xff" * 32
    b, _ = row_of(one(scale=0), -(10 ** 38 - 1))
    v = int.from_bytes(b[16:48], "little", signed=True)
    assert v == -(10 ** 38 - 1)


def test_null_decimal_sets_the_bit_and_no_bytes():
    b, _ = row_of(one(), None)
    assert b == bytes([1]) + bytes(7) + bytes(8)  # bitmap bit 0, slot left zero, no var bytes


def test_precision_is_checked():
    with pytest.raises(oracle.OracleUnsupported):
        row_of(one(scale=0), 10 ** 38)  # 39 digits > MAX_PRECISION 38
    with pytest.raises(oracle.OracleUnsupported):
        row_of(one(scale=2, precision=10), 10 ** 10)  # 11 digits > 10
    row_of(one(scale=2, precision=10), 10 ** 10 - 1)  # 10 digits: fine
    # the error survives later rows of the batch (the sizing pass overflows too)
    s = one(scale=0)
    cols = build_columns(s, [{"d": v} for v in (1, 2, 10 ** 38, 3, 4)])
    with pytest.raises(oracle.OracleUnsupported):
        oracle.encode(s, cols, 5, 1)


def test_decimal_words_round_trip():
    for v in (0, 1, -1, 2 ** 64, -(2 ** 64) - 5, 10 ** 38 - 1, -(10 ** 38 - 1), 2 ** 127 - 1, -(2 ** 127)):
        w = decimal_words(v, 0)
        assert decimal_value(w, 0) == v
    assert decimal_value(decimal_words(decimal.Decimal("-12.34"), 2), 2) == decimal.Decimal("-12.34")
    with pytest.raises(ValueError):
        decimal_words(decimal.Decimal("1.5"), 2)  # scale must equal the field's


def test_decode_round_trip_and_corrupt_high_bytes():
    s = Schema([Field("a", DataTypes.decimal(38, 18), True), Field("b", DataTypes.decimal(38, 0), False),
                DataTypes.array_field("l", Field("item", DataTypes.decimal(38, 18), True))])
    rng = np.random.default_rng(4)
    rows = []
    for i in range(200):
        rows.append({"a": None if i % 7 == 0 else int(rng.integers(-10 ** 18, 10 ** 18)),
                     "b": int(rng.integers(-2 ** 62, 2 ** 62)) * 10 ** 15,
                     "l": None if i % 5 == 0 else [None if j % 3 == 0 else j * 10 ** 20 - 7 for j in range(i % 9)]})
    cols = build_columns(s, rows)
    buf, offs = oracle.encode(s, cols, len(rows), 1)
    dec = oracle.decode(s, buf, offs, len(rows), 1)
    from helpers import columns_equal
    assert columns_equal(s, cols, dec) == []
    # a row whose 32 bytes are not a sign-extended decimal128: corrupt
    bad = buf.copy()
    row0 = 12  # frame 0's row (frame header 12 bytes); field b's 32 bytes follow the fixed part
    fixed = 8 + 3 * 8
    slot_b = int.from_bytes(bad[row0 + 16:row0 + 24].tobytes(), "little")
    at = row0 + (slot_b >> 32)
    bad[at + 20] ^= 0x40
    with pytest.raises(oracle.OracleError):
        oracle.decode(s, bad, offs, len(rows), 1)
    assert fixed == 32
