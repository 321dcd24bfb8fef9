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


# --- java.math.BigInteger fields ------------------------------------------------------
# BaseBinaryEncoderBuilder.java:192-194 writes writer.write(ordinal, value.toByteArray()):
# BinaryWriter.write(int, byte[]) -> writeUnaligned (BinaryWriter.java:167-194), i.e. the
# minimal big-endian two's complement (bitLength() / 8 + 1 bytes), zero-padded to 8, behind
# an (offset, length) slot; :559-560 reads it back as new BigInteger(bytes). The vectors
# below are BigInteger.toByteArray() worked by hand (java.math.BigInteger's documented
# contract; no JDK here).
BIGINT_VECTORS = [
    (0, "00"), (-1, "ff"), (1, "01"), (127, "7f"), (128, "0080"), (-128, "80"), (-129, "ff7f"),
    (255, "00ff"), (256, "0100"), (-256, "ff00"), (-257, "feff"), (32767, "7fff"), (32768, "008000"),
    (2 ** 63 - 1, "7fffffffffffffff"), (2 ** 63, "008000000000000000"), (-(2 ** 63), "8000000000000000"),
    (2 ** 127 - 1, "7f" + "ff" * 15), (-(2 ** 127), "80" + "00" * 15), (-(2 ** 127) + 1, "80" + "00" * 14 + "01"),
]


def big_schema(nullable=True):
    return Schema([Field("n", DataTypes.big_integer(), nullable)])


def test_java_biginteger_vectors_are_self_consistent():
    # the hand vectors against Python's own minimal two's complement (a second derivation)
    for v, hx in BIGINT_VECTORS:
        n = v.bit_length() if v >= 0 else (-v - 1).bit_length()
        assert len(hx) // 2 == n // 8 + 1
        assert bytes.fromhex(hx) == v.to_bytes(n // 8 + 1, "big", signed=True)


@pytest.mark.parametrize("v,hx", BIGINT_VECTORS)
def test_biginteger_row_bytes(v, hx):
    s = big_schema()
    cols = build_columns(s, [{"n": v}])
    buf, _ = oracle.encode(s, cols, 1, 0)
    b = buf.tobytes()
    want = bytes.fromhex(hx)
    pad = -len(want) % 8
    assert b[:8] == bytes(8)  # no null bit
    assert b[8:16] == (16 << 32 | len(want)).to_bytes(8, "little")  # (offset 16, toByteArray().length)
    assert b[16:] == want + bytes(pad)  # the bytes, then zeroOutPaddingBytes
    dec = oracle.decode(s, buf, np.array([0, len(b)], np.int64), 1, 0)
    assert decimal_value(dec[0].values[0], 0) == v


def test_biginteger_null_and_frames():
    s = big_schema()
    cols = build_columns(s, [{"n": None}, {"n": -129}])
    buf, offs = oracle.encode(s, cols, 2, 1)
    b = buf.tobytes()
    assert offs.tolist() == [0, 28, 28 + 12 + 24]
    assert b[12:20] == bytes([1]) + bytes(7) and b[20:28] == bytes(8)  # null: bit set, slot zero
    assert b[40 + 8:40 + 16] == (16 << 32 | 2).to_bytes(8, "little")
    assert b[40 + 16:] == bytes.fromhex("ff7f") + bytes(6)


def test_biginteger_corrupt_lengths():
    s = big_schema(False)
    cols = build_columns(s, [{"n": 5}])
    buf, offs = oracle.encode(s, cols, 1, 0)
    for size in (0, 17):  # "Zero length BigInteger"; more bytes than a decimal128 holds
        bad = np.zeros(16 + 24, np.uint8)
        bad[:16] = buf[:16]
        bad[8:12] = np.frombuffer(np.uint32(size).tobytes(), np.uint8)
        with pytest.raises(oracle.OracleError):
            oracle.decode(s, bad, np.array([0, len(bad)], np.int64), 1, 0)
    # a sign-extended (non-minimal) encoding is still a valid BigInteger: ff ff 7f = -129
    ok = np.zeros(24, np.uint8)
    ok[8:16] = np.frombuffer((16 << 32 | 3).to_bytes(8, "little"), np.uint8)
    ok[16:19] = [0xFF, 0xFF, 0x7F]
    dec = oracle.decode(s, ok, np.array([0, 24], np.int64), 1, 0)
    assert decimal_value(dec[0].values[0], 0) == -129


def test_biginteger_has_no_precision_check():
    s = big_schema()
    cols = build_columns(s, [{"n": 10 ** 38}, {"n": -(2 ** 127)}])  # 39 digits: fine for a BigInteger
    buf, offs = oracle.encode(s, cols, 2, 0)
    dec = oracle.decode(s, buf, offs, 2, 0)
    assert [decimal_value(dec[0].values[i], 0) for i in range(2)] == [10 ** 38, -(2 ** 127)]
