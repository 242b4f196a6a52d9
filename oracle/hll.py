"""stream-lib 2.7.0 HyperLogLog(log2m=8) + MurmurHash, restated.

TEST INFRASTRUCTURE — part of the oracle (see oracle/pinot_oracle.py header).

stream-lib is a third-party dependency absent from /root/reference
(`com.clearspring.analytics:stream` 2.7.0, reference pom.xml:702-705). Its call
sites are `DistinctCountHLLAggregationFunction.java:77-110,283-298,339-356`
(log2m = DEFAULT_LOG2M = 8, `:36`). The published algorithm is restated here
and pinned by the reference's DISTINCTCOUNTHLL known answers
(`InterSegmentAggregationSingleValueQueriesTest.java:189-206`: 5977, 23825,
1886, 4492, 3592, 11889, 1324, 3197), checked in tests/test_oracle_kats.py.

All arithmetic is 32-bit two's complement; `>>>` is a logical shift.
"""
import math
import struct
import numpy as np

LOG2M = 8
M = 1 << LOG2M
ALPHA_MM = (0.7213 / (1 + 1.079 / M)) * M * M
_M32 = 0xFFFFFFFF
_MUR_M = 0x5bd1e995


def _i32(x):
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def hash_long(data):
    """MurmurHash.hashLong(long) — Integer values are widened (sign-extended) first."""
    data &= 0xFFFFFFFFFFFFFFFF
    m = _MUR_M
    h = 0
    k = ((data & _M32) * m) & _M32
    k ^= k >> 24
    h ^= (k * m) & _M32
    k = (((data >> 32) & _M32) * m) & _M32
    k ^= k >> 24
    h = (h * m) & _M32
    h ^= (k * m) & _M32
    h ^= h >> 13
    h = (h * m) & _M32
    h ^= h >> 15
    return _i32(h)


def hash_long_np(values):
    """Vectorised hash_long over an int64 numpy array (returns uint32 hashes)."""
    d = np.asarray(values, dtype=np.int64).view(np.uint64)
    m = np.uint64(_MUR_M)
    mask = np.uint64(_M32)
    k = ((d & mask) * m) & mask
    k ^= k >> np.uint64(24)
    h = (k * m) & mask
    k = (((d >> np.uint64(32)) & mask) * m) & mask
    k ^= k >> np.uint64(24)
    h = (h * m) & mask
    h ^= (k * m) & mask
    h ^= h >> np.uint64(13)
    h = (h * m) & mask
    h ^= h >> np.uint64(15)
    return h.astype(np.uint32)


def hash_bytes(data: bytes, seed=-1):
    """MurmurHash.hash(byte[], len, seed=-1) — used for STRING values (UNVERIFIED: no STRING HLL KAT)."""
    m = _MUR_M
    length = len(data)
    h = (seed ^ length) & _M32
    len4 = length >> 2
    sb = [b - 256 if b > 127 else b for b in data]  # Java signed bytes
    for i in range(len4):
        i4 = i << 2
        k = sb[i4 + 3] & _M32
        k = ((k << 8) | (data[i4 + 2])) & _M32
        k = ((k << 8) | (data[i4 + 1])) & _M32
        k = ((k << 8) | (data[i4 + 0])) & _M32
        k = (k * m) & _M32
        k ^= k >> 24
        k = (k * m) & _M32
        h = (h * m) & _M32
        h ^= k
    left = length - (len4 << 2)
    if left != 0:
        if left >= 3:
            h ^= (sb[length - 3] << 16) & _M32
        if left >= 2:
            h ^= (sb[length - 2] << 8) & _M32
        if left >= 1:
            h ^= sb[length - 1] & _M32
        h = (h * m) & _M32
    h ^= h >> 13
    h = (h * m) & _M32
    h ^= h >> 15
    return _i32(h)


def hash_value(value, data_type):
    """MurmurHash.hash(Object) dispatch for the boxed value types Pinot offers."""
    if data_type in ("INT", "LONG"):
        return hash_long(int(value))
    if data_type == "DOUBLE":
        return hash_long(struct.unpack("<q", struct.pack("<d", float(value)))[0])
    if data_type == "FLOAT":
        return hash_long(struct.unpack("<i", struct.pack("<f", float(value)))[0])
    return hash_bytes(str(value).encode("utf-8"))


def register_and_rank(h):
    """offerHashed: j = h >>> (32 - log2m); r = nlz((h << log2m) | (1 << (log2m-1)) + 1) + 1."""
    h &= _M32
    j = h >> (32 - LOG2M)
    w = ((h << LOG2M) | ((1 << (LOG2M - 1)) + 1)) & _M32
    r = 32 - w.bit_length() + 1
    return j, r


def register_and_rank_np(h):
    h = np.asarray(h, dtype=np.uint32).astype(np.uint64)
    j = (h >> np.uint64(32 - LOG2M)).astype(np.int32)
    w = ((h << np.uint64(LOG2M)) | np.uint64((1 << (LOG2M - 1)) + 1)) & np.uint64(_M32)
    # nlz of 32-bit w (w != 0 always, bit 7 set)
    _, bitlen = np.frexp(w.astype(np.float64))  # exact bit length of w (< 2**53)
    nlz = 32 - bitlen.astype(np.int32)
    return j, (nlz + 1).astype(np.int32)


def java_round(x):
    """Math.round(double): floor(x + 0.5), +inf -> Long.MAX_VALUE."""
    if math.isinf(x) and x > 0:
        return 9223372036854775807
    if math.isnan(x):
        return 0
    return int(math.floor(x + 0.5))


def cardinality(registers):
    """HyperLogLog.cardinality() for log2m=8."""
    s = 0.0
    zeros = 0.0
    for v in registers:
        v = int(v)
        s += 1.0 / (1 << v)
        if v == 0:
            zeros += 1
    est = ALPHA_MM * (1.0 / s)
    if est <= 2.5 * M:
        lc = M * math.log(M / zeros) if zeros > 0 else float("inf")
        return java_round(lc)
    return java_round(est)


class HyperLogLog:
    def __init__(self):
        self.reg = np.zeros(M, dtype=np.int32)

    def offer_hashes(self, hashes):
        j, r = register_and_rank_np(hashes)
        np.maximum.at(self.reg, j, r)

    def add_all(self, other):
        np.maximum(self.reg, other.reg, out=self.reg)

    def cardinality(self):
        return cardinality(self.reg)
