"""CPU oracle for the pruners' bloom filters and partition functions.

TEST INFRASTRUCTURE (see pinot_oracle.py's header): only tests/ use it, as the checker of the library's pruners.
PC = pinot-core/src/main/java/org/apache/pinot/core.

Bloom filter: Pinot's GuavaOnHeapBloomFilter (PC/bloom/GuavaOnHeapBloomFilter.java) over
com.google.common.hash.BloomFilter of guava 20.0 (pom.xml:317-320) — not in the container, so its published algorithm
is restated: Funnels.stringFunnel(UTF-8) of value.toString(), Hashing.murmur3_128() (MurmurHash3_x64_128, seed 0),
strategy MURMUR128_MITZ_64 (ordinal 1; MITZ_32, ordinal 0, for reading). File = BE int type (GUAVA_ON_HEAP = 1),
BE int version (1) (BloomFilterCreator.java:57-64), then BloomFilter.writeTo: byte strategy, byte numHashFunctions,
BE int word count, BE long words. Sizing: BloomFilterCreator.java:48-53, BloomFilterUtil.java (pinned by the known
answers of BloomFilterCreatorTest.testBloomFilterUtil), BloomFilter.create's optimalNumOfBits /
optimalNumOfHashFunctions. Bit positions: parity unpinned (no Java-written .bloom file in the reference).

Partition functions: PC/data/partition/{Modulo,Murmur,ByteArray,HashCode}PartitionFunction.java.
"""
import math
import struct

M64 = (1 << 64) - 1
LONG_MAX = (1 << 63) - 1


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M64
    k ^= k >> 33
    return k


def murmur3_x64_128(data: bytes):
    """MurmurHash3_x64_128 with seed 0: (h1, h2) as unsigned 64-bit (Guava's HashCode bytes are h1, h2 LE)."""
    c1, c2 = 0x87c37b91114253d5, 0x4cf5ad432745937f
    h1 = h2 = 0
    n = len(data)
    nblocks = n // 16
    for i in range(nblocks):
        k1, k2 = struct.unpack_from("<QQ", data, 16 * i)
        k1 = (k1 * c1) & M64
        k1 = _rotl(k1, 31)
        k1 = (k1 * c2) & M64
        h1 ^= k1
        h1 = _rotl(h1, 27)
        h1 = (h1 + h2) & M64
        h1 = (h1 * 5 + 0x52dce729) & M64
        k2 = (k2 * c2) & M64
        k2 = _rotl(k2, 33)
        k2 = (k2 * c1) & M64
        h2 ^= k2
        h2 = _rotl(h2, 31)
        h2 = (h2 + h1) & M64
        h2 = (h2 * 5 + 0x38495ab5) & M64
    tail = data[16 * nblocks:]
    k1 = k2 = 0
    if len(tail) > 8:
        for i in range(len(tail) - 1, 7, -1):
            k2 ^= tail[i] << (8 * (i - 8))
        k2 = (k2 * c2) & M64
        k2 = _rotl(k2, 33)
        k2 = (k2 * c1) & M64
        h2 ^= k2
    if tail:
        for i in range(min(len(tail), 8) - 1, -1, -1):
            k1 ^= tail[i] << (8 * i)
        k1 = (k1 * c1) & M64
        k1 = _rotl(k1, 31)
        k1 = (k1 * c2) & M64
        h1 ^= k1
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    h1 = _fmix(h1)
    h2 = _fmix(h2)
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    return h1, h2


def _java_round(x):
    return math.floor(x + 0.5)


def compute_num_bits(cardinality, p):
    """BloomFilterUtil.computeNumBits."""
    return int(math.ceil((cardinality * math.log(p)) / math.log(1.0 / math.pow(2.0, math.log(2.0)))))


def compute_num_hash_functions(cardinality, num_bits):
    """BloomFilterUtil.computeNumberOfHashFunctions."""
    return int(max(1.0, _java_round((num_bits / cardinality) * math.log(2.0))))


def compute_max_false_pos_probability(cardinality, k, num_bits):
    return math.pow(1.0 - math.exp(-1.0 * k / (num_bits / cardinality)), k)


class BloomFilter:
    def __init__(self, strategy, k, words):
        self.strategy, self.k, self.words = strategy, k, list(words)

    @classmethod
    def for_cardinality(cls, cardinality):
        """BloomFilterCreator(indexDir, column, cardinality) -> BloomFilter.create(stringFunnel, cardinality, fpp)."""
        mb_in_bits, fpp = 8388608, 0.05
        if cardinality > 0 and compute_num_bits(cardinality, fpp) > mb_in_bits:
            k = compute_num_hash_functions(cardinality, mb_in_bits)
            fpp = compute_max_false_pos_probability(cardinality, k, mb_in_bits)
        n = max(cardinality, 1)
        num_bits = int(-n * math.log(fpp) / (math.log(2) * math.log(2)))
        k = max(1, int(_java_round(num_bits / n * math.log(2))))
        return cls(1, k, [0] * ((num_bits + 63) // 64))

    def _bits(self, s):
        h1, h2 = murmur3_x64_128(s.encode("utf-8"))
        size = len(self.words) * 64
        if self.strategy == 0:
            def s32(x):
                x &= 0xFFFFFFFF
                return x - (1 << 32) if x >> 31 else x
            a, c = s32(h1), s32(h1 >> 32)
            for i in range(1, self.k + 1):
                comb = s32(a + i * c)
                if comb < 0:
                    comb = ~comb
                yield comb % size
            return
        comb = h1
        for _ in range(self.k):
            yield (comb & LONG_MAX) % size
            comb = (comb + h2) & M64

    def put(self, s):
        for b in self._bits(s):
            self.words[b >> 6] |= 1 << (b & 63)

    def might_contain(self, s):
        return all((self.words[b >> 6] >> (b & 63)) & 1 for b in self._bits(s))

    def to_bytes(self):
        out = struct.pack(">iiBBi", 1, 1, self.strategy, self.k, len(self.words))
        return out + b"".join(struct.pack(">Q", w) for w in self.words)

    @classmethod
    def from_bytes(cls, b):
        typ, ver, strategy, k, n = struct.unpack_from(">iiBBi", b, 0)
        assert typ == 1 and ver == 1 and len(b) == 14 + 8 * n
        return cls(strategy, k, struct.unpack_from(">%dQ" % n, b, 14))


# ---------------------------------------------------------------- partition functions
def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def kafka_murmur2(data: bytes):
    """MurmurPartitionFunction.murmur2 (Kafka Utils.murmur2, seed 0x9747b28c)."""
    m, r = 0x5bd1e995, 24
    n = len(data)
    h = (0x9747b28c ^ n) & 0xFFFFFFFF
    for i in range(n // 4):
        k = data[4 * i] | (data[4 * i + 1] << 8) | (data[4 * i + 2] << 16) | (data[4 * i + 3] << 24)
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> r
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
    t = n & ~3
    rem = n % 4
    if rem == 3:
        h ^= data[t + 2] << 16
    if rem >= 2:
        h ^= data[t + 1] << 8
    if rem >= 1:
        h ^= data[t]
        h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return _i32(h)


def java_string_hash(s):
    """String.hashCode over UTF-16 code units."""
    b = s.encode("utf-16-be")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + ((b[i] << 8) | b[i + 1])) & 0xFFFFFFFF
    return _i32(h)


def java_hash_code(data_type, value):
    """hashCode() of the boxed Integer / Long / Float / Double / String."""
    if data_type == "INT":
        return _i32(value)
    if data_type == "LONG":
        u = value & M64
        return _i32(u ^ (u >> 32))
    if data_type == "FLOAT":
        u = 0x7fc00000 if math.isnan(value) else struct.unpack(">I", struct.pack(">f", value))[0]
        return _i32(u)
    if data_type == "DOUBLE":
        u = 0x7ff8000000000000 if math.isnan(value) else struct.unpack(">Q", struct.pack(">d", value))[0]
        return _i32(u ^ (u >> 32))
    return java_string_hash(value)


def _java_mod(a, n):
    r = abs(a) % n
    return -r if a < 0 else r


def partition_of(function, num_partitions, data_type, value, to_string):
    """PartitionFunction.getPartition of the typed value; to_string = the value's Java toString."""
    f = function.lower()
    if f == "modulo":
        if data_type == "INT":
            return _java_mod(value, num_partitions)
        if data_type == "STRING":
            return _java_mod(int(value), num_partitions)
        raise ValueError("Illegal argument for partitioning, expected Integer")
    if f == "murmur":
        return (kafka_murmur2(to_string.encode("utf-8")) & 0x7fffffff) % num_partitions
    if f == "bytearray":
        h = 1
        for b in to_string.encode("utf-8"):
            h = (31 * h + (b - 256 if b > 127 else b)) & 0xFFFFFFFF
        h = _i32(h)
        a = 0 if h == -(1 << 31) else abs(h)
        return a % num_partitions
    if f == "hashcode":
        h = java_hash_code(data_type, value)
        a = h if h == -(1 << 31) else abs(h)
        return _java_mod(a, num_partitions)
    raise ValueError("No enum constant for: " + function)
