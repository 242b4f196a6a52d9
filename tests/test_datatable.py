"""DataTable bytes (IntermediateResultsBlock.getDataTable -> DataTableImplV2.toBytes): the oracle codec, and the
library's pinot_datatable_aggregation — host code, so it runs here without a GPU — byte for byte against the
oracle's restatement of the Java writer. GPU-produced results: tests/test_gpu_datatable.py."""
import ctypes as C
import math
import struct

import numpy as np

import datatable as D
from pinot_amd import _lib, compile_pql
from pinot_amd.executor import QueryMarshal

STATS = dict(num_docs_scanned=12345, num_entries_scanned_in_filter=678901, num_entries_scanned_post_filter=24690,
             num_total_raw_docs=30000, num_segments_processed=3, num_segments_matched=2)


def _exec_stats():
    s = _lib.ExecStats()
    for k, v in STATS.items():
        setattr(s, k, v)
    return s


def test_java_string_hash_and_hashmap_order():
    # String.hashCode: s[0]*31^(n-1) + ... + s[n-1] (int overflow); HashMap buckets (h ^ h >>> 16) & (cap - 1)
    assert D.java_string_hash("") == 0
    assert D.java_string_hash("a") == 97 and D.java_string_hash("ab") == 97 * 31 + 98
    assert D.java_string_hash("polygenelubricants") == (-2147483648) & 0xFFFFFFFF  # the classic Integer.MIN_VALUE
    assert D.java_hashmap_order([3, 1, 2]) == [1, 2, 0]
    assert D.java_hashmap_order(list(range(20))) == list(range(20))  # Integer keys below the capacity: ascending
    # capacity grows past 12 entries: keys 16 and 0 collide in a 16-slot table but not in a 32-slot one
    assert D.java_hashmap_order([16] + list(range(12))) == [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 0]


def test_hll_register_words_round_trip():
    regs = [(7 * p + 3) % 26 for p in range(256)]
    b = D.hll_to_bytes(regs)
    assert len(b) == 8 + 43 * 4 and struct.unpack(">ii", b[:8]) == (8, 172)
    assert D.hll_from_bytes(b) == regs
    # register p lives in word p / 6 at bit 5 * (p % 6): register 7 = word 1 bits 5..9
    w1 = struct.unpack(">I", b[8 + 4:8 + 8])[0]
    assert (w1 >> 5) & 0x1F == regs[7]


def test_oracle_codec_round_trip():
    q = compile_pql("SELECT COUNT(*), SUM(met), MIN(met), MAX(met), AVG(met), DISTINCTCOUNTHLL(dim0) FROM t")
    vals = [42, 1.5e10, -3.0, math.inf, (7.25, 9), [p % 19 for p in range(256)]]
    d = D.decode(D.encode_aggregation(q, vals, STATS, server=(4, 17, 99)))
    assert d["rows"] == 1 and d["columns"] == 6
    assert [n for n, _ in d["schema"]] == ["count_star", "sum_met", "min_met", "max_met", "avg_met",
                                           "distinctCountHLL_dim0"]
    assert [t for _, t in d["schema"]] == ["LONG", "DOUBLE", "DOUBLE", "DOUBLE", "OBJECT", "OBJECT"]
    assert d["cells"][0] == vals
    md = dict(d["metadata"])
    assert md["numDocsScanned"] == "12345" and md["numSegmentsMatched"] == "2" and md["requestId"] == "99"
    assert md["timeUsedMs"] == "17" and md["numSegmentsQueried"] == "4" and "numGroupsLimitReached" not in md


def _native_aggregation(query, results, server=None):
    lib = _lib.load()
    m = QueryMarshal(query)
    stats = _exec_stats()
    srv = C.byref(_lib.DataTableServer(*server)) if server else None
    need = C.c_uint64()
    _lib.check(lib.pinot_datatable_aggregation(C.byref(m.q), results, C.byref(stats), srv, None, 0, C.byref(need)))
    buf = C.create_string_buffer(need.value)
    _lib.check(lib.pinot_datatable_aggregation(C.byref(m.q), results, C.byref(stats), srv, buf, need.value,
                                               C.byref(need)))
    small = C.create_string_buffer(4)
    assert lib.pinot_datatable_aggregation(C.byref(m.q), results, C.byref(stats), srv, small, 4, C.byref(need)) != 0
    return buf.raw


def test_native_aggregation_datatable_matches_oracle_bytes():
    rng = np.random.default_rng(3)
    for server in (None, (8, 123, -1), (1, 0, 77)):
        q = compile_pql("SELECT COUNT(*), SUM(m1), AVG(m2), MIN(m1), MAX(m3), DISTINCTCOUNTHLL(d1) FROM t")
        res = (_lib.AggResult * 6)()
        regs = rng.integers(0, 26, 256).astype(np.uint8)
        res[0].count = 123456789012
        res[1].value = float(rng.normal() * 1e12)
        res[2].value, res[2].count = 0.1 + 0.2, 3
        res[3].value = math.inf  # MIN over no docs
        res[4].value = -12.5
        for i in range(256):
            res[5].hll_registers[i] = int(regs[i])
        exp = D.encode_aggregation(q, [123456789012, res[1].value, (0.1 + 0.2, 3), math.inf, -12.5, regs.tolist()],
                                   STATS, server=server)
        assert _native_aggregation(q, res, server) == exp


def test_native_aggregation_datatable_rejects_bad_arguments():
    lib = _lib.load()
    q = QueryMarshal(compile_pql("SELECT COUNT(*) FROM t"))
    need = C.c_uint64()
    assert lib.pinot_datatable_aggregation(C.byref(q.q), None, None, None, None, 0, C.byref(need)) != 0
    assert lib.pinot_gpu_last_error()
