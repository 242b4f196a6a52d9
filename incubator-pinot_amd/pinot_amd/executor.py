"""Host-side mirror of Pinot's server query executor over the MI355X engine.

Shapes follow the reference so callers (and the parity tests) read like Pinot's own tests:
  * `ServerQueryExecutor.process_query(query, segments)` ~ `ServerQueryExecutorV1Impl.processQuery`
    (pinot-core/.../query/executor/ServerQueryExecutorV1Impl.java:100-267), returning the combined
    intermediate result (`IntermediateResultsBlock`) and `ExecutionStatistics`.
  * aggregation-only results: list per function of COUNT -> int, SUM/MIN/MAX -> float,
    AVG -> AvgPair(sum, count), DISTINCTCOUNTHLL -> HyperLogLog (registers + cardinality()).
  * group-by results: {group_key_string: [intermediate value per function]} as produced by
    `CombineGroupByOperator` (CombineGroupByOperator.java:104-228), trimmed like
    `AggregationGroupByTrimmingService` (:52-116) when it is larger than the trim threshold.
  * `BrokerReduce.reduce` ~ `BrokerReduceService` final results (formatted strings).
All compute happens in libpinot_gpu.so; this module only marshals arguments.
"""
import ctypes as C
import math
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, sv_name
from .pql import compile_pql
from .segment import Segment


@dataclass
class AvgPair:
    """`AvgPair` (query/aggregation/function/customobject/AvgPair.java:25-45)."""
    sum: float
    count: int


class HyperLogLog:
    """Merged stream-lib HyperLogLog(log2m=8) registers as the device produced them."""

    def __init__(self, registers, cardinality):
        if isinstance(registers, (bytes, bytearray)):
            registers = np.frombuffer(bytes(registers), dtype=np.uint8)
        self.registers = np.array(registers, dtype=np.uint8)
        self._card = int(cardinality)

    def cardinality(self):
        return self._card


@dataclass
class ExecutionStatistics:
    """`ExecutionStatistics` (pinot-core/.../operator/ExecutionStatistics.java:24-90)."""
    num_docs_scanned: int
    num_entries_scanned_in_filter: int
    num_entries_scanned_post_filter: int
    num_total_raw_docs: int
    num_segments_processed: int = 0
    device_ms: float = 0.0
    host_ms: float = 0.0
    num_segments_matched: int = 0


class GpuSegment:
    def __init__(self, engine, handle, name, num_docs):
        self.engine = engine
        self.handle = handle
        self.name = name
        self.num_docs = num_docs

    def device_bytes(self):
        out = C.c_uint64()
        check(self.engine.lib.pinot_gpu_segment_device_bytes(self.engine.ptr, self.handle, C.byref(out)))
        return out.value

    def attach_star_tree(self, segment: Segment, tree_bytes: bytes, dimensions, dims, metrics):
        """pinot_gpu_segment_attach_star_tree: the segment's star-tree v2 — the OffHeapStarTree bytes, the split-order
        dimensions' star-doc dictIds (int [num_star_docs, num_dims], STAR as 0; encoded with the segment's
        dictionaries) and the pair columns {"count__*": int64, "sum__x" / "min__x" / "max__x": float64,
        "avg__x": (sum float64, count int64), "distinctCountHLL__x": uint8 registers [num_star_docs, 256]}; the
        HyperLogLogs travel as their HyperLogLog.getBytes values in a raw STRING-layout column."""
        from .segment import Column, Segment as Seg, build_column, pack_fixed_bit
        n = int(np.asarray(dims).shape[0])
        cols = {}
        for j, d in enumerate(dimensions):
            pc = segment.column(d)
            cols[d] = Column(name=d, data_type=pc.data_type, cardinality=pc.cardinality, bits=pc.bits,
                             is_sorted=False, has_inverted_index=False, num_docs=n, dictionary=pc.dictionary,
                             string_width=pc.string_width, fwd=pack_fixed_bit(np.asarray(dims)[:, j], pc.bits),
                             padding=pc.padding)
        for name, vals in metrics.items():
            if getattr(vals, "ndim", 1) == 2:  # HyperLogLog registers [n, 256] -> getBytes values, raw var-byte
                enc = [_hll_bytes(r) for r in np.asarray(vals)]
                offs = np.zeros(n + 1, dtype=np.int64)
                offs[1:] = np.cumsum([len(b) for b in enc])
                c = Column(name=name, data_type="STRING", cardinality=0, bits=0, is_sorted=False,
                           has_inverted_index=False, num_docs=n, dictionary=b"", encoding="raw")
                c.fwd = offs.astype(">i4").tobytes() + b"".join(enc)
                cols[name] = c
                continue
            if isinstance(vals, tuple):  # an AvgPair column "avg__x": its halves "avg__x.sum" / "avg__x.count"
                cols[name + ".sum"] = build_column(name + ".sum", np.asarray(vals[0], dtype=np.float64), "DOUBLE", raw=True)
                cols[name + ".count"] = build_column(name + ".count", np.asarray(vals[1], dtype=np.int64), "LONG", raw=True)
                continue
            v = np.asarray(vals)
            cols[name] = build_column(name, v, "LONG" if v.dtype.kind in "iu" else "DOUBLE", raw=True)
        docs = Seg(name=segment.name + "$startree", num_docs=n, columns=cols)
        desc, keep = segment_desc(docs)
        tb = C.create_string_buffer(bytes(tree_bytes), len(tree_bytes))
        sd = _lib.StarTreeDesc(C.cast(tb, C.c_void_p), len(tree_bytes), C.pointer(desc))
        check(self.engine.lib.pinot_gpu_segment_attach_star_tree(self.engine.ptr, self.handle, C.byref(sd)))
        del keep

    def release(self):
        if self.handle is not None:
            check(self.engine.lib.pinot_gpu_segment_release(self.engine.ptr, self.handle))
            self.handle = None


def _hll_bytes(regs):
    """stream-lib HyperLogLog.getBytes (log2m 8): BE int 8, BE int 172, the RegisterSet's 43 BE int words (register p
    at bit 5 * (p % 6) of word p / 6)."""
    r = np.zeros(258, dtype=np.uint32)
    r[:256] = np.asarray(regs, dtype=np.uint32)
    words = (r.reshape(43, 6) << (5 * np.arange(6, dtype=np.uint32))).sum(axis=1, dtype=np.uint32)
    return np.array([8, 172], dtype=">i4").tobytes() + words.astype(">u4").tobytes()


def segment_desc(seg: Segment):
    """pinot_segment_desc over the segment's column buffers; the second value keeps the buffers alive."""
    keep = []
    cols = (_lib.ColumnDesc * max(len(seg.columns), 1))()
    for i, col in enumerate(seg.columns.values()):
        d = cols[i]
        name = col.name.encode()
        keep.append(name)
        d.name = name
        d.data_type = _lib.DATA_TYPE[col.data_type]
        d.cardinality = col.cardinality
        d.bits_per_value = col.bits
        d.is_sorted = int(col.is_sorted)
        d.has_inverted_index = int(col.has_inverted_index and not col.is_sorted)
        d.string_width = col.string_width
        d.padding_byte = col.padding if col.data_type == "STRING" else 0
        d.encoding = 1 if getattr(col, "encoding", "dictionary") == "raw" else 0
        if getattr(col, "min_value", None) is not None:
            mn, mx = col.min_value.encode(), col.max_value.encode()
            keep += [mn, mx]
            d.min_value, d.max_value = mn, mx
        bloom = getattr(col, "bloom_filter", None)
        if bloom is not None:
            bbuf = C.create_string_buffer(bytes(bloom), max(len(bloom), 1))
            keep.append(bbuf)
            d.bloom_filter, d.bloom_filter_len = C.cast(bbuf, C.c_void_p), len(bloom)
        d.create_bloom_filter = int(bool(getattr(col, "create_bloom_filter", False)))
        if getattr(col, "multi_value", False):
            d.multi_value = 1
            d.total_number_of_entries = int(col.total_entries)
            d.max_number_of_multi_values = int(col.max_multi_values)
        if getattr(col, "partition_function", None):
            fn = col.partition_function.encode()
            keep.append(fn)
            d.partition_function, d.num_partitions = fn, int(col.num_partitions)
            if col.partitions is None:
                d.num_partition_values = -1
            else:
                pv = (C.c_int32 * max(len(col.partitions), 1))(*col.partitions)
                keep.append(pv)
                d.partition_values, d.num_partition_values = C.cast(pv, C.c_void_p), len(col.partitions)
        for field, data in (("dictionary", col.dictionary), ("forward_index", col.fwd),
                            ("sorted_index", col.sorted_index), ("inverted_index", col.inverted)):
            if data is None:
                continue
            buf = C.create_string_buffer(bytes(data), len(data)) if len(data) else C.create_string_buffer(1)
            keep.append(buf)
            setattr(d, field, C.cast(buf, C.c_void_p))
            setattr(d, field + "_len", len(data))
    sname = seg.name.encode()
    keep += [sname, cols]
    return _lib.SegmentDesc(sname, seg.num_docs, len(seg.columns), cols), keep


def segment_dir_info(index_dir: str):
    """pinot_gpu_segment_dir_info: (num_docs, served columns, left-out columns) of a segment directory, read and
    checked on the host only."""
    lib = _lib.load()
    n, c, k = C.c_int32(), C.c_int32(), C.c_int32()
    check(lib.pinot_gpu_segment_dir_info(os.fsencode(index_dir), C.byref(n), C.byref(c), C.byref(k)))
    return n.value, c.value, k.value


def raw_forward_index_values(buf: bytes, data_type: str, num_docs: int):
    """pinot_segment_read_raw_forward_index: a fixed-width raw forward index file (.sv.raw.fwd) read by the library's
    FixedByteChunkSingleValueReader restatement on the host, as a numpy array."""
    dt = {"INT": (0, np.int32), "LONG": (1, np.int64), "FLOAT": (2, np.float32), "DOUBLE": (3, np.float64)}[data_type]
    out = np.zeros(max(num_docs, 1), dtype=dt[1])
    check(_lib.load().pinot_segment_read_raw_forward_index(bytes(buf), len(buf), dt[0], num_docs,
                                                    out.ctypes.data_as(C.c_void_p)))
    return out[:num_docs]


def validate_segment(seg: Segment) -> None:
    """pinot_gpu_segment_validate: the registration checks on the host alone (no engine, no GPU);
    raises PinotGpuError (BAD_ARG) naming the first bad column."""
    lib = _lib.load()
    desc, _keep = segment_desc(seg)
    check(lib.pinot_gpu_segment_validate(C.byref(desc)))


def prune_segment(seg: Segment, query, pruners=_lib.PRUNER_DEFAULT) -> bool:
    """pinot_segment_prune: SegmentPrunerService.prune for one segment, on the host alone (no engine, no GPU)."""
    lib = _lib.load()
    if isinstance(query, str):
        query = compile_pql(query)
    desc, _keep = segment_desc(seg)
    m = QueryMarshal(query)
    out = C.c_int32()
    check(lib.pinot_segment_prune(C.byref(desc), C.byref(m.q), int(pruners), C.byref(out)))
    return bool(out.value)


def empty_datatable(query, total_docs, server=None, num_groups_limit=100000):
    """pinot_datatable_empty: the DataTable processQuery answers when every segment was pruned."""
    lib = _lib.load()
    if isinstance(query, str):
        query = compile_pql(query)
    m = QueryMarshal(query, num_groups_limit)
    srv = C.byref(_lib.DataTableServer(*server)) if server else None
    need = C.c_uint64()
    check(lib.pinot_datatable_empty(C.byref(m.q), int(total_docs), srv, None, 0, C.byref(need)))
    buf = C.create_string_buffer(max(need.value, 1))
    check(lib.pinot_datatable_empty(C.byref(m.q), int(total_docs), srv, buf, need.value, C.byref(need)))
    return buf.raw[:need.value]


def _empty_result(query):
    """The combined result of zero segments: the functions' empty holders (extractAggregationResult of a fresh
    holder, DataTableBuilder.java:336-343) or an empty group map."""
    if query.get("group_by"):
        return {}
    out = []
    for a in query["aggregations"]:
        f = sv_name(a["function"])
        out.append({"COUNT": 0, "SUM": 0.0, "MIN": math.inf, "MAX": -math.inf}.get(f) if f not in (
            "AVG", "DISTINCTCOUNTHLL") else AvgPair(0.0, 0) if f == "AVG" else HyperLogLog(bytes(256), 0))
    return out


def _pruned_stats(total_docs):
    return ExecutionStatistics(0, 0, 0, total_docs, 0, 0.0, 0.0, 0)


class GpuEngine:
    """One engine per HIP device (`QueryExecutor.init/start/shutDown`)."""

    def __init__(self, device=0, config=None, _server_engine=None):
        self.lib = _lib.load()
        self.index = 0
        self.owned = _server_engine is None
        if _server_engine is not None:  # (server, index): an engine the server owns
            server, self.index = _server_engine
            ptr = C.c_void_p()
            check(self.lib.pinot_gpu_server_engine(server.ptr, self.index, C.byref(ptr)))
            self.ptr = ptr
            self.device = device
            self._server = server
            return
        ptr = C.c_void_p()
        check(self.lib.pinot_gpu_engine_create(device, config.encode() if config else None, C.byref(ptr)))
        self.ptr = ptr
        self.device = device

    def close(self):
        if self.ptr and self.owned:
            check(self.lib.pinot_gpu_engine_destroy(self.ptr))
        self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- segments
    def register(self, seg: Segment) -> GpuSegment:
        desc, _keep = segment_desc(seg)
        h = C.c_int64()
        check(self.lib.pinot_gpu_segment_register(self.ptr, C.byref(desc), C.byref(h)))
        return GpuSegment(self, h.value, seg.name, seg.num_docs)

    def transcode_raw(self, seg: Segment, column: str, on_device: bool = True):
        """pinot_gpu_transcode_raw: a raw column's dictionary form as registration builds it — (cardinality,
        bits per value, dictionary bytes, packed forward-index bytes); on the GPU when on_device (numeric columns)."""
        desc, _keep = segment_desc(seg)
        names = list(seg.columns)
        d = desc.columns[names.index(column)]
        card, bits = C.c_int32(), C.c_int32()
        dl, fl = C.c_uint64(), C.c_uint64()
        args = (self.ptr, C.byref(d), seg.num_docs, int(on_device), C.byref(card), C.byref(bits))
        check(self.lib.pinot_gpu_transcode_raw(*args, None, 0, C.byref(dl), None, 0, C.byref(fl)))
        dic = C.create_string_buffer(max(dl.value, 1))
        fwd = C.create_string_buffer(max(fl.value, 1))
        check(self.lib.pinot_gpu_transcode_raw(*args, dic, dl.value, C.byref(dl), fwd, fl.value, C.byref(fl)))
        return card.value, bits.value, dic.raw[:dl.value], fwd.raw[:fl.value]

    def load(self, index_dir: str) -> GpuSegment:
        """pinot_gpu_segment_load: a Pinot segment directory (v1/v2 files or v3 columns.psf) straight to HBM."""
        h = C.c_int64()
        check(self.lib.pinot_gpu_segment_load(self.ptr, os.fsencode(index_dir), C.byref(h)))
        n = C.c_int32()
        check(self.lib.pinot_gpu_segment_dir_info(os.fsencode(index_dir), C.byref(n), None, None))
        return GpuSegment(self, h.value, os.path.basename(os.path.normpath(index_dir)), n.value)

    def acquire(self, index_dir: str):
        """pinot_gpu_segment_acquire: the device segment cache (segment name + creation.meta CRC). Returns
        (GpuSegment, cache_hit); a hit is the cached copy's handle, a changed CRC replaces the old copy in the cache.
        Every returned GpuSegment holds one reference: release() returns it, the last one drops the device copy."""
        h, hit = C.c_int64(), C.c_int32()
        check(self.lib.pinot_gpu_segment_acquire(self.ptr, os.fsencode(index_dir), C.byref(h), C.byref(hit)))
        n = C.c_int32()
        check(self.lib.pinot_gpu_segment_dir_info(os.fsencode(index_dir), C.byref(n), None, None))
        return GpuSegment(self, h.value, os.path.basename(os.path.normpath(index_dir)), n.value), bool(hit.value)

    SYNTH_KIND = {"random": 0, "sorted": 1, "inverted": 2}

    def register_synthetic(self, name, num_docs, columns, seed):
        """Bench tooling: columns = [(name, cardinality[, kind])] with kind "random" (generated in HBM),
        "sorted" or "inverted" (bitmap inverted index, built on the host); see include/pinot_gpu.h."""
        names = (C.c_char_p * len(columns))(*[c[0].encode() for c in columns])
        cards = (C.c_int32 * len(columns))(*[int(c[1]) for c in columns])
        kinds = (C.c_int32 * len(columns))(*[self.SYNTH_KIND[c[2] if len(c) > 2 else "random"] for c in columns])
        h = C.c_int64()
        check(self.lib.pinot_gpu_segment_register_synthetic_ex(self.ptr, name.encode(), int(num_docs), len(columns),
                                                               names, cards, kinds, C.c_uint64(seed), C.byref(h)))
        return GpuSegment(self, h.value, name, num_docs)

    def set_config(self, config):
        check(self.lib.pinot_gpu_engine_set_config(self.ptr, config.encode()))

    def synchronize(self):
        check(self.lib.pinot_gpu_synchronize(self.ptr))

    def last_kernel_ms(self, kind):
        ms = C.c_double()
        n = C.c_int64()
        check(self.lib.pinot_gpu_last_kernel_ms(self.ptr, kind, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def stat(self, name):
        """Engine counter (pinot_gpu_engine_stat): "group.ring_queries", "group.ring_fallbacks"."""
        v = C.c_int64()
        check(self.lib.pinot_gpu_engine_stat(self.ptr, name.encode(), C.byref(v)))
        return v.value

    # ---------------------------------------------------------------- filter
    def filter(self, seg: GpuSegment, filter_tree):
        """`BaseFilterOperator.nextBlock().getBlockDocIdSet()` as a dense bitset + count."""
        m = QueryMarshal({"aggregations": [{"function": "COUNT", "column": "*"}], "filter": filter_tree,
                          "group_by": None})
        nwords = (seg.num_docs + 63) // 64
        bits = np.zeros(max(nwords, 1), dtype=np.uint64)
        cnt = C.c_int64()
        check(self.lib.pinot_gpu_filter(self.ptr, seg.handle, m.q.num_filter_nodes, m.q.filter,
                                        bits.ctypes.data_as(C.c_void_p), C.byref(cnt)))
        return bits[:nwords], cnt.value


def _postfix(tree, out, keep):
    if tree is None:
        return
    op = tree["operator"]
    if op in ("AND", "OR"):
        for c in tree["children"]:
            _postfix(c, out, keep)
        n = _lib.FilterNode()
        n.op = _lib.FILTER_OP[op]
        n.num_children = len(tree["children"])
        out.append(n)
        return
    n = _lib.FilterNode()
    n.op = _lib.FILTER_OP[op]
    col = tree["column"].encode()
    vals = [v.encode() for v in tree["values"]]
    arr = (C.c_char_p * len(vals))(*vals)
    keep.extend([col, vals, arr])
    n.column = col
    n.num_values = len(vals)
    n.values = arr
    out.append(n)


class QueryMarshal:
    """Query dict -> `pinot_query` (keeps every buffer alive for the duration of the call)."""

    def __init__(self, query, num_groups_limit=100000, max_init_group_holder_capacity=10000, timeout_ms=0, pruners=0):
        self.keep = []
        nodes = []
        _postfix(query.get("filter"), nodes, self.keep)
        self.nodes = (_lib.FilterNode * max(len(nodes), 1))(*nodes)
        aggs = query["aggregations"]
        self.aggs = (_lib.AggSpec * len(aggs))()
        for i, a in enumerate(aggs):
            fn = a["function"].upper()
            if fn not in _lib.AGG_FN:
                raise _lib.PinotGpuError(4, "unsupported aggregation function " + fn)
            self.aggs[i].function = _lib.AGG_FN[fn]
            c = a["column"].encode()
            self.keep.append(c)
            self.aggs[i].column = c
        gb = query.get("group_by")
        gcols = [c.encode() for c in gb["columns"]] if gb else []
        self.keep.append(gcols)
        self.gcols = (C.c_char_p * max(len(gcols), 1))(*gcols)
        self.q = _lib.Query(len(nodes), self.nodes, len(aggs), self.aggs, len(gcols), self.gcols,
                            num_groups_limit, max_init_group_holder_capacity, int(timeout_ms), int(pruners))


class GroupByResult:
    """Non-empty groups of a device group-by, with their intermediate values."""

    def __init__(self, lib, ptr, query):
        self.lib = lib
        self.ptr = ptr
        self.query = query

    def __del__(self):
        if getattr(self, "ptr", None):
            self.lib.pinot_groupby_free(self.ptr)
            self.ptr = None

    def num_groups(self):
        return self.lib.pinot_groupby_num_groups(self.ptr)

    def keys(self):
        """Every group key string through one bulk export call (pinot_groupby_export_keys)."""
        buf, offs = self.key_bytes()
        text = buf.decode("utf-8")
        if len(text) == len(buf):  # ASCII: byte offsets are character offsets
            return [text[offs[g]:offs[g + 1]] for g in range(offs.shape[0] - 1)]
        return [buf[offs[g]:offs[g + 1]].decode("utf-8") for g in range(offs.shape[0] - 1)]

    def key_bytes(self):
        n = self.num_groups()
        offs = np.zeros(n + 1, dtype=np.int64)
        need = C.c_uint64()
        check(self.lib.pinot_groupby_export_keys(self.ptr, None, 0, offs.ctypes.data_as(C.c_void_p), C.byref(need)))
        buf = C.create_string_buffer(max(need.value, 1))
        check(self.lib.pinot_groupby_export_keys(self.ptr, buf, need.value, offs.ctypes.data_as(C.c_void_p),
                                                 C.byref(need)))
        return buf.raw[:need.value], offs

    def trimmed_groups(self, top_n, fn):
        """Group indices of function fn's trimmed map (AggregationGroupByTrimmingService, native)."""
        k = C.c_int64()
        check(self.lib.pinot_groupby_trim(self.ptr, int(top_n), fn, None, C.byref(k)))
        out = np.zeros(max(k.value, 1), dtype=np.int64)
        check(self.lib.pinot_groupby_trim(self.ptr, int(top_n), fn, out.ctypes.data_as(C.c_void_p), C.byref(k)))
        return out[:k.value]

    def raw_keys(self):
        n = self.num_groups()
        out = np.zeros(max(n, 1), dtype=np.int64)
        check(self.lib.pinot_groupby_raw_keys(self.ptr, out.ctypes.data_as(C.c_void_p)))
        return out[:n]

    def function_values(self, fn):
        n = self.num_groups()
        counts = np.zeros(max(n, 1), dtype=np.int64)
        vals = np.zeros(max(n, 1), dtype=np.float64)
        check(self.lib.pinot_groupby_values(self.ptr, fn, counts.ctypes.data_as(C.c_void_p),
                                            vals.ctypes.data_as(C.c_void_p)))
        return counts[:n], vals[:n]

    def hll(self, fn):
        n = self.num_groups()
        regs = np.zeros((max(n, 1), 256), dtype=np.uint8)
        cards = np.zeros(max(n, 1), dtype=np.int64)
        check(self.lib.pinot_groupby_hll(self.ptr, fn, regs.ctypes.data_as(C.c_void_p),
                                         cards.ctypes.data_as(C.c_void_p)))
        return regs[:n], cards[:n]

    def data_table(self, marshal, stats, trim_top_n=None, server=None, zero_copy=False):
        """DataTable bytes of this result (pinot_datatable_group_by), each function's map trimmed to its own top
        groups (AggregationGroupByTrimmingService) when trim_top_n is given. zero_copy: a read-only memoryview of the
        result's own buffer (it keeps this result alive), as a transport would hand the native bytes on."""
        na = len(self.query["aggregations"])
        groups = nums = None
        if trim_top_n is not None:
            kept = [self.trimmed_groups(trim_top_n, i) for i in range(na)]
            groups = (C.c_void_p * na)(*[k.ctypes.data_as(C.c_void_p) for k in kept])
            nums = (C.c_int64 * na)(*[k.shape[0] for k in kept])
        data, size = C.c_void_p(), C.c_uint64()
        check(self.lib.pinot_datatable_group_by(C.byref(marshal.q), self.ptr, groups, nums, C.byref(stats), server,
                                                C.byref(data), C.byref(size)))
        if not size.value:
            return b""
        if zero_copy:
            view = (C.c_ubyte * size.value).from_address(data.value)
            view.owner = self  # the bytes live in the native result until it is freed
            return memoryview(view).cast("B").toreadonly()
        return C.string_at(data, size.value)

    def to_map(self, trim_top_n=None):
        """{string_key: [intermediate result per function]} (the CombineGroupByOperator result map).

        trim_top_n: apply AggregationGroupByTrimmingService.trimIntermediateResultsMap (native): the reference
        returns one map per function, so a group trimmed from function i's map carries None at position i."""
        keys = self.keys()
        cols = []
        for i, a in enumerate(self.query["aggregations"]):
            f = sv_name(a["function"])
            if f == "DISTINCTCOUNTHLL":
                regs, cards = self.hll(i)
                cols.append([HyperLogLog(regs[g], cards[g]) for g in range(len(keys))])
                continue
            counts, vals = self.function_values(i)
            if f == "COUNT":
                cols.append([int(c) for c in counts])
            elif f == "AVG":
                cols.append([AvgPair(float(v), int(c)) for v, c in zip(vals, counts)])
            else:
                cols.append([float(v) for v in vals])
        if trim_top_n is None:
            return {k: [col[g] for col in cols] for g, k in enumerate(keys)}
        kept = [self.trimmed_groups(trim_top_n, i) for i in range(len(cols))]
        if all(k.shape[0] == len(keys) for k in kept):
            return {k: [col[g] for col in cols] for g, k in enumerate(keys)}
        out = {}
        for i, (col, sel) in enumerate(zip(cols, kept)):
            for g in sel.tolist():
                out.setdefault(keys[g], [None] * len(cols))[i] = col[g]
        return out


class GpuServer:
    """Multi-GPU server (pinot_gpu_server_*): one engine per device and RCCL communicators inside the library.

    GpuServer(devices=[0, 1, ...]) serves several GPUs from this process; GpuServer.rank(device, nranks, rank, uid)
    is one rank of a multi-process server (uid from GpuServer.unique_id() on rank 0, shared out of band)."""

    def __init__(self, devices=(0,), config=None, _ptr=None, _devices=None):
        self.lib = _lib.load()
        if _ptr is None:
            devs = (C.c_int32 * len(devices))(*devices)
            ptr = C.c_void_p()
            check(self.lib.pinot_gpu_server_create(devs, len(devices), config.encode() if config else None, C.byref(ptr)))
            _ptr, _devices = ptr, list(devices)
        self.ptr = _ptr
        self.engines = [GpuEngine(d, _server_engine=(self, i)) for i, d in enumerate(_devices)]

    @staticmethod
    def unique_id():
        lib = _lib.load()
        buf = (C.c_uint8 * 128)()
        check(lib.pinot_gpu_server_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rank(cls, device, nranks, rank, uid, config=None):
        lib = _lib.load()
        ptr = C.c_void_p()
        ub = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(lib.pinot_gpu_server_create_rank(device, nranks, rank, ub, config.encode() if config else None,
                                               C.byref(ptr)))
        srv = cls(_ptr=ptr, _devices=[device])
        srv.multi_process = True
        return srv

    PHASES = ("local", "exchange", "partials", "agree", "reduce_scatter", "finalize", "gather_d2h", "total")

    def last_phases(self):
        """pinot_gpu_server_last_phases: host ms per phase of the last query on the first engine's rank."""
        ms = (C.c_double * 8)()
        check(self.lib.pinot_gpu_server_last_phases(self.ptr, ms, 8))
        return dict(zip(self.PHASES, list(ms)))

    def close(self):
        if self.ptr:
            for e in self.engines:
                e.ptr = None
            check(self.lib.pinot_gpu_server_destroy(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ServerExecutor:
    """`ServerQueryExecutorV1Impl.processQuery` over segments spread across a GpuServer's GPUs: the library runs
    each GPU's share and combines them (pinot_gpu_server_aggregate / _group_by)."""

    def __init__(self, server: GpuServer, num_groups_limit=100000, max_init_group_holder_capacity=10000, timeout_ms=0,
                 pruners=_lib.PRUNER_DEFAULT):
        self.server = server
        self.num_groups_limit = num_groups_limit
        self.max_init = max_init_group_holder_capacity
        self.timeout_ms = timeout_ms
        self.pruners = pruners

    def _refs(self, segments):
        arr = (_lib.SegmentRef * max(len(segments), 1))()
        for i, s in enumerate(segments):
            arr[i].engine = s.engine.index
            arr[i].handle = s.handle
        return arr

    def _query(self, query):
        if isinstance(query, PreparedQuery):
            return query.query, query.marshal
        if isinstance(query, str):
            query = compile_pql(query)
        return query, self._marshal(query)

    def group_by_result(self, query, segments, top_n=None):
        """(native result, stats) of the merged group-by; top_n: the server's trimmed answer
        (pinot_gpu_server_group_by_top: each rank trims its own key range before the gather to rank 0)."""
        res, stats, _ = self._group_by(query, segments, top_n)
        return res, _stats(stats)

    def _group_by(self, query, segments, top_n):
        query, m = self._query(query)
        lib = self.server.lib
        stats = _lib.ExecStats()
        out = C.c_void_p()
        refs = self._refs(segments)
        if top_n:
            check(lib.pinot_gpu_server_group_by_top(self.server.ptr, refs, len(segments), C.byref(m.q), top_n,
                                                    C.byref(out), C.byref(stats)))
        else:
            check(lib.pinot_gpu_server_group_by(self.server.ptr, refs, len(segments), C.byref(m.q), C.byref(out),
                                                C.byref(stats)))
        return GroupByResult(lib, out, query), stats, m

    def process_query_datatable(self, query, segments, trim=True, server=None, zero_copy=False):
        """The server's answer to the broker as DataTable bytes (rank 0's; the other ranks' results are empty):
        group-bys trimmed per function on the device across the ranks when `trim`."""
        query, m = self._query(query)
        if not query.get("group_by"):
            raise ValueError("process_query_datatable on the multi-GPU server serves group-by queries")
        top_n = query["group_by"].get("top_n", 10) if trim else None
        res, stats, m = self._group_by(PreparedQuery(query, m), segments, top_n)
        srv = C.byref(_lib.DataTableServer(*server)) if server else None
        return res.data_table(m, stats, top_n, srv, zero_copy), _stats(stats)

    def process_query(self, query, segments, trim=True, as_result=False):
        """Every rank calls this with its own segments (possibly none): pruning (the executor's pruners, carried in
        the query) and the merge across GPUs / ranks happen inside the library, where a failure on any rank fails
        every rank with the same status instead of leaving peers in a collective."""
        query, m = self._query(query)
        lib = self.server.lib
        refs = self._refs(segments)
        stats = _lib.ExecStats()
        if query.get("group_by"):
            out = C.c_void_p()
            check(lib.pinot_gpu_server_group_by(self.server.ptr, refs, len(segments), C.byref(m.q), C.byref(out),
                                                C.byref(stats)))
            res = GroupByResult(lib, out, query)
            if not as_result:
                res = res.to_map(trim_top_n=query["group_by"].get("top_n", 10) if trim else None)
        else:
            n = len(query["aggregations"])
            out = (_lib.AggResult * n)()
            check(lib.pinot_gpu_server_aggregate(self.server.ptr, refs, len(segments), C.byref(m.q), out,
                                                 C.byref(stats)))
            res = [_agg_value(sv_name(a["function"]), out[i]) for i, a in enumerate(query["aggregations"])]
        return res, _stats(stats)

    def _marshal(self, query):
        return QueryMarshal(query, self.num_groups_limit, self.max_init, self.timeout_ms, self.pruners)

    def prepare(self, query):
        if isinstance(query, str):
            query = compile_pql(query)
        return PreparedQuery(query, self._marshal(query))


def _segment_handles(segments):
    arr = (C.c_int64 * len(segments))(*[s.handle for s in segments])
    return arr


@dataclass
class PreparedQuery:
    query: dict
    marshal: "QueryMarshal"


class ServerQueryExecutor:
    """`ServerQueryExecutorV1Impl.processQuery` over GPU-resident segments of one engine."""

    def __init__(self, engine: GpuEngine, num_groups_limit=100000, max_init_group_holder_capacity=10000,
                 timeout_ms=0, pruners=_lib.PRUNER_DEFAULT):
        self.engine = engine
        self.num_groups_limit = num_groups_limit
        self.max_init = max_init_group_holder_capacity
        self.timeout_ms = timeout_ms
        self.pruners = pruners  # pinot_pruner bits (0 = no pruning); default: the server's default pruner list

    def prune(self, query, segments):
        """ServerQueryExecutorV1Impl.pruneSegments (:270-294): (segments kept, totalDocs over all of them)."""
        m = query.marshal if isinstance(query, PreparedQuery) else QueryMarshal(
            compile_pql(query) if isinstance(query, str) else query)
        kept, total, _ = self._prune(m, segments)
        return kept, total

    def _prune(self, m, segments):
        handles = _segment_handles(segments)
        pruned = (C.c_uint8 * max(len(segments), 1))()
        total = C.c_int64()
        check(self.engine.lib.pinot_gpu_prune_segments(self.engine.ptr, handles, len(segments), C.byref(m.q),
                                                       int(self.pruners), pruned, C.byref(total)))
        if not any(pruned[:len(segments)]):
            return segments, total.value, handles  # the common case: the handle array is reused for the plan
        kept = [sg for i, sg in enumerate(segments) if not pruned[i]]
        return kept, total.value, (_segment_handles(kept) if kept else None)

    def prepare(self, query):
        """Compile + marshal a query once (a prepared statement); process_query accepts the result.
        Only the ctypes argument structs are reused: every execution still plans, resolves predicates
        against each segment's dictionary and runs the device path."""
        if isinstance(query, str):
            query = compile_pql(query)
        return PreparedQuery(query, QueryMarshal(query, self.num_groups_limit, self.max_init, self.timeout_ms,
                                                 self.pruners))

    def process_query(self, query, segments, trim=True):
        """processQuery: the library prunes (the executor's pruners travel in the query), plans and runs the rest;
        totalDocs counts every segment, an all-pruned query gives the empty result."""
        if isinstance(query, PreparedQuery):
            query, m = query.query, query.marshal
        else:
            if isinstance(query, str):
                query = compile_pql(query)
            m = QueryMarshal(query, self.num_groups_limit, self.max_init, self.timeout_ms, self.pruners)
        lib = self.engine.lib
        if not segments:
            return _empty_result(query), _pruned_stats(0)
        handles = _segment_handles(segments)
        stats = _lib.ExecStats()
        if query.get("group_by"):
            out = C.c_void_p()
            top_n = query["group_by"].get("top_n", 10) if trim else None
            if top_n:  # CombineGroupByOperator's trim on the device: only the kept groups leave it
                check(lib.pinot_gpu_group_by_top(self.engine.ptr, handles, len(segments), C.byref(m.q), top_n,
                                                 C.byref(out), C.byref(stats)))
            else:
                check(lib.pinot_gpu_group_by(self.engine.ptr, handles, len(segments), C.byref(m.q), C.byref(out),
                                             C.byref(stats)))
            res = GroupByResult(lib, out, query).to_map(trim_top_n=top_n)
        else:
            n = len(query["aggregations"])
            out = (_lib.AggResult * n)()
            check(lib.pinot_gpu_aggregate(self.engine.ptr, handles, len(segments), C.byref(m.q), out,
                                          C.byref(stats)))
            res = [_agg_value(sv_name(a["function"]), out[i]) for i, a in enumerate(query["aggregations"])]
        return res, _stats(stats)

    def process_query_datatable(self, query, segments, trim=True, server=None, zero_copy=False):
        """`processQuery` as the server answers the broker: the combined result as DataTable bytes
        (IntermediateResultsBlock.getDataTable -> DataTableImplV2.toBytes, built natively by pinot_datatable_*).
        Group-by maps are trimmed per function like CombineGroupByOperator when `trim`; `server` =
        (numSegmentsQueried, timeUsedMs, requestId or -1) adds the server's own metadata keys."""
        if isinstance(query, PreparedQuery):
            query, m = query.query, query.marshal
        else:
            if isinstance(query, str):
                query = compile_pql(query)
            m = QueryMarshal(query, self.num_groups_limit, self.max_init, self.timeout_ms)
        lib = self.engine.lib
        srv = C.byref(_lib.DataTableServer(*server)) if server else None
        total = None
        handles = None
        if self.pruners:
            segments, total, handles = self._prune(m, segments)
            if not segments:  # every segment pruned: buildEmptyDataTable (:187-196)
                need = C.c_uint64()
                check(lib.pinot_datatable_empty(C.byref(m.q), total, srv, None, 0, C.byref(need)))
                buf = C.create_string_buffer(max(need.value, 1))
                check(lib.pinot_datatable_empty(C.byref(m.q), total, srv, buf, need.value, C.byref(need)))
                return buf.raw[:need.value], _pruned_stats(total)
        if handles is None:
            handles = _segment_handles(segments)
        stats = _lib.ExecStats()
        if query.get("group_by"):
            out = C.c_void_p()
            top_n = query["group_by"].get("top_n", 10) if trim else None
            if top_n:
                check(lib.pinot_gpu_group_by_top(self.engine.ptr, handles, len(segments), C.byref(m.q), top_n,
                                                 C.byref(out), C.byref(stats)))
            else:
                check(lib.pinot_gpu_group_by(self.engine.ptr, handles, len(segments), C.byref(m.q), C.byref(out),
                                             C.byref(stats)))
            if total is not None:
                stats.num_total_raw_docs = total
            res = GroupByResult(lib, out, query)
            return res.data_table(m, stats, top_n, srv, zero_copy), _stats(stats)
        n = len(query["aggregations"])
        out = (_lib.AggResult * n)()
        check(lib.pinot_gpu_aggregate(self.engine.ptr, handles, len(segments), C.byref(m.q), out, C.byref(stats)))
        if total is not None:
            stats.num_total_raw_docs = total
        need = C.c_uint64()
        check(lib.pinot_datatable_aggregation(C.byref(m.q), out, C.byref(stats), srv, None, 0, C.byref(need)))
        buf = C.create_string_buffer(max(need.value, 1))
        check(lib.pinot_datatable_aggregation(C.byref(m.q), out, C.byref(stats), srv, buf, need.value, C.byref(need)))
        return buf.raw[:need.value], _stats(stats)

    def group_by_result(self, query, segments, top_n=None):
        """Raw device group-by result object: every group, or with top_n the device-trimmed result the server hands to
        its DataTable (pinot_gpu_group_by_top: the union of the functions' trimmed maps)."""
        if isinstance(query, PreparedQuery):
            query, m = query.query, query.marshal
        else:
            if isinstance(query, str):
                query = compile_pql(query)
            m = QueryMarshal(query, self.num_groups_limit, self.max_init, self.timeout_ms, self.pruners)
        out = C.c_void_p()
        stats = _lib.ExecStats()
        if top_n:
            check(self.engine.lib.pinot_gpu_group_by_top(self.engine.ptr, _segment_handles(segments), len(segments),
                                                         C.byref(m.q), int(top_n), C.byref(out), C.byref(stats)))
        else:
            check(self.engine.lib.pinot_gpu_group_by(self.engine.ptr, _segment_handles(segments), len(segments),
                                                     C.byref(m.q), C.byref(out), C.byref(stats)))
        return GroupByResult(self.engine.lib, out, query), stats


def _stats(s):
    return ExecutionStatistics(s.num_docs_scanned, s.num_entries_scanned_in_filter, s.num_entries_scanned_post_filter,
                               s.num_total_raw_docs, s.num_segments_processed, s.device_ms, s.host_ms,
                               s.num_segments_matched)


def _agg_value(f, r):
    if f == "COUNT":
        return int(r.count)
    if f in ("SUM", "MIN", "MAX"):
        return float(r.value)
    if f == "AVG":
        return AvgPair(float(r.value), int(r.count))
    if f == "DISTINCTCOUNTHLL":
        return HyperLogLog(bytes(r.hll_registers), r.hll_cardinality)
    raise ValueError(f)


# ---------------------------------------------------------------------- results handling
def final_result(f, v):
    """`AggregationFunction.extractFinalResult`: AVG -> sum/count or -inf (AvgAggregationFunction.java:35,222-230)."""
    f = sv_name(f)
    if f == "AVG":
        return v.sum / v.count if v.count else -math.inf
    if f == "DISTINCTCOUNTHLL":
        return v.cardinality()
    return v


def merge(f, a, b):
    f = sv_name(f)
    if f in ("COUNT", "SUM"):
        return a + b
    if f == "MIN":
        return min(a, b)
    if f == "MAX":
        return max(a, b)
    if f == "AVG":
        return AvgPair(a.sum + b.sum, a.count + b.count)
    if f == "DISTINCTCOUNTHLL":
        regs = np.maximum(a.registers, b.registers)
        from ._hll import cardinality
        return HyperLogLog(regs, cardinality(regs))
    raise ValueError(f)


def trim_intermediate_results(query, result, trim_size=None):
    """`AggregationGroupByTrimmingService.trimIntermediateResultsMap` (:52-116) over an untrimmed result map, with
    the native rule (pinot_groupby_trim): above 4 * max(5*topN, 5000) groups each function keeps its own
    max(5*topN, 5000) best groups (MIN ascending, others descending); a group trimmed from function i's map carries
    None at position i (the reference returns one map per function)."""
    top_n = query["group_by"].get("top_n", 10)
    keep_n = trim_size if trim_size is not None else max(5 * top_n, 5000)
    if len(result) <= 4 * keep_n:
        return result
    out = {}
    for i, a in enumerate(query["aggregations"]):
        f = sv_name(a["function"])
        items = sorted(result.items(), key=lambda kv: final_result(f, kv[1][i]), reverse=(f != "MIN"))
        for k, v in items[:keep_n]:
            out.setdefault(k, [None] * len(v))[i] = v[i]
    return out


def format_value(f, v):
    """Broker string form (`String.format("%.5f")` for doubles, plain integers otherwise)."""
    v = final_result(f, v)
    if sv_name(f) in ("COUNT", "DISTINCTCOUNTHLL"):
        return str(int(v))
    return "%.5f" % v


class BrokerReduce:
    """`BrokerReduceService` over several server results of one query."""

    @staticmethod
    def reduce_datatables(query, tables, top_n=None):
        """pinot_broker_reduce: BrokerReduceService.reduceOnDataTable over the servers' DataTable bytes, in the
        library; returns the BrokerResponseNative as a dict (values formatted by AggregationFunctionUtils)."""
        import json
        lib = _lib.load()
        if isinstance(query, str):
            query = compile_pql(query)
        if top_n is None:
            top_n = (query.get("group_by") or {}).get("top_n", 10)
        m = QueryMarshal(query)
        n = len(tables)
        keep = [C.create_string_buffer(bytes(t), max(len(t), 1)) for t in tables]
        ptrs = (C.c_void_p * max(n, 1))(*[C.cast(b, C.c_void_p) for b in keep])
        lens = (C.c_uint64 * max(n, 1))(*[len(t) for t in tables])
        need = C.c_uint64()
        check(lib.pinot_broker_reduce(C.byref(m.q), n, ptrs, lens, int(top_n), None, 0, C.byref(need)))
        buf = C.create_string_buffer(max(need.value, 1))
        check(lib.pinot_broker_reduce(C.byref(m.q), n, ptrs, lens, int(top_n), buf, need.value, C.byref(need)))
        return json.loads(buf.raw[:need.value].decode("utf-8"))

    @staticmethod
    def reduce(query, server_results):
        fns = [sv_name(a["function"]) for a in query["aggregations"]]
        if query.get("group_by"):
            # per function (the servers' trimmed maps are per function: None = trimmed there)
            merged = [{} for _ in fns]
            for r in server_results:
                for k, vals in r.items():
                    for i, (f, v) in enumerate(zip(fns, vals)):
                        if v is None:
                            continue
                        merged[i][k] = merge(f, merged[i][k], v) if k in merged[i] else v
            top_n = query["group_by"].get("top_n", 10)
            out = []
            for i, f in enumerate(fns):
                items = sorted(((k, final_result(f, v)) for k, v in merged[i].items()), key=lambda kv: kv[1],
                               reverse=(f != "MIN"))[:top_n]
                out.append([(k, ("%d" % v) if f in ("COUNT", "DISTINCTCOUNTHLL") else "%.5f" % v) for k, v in items])
            return out
        acc = None
        for r in server_results:
            acc = list(r) if acc is None else [merge(f, x, y) for f, x, y in zip(fns, acc, r)]
        return [format_value(f, v) for f, v in zip(fns, acc)]
