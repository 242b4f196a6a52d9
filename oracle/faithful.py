"""ctypes driver of oracle/faithful.c (TEST INFRASTRUCTURE / CPU baseline; see pinot_oracle.py header).

Runs the reference-faithful per-doc executor for the scan-filter AND + COUNT/SUM query shape of the
bench (BASELINE.json configs[1]) over synthetic segments generated on the host."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libfaithful.so")


class Leaf(C.Structure):
    _fields_ = [("fwd", C.c_void_p), ("bits", C.c_int), ("kind", C.c_int), ("lo", C.c_int32), ("hi", C.c_int32),
                ("member", C.c_void_p)]


class Task(C.Structure):
    _fields_ = [("num_docs", C.c_int32), ("nleaves", C.c_int), ("leaves", C.POINTER(Leaf)),
                ("metric_fwd", C.c_void_p), ("metric_bits", C.c_int), ("metric_dict", C.c_void_p),
                ("count", C.c_int64), ("sum", C.c_double)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("oracle/build/libfaithful.so missing: make -C oracle")
        _lib = C.CDLL(LIB)
        _lib.pinot_faithful_run.argtypes = [C.POINTER(Task), C.c_int, C.c_int, C.POINTER(C.c_int64),
                                            C.POINTER(C.c_double)]
        _lib.pinot_fast_run.argtypes = [C.POINTER(Task), C.c_int, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_double)]
        _lib.pinot_synth_column.argtypes = [C.c_uint64, C.c_int, C.c_int32, C.c_int, C.c_int64, C.c_void_p]
        _lib.pinot_faithful_read_int.argtypes = [C.c_void_p, C.c_int32, C.c_int]
        _lib.pinot_faithful_read_int.restype = C.c_int32
        assert _lib.pinot_faithful_task_size() == C.sizeof(Task)
        assert _lib.pinot_faithful_leaf_size() == C.sizeof(Leaf)
    return _lib


def bits_for(card):
    return max(1, int(card - 1).bit_length())


def synth_column(seed, col_index, card, num_docs):
    lib = load()
    b = bits_for(card)
    buf = np.zeros((num_docs * b + 7) // 8 + 8, dtype=np.uint8)
    lib.pinot_synth_column(C.c_uint64(seed), col_index, card, b, num_docs, buf.ctypes.data_as(C.c_void_p))
    return buf


class SyntheticTable:
    """Host copy of synthetic segments: columns [(name, card)], segment s uses seed base_seed + s."""

    def __init__(self, columns, num_docs, num_segments, base_seed, needed):
        self.columns = list(columns)
        self.num_docs = num_docs
        self.segments = []
        for s in range(num_segments):
            cols = {}
            for i, (name, card) in enumerate(self.columns):
                if name in needed:
                    cols[name] = synth_column(base_seed + s, i, card, num_docs)
            self.segments.append(cols)

    def card(self, name):
        return dict(self.columns)[name]


def run_and_count_sum(table, leaves, metric, threads, optimized=False):
    """leaves: [(column, ("RANGE", lo, hi)) | (column, ("IN", [dictIds]))]; returns (count, sum).
    optimized: the batch-unpack executor (pinot_fast_run) instead of the reference-faithful one."""
    lib = load()
    keep = []
    tasks = (Task * len(table.segments))()
    metric_dict = np.arange(table.card(metric), dtype=np.float64) if metric else None  # identity dictionary
    for si, cols in enumerate(table.segments):
        arr = (Leaf * max(1, len(leaves)))()
        for li, (col, pred) in enumerate(leaves):
            arr[li].fwd = cols[col].ctypes.data
            arr[li].bits = bits_for(table.card(col))
            if pred[0] == "RANGE":
                arr[li].kind, arr[li].lo, arr[li].hi = 0, pred[1], pred[2]
            else:
                m = np.zeros(table.card(col), dtype=np.uint8)
                m[list(pred[1])] = 1
                keep.append(m)
                arr[li].kind = 1
                arr[li].member = m.ctypes.data
        keep.append(arr)
        t = tasks[si]
        t.num_docs = table.num_docs
        t.nleaves = len(leaves)
        t.leaves = arr
        if metric:
            t.metric_fwd = cols[metric].ctypes.data
            t.metric_bits = bits_for(table.card(metric))
            t.metric_dict = metric_dict.ctypes.data
    cnt = C.c_int64()
    sm = C.c_double()
    (lib.pinot_fast_run if optimized else lib.pinot_faithful_run)(tasks, len(table.segments), threads, C.byref(cnt),
                                                                   C.byref(sm))
    return cnt.value, sm.value


class GroupTask(C.Structure):
    _fields_ = [("num_docs", C.c_int32), ("nleaves", C.c_int), ("leaves", C.POINTER(Leaf)),
                ("g0_fwd", C.c_void_p), ("g1_fwd", C.c_void_p), ("g0_bits", C.c_int), ("g1_bits", C.c_int),
                ("g0_card", C.c_int32), ("m_fwd", C.c_void_p), ("m_bits", C.c_int), ("h_fwd", C.c_void_p),
                ("h_bits", C.c_int), ("ngroups", C.c_int32), ("keys", C.c_void_p), ("sum", C.c_void_p),
                ("cnt", C.c_void_p), ("regs", C.c_void_p)]


def run_group_by(table, leaves, g0, g1, metric, hll_col, threads):
    """Config-4 shape: GROUP BY g0, g1 with SUM / AVG(metric) and DISTINCTCOUNTHLL(hll_col) per segment (INT_MAP
    holder, per-group double sums, AvgPair, HyperLogLog), then the cross-segment combine. Returns
    (groups, total count, total sum)."""
    lib = load()
    lib.pinot_faithful_group_run.argtypes = [C.POINTER(GroupTask), C.c_int, C.c_int, C.c_int64,
                                             C.POINTER(C.c_int64), C.POINTER(C.c_double)]
    lib.pinot_faithful_group_run.restype = C.c_int64
    assert lib.pinot_faithful_group_task_size() == C.sizeof(GroupTask)
    keep = []
    tasks = (GroupTask * len(table.segments))()
    for si, cols in enumerate(table.segments):
        arr = (Leaf * max(1, len(leaves)))()
        for li, (col, pred) in enumerate(leaves):
            arr[li].fwd = cols[col].ctypes.data
            arr[li].bits = bits_for(table.card(col))
            arr[li].kind, arr[li].lo, arr[li].hi = 0, pred[1], pred[2]
        keep.append(arr)
        t = tasks[si]
        t.num_docs = table.num_docs
        t.nleaves = len(leaves)
        t.leaves = arr
        t.g0_fwd, t.g0_bits, t.g0_card = cols[g0].ctypes.data, bits_for(table.card(g0)), table.card(g0)
        t.g1_fwd, t.g1_bits = cols[g1].ctypes.data, bits_for(table.card(g1))
        t.m_fwd, t.m_bits = cols[metric].ctypes.data, bits_for(table.card(metric))
        if hll_col is not None:  # None: no DISTINCTCOUNTHLL in the query
            t.h_fwd, t.h_bits = cols[hll_col].ctypes.data, bits_for(table.card(hll_col))
    tc, ts = C.c_int64(), C.c_double()
    groups = lib.pinot_faithful_group_run(tasks, len(table.segments), threads, table.card(g0) * table.card(g1),
                                          C.byref(tc), C.byref(ts))
    return groups, tc.value, ts.value
