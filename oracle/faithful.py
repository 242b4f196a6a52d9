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


def run_and_count_sum(table, leaves, metric, threads):
    """leaves: [(column, ("RANGE", lo, hi)) | (column, ("IN", [dictIds]))]; returns (count, sum)."""
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
    lib.pinot_faithful_run(tasks, len(table.segments), threads, C.byref(cnt), C.byref(sm))
    return cnt.value, sm.value
