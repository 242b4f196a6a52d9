"""ctypes binding of libpinot_gpu.so (include/pinot_gpu.h).

The library is the product: HIP kernels + C++ engine. There is no CPU fallback anywhere in
this package — if the .so is missing or no HIP device exists, every entry point raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpinot_gpu.so")

PINOT_OK = 0
STATUS = {0: "PINOT_OK", 1: "PINOT_ERR_BAD_ARG", 2: "PINOT_ERR_OOM", 3: "PINOT_ERR_DEVICE",
          4: "PINOT_ERR_UNSUPPORTED", 5: "PINOT_ERR_BAD_QUERY", 6: "PINOT_ERR_TIMEOUT"}
PINOT_ERR_TIMEOUT = 6
DATA_TYPE = {"INT": 0, "LONG": 1, "FLOAT": 2, "DOUBLE": 3, "STRING": 4}
FILTER_OP = {"AND": 0, "OR": 1, "EQUALITY": 2, "NOT": 3, "RANGE": 4, "IN": 5, "NOT_IN": 6}
def sv_name(f):
    """The single-value function a multi-value one shares its intermediate result, merge and final result with
    (CountMVAggregationFunction extends CountAggregationFunction, ...): "COUNTMV" -> "COUNT"."""
    f = f.upper()
    return f[:-2] if f.endswith("MV") and f[:-2] in ("COUNT", "SUM", "MIN", "MAX", "AVG", "DISTINCTCOUNTHLL") else f


AGG_FN = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "AVG": 4, "DISTINCTCOUNTHLL": 5,
          "COUNTMV": 6, "SUMMV": 7, "MINMV": 8, "MAXMV": 9, "AVGMV": 10, "DISTINCTCOUNTHLLMV": 11}
# pinot_pruner bits; the server's default list (DefaultHelixStarterServerConfig.java:60-65)
PRUNER = {"DataSchemaSegmentPruner": 1, "ColumnValueSegmentPruner": 2, "ValidSegmentPruner": 4,
          "PartitionSegmentPruner": 8}
PRUNER_DEFAULT = 15

# every symbol include/pinot_gpu.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "pinot_gpu_last_error", "pinot_gpu_abi_version", "pinot_gpu_device_count",
    "pinot_gpu_engine_create", "pinot_gpu_engine_destroy", "pinot_gpu_engine_set_config",
    "pinot_gpu_segment_register", "pinot_gpu_segment_release", "pinot_gpu_segment_validate",
    "pinot_gpu_segment_load", "pinot_gpu_segment_acquire", "pinot_gpu_segment_attach_star_tree",
    "pinot_gpu_segment_dir_info",
    "pinot_gpu_segment_device_bytes", "pinot_gpu_filter", "pinot_gpu_aggregate", "pinot_gpu_group_by", "pinot_gpu_group_by_top",
    "pinot_groupby_num_groups", "pinot_groupby_num_columns", "pinot_groupby_key", "pinot_groupby_values",
    "pinot_groupby_hll", "pinot_groupby_raw_keys", "pinot_groupby_export_keys", "pinot_groupby_trim",
    "pinot_groupby_free", "pinot_datatable_aggregation", "pinot_datatable_group_by", "pinot_datatable_empty",
    "pinot_gpu_prune_segments", "pinot_segment_prune", "pinot_gpu_server_prune_segments", "pinot_broker_reduce",
    "pinot_gpu_group_by_layout", "pinot_gpu_group_by_partial", "pinot_gpu_group_by_finalize",
    "pinot_gpu_segment_register_synthetic", "pinot_gpu_segment_register_synthetic_ex", "pinot_gpu_synchronize",
    "pinot_gpu_last_kernel_ms", "pinot_gpu_engine_stat", "pinot_segment_read_raw_forward_index",
    "pinot_gpu_server_create", "pinot_gpu_server_unique_id", "pinot_gpu_server_create_rank", "pinot_gpu_server_destroy",
    "pinot_gpu_server_num_engines", "pinot_gpu_server_engine", "pinot_gpu_server_aggregate", "pinot_gpu_server_group_by",
    "pinot_gpu_server_last_phases", "pinot_gpu_transcode_raw", "pinot_gpu_server_group_by_top",
]


class PinotGpuError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("%s: %s" % (STATUS.get(status, status), msg))
        self.status = status


class ColumnDesc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data_type", C.c_int32), ("cardinality", C.c_int32),
                ("bits_per_value", C.c_int32), ("is_sorted", C.c_int32), ("has_inverted_index", C.c_int32),
                ("string_width", C.c_int32), ("padding_byte", C.c_int32), ("encoding", C.c_int32),
                ("dictionary", C.c_void_p), ("dictionary_len", C.c_uint64),
                ("forward_index", C.c_void_p), ("forward_index_len", C.c_uint64),
                ("sorted_index", C.c_void_p), ("sorted_index_len", C.c_uint64),
                ("inverted_index", C.c_void_p), ("inverted_index_len", C.c_uint64),
                ("min_value", C.c_char_p), ("max_value", C.c_char_p),
                ("bloom_filter", C.c_void_p), ("bloom_filter_len", C.c_uint64), ("create_bloom_filter", C.c_int32),
                ("num_partitions", C.c_int32), ("partition_function", C.c_char_p),
                ("partition_values", C.c_void_p), ("num_partition_values", C.c_int32), ("multi_value", C.c_int32),
                ("max_number_of_multi_values", C.c_int32), ("total_number_of_entries", C.c_int64)]


class SegmentDesc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("num_docs", C.c_int32), ("num_columns", C.c_int32),
                ("columns", C.POINTER(ColumnDesc))]


class StarTreeDesc(C.Structure):
    _fields_ = [("tree", C.c_void_p), ("tree_len", C.c_uint64), ("docs", C.POINTER(SegmentDesc))]


class FilterNode(C.Structure):
    _fields_ = [("op", C.c_int32), ("num_children", C.c_int32), ("column", C.c_char_p),
                ("num_values", C.c_int32), ("values", C.POINTER(C.c_char_p))]


class AggSpec(C.Structure):
    _fields_ = [("function", C.c_int32), ("column", C.c_char_p)]


class Query(C.Structure):
    _fields_ = [("num_filter_nodes", C.c_int32), ("filter", C.POINTER(FilterNode)),
                ("num_aggregations", C.c_int32), ("aggregations", C.POINTER(AggSpec)),
                ("num_group_by", C.c_int32), ("group_by", C.POINTER(C.c_char_p)),
                ("num_groups_limit", C.c_int32), ("max_init_group_holder_capacity", C.c_int32),
                ("timeout_ms", C.c_int32), ("pruners", C.c_int32)]


class ExecStats(C.Structure):
    _fields_ = [("num_docs_scanned", C.c_int64), ("num_entries_scanned_in_filter", C.c_int64),
                ("num_entries_scanned_post_filter", C.c_int64), ("num_total_raw_docs", C.c_int64),
                ("num_segments_processed", C.c_int64), ("device_ms", C.c_double),
                ("host_ms", C.c_double), ("num_segments_matched", C.c_int64)]


class DataTableServer(C.Structure):
    _fields_ = [("num_segments_queried", C.c_int64), ("time_used_ms", C.c_int64), ("request_id", C.c_int64)]


class AggResult(C.Structure):
    _fields_ = [("count", C.c_int64), ("value", C.c_double), ("exact_sum", C.c_int64),
                ("has_exact_sum", C.c_int32), ("reserved", C.c_int32), ("hll_cardinality", C.c_int64),
                ("hll_registers", C.c_uint8 * 256)]


class SegmentRef(C.Structure):
    _fields_ = [("engine", C.c_int32), ("reserved", C.c_int32), ("handle", C.c_int64)]


class PartialLayout(C.Structure):
    _fields_ = [("num_keys", C.c_int64), ("num_aggregations", C.c_int32), ("reserved", C.c_int32),
                ("acc_kind", C.c_int32 * 8), ("group_dictionary_fingerprint", C.c_uint64)]


_lib = None


def _share_hip_runtime_with_torch():
    """One HIP runtime per process. PyTorch-ROCm bundles its own libamdhip64 / libhsa-runtime64 (same
    sonames as /opt/rocm's). If this library loaded /opt/rocm's copy first, torch would later load a
    second runtime and fail to see the GPU ("No HIP GPUs are available"), which breaks the RCCL combine
    in the same process. When torch is installed, its runtime files are loaded (RTLD_GLOBAL, without
    importing torch) so this library binds to them, exactly as when torch is imported first.
    PINOT_GPU_HIP_RUNTIME=system keeps /opt/rocm's runtime."""
    if os.environ.get("PINOT_GPU_HIP_RUNTIME") == "system":
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    tlib = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        f = os.path.join(tlib, name)
        if os.path.exists(f):
            C.CDLL(f, mode=C.RTLD_GLOBAL)


def load(path=None):
    """Load libpinot_gpu.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # PINOT_GPU_LIB: another build of the same library (timing experiments on diagnostic builds); default the in-tree one
    p = path or os.environ.get("PINOT_GPU_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise PinotGpuError(3, "libpinot_gpu.so not built (%s); run `make -C incubator-pinot_amd`" % p)
    _share_hip_runtime_with_torch()
    lib = C.CDLL(p)
    P = C.c_void_p
    i32, i64, u64 = C.c_int32, C.c_int64, C.c_uint64
    sig = {
        "pinot_gpu_last_error": (C.c_char_p, []),
        "pinot_gpu_abi_version": (i32, []),
        "pinot_gpu_device_count": (i32, []),
        "pinot_gpu_engine_create": (i32, [i32, C.c_char_p, C.POINTER(P)]),
        "pinot_gpu_engine_destroy": (i32, [P]),
        "pinot_gpu_engine_set_config": (i32, [P, C.c_char_p]),
        "pinot_gpu_segment_register": (i32, [P, C.POINTER(SegmentDesc), C.POINTER(i64)]),
        "pinot_gpu_segment_release": (i32, [P, i64]),
        "pinot_gpu_segment_validate": (i32, [C.POINTER(SegmentDesc)]),
        "pinot_gpu_transcode_raw": (i32, [P, C.POINTER(ColumnDesc), i32, i32, C.POINTER(i32), C.POINTER(i32), P, u64,
                                          C.POINTER(u64), P, u64, C.POINTER(u64)]),
        "pinot_gpu_segment_load": (i32, [P, C.c_char_p, C.POINTER(i64)]),
        "pinot_gpu_segment_acquire": (i32, [P, C.c_char_p, C.POINTER(i64), C.POINTER(i32)]),
        "pinot_gpu_segment_attach_star_tree": (i32, [P, i64, C.POINTER(StarTreeDesc)]),
        "pinot_gpu_segment_dir_info": (i32, [C.c_char_p, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
        "pinot_gpu_segment_device_bytes": (i32, [P, i64, C.POINTER(u64)]),
        "pinot_gpu_filter": (i32, [P, i64, i32, C.POINTER(FilterNode), P, C.POINTER(i64)]),
        "pinot_gpu_aggregate": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), C.POINTER(AggResult),
                                      C.POINTER(ExecStats)]),
        "pinot_gpu_group_by": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), C.POINTER(P), C.POINTER(ExecStats)]),
        "pinot_gpu_group_by_top": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), i32, C.POINTER(P),
                                         C.POINTER(ExecStats)]),
        "pinot_groupby_num_groups": (i64, [P]),
        "pinot_groupby_num_columns": (i32, [P]),
        "pinot_groupby_key": (C.c_char_p, [P, i64]),
        "pinot_groupby_values": (i32, [P, i32, P, P]),
        "pinot_groupby_hll": (i32, [P, i32, P, P]),
        "pinot_groupby_raw_keys": (i32, [P, P]),
        "pinot_groupby_export_keys": (i32, [P, P, u64, P, C.POINTER(u64)]),
        "pinot_groupby_trim": (i32, [P, i32, i32, P, C.POINTER(i64)]),
        "pinot_datatable_aggregation": (i32, [C.POINTER(Query), P, C.POINTER(ExecStats), C.POINTER(DataTableServer),
                                              P, u64, C.POINTER(u64)]),
        "pinot_datatable_group_by": (i32, [C.POINTER(Query), P, P, P, C.POINTER(ExecStats),
                                           C.POINTER(DataTableServer), C.POINTER(P), C.POINTER(u64)]),
        "pinot_datatable_empty": (i32, [C.POINTER(Query), i64, C.POINTER(DataTableServer), P, u64, C.POINTER(u64)]),
        "pinot_gpu_prune_segments": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), i32, P, C.POINTER(i64)]),
        "pinot_segment_prune": (i32, [C.POINTER(SegmentDesc), C.POINTER(Query), i32, C.POINTER(i32)]),
        "pinot_gpu_server_prune_segments": (i32, [P, C.POINTER(SegmentRef), i32, C.POINTER(Query), i32, P,
                                                  C.POINTER(i64)]),
        "pinot_broker_reduce": (i32, [C.POINTER(Query), i32, C.POINTER(P), C.POINTER(u64), i32, P, u64,
                                      C.POINTER(u64)]),
        "pinot_groupby_free": (None, [P]),
        "pinot_gpu_group_by_layout": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), C.POINTER(PartialLayout)]),
        "pinot_gpu_group_by_partial": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), P, C.POINTER(P),
                                             C.POINTER(ExecStats)]),
        "pinot_gpu_group_by_finalize": (i32, [P, C.POINTER(i64), i32, C.POINTER(Query), P, C.POINTER(P),
                                              C.POINTER(P)]),
        "pinot_gpu_segment_register_synthetic": (i32, [P, C.c_char_p, i32, i32, C.POINTER(C.c_char_p),
                                                       C.POINTER(i32), u64, C.POINTER(i64)]),
        "pinot_gpu_segment_register_synthetic_ex": (i32, [P, C.c_char_p, i32, i32, C.POINTER(C.c_char_p),
                                                          C.POINTER(i32), C.POINTER(i32), u64, C.POINTER(i64)]),
        "pinot_gpu_synchronize": (i32, [P]),
        "pinot_gpu_last_kernel_ms": (i32, [P, i32, C.POINTER(C.c_double), C.POINTER(i64)]),
        "pinot_gpu_engine_stat": (i32, [P, C.c_char_p, C.POINTER(i64)]),
        "pinot_segment_read_raw_forward_index": (i32, [C.c_char_p, u64, i32, i32, P]),
        "pinot_gpu_server_create": (i32, [C.POINTER(i32), i32, C.c_char_p, C.POINTER(P)]),
        "pinot_gpu_server_unique_id": (i32, [P]),
        "pinot_gpu_server_create_rank": (i32, [i32, i32, i32, P, C.c_char_p, C.POINTER(P)]),
        "pinot_gpu_server_destroy": (i32, [P]),
        "pinot_gpu_server_num_engines": (i32, [P]),
        "pinot_gpu_server_engine": (i32, [P, i32, C.POINTER(P)]),
        "pinot_gpu_server_aggregate": (i32, [P, C.POINTER(SegmentRef), i32, C.POINTER(Query), C.POINTER(AggResult),
                                             C.POINTER(ExecStats)]),
        "pinot_gpu_server_group_by": (i32, [P, C.POINTER(SegmentRef), i32, C.POINTER(Query), C.POINTER(P),
                                            C.POINTER(ExecStats)]),
        "pinot_gpu_server_group_by_top": (i32, [P, C.POINTER(SegmentRef), i32, C.POINTER(Query), i32, C.POINTER(P),
                                                C.POINTER(ExecStats)]),
        "pinot_gpu_server_last_phases": (i32, [P, C.POINTER(C.c_double), i32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status):
    if status != PINOT_OK:
        msg = _lib.pinot_gpu_last_error().decode("utf-8", "replace") if _lib else ""
        raise PinotGpuError(status, msg)
