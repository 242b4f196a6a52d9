"""pinot_amd — MI355X-native executor for Pinot's segment query hot path.

The compute lives in libpinot_gpu.so (HIP kernels for gfx950 + C++ engine, C-ABI in
include/pinot_gpu.h). This package is the host-side mirror of Pinot's operator interface
(ServerQueryExecutorV1Impl / AggregationOperator / AggregationGroupByOperator / Combine*) over
that library, plus the segment-format writer used to feed it.
"""
from .segment import Segment, Column, build_segment, build_column, num_bits_per_value, pack_fixed_bit  # noqa: F401
from .pql import compile_pql, PqlCompilationException  # noqa: F401
from .executor import (GpuEngine, GpuSegment, GpuServer, ServerExecutor, ServerQueryExecutor, BrokerReduce,  # noqa: F401
                       AvgPair, HyperLogLog,
                       ExecutionStatistics, trim_intermediate_results, final_result, format_value,
                       validate_segment, segment_dir_info, raw_forward_index_values, prune_segment,
                       empty_datatable)
from ._lib import PinotGpuError, load as load_library  # noqa: F401
