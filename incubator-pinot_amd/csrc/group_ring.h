// Shape limits of the ring-partitioned group-by plan (group_ring.hip), shared with its planner (executor.cpp).
#pragma once

namespace pinot {
// Column slots of the ring decoder: at most kRingGroupCols group columns and kRingAggCols distinct aggregated columns
// (a record's dictId fields), each at most kGroupLwMaxBits wide.
constexpr int kRingGroupCols = 2, kRingAggCols = 2;
// Partitions (of K <= 1024 consecutive keys) a ring block holds in LDS: a 16-entry bucket (144-B stride) + two counters each.
constexpr int kRingMaxPartitions = 1024;
}  // namespace pinot
