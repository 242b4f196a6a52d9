// Device selection of each function's trimSize best groups for the server trim (executor.cpp device_trim), without
// sorting: AggregationGroupByTrimmingService.trimIntermediateResultsMap (:71-116) keeps, per function, the trimSize
// first groups in getSorter's order (:160-176: MIN ascending, the others descending; AVG by sum / count, HLL by
// cardinality) with ties in ascending raw key order. A radix select over each function's order-preserving u64 key
// finds the trimSize-th key K (eight 8-bit digit rounds, every function at once), then every group with a key below K
// and the first ties of K in group order are marked.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace pinot {

constexpr int kTrimMaxFns = 8;

struct TrimFn {
  const double *vals;  // the function's comparable value per group (k_group_final's out_values)
  int32_t avg, asc;    // AVG: value / count; MIN: ascending (the others descending)
};

size_t trim_radix_scratch_bytes(long long n, int nf);
// flags[i] = bit f set for every function f that keeps group i (T <= n); counts: the groups' doc counts (AVG).
void launch_trim_radix(const TrimFn *fns, int nf, const long long *counts, long long n, long long T, uint32_t *flags,
                       void *scratch, size_t scratch_bytes, hipStream_t stream);

// ids[i][j] = global id of group column j in key keys[i] + key_base (mixed radix, column 0 least significant:
// DictionaryBasedGroupKeyGenerator's raw key): the kept groups' key tuples, so the DataTable writer does no division.
constexpr int kDigitsMaxCols = 16;
struct KeyDigits {
  long long card[kDigitsMaxCols];
  int32_t nc;
};
void launch_key_digits(const long long *keys, long long n, long long key_base, const KeyDigits &kd, int32_t *ids,
                       hipStream_t stream);

}  // namespace pinot
