// Multi-value group-by over a hashed key space (kernels.hip): the group columns' cardinality product is beyond the
// dense limit (the reference's LONG_MAP / ARRAY_MAP holder shapes, DictionaryBasedGroupKeyGenerator.java:79-126), so
// a key is the slot of its global-id tuple's 64-bit fingerprint in an open-addressing table. An insert pass over the
// matching docs' key products fills the table (the winner of a slot's CAS writes the tuple beside it); the
// accumulation and first-appearance passes find each key's slot and compare the tuple stored there with their own:
// a fingerprint collision is reported (`verify_err`) and the host retries with another seed, never merges.
#pragma once
#include "kernels.h"

namespace pinot {

struct MvHash {
  unsigned long long *htable;  // [hcap] fingerprints, 0 = empty
  int32_t *tuples;             // [hcap][n_gcols] global ids of each occupied slot's key
  long long hcap;              // power of two >= 2 x the keys the matching docs yield
  unsigned long long hseed;
  uint32_t *verify_err;        // set when a key's tuple differs from its slot's
};

// Σ over the matching docs of Π (entries of each group column): the keys the docs yield (u64 atomically added).
void launch_mv_key_count(const MvGroupArgs &a, unsigned long long *total, hipStream_t stream);
// Inserts every matching doc's keys into the table.
void launch_mv_hash_insert(const MvGroupArgs &a, const MvHash &h, hipStream_t stream);
// k_group_by_mv / k_first_pos_mv with key = slot (a.stride unused).
void launch_group_by_mv_hashed(const MvGroupArgs &a, const MvHash &h, hipStream_t stream);
void launch_first_pos_mv_hashed(const MvGroupArgs &a, const MvHash &h, unsigned long long *first_pos,
                                hipStream_t stream);
// ids[i][j] = tuples[slots[i]][j]: the result groups' global-id tuples.
void launch_mv_hash_tuples(const MvHash &h, int n_gcols, const long long *slots, long long n, int32_t *ids,
                           hipStream_t stream);

}  // namespace pinot
