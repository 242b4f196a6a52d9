// Host micro-benchmark of the group-by DataTable writer (pinot::group_by_datatable) on a config-4-shaped trimmed
// result: 15,000 groups over two 1,000-value INT group columns, SUM / AVG / DISTINCTCOUNTHLL with 5,000 kept groups
// each. Runs without a GPU (registers on the host). Build: see scripts/host/Makefile.
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "engine.h"

int main(int argc, char **argv) {
  using namespace pinot;
  const int nf = argc > 1 ? atoi(argv[1]) : 3;  // first nf functions of SUM, AVG, HLL (or only HLL with -1)
  const int64_t n = 15000;
  GroupByResult r;
  r.num_columns = 2;
  r.functions = {PINOT_AGG_SUM, PINOT_AGG_AVG, PINOT_AGG_DISTINCTCOUNTHLL};
  r.gcard = {1000, 1000};
  r.gvalues.assign(2, {});
  for (int j = 0; j < 2; j++)
    for (int v = 0; v < 1000; v++) r.gvalues[j].push_back(std::to_string(v));
  std::mt19937_64 rng(7);
  r.raw_keys.resize(n);
  for (int64_t g = 0; g < n; g++) r.raw_keys[g] = g * 66;
  r.counts.assign(1, HostVec<int64_t>(n));
  r.counts_shared = true;
  r.values.assign(3, HostVec<double>(n));
  r.hll_card.assign(3, HostVec<int64_t>(n));
  r.hll.assign(3, {});
  r.hll[2].resize(n * 256);
  for (int64_t g = 0; g < n; g++) {
    r.counts[0][g] = 800 + (int64_t)(rng() % 50);
    r.values[0][g] = r.values[1][g] = (double)(rng() % 1000000);
  }
  for (auto &b : r.hll[2]) b = (uint8_t)(rng() % 12);
  std::vector<std::vector<int64_t>> kept(3);
  for (int f = 0; f < 3; f++)
    for (int64_t g = 0; g < 5000; g++) kept[f].push_back((g * 3 + f) % n);
  const int64_t *groups[3] = {kept[0].data(), kept[1].data(), kept[2].data()};
  int64_t nums[3] = {5000, 5000, 5000};
  pinot_agg_spec specs[3] = {{PINOT_AGG_SUM, "d8"}, {PINOT_AGG_AVG, "d8"}, {PINOT_AGG_DISTINCTCOUNTHLL, "d5"}};
  pinot_query q{};
  q.aggregations = specs;
  q.num_aggregations = nf < 0 ? 1 : nf;
  if (nf < 0) {  // HLL only
    specs[0] = specs[2];
    groups[0] = groups[2];
    r.functions = {PINOT_AGG_DISTINCTCOUNTHLL};
    r.values.resize(1);
    r.hll[0].swap(r.hll[2]);
    r.hll.resize(1);
    r.hll_card.resize(1);
  } else {
    r.functions.resize(nf);
    r.values.resize(nf);
    r.hll.resize(nf);
    r.hll_card.resize(nf);
  }
  const char *gb[2] = {"d6", "d7"};
  q.group_by = gb;
  q.num_group_by = 2;
  q.num_groups_limit = 1000000;
  pinot_exec_stats st{};
  size_t bytes = 0;
  double best = 1e9;
  for (int it = 0; it < 20; it++) {
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<uint8_t> dt = group_by_datatable(q, r, groups, nums, st, nullptr);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    best = ms < best ? ms : best;
    bytes = dt.size();
  }
  printf("group_by_datatable: %zu bytes, best %.3f ms\n", bytes, best);
  return 0;
}
