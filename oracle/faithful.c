/*
 * faithful.c — reference-faithful CPU executor for the bench workload (TEST INFRASTRUCTURE / CPU baseline).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, as the
 * checker or the reported CPU baseline — never as the product path.
 *
 * The stock Pinot executor is Java and cannot run here (no JDK, no jars). This is a
 * C restatement of the same per-doc algorithm, structure for structure (PC = pinot-core/src/main/java/
 * org/apache/pinot/core):
 *   read_int            PinotDataBitSet.readInt, byte-wise (PC/io/util/PinotDataBitSet.java:79-100)
 *   scan_next/advance   SVScanDocIdIterator.next/advance (PC/operator/dociditerators/SVScanDocIdIterator.java:96-128)
 *   and_next            AndDocIdIterator.next leapfrog (PC/operator/dociditerators/AndDocIdIterator.java:87-122)
 *   block loop          DocIdSetOperator: <= 10000 docIds per block (PC/operator/DocIdSetOperator.java:60-85)
 *   fetch + aggregate   DataFetcher.fetchDictIds -> Dictionary.readDoubleValues -> SumAggregationFunction
 *                       (double accumulator, PC/query/aggregation/function/SumAggregationFunction.java:64-72)
 *   segment tasks       one task per segment on a worker pool (CombineOperator.java:83-161)
 * plus the synthetic generator restated from the HBM generator (see oracle/synth.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EOF_DOC INT32_MIN
#define MAX_DOCS_PER_CALL 10000

static inline int32_t read_int(const uint8_t *buf, int32_t index, int bits) {
  const int64_t bit_offset = (int64_t)index * bits;
  int32_t byte_offset = (int32_t)(bit_offset / 8);
  const int bit_in_first = (int)(bit_offset % 8);
  int32_t cur = buf[byte_offset] & (0xFF >> bit_in_first);
  int left = bits - (8 - bit_in_first);
  if (left <= 0) return (int32_t)((uint32_t)cur >> -left);
  while (left > 8) {
    cur = (cur << 8) | buf[++byte_offset];
    left -= 8;
  }
  return (cur << left) | (buf[byte_offset + 1] >> (8 - left));
}

/* ------------------------------------------------------------------ predicates (dictionary based) */
typedef struct {
  const uint8_t *fwd;
  int bits;
  int kind;              /* 0: RANGE [lo, hi) ; 1: IN membership over dictIds */
  int32_t lo, hi;
  const uint8_t *member; /* kind 1: member[dictId] != 0 */
} pinot_leaf;

static inline int apply_sv(const pinot_leaf *l, int32_t dict_id) {
  return l->kind == 0 ? (l->lo <= dict_id && l->hi > dict_id) : l->member[dict_id] != 0;
}

typedef struct {
  const pinot_leaf *leaf;
  int32_t cur, end;
} scan_iter;

static int32_t scan_next(scan_iter *it) {
  if (it->cur == EOF_DOC) return EOF_DOC;
  while (it->cur < it->end) {
    it->cur++;
    if (apply_sv(it->leaf, read_int(it->leaf->fwd, it->cur, it->leaf->bits))) return it->cur;
  }
  it->cur = EOF_DOC;
  return EOF_DOC;
}

static int32_t scan_advance(scan_iter *it, int32_t target) {
  if (it->cur == EOF_DOC) return EOF_DOC;
  if (target > it->end) {
    it->cur = EOF_DOC;
    return EOF_DOC;
  }
  if (it->cur >= target) return it->cur;
  it->cur = target - 1;
  return scan_next(it);
}

typedef struct {
  scan_iter *its;
  int n;
  int32_t current_max;
  int done;
} and_iter;

static int32_t and_next(and_iter *a) {
  if (a->done) return EOF_DOC;
  a->current_max = a->current_max + 1;
  for (int i = 0; i < a->n; i++) {
    int32_t p = scan_advance(&a->its[i], a->current_max);
    if (p == EOF_DOC) {
      a->done = 1;
      return EOF_DOC;
    }
    if (p > a->current_max) {
      a->current_max = p;
      if (i > 0) i = -1;
    }
  }
  return a->current_max;
}

/* ------------------------------------------------------------------ one segment */
typedef struct {
  /* inputs */
  int32_t num_docs;
  int nleaves;
  const pinot_leaf *leaves;
  const uint8_t *metric_fwd;
  int metric_bits;
  const double *metric_dict;
  /* outputs */
  int64_t count;
  double sum;
} pinot_segment_task;

static void run_segment(pinot_segment_task *t) {
  scan_iter its[16];
  for (int i = 0; i < t->nleaves; i++) {
    its[i].leaf = &t->leaves[i];
    its[i].cur = -1;
    its[i].end = t->num_docs - 1; /* inclusive end docId (ScanBasedFilterOperator.java:40-42) */
  }
  and_iter a = {its, t->nleaves, -1, 0};
  int32_t *doc_ids = (int32_t *)malloc(sizeof(int32_t) * MAX_DOCS_PER_CALL);
  int32_t *dict_ids = (int32_t *)malloc(sizeof(int32_t) * MAX_DOCS_PER_CALL);
  double *values = (double *)malloc(sizeof(double) * MAX_DOCS_PER_CALL);
  int64_t count = 0;
  double sum = 0.0;
  for (;;) {
    int n = 0;
    int32_t d;
    while (n < MAX_DOCS_PER_CALL && (d = (t->nleaves ? and_next(&a) : (a.current_max + 1 < t->num_docs
                                                                          ? ++a.current_max : EOF_DOC))) != EOF_DOC)
      doc_ids[n++] = d;
    if (n == 0) break;
    count += n; /* CountAggregationFunction: length of the block */
    if (t->metric_fwd) {
      for (int i = 0; i < n; i++) dict_ids[i] = read_int(t->metric_fwd, doc_ids[i], t->metric_bits);
      for (int i = 0; i < n; i++) values[i] = t->metric_dict[dict_ids[i]];
      for (int i = 0; i < n; i++) sum += values[i];
    }
    if (n < MAX_DOCS_PER_CALL) break;
  }
  free(doc_ids);
  free(dict_ids);
  free(values);
  t->count = count;
  t->sum = sum;
}

typedef struct {
  pinot_segment_task *tasks;
  int ntasks;
  int next;
  pthread_mutex_t mu;
} pool_t;

static void *worker(void *arg) {
  pool_t *p = (pool_t *)arg;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    int i = p->next++;
    pthread_mutex_unlock(&p->mu);
    if (i >= p->ntasks) break;
    run_segment(&p->tasks[i]);
  }
  return NULL;
}

/* Runs all segment tasks on `threads` workers; merges COUNT (sum) and SUM (in segment order). */
void pinot_faithful_run(pinot_segment_task *tasks, int ntasks, int threads, int64_t *count, double *sum) {
  pool_t p;
  p.tasks = tasks;
  p.ntasks = ntasks;
  p.next = 0;
  pthread_mutex_init(&p.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, worker, &p);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&p.mu);
  int64_t c = 0;
  double s = 0.0;
  for (int i = 0; i < ntasks; i++) {
    c += tasks[i].count;
    s += tasks[i].sum;
  }
  *count = c;
  *sum = s;
}

/* ------------------------------------------------------------------ optimised CPU variant (second baseline line)
 * beside the reference-faithful executor, an optimised CPU executor of the same query: the 64 docs
 * of a bitset word are unpacked together from the b big-endian 64-bit words holding them (no per-doc byte-wise
 * readInt), every leaf turns them into a 64-bit match mask, the metric is folded for the set bits with an exact
 * integer accumulator, and the work is split into 64 K-doc ranges (not whole segments) over the threads. Same
 * inputs (pinot_segment_task) and results as pinot_faithful_run. */
static inline uint64_t load_be64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

/* dictIds of docs [64 w, 64 w + 64) of a b-bit column (b <= 32) */
static inline void unpack64(const uint8_t *fwd, int b, int64_t w, uint32_t *out) {
  uint64_t W[33];
  const uint8_t *p = fwd + (size_t)w * 8 * b;
  for (int k = 0; k < b; k++) W[k] = load_be64(p + 8 * k);
  W[b] = 0;
  const uint64_t mask = (b == 64) ? ~0ull : ((1ull << b) - 1);
  for (int j = 0; j < 64; j++) {
    const int bit = j * b, k = bit >> 6, o = bit & 63;
    const uint64_t x = o ? (W[k] << o) | (W[k + 1] >> (64 - o)) : W[k];
    out[j] = (uint32_t)((x >> (64 - b)) & mask);
  }
}

typedef struct {
  pinot_segment_task *tasks;
  int ntasks;
  int64_t nranges, ranges_per_seg_max;
  int64_t *range_seg, *range_w0, *range_w1;
  int64_t *counts;
  int64_t *isums;
  int64_t next;
  pthread_mutex_t mu;
} fast_pool_t;

static void fast_range(fast_pool_t *fp, int64_t r) {
  const pinot_segment_task *t = &fp->tasks[fp->range_seg[r]];
  uint32_t ids[64];
  int64_t count = 0, isum = 0;
  for (int64_t w = fp->range_w0[r]; w < fp->range_w1[r]; w++) {
    const int64_t base = w * 64;
    uint64_t m = (t->num_docs - base >= 64) ? ~0ull : ((1ull << (t->num_docs - base)) - 1);
    for (int l = 0; l < t->nleaves && m; l++) {
      const pinot_leaf *lf = &t->leaves[l];
      unpack64(lf->fwd, lf->bits, w, ids);
      uint64_t lm = 0;
      if (lf->kind == 0) {
        for (int j = 0; j < 64; j++) lm |= (uint64_t)((uint32_t)(ids[j] - (uint32_t)lf->lo) < (uint32_t)(lf->hi - lf->lo)) << j;
      } else {
        for (int j = 0; j < 64; j++) lm |= (uint64_t)(lf->member[ids[j]] != 0) << j;
      }
      m &= lm;
    }
    if (!m) continue;
    count += __builtin_popcountll(m);
    if (t->metric_fwd) {
      unpack64(t->metric_fwd, t->metric_bits, w, ids);
      for (int j = 0; j < 64; j++)
        if ((m >> j) & 1) isum += (int64_t)t->metric_dict[ids[j]];
    }
  }
  fp->counts[r] = count;
  fp->isums[r] = isum;
}

static void *fast_worker(void *arg) {
  fast_pool_t *p = (fast_pool_t *)arg;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    const int64_t r = p->next++;
    pthread_mutex_unlock(&p->mu);
    if (r >= p->nranges) break;
    fast_range(p, r);
  }
  return NULL;
}

/* The metric dictionary must hold integral values (the bench's INT columns): sums are exact int64. */
void pinot_fast_run(pinot_segment_task *tasks, int ntasks, int threads, int64_t *count, double *sum) {
  const int64_t words_per_range = 1024; /* 64 K docs */
  int64_t nr = 0;
  for (int i = 0; i < ntasks; i++) nr += ((tasks[i].num_docs + 63) / 64 + words_per_range - 1) / words_per_range;
  fast_pool_t p;
  memset(&p, 0, sizeof(p));
  p.tasks = tasks;
  p.ntasks = ntasks;
  p.nranges = nr;
  p.range_seg = (int64_t *)malloc(sizeof(int64_t) * nr);
  p.range_w0 = (int64_t *)malloc(sizeof(int64_t) * nr);
  p.range_w1 = (int64_t *)malloc(sizeof(int64_t) * nr);
  p.counts = (int64_t *)calloc(nr, sizeof(int64_t));
  p.isums = (int64_t *)calloc(nr, sizeof(int64_t));
  int64_t r = 0;
  for (int i = 0; i < ntasks; i++) {
    const int64_t nw = (tasks[i].num_docs + 63) / 64;
    for (int64_t w0 = 0; w0 < nw; w0 += words_per_range, r++) {
      p.range_seg[r] = i;
      p.range_w0[r] = w0;
      p.range_w1[r] = w0 + words_per_range < nw ? w0 + words_per_range : nw;
    }
  }
  pthread_mutex_init(&p.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, fast_worker, &p);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&p.mu);
  int64_t c = 0, s = 0;
  for (int64_t i = 0; i < nr; i++) {
    c += p.counts[i];
    s += p.isums[i];
  }
  free(p.range_seg);
  free(p.range_w0);
  free(p.range_w1);
  free(p.counts);
  free(p.isums);
  *count = c;
  *sum = (double)s;
}

/* ------------------------------------------------------------------ group-by (config 4 shape)
 * AggregationGroupByOperator with DictionaryBasedGroupKeyGenerator's INT_MAP holder (cardinality product above
 * max.init.group.holder.capacity: raw key -> group id through an open-addressing int map, first-seen order,
 * IntMapBasedHolder.getGroupId :293-302; no group is dropped below num.groups.limit), per 10,000-doc block:
 * fetch the group-by dictIds (readInt per doc), build raw keys (:200-209), look up group ids; SUM / AVG:
 * DoubleGroupByResultHolder and AvgPair (sum, count) per group (SumAggregationFunction.aggregateGroupBySV :75-82,
 * AvgAggregationFunction :110-134); DISTINCTCOUNTHLL: a HyperLogLog(8) per group fed with MurmurHash.hashLong of
 * each doc's INT value (DistinctCountHLLAggregationFunction.aggregateGroupBySV :121-170). Then
 * CombineGroupByOperator merges the segments' results per group (here keyed by the raw key instead of the
 * '\t'-joined string, which only makes the baseline cheaper). */
static inline uint32_t murmur_hash_long(int64_t data) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0, k = (uint32_t)data * m;
  k ^= k >> 24;
  h ^= k * m;
  k = (uint32_t)((uint64_t)data >> 32) * m;
  k ^= k >> 24;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}

typedef struct {
  int32_t num_docs;
  int nleaves;
  const pinot_leaf *leaves;
  const uint8_t *g0_fwd, *g1_fwd; /* group-by columns (identity INT dictionaries) */
  int g0_bits, g1_bits;
  int32_t g0_card;
  const uint8_t *m_fwd;           /* SUM / AVG column */
  int m_bits;
  const uint8_t *h_fwd;           /* DISTINCTCOUNTHLL column (NULL: the query has none) */
  int h_bits;
  /* outputs (owned): groups in first-seen order */
  int32_t ngroups;
  int64_t *keys;
  double *sum;
  int64_t *cnt;
  uint8_t *regs; /* [ngroups][256] */
} pinot_group_task;

static void run_group_segment(pinot_group_task *t) {
  scan_iter its[16];
  for (int i = 0; i < t->nleaves; i++) {
    its[i].leaf = &t->leaves[i];
    its[i].cur = -1;
    its[i].end = t->num_docs - 1;
  }
  and_iter a = {its, t->nleaves, -1, 0};
  int32_t *doc_ids = (int32_t *)malloc(sizeof(int32_t) * MAX_DOCS_PER_CALL);
  int32_t *gids = (int32_t *)malloc(sizeof(int32_t) * MAX_DOCS_PER_CALL);
  /* Int2IntOpenHashMap: power-of-two table, linear probing, key -1 = free */
  int64_t cap = 1 << 16, cap_groups = 1 << 14, n = 0;
  int64_t *tk = (int64_t *)malloc(sizeof(int64_t) * cap);
  int32_t *tv = (int32_t *)malloc(sizeof(int32_t) * cap);
  for (int64_t i = 0; i < cap; i++) tk[i] = -1;
  int64_t *keys = (int64_t *)malloc(sizeof(int64_t) * cap_groups);
  double *sum = (double *)malloc(sizeof(double) * cap_groups);
  int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * cap_groups);
  uint8_t *regs = (uint8_t *)malloc((size_t)256 * cap_groups);
  for (;;) {
    int nd = 0;
    int32_t d;
    while (nd < MAX_DOCS_PER_CALL && (d = and_next(&a)) != EOF_DOC) doc_ids[nd++] = d;
    if (nd == 0) break;
    for (int i = 0; i < nd; i++) {  /* generateKeysForBlock */
      const int64_t raw = (int64_t)read_int(t->g1_fwd, doc_ids[i], t->g1_bits) * t->g0_card +
                          read_int(t->g0_fwd, doc_ids[i], t->g0_bits);
      uint64_t slot = (uint64_t)(raw * 0x9E3779B97F4A7C15ull) & (uint64_t)(cap - 1);
      while (tk[slot] != -1 && tk[slot] != raw) slot = (slot + 1) & (uint64_t)(cap - 1);
      if (tk[slot] == -1) {
        if (n == cap_groups) {
          cap_groups *= 2;
          keys = (int64_t *)realloc(keys, sizeof(int64_t) * cap_groups);
          sum = (double *)realloc(sum, sizeof(double) * cap_groups);
          cnt = (int64_t *)realloc(cnt, sizeof(int64_t) * cap_groups);
          regs = (uint8_t *)realloc(regs, (size_t)256 * cap_groups);
        }
        tk[slot] = raw;
        tv[slot] = (int32_t)n;
        keys[n] = raw;
        sum[n] = 0.0;
        cnt[n] = 0;
        memset(regs + (size_t)256 * n, 0, 256);
        n++;
        if (2 * n > cap) { /* rehash at load factor 1/2 */
          int64_t nc = cap * 2;
          int64_t *nk = (int64_t *)malloc(sizeof(int64_t) * nc);
          int32_t *nv = (int32_t *)malloc(sizeof(int32_t) * nc);
          for (int64_t j = 0; j < nc; j++) nk[j] = -1;
          for (int64_t j = 0; j < cap; j++)
            if (tk[j] != -1) {
              uint64_t s2 = (uint64_t)(tk[j] * 0x9E3779B97F4A7C15ull) & (uint64_t)(nc - 1);
              while (nk[s2] != -1) s2 = (s2 + 1) & (uint64_t)(nc - 1);
              nk[s2] = tk[j];
              nv[s2] = tv[j];
            }
          free(tk);
          free(tv);
          tk = nk;
          tv = nv;
          cap = nc;
          slot = (uint64_t)(raw * 0x9E3779B97F4A7C15ull) & (uint64_t)(cap - 1);
          while (tk[slot] != raw) slot = (slot + 1) & (uint64_t)(cap - 1);
        }
      }
      gids[i] = tv[slot];
    }
    for (int i = 0; i < nd; i++) { /* SUM(m) and AVG(m): dictionary value (identity) as double */
      const double v = (double)read_int(t->m_fwd, doc_ids[i], t->m_bits);
      sum[gids[i]] += v;
      cnt[gids[i]] += 1;
    }
    for (int i = 0; t->h_fwd && i < nd; i++) { /* DISTINCTCOUNTHLL(h): offer(hashLong(value)) */
      const uint32_t h = murmur_hash_long(read_int(t->h_fwd, doc_ids[i], t->h_bits));
      const uint32_t j = h >> 24;
      const uint32_t w = (h << 8) | 129u;
      const uint8_t r = (uint8_t)(__builtin_clz(w) + 1);
      uint8_t *g = regs + (size_t)256 * gids[i];
      if (g[j] < r) g[j] = r;
    }
    if (nd < MAX_DOCS_PER_CALL) break;
  }
  free(doc_ids);
  free(gids);
  free(tk);
  free(tv);
  t->ngroups = (int32_t)n;
  t->keys = keys;
  t->sum = sum;
  t->cnt = cnt;
  t->regs = regs;
}

typedef struct {
  pinot_group_task *tasks;
  int ntasks;
  int next;
  pthread_mutex_t mu;
} gpool_t;

static void *gworker(void *arg) {
  gpool_t *p = (gpool_t *)arg;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    int i = p->next++;
    pthread_mutex_unlock(&p->mu);
    if (i >= p->ntasks) break;
    run_group_segment(&p->tasks[i]);
  }
  return NULL;
}

typedef struct {
  pinot_group_task *tasks;
  int ntasks, nthreads;
  int64_t *mc;
  double *ms;
  uint8_t *mr;
} merge_ctx_t;

typedef struct {
  merge_ctx_t *m;
  int worker;
  int64_t groups;
} merge_arg_t;

static void *merge_worker(void *arg) {
  merge_arg_t *a = (merge_arg_t *)arg;
  merge_ctx_t *m = a->m;
  for (int i = 0; i < m->ntasks; i++) {
    const pinot_group_task *t = &m->tasks[i];
    for (int32_t g = 0; g < t->ngroups; g++) {
      const int64_t k = t->keys[g];
      if (k % m->nthreads != a->worker) continue;
      if (!m->mc[k]) a->groups++;
      m->mc[k] += t->cnt[g];
      m->ms[k] += t->sum[g];
      if (!t->h_fwd) continue;
      uint8_t *dst = m->mr + (size_t)256 * k;
      const uint8_t *src = t->regs + (size_t)256 * g;
      for (int j = 0; j < 256; j++)
        if (dst[j] < src[j]) dst[j] = src[j];
    }
  }
  return NULL;
}

/* Runs the group-by tasks on `threads` workers, then the combine into a dense key space of `num_keys` (counts,
 * sums, registers merged per key). Returns the number of groups; total count / sum for the caller's check. */
int64_t pinot_faithful_group_run(pinot_group_task *tasks, int ntasks, int threads, int64_t num_keys, int64_t *total_count,
                                 double *total_sum) {
  gpool_t p;
  p.tasks = tasks;
  p.ntasks = ntasks;
  p.next = 0;
  pthread_mutex_init(&p.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, gworker, &p);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&p.mu);
  /* CombineGroupByOperator: merge every segment's groups (the reference merges concurrently into one
     ConcurrentHashMap; here `threads` workers each own the keys k with k % threads == worker) */
  merge_ctx_t m;
  m.tasks = tasks;
  m.ntasks = ntasks;
  m.nthreads = threads;
  m.mc = (int64_t *)calloc((size_t)num_keys, sizeof(int64_t));
  m.ms = (double *)calloc((size_t)num_keys, sizeof(double));
  m.mr = (uint8_t *)calloc((size_t)num_keys, 256);
  merge_arg_t *args = (merge_arg_t *)malloc(sizeof(merge_arg_t) * threads);
  th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) {
    args[i].m = &m;
    args[i].worker = i;
    args[i].groups = 0;
    pthread_create(&th[i], NULL, merge_worker, &args[i]);
  }
  int64_t groups = 0, tc = 0;
  double tsum = 0.0;
  for (int i = 0; i < threads; i++) {
    pthread_join(th[i], NULL);
    groups += args[i].groups;
  }
  free(th);
  free(args);
  for (int i = 0; i < ntasks; i++) {
    pinot_group_task *t = &tasks[i];
    for (int32_t g = 0; g < t->ngroups; g++) {
      tc += t->cnt[g];
      tsum += t->sum[g];
    }
    free(t->keys);
    free(t->sum);
    free(t->cnt);
    free(t->regs);
  }
  free(m.mc);
  free(m.ms);
  free(m.mr);
  *total_count = tc;
  *total_sum = tsum;
  return groups;
}

int pinot_faithful_group_task_size(void) { return (int)sizeof(pinot_group_task); }

int32_t pinot_faithful_read_int(const uint8_t *buf, int32_t index, int bits) { return read_int(buf, index, bits); }

int pinot_faithful_task_size(void) { return (int)sizeof(pinot_segment_task); }
int pinot_faithful_leaf_size(void) { return (int)sizeof(pinot_leaf); }

/* ------------------------------------------------------------------ synthetic generator (host twin of k_synth_column) */
static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Packs ceil(num_docs*bits/8) bytes MSB-first (PinotDataBitSet.writeInt layout) into out (zeroed by caller). */
void pinot_synth_column(uint64_t seed, int col_index, int32_t card, int bits, int64_t num_docs, uint8_t *out) {
  const uint64_t cseed = seed ^ ((uint64_t)(col_index + 1) * 0xD1B54A32D192ED03ull);
  uint64_t acc = 0;
  int nb = 0;
  int64_t o = 0;
  for (int64_t d = 0; d < num_docs; d++) {
    uint64_t v = d < card ? (uint64_t)d : splitmix64(cseed ^ ((uint64_t)d * 0x9E3779B97F4A7C15ull)) % (uint64_t)card;
    acc = (acc << bits) | v;
    nb += bits;
    while (nb >= 8) {
      out[o++] = (uint8_t)(acc >> (nb - 8));
      nb -= 8;
    }
    acc &= nb ? ((1ull << nb) - 1) : 0;
  }
  if (nb) out[o] = (uint8_t)(acc << (8 - nb));
}
