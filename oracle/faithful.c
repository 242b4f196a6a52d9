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
