/*
 * oracle/rmat.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg:
 *
 *  1. rmat_edges: the same counter-based Graph500-style R-MAT generator as
 *     csrc/graph_gen.hip (bit-identical edges for a given seed).
 *  2. Closed-form counts of the north-star patterns (independent of any join
 *     implementation):
 *       1-hop  (a:L)-->(b)        = Σ_rels [a ∈ S_a]·[b ∈ S_b]
 *       2-hop  (a)-->(b)-->(c), r1<>r2
 *              = Σ_b in(b)·out(b) − #self-loops        
 *  3. pipeline_2hop: the Flink physical plan shape of
 *       S_a ⋈[a=start(r1)] R1 ⋈[end(r1)=b] S_b ⋈[b=start(r2)] R2 ⋈[end(r2)=c] S_c,
 *       Filter(NOT(r1 = r2)), count(*)
 *     as lowered by RelationalPlanner.scala:130-165 and executed by Flink's
 *     hash joins (FlinkTable.join, FlinkTable.scala:171-187): hash tables are
 *     built on the node scans and on R2 keyed by start(r2); every r1 row
 *     probes them tuple-at-a-time and every joined row is produced and
 *     counted.  Parallelism = threads (LocalEnvironment default = cores,
 *     flink-cypher/.../api/CAPFSession.scala:81).  This is the CPU baseline.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t oracle_splitmix64(uint64_t x) { return splitmix64(x); }

/* Edge e: for level l, u = 32-bit draw; quadrant by integer thresholds. */
void rmat_edges(int scale, uint64_t seed, uint32_t ta, uint32_t tab, uint32_t tabc, int64_t first,
                int64_t count, int64_t *src, int64_t *dst) {
  const uint64_t key = splitmix64(seed);
  for (int64_t k = 0; k < count; ++k) {
    const uint64_t e = (uint64_t)(first + k);
    uint64_t s = 0, d = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
      if ((l & 1) == 0) r = splitmix64(key + e * 32ull + (uint64_t)(l >> 1));
      const uint32_t u = (l & 1) ? (uint32_t)(r >> 32) : (uint32_t)r;
      const uint32_t q = u < ta ? 0u : (u < tab ? 1u : (u < tabc ? 2u : 3u));
      const int bit = scale - 1 - l;
      s |= (uint64_t)(q >> 1) << bit;
      d |= (uint64_t)(q & 1) << bit;
    }
    src[k] = (int64_t)s;
    dst[k] = (int64_t)d;
  }
}

/* Person label bit of node v (same hash as csrc/graph_gen.hip). */
void node_labels(int64_t base, int64_t n, uint64_t seed, uint8_t *out) {
  const uint64_t lkey = splitmix64(seed ^ 0x1ABE1ull);
  for (int64_t k = 0; k < n; ++k) out[k] = (uint8_t)(splitmix64(lkey + (uint64_t)(base + k)) >> 63);
}

/* ---------------------------------------------------------- closed forms */
/* 1-hop with per-node membership flags of S_a and S_b over ids [0, n). */
uint64_t count_1hop(const int64_t *src, const int64_t *dst, int64_t m, const uint8_t *in_a,
                    const uint8_t *in_b, int64_t n) {
  uint64_t c = 0;
  for (int64_t e = 0; e < m; ++e) {
    int64_t s = src[e], d = dst[e];
    if (s < 0 || s >= n || d < 0 || d >= n) continue;
    c += (uint64_t)(in_a ? in_a[s] : 1) * (uint64_t)(in_b ? in_b[d] : 1);
  }
  return c;
}

/* 2-hop (a)-->(b)-->(c) with r1 <> r2 over a dense node range [0, n). */
uint64_t count_2hop(const int64_t *src, const int64_t *dst, int64_t m, int64_t n) {
  uint32_t *in = (uint32_t *)calloc((size_t)n, 4), *out = (uint32_t *)calloc((size_t)n, 4);
  uint64_t loops = 0, total = 0;
  for (int64_t e = 0; e < m; ++e) {
    int64_t s = src[e], d = dst[e];
    if (s < 0 || s >= n || d < 0 || d >= n) continue;
    in[d]++;
    out[s]++;
    loops += s == d;
  }
  for (int64_t v = 0; v < n; ++v) total += (uint64_t)in[v] * out[v];
  free(in);
  free(out);
  return total - loops;
}

/* Directed triangle (a)-->(b)-->(c)-->(a) with pairwise distinct rels over a
 * dense node range [0, n) — brute force over rels (RelationalPlanner's
 * Expand, Expand, ExpandInto join chain + the uniqueness filter,
 * RelationalPlanner.scala:130-189): for every r1 = a->b, every r2 = b->c
 * (r2 != r1), every r3 = c->a (r3 != r1, r2).  Small scales only.          */
uint64_t count_triangle_brute(const int64_t *src, const int64_t *dst, int64_t m, int64_t n) {
  int64_t *off = (int64_t *)calloc((size_t)n + 1, 8), *pos = (int64_t *)malloc((size_t)n * 8);
  int64_t *adj = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
  for (int64_t e = 0; e < m; ++e)
    if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) off[src[e] + 1]++;
  for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
  memcpy(pos, off, (size_t)n * 8);
  for (int64_t e = 0; e < m; ++e)
    if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) adj[pos[src[e]]++] = e;
  uint64_t c = 0;
  for (int64_t r1 = 0; r1 < m; ++r1) {
    const int64_t a = src[r1], b = dst[r1];
    if (a < 0 || a >= n || b < 0 || b >= n) continue;
    for (int64_t i = off[b]; i < off[b + 1]; ++i) {
      const int64_t r2 = adj[i];
      if (r2 == r1) continue;
      const int64_t cc = dst[r2];
      for (int64_t k = off[cc]; k < off[cc + 1]; ++k) {
        const int64_t r3 = adj[k];
        if (dst[r3] == a && r3 != r1 && r3 != r2) ++c;
      }
    }
  }
  free(off);
  free(pos);
  free(adj);
  return c;
}

/* Per-node in/out degree histograms (for the distributed-count tests). */
void degree_hists(const int64_t *src, const int64_t *dst, int64_t m, int64_t base, int64_t n,
                  uint32_t *in, uint32_t *out, int64_t *loops) {
  memset(in, 0, (size_t)n * 4);
  memset(out, 0, (size_t)n * 4);
  int64_t l = 0;
  for (int64_t e = 0; e < m; ++e) {
    int64_t s = src[e] - base, d = dst[e] - base;
    if (s < 0 || s >= n || d < 0 || d >= n) continue;
    in[d]++;
    out[s]++;
    l += s == d;
  }
  *loops = l;
}

/* ------------------------------------------------- Flink-shaped pipeline */
typedef struct {
  /* open-addressing hash set of node ids (S_a = S_b = S_c = all nodes) */
  int64_t *node_keys;
  uint64_t node_mask;
  /* R2 hash table keyed by start(r2): bucket → rows (chained, CSR layout) */
  int64_t *r2_off;    /* nb + 1 bucket offsets */
  int64_t *r2_rows;   /* rows grouped by bucket */
  uint64_t r2_mask;
  const int64_t *src, *dst, *id;
} JoinState;

static inline uint64_t hmix(int64_t k) {
  uint64_t x = (uint64_t)k;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

static int node_probe(const JoinState *js, int64_t k) {
  uint64_t s = hmix(k) & js->node_mask;
  for (;;) {
    int64_t c = js->node_keys[s];
    if (c == k) return 1;
    if (c == INT64_MIN) return 0;
    s = (s + 1) & js->node_mask;
  }
}

typedef struct {
  const JoinState *js;
  int64_t lo, hi;
  uint64_t count;
} ProbeTask;

static void *probe_worker(void *arg) {
  ProbeTask *t = (ProbeTask *)arg;
  const JoinState *js = t->js;
  uint64_t c = 0;
  for (int64_t r1 = t->lo; r1 < t->hi; ++r1) {
    const int64_t a = js->src[r1], b = js->dst[r1];
    if (!node_probe(js, a)) continue;      /* S_a ⋈ R1 */
    if (!node_probe(js, b)) continue;      /* ⋈ S_b    */
    const uint64_t bk = hmix(b) & js->r2_mask;
    for (int64_t j = js->r2_off[bk]; j < js->r2_off[bk + 1]; ++j) {   /* ⋈ R2 */
      const int64_t r2 = js->r2_rows[j];
      if (js->src[r2] != b) continue;
      if (!node_probe(js, js->dst[r2])) continue;                     /* ⋈ S_c */
      if (js->id[r1] != js->id[r2]) ++c;   /* Filter(NOT(r1 = r2)), count(*) */
    }
  }
  t->count = c;
  return NULL;
}

typedef struct {
  JoinState js;
  int64_t n_nodes, m;
  /* config 4: R3 keyed by (start, end) (pipeline_build_pairs), or null */
  int64_t *r3_off, *r3_rows;
  uint64_t r3_mask;
} Pipeline;

typedef struct {
  JoinState *js;
  int64_t m;
  uint64_t blo, bhi; /* bucket range owned by this builder */
  int64_t *fill;
  int phase;
} BuildTask;

static void *build_worker(void *arg) {
  BuildTask *t = (BuildTask *)arg;
  JoinState *js = t->js;
  for (int64_t r = 0; r < t->m; ++r) {
    uint64_t b = hmix(js->src[r]) & js->r2_mask;
    if (b < t->blo || b >= t->bhi) continue;
    if (t->phase == 0)
      js->r2_off[b + 1]++;
    else
      js->r2_rows[js->r2_off[b] + t->fill[b]++] = r;
  }
  return NULL;
}

void pipeline_free(void *handle);

/* Build phase: hash set on the node scan, bucketed hash table on R2 by start
 * id (partitioned over `threads` builders by bucket range). */
void *pipeline_build(const int64_t *node_ids, int64_t n_nodes, const int64_t *id,
                     const int64_t *src, const int64_t *dst, int64_t m, int threads) {
  if (threads < 1) threads = 1;
  Pipeline *p = (Pipeline *)calloc(1, sizeof(Pipeline));
  JoinState *js = &p->js;
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)n_nodes) cap <<= 1;
  js->node_mask = cap - 1;
  js->node_keys = (int64_t *)malloc(cap * 8);
  for (uint64_t i = 0; i < cap; ++i) js->node_keys[i] = INT64_MIN;
  for (int64_t i = 0; i < n_nodes; ++i) {
    uint64_t s = hmix(node_ids[i]) & js->node_mask;
    while (js->node_keys[s] != INT64_MIN && js->node_keys[s] != node_ids[i]) s = (s + 1) & js->node_mask;
    js->node_keys[s] = node_ids[i];
  }
  uint64_t nb = 1024;
  while (nb < (uint64_t)m) nb <<= 1;
  js->r2_mask = nb - 1;
  js->r2_off = (int64_t *)calloc(nb + 1, 8);
  js->r2_rows = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
  int64_t *fill = (int64_t *)calloc(nb, 8);
  js->src = src;
  js->dst = dst;
  js->id = id;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  BuildTask *tasks = (BuildTask *)malloc(sizeof(BuildTask) * threads);
  for (int phase = 0; phase < 2; ++phase) {
    if (phase == 1)
      for (uint64_t b = 0; b < nb; ++b) js->r2_off[b + 1] += js->r2_off[b];
    for (int t = 0; t < threads; ++t) {
      tasks[t].js = js;
      tasks[t].m = m;
      tasks[t].blo = nb * (uint64_t)t / threads;
      tasks[t].bhi = nb * (uint64_t)(t + 1) / threads;
      tasks[t].fill = fill;
      tasks[t].phase = phase;
      pthread_create(&th[t], NULL, build_worker, &tasks[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  free(th);
  free(tasks);
  free(fill);
  p->n_nodes = n_nodes;
  p->m = m;
  return p;
}

/* Probe phase over r1 rows [lo, hi) with `threads` workers (contiguous r1
 * ranges: R-MAT edge order is random, so the load is even). */
uint64_t pipeline_probe(void *handle, int64_t lo, int64_t hi, int threads) {
  Pipeline *p = (Pipeline *)handle;
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  ProbeTask *tasks = (ProbeTask *)malloc(sizeof(ProbeTask) * threads);
  int64_t span = hi - lo;
  for (int t = 0; t < threads; ++t) {
    tasks[t].js = &p->js;
    tasks[t].lo = lo + span * t / threads;
    tasks[t].hi = lo + span * (t + 1) / threads;
    tasks[t].count = 0;
    pthread_create(&th[t], NULL, probe_worker, &tasks[t]);
  }
  uint64_t c = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    c += tasks[t].count;
  }
  free(th);
  free(tasks);
  return c;
}

/* --------------------------- config 4: the triangle, Flink plan shape
 * Expand, Expand, ExpandInto (RelationalPlanner.scala:130-189): the wedges
 * S_a ⋈ R1 ⋈ S_b ⋈ R2 ⋈ S_c through the start-keyed R2 table above, then the
 * closing rel R3 by a hash join on the TWO keys (start(r3) = c, end(r3) = a)
 * — a (start, end)-keyed table built here — and the uniqueness filters
 * NOT(r1 = r2), NOT(r1 = r3), NOT(r2 = r3); count(*).  Every wedge is
 * materialised and probed, as the relational plan does (no degree order, no
 * set intersection). */
static inline uint64_t pair_key(int64_t s, int64_t d) { return hmix(s) ^ (hmix(d) * 0x9e3779b97f4a7c15ull); }

typedef struct {
  Pipeline *p;
  uint64_t blo, bhi;
  int64_t *fill;
  int phase;
} PairBuildTask;

static void *pair_build_worker(void *arg) {
  PairBuildTask *t = (PairBuildTask *)arg;
  Pipeline *p = t->p;
  for (int64_t r = 0; r < p->m; ++r) {
    uint64_t b = pair_key(p->js.src[r], p->js.dst[r]) & p->r3_mask;
    if (b < t->blo || b >= t->bhi) continue;
    if (t->phase == 0)
      p->r3_off[b + 1]++;
    else
      p->r3_rows[p->r3_off[b] + t->fill[b]++] = r;
  }
  return NULL;
}

void pipeline_build_pairs(void *handle, int threads) {
  Pipeline *p = (Pipeline *)handle;
  if (threads < 1) threads = 1;
  uint64_t nb = 1024;
  while (nb < (uint64_t)p->m) nb <<= 1;
  p->r3_mask = nb - 1;
  p->r3_off = (int64_t *)calloc(nb + 1, 8);
  p->r3_rows = (int64_t *)malloc((size_t)(p->m > 0 ? p->m : 1) * 8);
  int64_t *fill = (int64_t *)calloc(nb, 8);
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  PairBuildTask *tasks = (PairBuildTask *)malloc(sizeof(PairBuildTask) * threads);
  for (int phase = 0; phase < 2; ++phase) {
    if (phase == 1)
      for (uint64_t b = 0; b < nb; ++b) p->r3_off[b + 1] += p->r3_off[b];
    for (int t = 0; t < threads; ++t) {
      tasks[t].p = p;
      tasks[t].blo = nb * (uint64_t)t / threads;
      tasks[t].bhi = nb * (uint64_t)(t + 1) / threads;
      tasks[t].fill = fill;
      tasks[t].phase = phase;
      pthread_create(&th[t], NULL, pair_build_worker, &tasks[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  free(th);
  free(tasks);
  free(fill);
}

typedef struct {
  const Pipeline *p;
  int64_t lo, hi;
  uint64_t count, wedges;
} WedgeTask;

static void *wedge_worker(void *arg) {
  WedgeTask *t = (WedgeTask *)arg;
  const Pipeline *p = t->p;
  const JoinState *js = &p->js;
  uint64_t c = 0, w = 0;
  for (int64_t r1 = t->lo; r1 < t->hi; ++r1) {
    const int64_t a = js->src[r1], b = js->dst[r1];
    if (!node_probe(js, a) || !node_probe(js, b)) continue;
    const uint64_t bk = hmix(b) & js->r2_mask;
    for (int64_t j = js->r2_off[bk]; j < js->r2_off[bk + 1]; ++j) {  /* ⋈ R2 on end(r1) = start(r2) */
      const int64_t r2 = js->r2_rows[j];
      if (js->src[r2] != b) continue;
      const int64_t cc = js->dst[r2];
      if (!node_probe(js, cc)) continue;
      if (js->id[r1] == js->id[r2]) continue;                       /* NOT(r1 = r2) */
      ++w;                                                           /* a wedge row */
      const uint64_t pk = pair_key(cc, a) & p->r3_mask;              /* ⋈ R3 on (start, end) = (c, a) */
      for (int64_t k = p->r3_off[pk]; k < p->r3_off[pk + 1]; ++k) {
        const int64_t r3 = p->r3_rows[k];
        if (js->src[r3] != cc || js->dst[r3] != a) continue;
        if (js->id[r3] != js->id[r1] && js->id[r3] != js->id[r2]) ++c;
      }
    }
  }
  t->count = c;
  t->wedges = w;
  return NULL;
}

/* Triangle rows of r1 rows [lo, hi); *wedges = the wedge rows probed. */
uint64_t pipeline_triangles(void *handle, int64_t lo, int64_t hi, int threads, uint64_t *wedges) {
  Pipeline *p = (Pipeline *)handle;
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  WedgeTask *tasks = (WedgeTask *)malloc(sizeof(WedgeTask) * threads);
  const int64_t span = hi - lo;
  for (int t = 0; t < threads; ++t) {
    tasks[t].p = p;
    tasks[t].lo = lo + span * t / threads;
    tasks[t].hi = lo + span * (t + 1) / threads;
    pthread_create(&th[t], NULL, wedge_worker, &tasks[t]);
  }
  uint64_t c = 0, w = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    c += tasks[t].count;
    w += tasks[t].wedges;
  }
  free(th);
  free(tasks);
  if (wedges) *wedges = w;
  return c;
}

void pipeline_free(void *handle) {
  Pipeline *p = (Pipeline *)handle;
  if (!p) return;
  free(p->r3_off);
  free(p->r3_rows);
  free(p->js.node_keys);
  free(p->js.r2_off);
  free(p->js.r2_rows);
  free(p);
}

/* ------------------------------- config 2: (a:Person)-->(b) count, Flink shape
 * S_a (Person scan) ⋈[a = start(r)] R ⋈[end(r) = b] S_b (all nodes): the two
 * hash-join builds on the node scans (open-addressing sets, as above), then the
 * rels stream through both probes on `threads` workers (contiguous rel ranges)
 * and the matches are counted — RelationalPlanner.scala:130-165 with the label
 * pushed into the S_a scan (ScanGraph.scala:59-105). */
typedef struct {
  int64_t *keys;
  uint64_t mask;
} IdSet;

static void idset_build(IdSet *h, const int64_t *ids, int64_t n) {
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)n) cap <<= 1;
  h->mask = cap - 1;
  h->keys = (int64_t *)malloc(cap * 8);
  for (uint64_t i = 0; i < cap; ++i) h->keys[i] = INT64_MIN;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t s = hmix(ids[i]) & h->mask;
    while (h->keys[s] != INT64_MIN && h->keys[s] != ids[i]) s = (s + 1) & h->mask;
    h->keys[s] = ids[i];
  }
}

static int idset_has(const IdSet *h, int64_t k) {
  uint64_t s = hmix(k) & h->mask;
  for (;;) {
    int64_t c = h->keys[s];
    if (c == k) return 1;
    if (c == INT64_MIN) return 0;
    s = (s + 1) & h->mask;
  }
}

typedef struct {
  const IdSet *a, *b;
  const int64_t *src, *dst;
  int64_t lo, hi;
  uint64_t count;
} OneHopTask;

static void *onehop_worker(void *arg) {
  OneHopTask *t = (OneHopTask *)arg;
  uint64_t c = 0;
  for (int64_t r = t->lo; r < t->hi; ++r)
    if (idset_has(t->a, t->src[r]) && idset_has(t->b, t->dst[r])) ++c;
  t->count = c;
  return NULL;
}

uint64_t onehop_label_count(const int64_t *person_ids, int64_t n_person, const int64_t *node_ids, int64_t n_nodes,
                            const int64_t *src, const int64_t *dst, int64_t m, int threads) {
  if (threads < 1) threads = 1;
  IdSet a, b;
  idset_build(&a, person_ids, n_person);
  idset_build(&b, node_ids, n_nodes);
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  OneHopTask *tasks = (OneHopTask *)malloc(sizeof(OneHopTask) * threads);
  for (int t = 0; t < threads; ++t) {
    tasks[t].a = &a;
    tasks[t].b = &b;
    tasks[t].src = src;
    tasks[t].dst = dst;
    tasks[t].lo = m * t / threads;
    tasks[t].hi = m * (t + 1) / threads;
    pthread_create(&th[t], NULL, onehop_worker, &tasks[t]);
  }
  uint64_t c = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    c += tasks[t].count;
  }
  free(th);
  free(tasks);
  free(a.keys);
  free(b.keys);
  return c;
}

/* ------------------------------------------- full-size counts (fixtures) */
/* Streaming closed forms at the headline sizes (R-MAT s22/s24): every thread
 * generates its contiguous edge range with rmat_edges' arithmetic and keeps
 * private in/out degree histograms; nothing of size M is ever stored.
 * out[0] = Σ_b in(b)·out(b) − self-loops  (2-hop, (a)-->(b)-->(c), r1 <> r2)
 * out[1] = self-loops
 * out[2] = #rels whose source carries the Person label (config 2,
 *          (a:Person)-->(b): b ranges over every node table)
 * out[3] = max in-degree, out[4] = max out-degree                            */
typedef struct {
  int scale;
  uint64_t seed;
  uint32_t ta, tab, tabc;
  int64_t lo, hi, n;
  const uint8_t *person;
  uint32_t *in, *out;
  uint64_t loops, person_rels;
} StreamTask;

static void *stream_worker(void *arg) {
  StreamTask *t = (StreamTask *)arg;
  enum { CH = 1 << 16 };
  int64_t *s = (int64_t *)malloc(CH * 8), *d = (int64_t *)malloc(CH * 8);
  for (int64_t e = t->lo; e < t->hi; e += CH) {
    const int64_t c = t->hi - e < CH ? t->hi - e : CH;
    rmat_edges(t->scale, t->seed, t->ta, t->tab, t->tabc, e, c, s, d);
    for (int64_t k = 0; k < c; ++k) {
      t->out[s[k]]++;
      t->in[d[k]]++;
      t->loops += s[k] == d[k];
      t->person_rels += t->person[s[k]];
    }
  }
  free(s);
  free(d);
  return NULL;
}

void rmat_stream_counts(int scale, uint64_t seed, uint32_t ta, uint32_t tab, uint32_t tabc, int64_t m,
                        int threads, uint64_t *res) {
  if (threads < 1) threads = 1;
  const int64_t n = (int64_t)1 << scale;
  uint8_t *person = (uint8_t *)malloc((size_t)n);
  node_labels(0, n, seed, person);
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  StreamTask *ts = (StreamTask *)calloc((size_t)threads, sizeof(StreamTask));
  for (int i = 0; i < threads; ++i) {
    StreamTask *t = &ts[i];
    t->scale = scale;
    t->seed = seed;
    t->ta = ta;
    t->tab = tab;
    t->tabc = tabc;
    t->lo = m * i / threads;
    t->hi = m * (i + 1) / threads;
    t->n = n;
    t->person = person;
    t->in = (uint32_t *)calloc((size_t)n, 4);
    t->out = (uint32_t *)calloc((size_t)n, 4);
    pthread_create(&th[i], NULL, stream_worker, t);
  }
  uint64_t loops = 0, person_rels = 0;
  for (int i = 0; i < threads; ++i) {
    pthread_join(th[i], NULL);
    loops += ts[i].loops;
    person_rels += ts[i].person_rels;
  }
  uint64_t total = 0, max_in = 0, max_out = 0;
  for (int64_t v = 0; v < n; ++v) {
    uint64_t a = 0, b = 0;
    for (int i = 0; i < threads; ++i) {
      a += ts[i].in[v];
      b += ts[i].out[v];
    }
    total += a * b;
    if (a > max_in) max_in = a;
    if (b > max_out) max_out = b;
  }
  for (int i = 0; i < threads; ++i) {
    free(ts[i].in);
    free(ts[i].out);
  }
  free(ts);
  free(th);
  free(person);
  res[0] = total - loops;
  res[1] = loops;
  res[2] = person_rels;
  res[3] = max_in;
  res[4] = max_out;
}

/* Directed triangle count by a method independent of csrc/triangle.hip (which
 * orients an undirected simple graph by degree):
 *   count = trace(A³) − Σ_x (L³ − L(L−1)(L−2)),   L = A[x][x]
 * (closed walks a→b→c→a of rels; only three self-loops at one node can reuse
 * a rel), with trace(A³) = Σ_{(a,b)} A[a][b] · Σ_c A[b][c]·A[c][a] evaluated
 * by intersecting b's sorted out-list with a's sorted in-list (both with
 * multiplicities; binary search of the shorter list into the longer).
 * Threads take 64-node chunks of a from a shared counter (hub skew).        */
typedef struct {
  const int64_t *ooff, *ioff;
  const int64_t *onb, *inb;  /* distinct neighbours, sorted */
  const uint32_t *omul, *imul;
  int64_t n;
  int64_t *next; /* shared chunk counter */
  pthread_mutex_t *mu;
  uint64_t sum;
} TriTask;

static uint64_t isect(const int64_t *x, const uint32_t *xm, int64_t nx, const int64_t *y,
                      const uint32_t *ym, int64_t ny) {
  uint64_t s = 0;
  if (nx > ny) {
    const int64_t *t = x; x = y; y = t;
    const uint32_t *tm = xm; xm = ym; ym = tm;
    int64_t tn = nx; nx = ny; ny = tn;
  }
  if (nx == 0) return 0;
  if (ny < 16 * nx) { /* merge */
    int64_t i = 0, j = 0;
    while (i < nx && j < ny) {
      if (x[i] < y[j]) ++i;
      else if (x[i] > y[j]) ++j;
      else { s += (uint64_t)xm[i] * ym[j]; ++i; ++j; }
    }
    return s;
  }
  int64_t lo = 0;
  for (int64_t i = 0; i < nx; ++i) { /* x sorted: search window only moves right */
    int64_t a = lo, b = ny;
    while (a < b) {
      int64_t mid = (a + b) >> 1;
      if (y[mid] < x[i]) a = mid + 1; else b = mid;
    }
    lo = a;
    if (a < ny && y[a] == x[i]) s += (uint64_t)xm[i] * ym[a];
  }
  return s;
}

static void *tri_worker(void *arg) {
  TriTask *t = (TriTask *)arg;
  uint64_t sum = 0;
  for (;;) {
    pthread_mutex_lock(t->mu);
    int64_t a0 = *t->next;
    *t->next += 64;
    pthread_mutex_unlock(t->mu);
    if (a0 >= t->n) break;
    int64_t a1 = a0 + 64 < t->n ? a0 + 64 : t->n;
    for (int64_t a = a0; a < a1; ++a)
      for (int64_t k = t->ooff[a]; k < t->ooff[a + 1]; ++k) {
        const int64_t b = t->onb[k];
        sum += (uint64_t)t->omul[k] * isect(t->onb + t->ooff[b], t->omul + t->ooff[b], t->ooff[b + 1] - t->ooff[b],
                                            t->inb + t->ioff[a], t->imul + t->ioff[a], t->ioff[a + 1] - t->ioff[a]);
      }
  }
  t->sum = sum;
  return NULL;
}

static int cmp_i64(const void *a, const void *b) {
  const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
  return x < y ? -1 : x > y;
}

/* CSR of distinct sorted neighbours with multiplicities: key[e] → val[e]. */
static void build_mcsr(const int64_t *key, const int64_t *val, int64_t m, int64_t n, int64_t **off_o,
                       int64_t **nb_o, uint32_t **mul_o) {
  int64_t *off = (int64_t *)calloc((size_t)n + 1, 8), *pos = (int64_t *)malloc((size_t)n * 8);
  int64_t *adj = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
  for (int64_t e = 0; e < m; ++e) off[key[e] + 1]++;
  for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
  memcpy(pos, off, (size_t)n * 8);
  for (int64_t e = 0; e < m; ++e) adj[pos[key[e]]++] = val[e];
  int64_t *noff = (int64_t *)calloc((size_t)n + 1, 8);
  uint32_t *mul = (uint32_t *)malloc((size_t)(m > 0 ? m : 1) * 4);
  int64_t w = 0;
  for (int64_t v = 0; v < n; ++v) {
    int64_t b = off[v], e = off[v + 1];
    qsort(adj + b, (size_t)(e - b), 8, cmp_i64);
    noff[v] = w;
    for (int64_t i = b; i < e;) {
      int64_t j = i;
      while (j < e && adj[j] == adj[i]) ++j;
      adj[w] = adj[i];
      mul[w] = (uint32_t)(j - i);
      ++w;
      i = j;
    }
  }
  noff[n] = w;
  free(off);
  free(pos);
  *off_o = noff;
  *nb_o = adj;
  *mul_o = mul;
}

uint64_t count_triangle_trace(const int64_t *src, const int64_t *dst, int64_t m, int64_t n, int threads) {
  if (threads < 1) threads = 1;
  /* ids outside [0, n) never match a node scan: drop those rels */
  int64_t *s = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8), *d = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
  int64_t mm = 0;
  for (int64_t e = 0; e < m; ++e)
    if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) {
      s[mm] = src[e];
      d[mm] = dst[e];
      ++mm;
    }
  int64_t *ooff, *onb, *ioff, *inb;
  uint32_t *omul, *imul;
  build_mcsr(s, d, mm, n, &ooff, &onb, &omul);
  build_mcsr(d, s, mm, n, &ioff, &inb, &imul);
  uint64_t bad = 0;
  {
    uint32_t *L = (uint32_t *)calloc((size_t)n, 4);
    for (int64_t e = 0; e < mm; ++e) L[s[e]] += s[e] == d[e];
    for (int64_t v = 0; v < n; ++v) {
      const uint64_t l = L[v];
      if (l) bad += l * l * l - l * (l - 1) * (l - 2);
    }
    free(L);
  }
  free(s);
  free(d);
  int64_t next = 0;
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  TriTask *ts = (TriTask *)calloc((size_t)threads, sizeof(TriTask));
  for (int i = 0; i < threads; ++i) {
    ts[i].ooff = ooff; ts[i].ioff = ioff; ts[i].onb = onb; ts[i].inb = inb;
    ts[i].omul = omul; ts[i].imul = imul; ts[i].n = n; ts[i].next = &next; ts[i].mu = &mu;
    pthread_create(&th[i], NULL, tri_worker, &ts[i]);
  }
  uint64_t tr = 0;
  for (int i = 0; i < threads; ++i) {
    pthread_join(th[i], NULL);
    tr += ts[i].sum;
  }
  free(th);
  free(ts);
  free(ooff); free(onb); free(omul); free(ioff); free(inb); free(imul);
  return tr - bad;
}

/* ------------------------------------------------------------------------
 * Config 5 (BASELINE.json):
 *   MATCH (a:L)-[:T*1..u]->(b:L) WITH DISTINCT a, b WITH a, count(*) AS reach
 *   RETURN reach, count(*) AS n
 * on nodes [0, n), every node a source and a target.
 *
 * reach_bitset: reach[a] = |{b : some walk a → b of length 1..u}| by a
 * breadth-first search from 64 sources at a time (bit j of a uint64 per node
 * = source s0 + j), pushing each node's NEW bits along its out-edges (CSR by
 * source).  Lower bound 1 on a walk-reachability plan equals the relational
 * plan's DISTINCT (a, b) pairs of isomorphic paths (a closed sub-walk between
 * two uses of one rel can be cut out: VarLengthExpandPlanner.scala:82-259
 * with the isomorphism filter :178-179; pinned by tests/test_ldbc_config5.py
 * against path enumeration).  Independent of the GPU kernels: push from the
 * source side over a CSR by source; the GPU pulls over a CSR by target.
 *
 * reach_paths: the relational plan's shape for a sample of sources — every
 * path of 1..u rels with pairwise distinct rel ids (the join chain plus
 * isomorphism filters), its end node deduplicated per source (DISTINCT a, b),
 * counted per source (GROUP BY a) — the Flink-shaped CPU baseline.
 * ---------------------------------------------------------------------- */
typedef struct {
  const int64_t *off, *adj;  /* CSR by source: out-neighbours (rel order) */
  int64_t n, chunks;
  int upper;
  int64_t *next;             /* shared chunk counter */
  pthread_mutex_t *mu;
  int64_t *reach;            /* out: per node */
} ReachTask;

static void build_csr(const int64_t *src, const int64_t *dst, int64_t m, int64_t n, int64_t **off_o,
                      int64_t **adj_o, int64_t **rid_o) {
  int64_t *off = (int64_t *)calloc((size_t)n + 1, 8);
  for (int64_t e = 0; e < m; ++e)
    if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) off[src[e] + 1]++;
  for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
  int64_t *pos = (int64_t *)malloc((size_t)(n + 1) * 8);
  memcpy(pos, off, (size_t)(n + 1) * 8);
  int64_t *adj = (int64_t *)malloc((size_t)(off[n] > 0 ? off[n] : 1) * 8);
  int64_t *rid = rid_o ? (int64_t *)malloc((size_t)(off[n] > 0 ? off[n] : 1) * 8) : NULL;
  for (int64_t e = 0; e < m; ++e)
    if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) {
      const int64_t p = pos[src[e]]++;
      adj[p] = dst[e];
      if (rid) rid[p] = e;
    }
  free(pos);
  *off_o = off;
  *adj_o = adj;
  if (rid_o) *rid_o = rid;
}

static void *reach_worker(void *arg) {
  ReachTask *t = (ReachTask *)arg;
  const int64_t n = t->n;
  uint64_t *vis = (uint64_t *)malloc((size_t)n * 8), *cur = (uint64_t *)malloc((size_t)n * 8),
           *nxt = (uint64_t *)malloc((size_t)n * 8);
  for (;;) {
    pthread_mutex_lock(t->mu);
    const int64_t c = (*t->next)++;
    pthread_mutex_unlock(t->mu);
    if (c >= t->chunks) break;
    const int64_t s0 = c * 64, ns = n - s0 < 64 ? n - s0 : 64;
    memset(vis, 0, (size_t)n * 8);
    memset(cur, 0, (size_t)n * 8);
    /* level 1: the sources' own out-edges */
    for (int64_t j = 0; j < ns; ++j)
      for (int64_t p = t->off[s0 + j]; p < t->off[s0 + j + 1]; ++p) cur[t->adj[p]] |= 1ull << j;
    for (int64_t v = 0; v < n; ++v) vis[v] = cur[v];
    for (int level = 2; level <= t->upper; ++level) {
      memset(nxt, 0, (size_t)n * 8);
      for (int64_t v = 0; v < n; ++v) {
        const uint64_t f = cur[v];
        if (!f) continue;
        for (int64_t p = t->off[v]; p < t->off[v + 1]; ++p) nxt[t->adj[p]] |= f;
      }
      for (int64_t v = 0; v < n; ++v) {
        const uint64_t fresh = nxt[v] & ~vis[v];
        cur[v] = fresh;
        vis[v] |= fresh;
      }
    }
    int64_t cnt[64] = {0};
    for (int64_t v = 0; v < n; ++v)
      for (uint64_t w = vis[v]; w; w &= w - 1) cnt[__builtin_ctzll(w)]++;
    for (int64_t j = 0; j < ns; ++j) t->reach[s0 + j] = cnt[j];
  }
  free(vis);
  free(cur);
  free(nxt);
  return NULL;
}

void reach_bitset(const int64_t *src, const int64_t *dst, int64_t m, int64_t n, int upper, int threads,
                  int64_t *reach) {
  if (threads < 1) threads = 1;
  int64_t *off, *adj;
  build_csr(src, dst, m, n, &off, &adj, NULL);
  int64_t next = 0;
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  ReachTask *ts = (ReachTask *)calloc((size_t)threads, sizeof(ReachTask));
  for (int i = 0; i < threads; ++i) {
    ts[i].off = off; ts[i].adj = adj; ts[i].n = n; ts[i].chunks = (n + 63) / 64;
    ts[i].upper = upper; ts[i].next = &next; ts[i].mu = &mu; ts[i].reach = reach;
    pthread_create(&th[i], NULL, reach_worker, &ts[i]);
  }
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  free(th);
  free(ts);
  free(off);
  free(adj);
}

typedef struct {
  const int64_t *off, *adj, *rid, *sources;
  int64_t nsrc, n;
  int upper;
  int64_t *next;
  pthread_mutex_t *mu;
  int64_t *reach, *paths;  /* out: per sampled source */
} PathTask;

static void *paths_worker(void *arg) {
  PathTask *t = (PathTask *)arg;
  uint8_t *seen = (uint8_t *)calloc((size_t)t->n, 1);
  int64_t *touched = (int64_t *)malloc((size_t)(t->n > 0 ? t->n : 1) * 8);
  for (;;) {
    pthread_mutex_lock(t->mu);
    const int64_t i = (*t->next)++;
    pthread_mutex_unlock(t->mu);
    if (i >= t->nsrc) break;
    const int64_t a = t->sources[i];
    int64_t nt = 0, paths = 0;
    /* e1: every rel leaving a */
    for (int64_t p1 = t->off[a]; p1 < t->off[a + 1]; ++p1) {
      const int64_t b1 = t->adj[p1], r1 = t->rid[p1];
      ++paths;
      if (!seen[b1]) { seen[b1] = 1; touched[nt++] = b1; }
      if (t->upper < 2) continue;
      /* e2 ≠ e1 */
      for (int64_t p2 = t->off[b1]; p2 < t->off[b1 + 1]; ++p2) {
        const int64_t r2 = t->rid[p2];
        if (r2 == r1) continue;
        const int64_t b2 = t->adj[p2];
        ++paths;
        if (!seen[b2]) { seen[b2] = 1; touched[nt++] = b2; }
        if (t->upper < 3) continue;
        /* e3 ∉ {e1, e2} */
        for (int64_t p3 = t->off[b2]; p3 < t->off[b2 + 1]; ++p3) {
          const int64_t r3 = t->rid[p3];
          if (r3 == r1 || r3 == r2) continue;
          const int64_t b3 = t->adj[p3];
          ++paths;
          if (!seen[b3]) { seen[b3] = 1; touched[nt++] = b3; }
        }
      }
    }
    for (int64_t k = 0; k < nt; ++k) seen[touched[k]] = 0;
    t->reach[i] = nt;
    t->paths[i] = paths;
  }
  free(seen);
  free(touched);
  return NULL;
}

/* upper ≤ 3.  Returns the number of paths enumerated (the relational plan's
 * rows before DISTINCT) over the sampled sources. */
int64_t reach_paths(const int64_t *src, const int64_t *dst, int64_t m, int64_t n, int upper,
                    const int64_t *sources, int64_t nsrc, int threads, int64_t *reach) {
  if (threads < 1) threads = 1;
  int64_t *off, *adj, *rid;
  build_csr(src, dst, m, n, &off, &adj, &rid);
  int64_t *paths = (int64_t *)calloc((size_t)(nsrc > 0 ? nsrc : 1), 8);
  int64_t next = 0;
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  PathTask *ts = (PathTask *)calloc((size_t)threads, sizeof(PathTask));
  for (int i = 0; i < threads; ++i) {
    ts[i].off = off; ts[i].adj = adj; ts[i].rid = rid; ts[i].sources = sources; ts[i].nsrc = nsrc;
    ts[i].n = n; ts[i].upper = upper; ts[i].next = &next; ts[i].mu = &mu; ts[i].reach = reach;
    ts[i].paths = paths;
    pthread_create(&th[i], NULL, paths_worker, &ts[i]);
  }
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  int64_t total = 0;
  for (int64_t i = 0; i < nsrc; ++i) total += paths[i];
  free(th);
  free(ts);
  free(paths);
  free(off);
  free(adj);
  free(rid);
  return total;
}
