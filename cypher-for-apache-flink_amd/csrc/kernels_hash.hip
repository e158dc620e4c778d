// kernels_hash.hip — HBM-resident hash tables for the materialising operators:
// equi-join (Table.join, FlinkTable.scala:171-187), DISTINCT
// (FlinkTable.scala:189-196, with Spark's dropDuplicates(cols) semantics,
// morpheus-spark-cypher/.../impl/table/SparkTable.scala:198-200) and GROUP BY
// aggregation (FlinkTable.group, FlinkTable.scala:123-150; aggregators
// FlinkSQLExprMapper.scala:281-287).  ORDER BY uses a stable radix sort.
//
// Open addressing with linear probing on uint32 row ids; key equality compares
// the key columns (multi-column keys, NULL == NULL for grouping, NULL never
// matches in a join — SQL semantics of the Flink `===` predicate).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr uint32_t EMPTY = 0xFFFFFFFFu;

struct KeyViews {
  const ColView *cols;  // device array of key column views
  int n;
};

__device__ inline uint64_t key_word(const ColView &c, int64_t r, bool &isnull) {
  if (c.type == CAPF_TYPE_NULL || !c.data || (c.valid && !c.valid[r])) {
    isnull = true;
    return 0;
  }
  isnull = false;
  if (c.type == CAPF_TYPE_BOOL) return ((const uint8_t *)c.data)[r] ? 1 : 0;
  if (c.type != CAPF_TYPE_FLOAT64) return (uint64_t)ld_int(c, r);
  uint64_t w = ((const uint64_t *)c.data)[r];
  if (w == 0x8000000000000000ull) w = 0;  // -0.0 == 0.0
  return w;
}

__device__ inline uint64_t hash_row(const ColView *cols, int n, int64_t r, bool &anynull) {
  uint64_t h = 0x243F6A8885A308D3ull;
  anynull = false;
  for (int k = 0; k < n; ++k) {
    bool nul;
    uint64_t w = key_word(cols[k], r, nul);
    anynull |= nul;
    h = fmix64(h ^ (nul ? 0x9E3779B97F4A7C15ull : w) ^ ((uint64_t)k << 56)) + (nul ? 1 : 0);
  }
  return h;
}

__device__ inline bool rows_equal(const ColView *a, int64_t ra, const ColView *b, int64_t rb,
                                  int n) {
  for (int k = 0; k < n; ++k) {
    bool na, nb;
    uint64_t wa = key_word(a[k], ra, na), wb = key_word(b[k], rb, nb);
    if (na != nb) return false;
    if (!na && wa != wb) return false;
  }
  return true;
}

// Insert every row (skip_null: rows with a NULL key are not inserted and get
// slot = EMPTY).  slot_min[slot] receives the smallest row id of the key, so
// group representatives are deterministic.
__global__ void k_ht_insert(const ColView *keys, int nkeys, int64_t n, uint32_t *slots,
                            uint32_t *slot_min, uint64_t mask, uint32_t *slot_of_row,
                            int skip_null) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    bool anynull;
    uint64_t h = hash_row(keys, nkeys, r, anynull);
    if (skip_null && anynull) {
      slot_of_row[r] = EMPTY;
      continue;
    }
    uint64_t slot = h & mask;
    while (true) {
      uint32_t cur = slots[slot];
      if (cur == EMPTY) {
        uint32_t old = atomicCAS(&slots[slot], EMPTY, (uint32_t)r);
        if (old == EMPTY) break;
        cur = old;
      }
      if (rows_equal(keys, cur, keys, r, nkeys)) break;
      slot = (slot + 1) & mask;
    }
    atomicMin(&slot_min[slot], (uint32_t)r);
    slot_of_row[r] = (uint32_t)slot;
  }
}

__global__ void k_rep_flags(const uint32_t *slot_of_row, const uint32_t *slot_min, int64_t n,
                            uint8_t *is_rep) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    uint32_t sl = slot_of_row[r];
    is_rep[r] = (sl != EMPTY && slot_min[sl] == (uint32_t)r) ? 1 : 0;
  }
}

__global__ void k_slot_gid(const int64_t *reps, int64_t ngroups, const uint32_t *slot_of_row,
                           int64_t *gid_of_slot) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * blockDim.x)
    gid_of_slot[slot_of_row[reps[g]]] = g;
}

__global__ void k_row_gid(const uint32_t *slot_of_row, const int64_t *gid_of_slot, int64_t n,
                          int64_t *gid) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    uint32_t sl = slot_of_row[r];
    gid[r] = sl == EMPTY ? -1 : gid_of_slot[sl];
  }
}

static BufPtr upload_views(Session *s, const std::vector<ColView> &v) {
  BufPtr b = s->alloc(sizeof(ColView) * std::max<size_t>(v.size(), 1));
  if (!v.empty())
    HIP_CHECK(hipMemcpyAsync(b->p, v.data(), sizeof(ColView) * v.size(), hipMemcpyHostToDevice,
                             s->stream));
  s->sync();
  return b;
}

static uint64_t table_capacity(int64_t n) {
  uint64_t cap = 1024;
  while (cap < (uint64_t)n * 2) cap <<= 1;
  return cap;
}

struct HashTable {
  BufPtr slots, slot_min, slot_of_row;
  uint64_t mask = 0;
  BufPtr views;
  int nkeys = 0;
};

static HashTable build_table(Session *s, const Data &d, const std::vector<int> &keys,
                             bool skip_null) {
  if (d.nrows >= (int64_t)EMPTY) not_impl("hash table over more than 2^32-1 rows");
  HashTable ht;
  std::vector<ColView> v;
  for (int k : keys) v.push_back(view_of(d.cols[k]));
  ht.views = upload_views(s, v);
  ht.nkeys = (int)keys.size();
  uint64_t cap = table_capacity(d.nrows);
  ht.mask = cap - 1;
  ht.slots = s->alloc(4 * cap);
  ht.slot_min = s->alloc(4 * cap);
  ht.slot_of_row = s->alloc(4 * std::max<int64_t>(d.nrows, 1));
  HIP_CHECK(hipMemsetAsync(ht.slots->p, 0xFF, 4 * cap, s->stream));
  HIP_CHECK(hipMemsetAsync(ht.slot_min->p, 0xFF, 4 * cap, s->stream));
  if (d.nrows > 0) {
    KernelTimer kt(s, "hash_build", 8.0 * d.nrows * keys.size());
    hipLaunchKernelGGL(k_ht_insert, dim3(grid_for(d.nrows, 256)), dim3(256), 0, s->stream,
                       (const ColView *)ht.views->p, ht.nkeys, d.nrows, (uint32_t *)ht.slots->p,
                       (uint32_t *)ht.slot_min->p, ht.mask, (uint32_t *)ht.slot_of_row->p,
                       skip_null ? 1 : 0);
    KERNEL_CHECK();
  }
  return ht;
}

// Dense group ids (0..ngroups-1, ordered by smallest row of the group).
static void dense_groups(Session *s, const HashTable &ht, int64_t n, Grouping &g) {
  BufPtr flags = s->alloc(std::max<int64_t>(n, 1));
  hipLaunchKernelGGL(k_rep_flags, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                     (const uint32_t *)ht.slot_of_row->p, (const uint32_t *)ht.slot_min->p, n,
                     (uint8_t *)flags->p);
  KERNEL_CHECK();
  g.rep_row = compact_flags(s, (const uint8_t *)flags->p, n, &g.ngroups);
  BufPtr gid_of_slot = s->alloc(8 * (ht.mask + 1));
  if (g.ngroups > 0) {
    hipLaunchKernelGGL(k_slot_gid, dim3(grid_for(g.ngroups, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.rep_row->p, g.ngroups,
                       (const uint32_t *)ht.slot_of_row->p, (int64_t *)gid_of_slot->p);
    KERNEL_CHECK();
  }
  g.group_of_row = s->alloc(8 * std::max<int64_t>(n, 1));
  hipLaunchKernelGGL(k_row_gid, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                     (const uint32_t *)ht.slot_of_row->p, (const int64_t *)gid_of_slot->p, n,
                     (int64_t *)g.group_of_row->p);
  KERNEL_CHECK();
}

__global__ void k_fill_i64(int64_t *p, int64_t v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

ColPtr scalar_i64_column(Session *s, int64_t v) {
  ColPtr col = make_column(s, Type::Int64, 1, false);
  hipLaunchKernelGGL(k_fill_i64, dim3(1), dim3(64), 0, s->stream, (int64_t *)col->data->p, v,
                     (int64_t)1);
  KERNEL_CHECK();
  col->host_i64.assign(1, v);
  return col;
}

Grouping group_rows(Session *s, const Data &d, const std::vector<int> &keys) {
  Grouping g;
  int64_t n = d.nrows;
  if (keys.empty()) {
    g.ngroups = n > 0 ? 1 : 0;
    g.group_of_row = s->alloc(8 * std::max<int64_t>(n, 1));
    g.rep_row = s->alloc(8);
    HIP_CHECK(hipMemsetAsync(g.rep_row->p, 0, 8, s->stream));
    if (n > 0) {
      hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                         (int64_t *)g.group_of_row->p, (int64_t)0, n);
      KERNEL_CHECK();
    }
    return g;
  }
  if (n == 0) {
    g.ngroups = 0;
    g.group_of_row = s->alloc(8);
    g.rep_row = s->alloc(8);
    return g;
  }
  HashTable ht = build_table(s, d, keys, false);
  dense_groups(s, ht, n, g);
  return g;
}

// ------------------------------------------------------------------ join
__global__ void k_count_group(const int64_t *gid, int64_t n, int64_t *cnt) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid[r];
    if (g >= 0) atomicAdd((unsigned long long *)&cnt[g], 1ull);
  }
}

__global__ void k_fill_csr(const int64_t *gid, int64_t n, const int64_t *off, int64_t *cursor,
                           int64_t *csr) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid[r];
    if (g < 0) continue;
    int64_t p = (int64_t)atomicAdd((unsigned long long *)&cursor[g], 1ull);
    csr[off[g] + p] = r;
  }
}

// Probe: find the build-side group of each probe row (-1: none / NULL key).
__global__ void k_probe(const ColView *pkeys, const ColView *bkeys, int nkeys, int64_t n,
                        const uint32_t *slots, uint64_t mask, const uint32_t *slot_of_row_b,
                        const int64_t *gid_of_row_b, const int64_t *gcnt, int64_t *pgid,
                        int64_t *out_cnt, int outer) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    bool anynull;
    uint64_t h = hash_row(pkeys, nkeys, r, anynull);
    int64_t g = -1;
    if (!anynull) {
      uint64_t slot = h & mask;
      while (true) {
        uint32_t cur = slots[slot];
        if (cur == EMPTY) break;
        if (rows_equal(bkeys, cur, pkeys, r, nkeys)) {
          g = gid_of_row_b[cur];
          break;
        }
        slot = (slot + 1) & mask;
      }
    }
    pgid[r] = g;
    int64_t c = g >= 0 ? gcnt[g] : 0;
    out_cnt[r] = (outer && c == 0) ? 1 : c;
  }
}

__global__ void k_join_emit(const int64_t *pgid, const int64_t *out_off, int64_t n,
                            const int64_t *goff, const int64_t *gcnt, const int64_t *csr,
                            int64_t *lidx, int64_t *ridx, int outer, uint8_t *bmatched) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = pgid[r];
    int64_t o = out_off[r];
    if (g < 0) {
      if (outer) {
        lidx[o] = r;
        ridx[o] = -1;
      }
      continue;
    }
    if (bmatched) bmatched[g] = 1;
    int64_t c = gcnt[g], b = goff[g];
    for (int64_t j = 0; j < c; ++j) {
      lidx[o + j] = r;
      ridx[o + j] = csr[b + j];
    }
  }
}

__global__ void k_unmatched(const int64_t *gid, const uint8_t *gmatched, int64_t n,
                            uint8_t *flags) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid[r];
    flags[r] = (g < 0 || !gmatched[g]) ? 1 : 0;
  }
}

__global__ void k_append_unmatched(const int64_t *rows, int64_t m, int64_t off, int64_t *lidx,
                                   int64_t *ridx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    lidx[off + i] = -1;
    ridx[off + i] = rows[i];
  }
}

JoinPairs hash_join(Session *s, const Data &l, const Data &r,
                    const std::vector<std::pair<int, int>> &keys, int32_t join_type) {
  std::vector<int> lk, rk;
  for (auto &kp : keys) {
    lk.push_back(kp.first);
    rk.push_back(kp.second);
  }
  const bool left_outer = join_type == CAPF_JOIN_LEFT_OUTER || join_type == CAPF_JOIN_FULL_OUTER;
  const bool right_outer = join_type == CAPF_JOIN_RIGHT_OUTER || join_type == CAPF_JOIN_FULL_OUTER;
  JoinPairs jp;
  // build side = right table
  HashTable ht = build_table(s, r, rk, true);
  Grouping g;
  int64_t nr = r.nrows, nl = l.nrows;
  if (nr > 0) dense_groups(s, ht, nr, g);
  BufPtr gcnt = s->alloc(8 * std::max<int64_t>(g.ngroups, 1));
  BufPtr goff = s->alloc(8 * std::max<int64_t>(g.ngroups, 1));
  BufPtr csr = s->alloc(8 * std::max<int64_t>(nr, 1));
  if (g.ngroups > 0) {
    HIP_CHECK(hipMemsetAsync(gcnt->p, 0, 8 * g.ngroups, s->stream));
    hipLaunchKernelGGL(k_count_group, dim3(grid_for(nr, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.group_of_row->p, nr, (int64_t *)gcnt->p);
    KERNEL_CHECK();
    exclusive_scan_i64(s, (const int64_t *)gcnt->p, (int64_t *)goff->p, g.ngroups);
    BufPtr cursor = s->alloc(8 * g.ngroups);
    HIP_CHECK(hipMemsetAsync(cursor->p, 0, 8 * g.ngroups, s->stream));
    hipLaunchKernelGGL(k_fill_csr, dim3(grid_for(nr, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.group_of_row->p, nr, (const int64_t *)goff->p,
                       (int64_t *)cursor->p, (int64_t *)csr->p);
    KERNEL_CHECK();
  }
  // probe with the left table
  std::vector<ColView> pv;
  for (int k : lk) pv.push_back(view_of(l.cols[k]));
  BufPtr pviews = upload_views(s, pv);
  BufPtr pgid = s->alloc(8 * std::max<int64_t>(nl, 1));
  BufPtr ocnt = s->alloc(8 * std::max<int64_t>(nl, 1));
  BufPtr ooff = s->alloc(8 * std::max<int64_t>(nl, 1));
  int64_t total = 0;
  if (nl > 0) {
    if (nr == 0) {
      // nothing to match: every probe row is unmatched
      hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(nl, 256)), dim3(256), 0, s->stream,
                         (int64_t *)pgid->p, (int64_t)-1, nl);
      hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(nl, 256)), dim3(256), 0, s->stream,
                         (int64_t *)ocnt->p, (int64_t)(left_outer ? 1 : 0), nl);
      KERNEL_CHECK();
    } else {
      KernelTimer kt(s, "hash_probe", 8.0 * nl * lk.size());
      hipLaunchKernelGGL(k_probe, dim3(grid_for(nl, 256)), dim3(256), 0, s->stream,
                         (const ColView *)pviews->p, (const ColView *)ht.views->p,
                         (int)lk.size(), nl, (const uint32_t *)ht.slots->p, ht.mask,
                         (const uint32_t *)ht.slot_of_row->p,
                         (const int64_t *)g.group_of_row->p, (const int64_t *)gcnt->p,
                         (int64_t *)pgid->p, (int64_t *)ocnt->p, left_outer ? 1 : 0);
      KERNEL_CHECK();
    }
    total = exclusive_scan_i64(s, (const int64_t *)ocnt->p, (int64_t *)ooff->p, nl);
  }
  int64_t extra = 0;
  BufPtr gmatched, unmatched_rows;
  if (right_outer) {
    gmatched = s->alloc(std::max<int64_t>(g.ngroups, 1));
    if (g.ngroups > 0) HIP_CHECK(hipMemsetAsync(gmatched->p, 0, g.ngroups, s->stream));
  }
  jp.left = s->alloc(8 * std::max<int64_t>(total + nr, 1));
  jp.right = s->alloc(8 * std::max<int64_t>(total + nr, 1));
  if (nl > 0 && total > 0) {
    KernelTimer kt(s, "join_emit", 16.0 * total);
    hipLaunchKernelGGL(k_join_emit, dim3(grid_for(nl, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)pgid->p, (const int64_t *)ooff->p, nl,
                       (const int64_t *)goff->p, (const int64_t *)gcnt->p,
                       (const int64_t *)csr->p, (int64_t *)jp.left->p, (int64_t *)jp.right->p,
                       left_outer ? 1 : 0, right_outer ? (uint8_t *)gmatched->p : nullptr);
    KERNEL_CHECK();
  }
  if (right_outer && nr > 0) {
    BufPtr flags = s->alloc(nr);
    hipLaunchKernelGGL(k_unmatched, dim3(grid_for(nr, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.group_of_row->p, (const uint8_t *)gmatched->p, nr,
                       (uint8_t *)flags->p);
    KERNEL_CHECK();
    unmatched_rows = compact_flags(s, (const uint8_t *)flags->p, nr, &extra);
    if (extra > 0) {
      hipLaunchKernelGGL(k_append_unmatched, dim3(grid_for(extra, 256)), dim3(256), 0,
                         s->stream, (const int64_t *)unmatched_rows->p, extra, total,
                         (int64_t *)jp.left->p, (int64_t *)jp.right->p);
      KERNEL_CHECK();
    }
  }
  jp.n = total + extra;
  return jp;
}

// ------------------------------------------------------------- aggregation
template <typename T>
__device__ inline T load_num(const ColView &c, int64_t r) {
  if (c.type == CAPF_TYPE_BOOL) return (T)((const uint8_t *)c.data)[r];
  if (c.type == CAPF_TYPE_FLOAT64) return (T)((const double *)c.data)[r];
  return (T)ld_int(c, r);
}

__device__ inline void atomic_min_f64(double *p, double v) {
  unsigned long long *a = (unsigned long long *)p;
  unsigned long long old = *a;
  while (v < __longlong_as_double(old)) {
    unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}
__device__ inline void atomic_max_f64(double *p, double v) {
  unsigned long long *a = (unsigned long long *)p;
  unsigned long long old = *a;
  while (v > __longlong_as_double(old)) {
    unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}

// acc: per group value (int64 or double), cnt: per group non-null count
__global__ void k_agg(const int64_t *gid, int64_t n, ColView arg, int kind, int fl, void *acc,
                      unsigned long long *cnt) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid ? gid[r] : 0;
    if (g < 0) continue;
    if (kind == CAPF_AGG_COUNT_STAR) {
      atomicAdd(&cnt[g], 1ull);
      continue;
    }
    if (arg.type == CAPF_TYPE_NULL || !arg.data || (arg.valid && !arg.valid[r])) continue;
    atomicAdd(&cnt[g], 1ull);
    if (kind == CAPF_AGG_COUNT) continue;
    if (fl) {
      double v = load_num<double>(arg, r);
      double *a = (double *)acc + g;
      if (kind == CAPF_AGG_SUM || kind == CAPF_AGG_AVG) atomicAdd(a, v);
      else if (kind == CAPF_AGG_MIN) atomic_min_f64(a, v);
      else atomic_max_f64(a, v);
    } else {
      long long v = load_num<long long>(arg, r);
      long long *a = (long long *)acc + g;
      if (kind == CAPF_AGG_SUM || kind == CAPF_AGG_AVG) atomicAdd((unsigned long long *)a, (unsigned long long)v);
      else if (kind == CAPF_AGG_MIN) atomicMin(a, v);
      else atomicMax(a, v);
    }
  }
}

__global__ void k_agg_final(int64_t ng, int kind, int fl, int out_type, const void *acc,
                            const unsigned long long *cnt, void *out, uint8_t *valid) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng;
       g += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long c = cnt[g];
    if (kind == CAPF_AGG_COUNT_STAR || kind == CAPF_AGG_COUNT) {
      ((int64_t *)out)[g] = (int64_t)c;
      valid[g] = 1;
      continue;
    }
    valid[g] = c > 0 ? 1 : 0;
    if (out_type == CAPF_TYPE_NULL) continue;
    if (fl) {
      double a = ((const double *)acc)[g];
      if (kind == CAPF_AGG_AVG && c > 0) a = a / (double)c;
      if (out_type == CAPF_TYPE_FLOAT64)
        ((double *)out)[g] = c > 0 ? a : 0.0;
      else
        ((int64_t *)out)[g] = c > 0 ? (int64_t)a : 0;
    } else {
      int64_t a = ((const int64_t *)acc)[g];
      if (kind == CAPF_AGG_AVG) {  // avg over INTEGER values: the exact int64 sum / count as a FLOAT
        ((double *)out)[g] = c > 0 ? (double)a / (double)c : 0.0;
        continue;
      }
      if (out_type == CAPF_TYPE_BOOL)
        ((uint8_t *)out)[g] = c > 0 ? (a != 0) : 0;
      else
        ((int64_t *)out)[g] = c > 0 ? a : 0;
    }
  }
}

// ---------------------------------------------------------- fp64 sum / avg
// sum and avg over FLOAT (FlinkSQLExprMapper.scala:281-287) must agree with the
// reference within 1e-12 relative error (north star) whatever the row order.
// An fp64 atomicAdd per row is order-dependent and uncompensated, so the rows
// are instead put in a fixed order — stable radix sort by group id, rows
// ascending within a group — and summed in double-double (TwoSum-compensated,
// Neumaier): per chunk of FS_CHUNK rows one wave, lane l taking rows l, l+64, …,
// then a fixed butterfly; per group one wave over its chunk partials.  The
// result is bit-identical from run to run and within ~2 ulp of the exact sum
// for any input whose exact sum is not the victim of catastrophic cancellation
// beyond the double-double's 106 bits.
constexpr int FS_CHUNK = 2048;

struct DD {
  double hi, lo;
};
__device__ inline DD dd_add_d(DD x, double v) {
  const double s = x.hi + v, bb = s - x.hi;
  return DD{s, x.lo + ((x.hi - (s - bb)) + (v - bb))};
}
__device__ inline DD dd_add(DD x, DD y) {
  const double s = x.hi + y.hi, bb = s - x.hi;
  return DD{s, x.lo + y.lo + ((x.hi - (s - bb)) + (y.hi - bb))};
}
// a fixed butterfly over the 64 lanes: every lane ends with the same sum
__device__ inline DD dd_wave_sum(DD x) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    DD y{__shfl_xor(x.hi, o, 64), __shfl_xor(x.lo, o, 64)};
    // combine in lane order (lower lane first) so both partners compute the same value
    x = (threadIdx.x & o) ? dd_add(y, x) : dd_add(x, y);
  }
  return x;
}
__device__ inline double dd_value(DD x) { return isfinite(x.hi) ? x.hi + x.lo : x.hi; }

// sort key per row: its group, or ng (sorted last) when the argument is NULL
__global__ void k_fs_keys(const int64_t *gid, ColView arg, int64_t n, int64_t ng, uint64_t *key, uint32_t *row,
                          unsigned long long *cnt) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid ? gid[r] : 0;
    if (g < 0 || (arg.valid && !arg.valid[r])) g = ng;
    else atomicAdd(&cnt[g], 1ull);
    key[r] = (uint64_t)g;
    row[r] = (uint32_t)r;
  }
}

// chunks per group → exclusive scan gives each group's first chunk
__global__ void k_fs_nchunks(const unsigned long long *cnt, int64_t ng, uint32_t *nch) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= ng; g += (int64_t)gridDim.x * blockDim.x)
    nch[g] = g < ng ? (uint32_t)((cnt[g] + FS_CHUNK - 1) / FS_CHUNK) : 0u;
}

// one wave per chunk: (group, chunk within group) found by a binary search over
// the groups' first chunks; rows [off[g] + c·FS_CHUNK, …) of the sorted order
// center non-null (stDev's second pass): each value is replaced by its squared
// deviation from its group's double-double mean, the square kept exactly as
// the pair (p, fma(d, d, −p))
__global__ __launch_bounds__(256) void k_fs_chunks(const uint32_t *rows, ColView arg, const int64_t *off,
                                                   const uint32_t *chunk0, int64_t ng, uint32_t nchunks,
                                                   const double2 *center, double2 *part) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * blockDim.x / 64;
  for (uint32_t c = wave; c < nchunks; c += nw) {
    int64_t lo = 0, hi = ng - 1;  // last g with chunk0[g] <= c
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (chunk0[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    const int64_t g = lo;
    const int64_t b = off[g] + (int64_t)(c - chunk0[g]) * FS_CHUNK;
    const int64_t e = min(off[g + 1], b + FS_CHUNK);
    DD acc{0.0, 0.0};
    if (center) {
      const double2 m = center[g];
      for (int64_t i = b + lane; i < e; i += 64) {
        const double d = (load_num<double>(arg, rows[i]) - m.x) - m.y;
        const double p = d * d;
        acc = dd_add(acc, DD{p, fma(d, d, -p)});
      }
    } else if (arg.type == CAPF_TYPE_FLOAT64) {
      for (int64_t i = b + lane; i < e; i += 64) acc = dd_add_d(acc, ((const double *)arg.data)[rows[i]]);
    } else {
      for (int64_t i = b + lane; i < e; i += 64) acc = dd_add_d(acc, load_num<double>(arg, rows[i]));
    }
    acc = dd_wave_sum(acc);
    if (lane == 0) part[c] = make_double2(acc.hi, acc.lo);
  }
}

// one wave per group over its chunk partials, then the final value
__global__ __launch_bounds__(256) void k_fs_groups(const double2 *part, const uint32_t *chunk0,
                                                   const unsigned long long *cnt, int64_t ng, int avg,
                                                   double *out, uint8_t *valid, double2 *dd_out) {
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * blockDim.x / 64;
  for (int64_t g = wave; g < ng; g += nw) {
    DD acc{0.0, 0.0};
    for (uint32_t c = chunk0[g] + lane; c < chunk0[g + 1]; c += 64) {
      const double2 p = part[c];
      acc = dd_add(acc, DD{p.x, p.y});
    }
    acc = dd_wave_sum(acc);
    if (lane == 0 && dd_out) {
      dd_out[g] = make_double2(acc.hi, acc.lo);
    } else if (lane == 0) {
      const unsigned long long n = cnt[g];
      const double v = dd_value(acc);
      out[g] = n > 0 ? (avg ? v / (double)n : v) : 0.0;
      valid[g] = n > 0 ? 1 : 0;
    }
  }
}

// The fixed summation order of a grouping: rows with a non-NULL argument
// sorted by group (stable), group offsets and the chunk layout of each group.
struct FsLayout {
  int64_t ng = 0;
  BufPtr srow, off, ch0, cnt;
  uint32_t nchunks = 0;
};

static FsLayout fs_layout(Session *s, const Grouping &g, int64_t nrows, const ColView &av) {
  FsLayout L;
  const int64_t ng = L.ng = g.ngroups;
  if (nrows >= (int64_t(1) << 32)) not_impl("FLOAT sum / avg / stDev over 2^32 or more rows");
  L.cnt = s->alloc(8 * (ng + 1));
  HIP_CHECK(hipMemsetAsync(L.cnt->p, 0, 8 * (ng + 1), s->stream));
  const int64_t n1 = std::max<int64_t>(nrows, 1);
  BufPtr key = s->alloc(8 * n1), skey = s->alloc(8 * n1), row = s->alloc(4 * n1);
  L.srow = s->alloc(4 * n1);
  KernelTimer kt(s, "group_fsum", 16.0 * nrows);
  if (nrows > 0) {
    hipLaunchKernelGGL(k_fs_keys, dim3(grid_for(nrows, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.group_of_row->p, av, nrows, ng, (uint64_t *)key->p, (uint32_t *)row->p,
                       (unsigned long long *)L.cnt->p);
    KERNEL_CHECK();
    int bits = 1;
    while (bits < 64 && (uint64_t(1) << bits) <= (uint64_t)ng) ++bits;
    size_t tmp = 0;
    HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp, (const uint64_t *)key->p, (uint64_t *)skey->p,
                                        (const uint32_t *)row->p, (uint32_t *)L.srow->p, (size_t)nrows, 0, bits,
                                        s->stream));
    BufPtr t = s->alloc(std::max<size_t>(tmp, 16));
    HIP_CHECK(rocprim::radix_sort_pairs(t->p, tmp, (const uint64_t *)key->p, (uint64_t *)skey->p,
                                        (const uint32_t *)row->p, (uint32_t *)L.srow->p, (size_t)nrows, 0, bits,
                                        s->stream));
  }
  // group offsets in the sorted order and first chunks
  L.off = s->alloc(8 * (ng + 1));
  BufPtr nch = s->alloc(4 * (ng + 1));
  L.ch0 = s->alloc(4 * (ng + 1));
  exclusive_scan_i64(s, (const int64_t *)L.cnt->p, (int64_t *)L.off->p, ng + 1);
  hipLaunchKernelGGL(k_fs_nchunks, dim3(grid_for(ng + 1, 256)), dim3(256), 0, s->stream,
                     (const unsigned long long *)L.cnt->p, ng, (uint32_t *)nch->p);
  KERNEL_CHECK();
  BufPtr tot = s->alloc(16);
  exclusive_scan_u32_async(s, (const uint32_t *)nch->p, (uint32_t *)L.ch0->p, ng + 1, (uint32_t *)tot->p);
  HIP_CHECK(hipMemcpyAsync(&L.nchunks, (const uint32_t *)L.ch0->p + ng, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  return L;
}

// One compensated pass over the layout: per group the double-double sum of
// the values (center null) or of the squared deviations from center[g];
// avg / sum finals into (out, valid), or the raw sums into dd_out.
static void fs_pass(Session *s, const FsLayout &L, const ColView &av, const double2 *center, int avg,
                    double *out, uint8_t *valid, double2 *dd_out) {
  BufPtr part = s->alloc(16 * std::max<uint32_t>(L.nchunks, 1));
  if (L.nchunks > 0) {
    hipLaunchKernelGGL(k_fs_chunks, dim3(grid_for((int64_t)L.nchunks * 64, 256, (int64_t)s->num_cus * 64)),
                       dim3(256), 0, s->stream, (const uint32_t *)L.srow->p, av, (const int64_t *)L.off->p,
                       (const uint32_t *)L.ch0->p, L.ng, L.nchunks, center, (double2 *)part->p);
    KERNEL_CHECK();
  }
  hipLaunchKernelGGL(k_fs_groups, dim3(grid_for(L.ng * 64, 256, (int64_t)s->num_cus * 64)), dim3(256), 0,
                     s->stream, (const double2 *)part->p, (const uint32_t *)L.ch0->p,
                     (const unsigned long long *)L.cnt->p, L.ng, avg, out, valid, dd_out);
  KERNEL_CHECK();
}

static void fp64_sum_groups(Session *s, const Grouping &g, int64_t nrows, const ColPtr &arg, bool avg,
                            const ColPtr &o) {
  force(arg);
  const ColView av = view_of(arg);
  FsLayout L = fs_layout(s, g, nrows, av);
  fs_pass(s, L, av, nullptr, avg ? 1 : 0, (double *)o->data->p, (uint8_t *)o->valid->p, nullptr);
}

// ------------------------------------------------------------ stDev / stDevP
// StDev / StDevP (Expr.scala:1120-1128 → Flink stddevSamp / stddevPop,
// FlinkSQLExprMapper.scala:223-224) over the same fixed order as sum: the
// double-double mean of each group (pass 1 ÷ n, a DD quotient), then the
// double-double sum of squared deviations (pass 2), sqrt(M2 / (n − 1)) or
// sqrt(M2 / n).  The deviations are taken from the DD mean, so the result
// stays within a few ulp of the exact value also when mean ≫ spread.
__global__ void k_dd_mean(const double2 *sum, const unsigned long long *cnt, int64_t ng, double2 *mean) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = cnt[g];
    if (c == 0) {
      mean[g] = make_double2(0.0, 0.0);
      continue;
    }
    const double n = (double)c, q1 = sum[g].x / n;
    const double r = fma(-q1, n, sum[g].x) + sum[g].y;  // sum − q1·n, exact in its first term
    mean[g] = make_double2(q1, r / n);
  }
}

__global__ void k_stdev_final(const double2 *m2, const unsigned long long *cnt, int64_t ng, int samp, double *out,
                              uint8_t *valid) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = cnt[g];
    const bool ok = samp ? c >= 2 : c >= 1;
    valid[g] = ok ? 1 : 0;
    const double ss = m2[g].x + m2[g].y;
    out[g] = ok ? sqrt(ss / (double)(samp ? c - 1 : c)) : 0.0;
  }
}

static void stdev_groups(Session *s, const Grouping &g, int64_t nrows, const ColPtr &arg, bool samp,
                         const ColPtr &o) {
  force(arg);
  const ColView av = view_of(arg);
  FsLayout L = fs_layout(s, g, nrows, av);
  const int64_t ng = L.ng;
  BufPtr sums = s->alloc(16 * ng), mean = s->alloc(16 * ng), m2 = s->alloc(16 * ng);
  fs_pass(s, L, av, nullptr, 0, nullptr, nullptr, (double2 *)sums->p);
  hipLaunchKernelGGL(k_dd_mean, dim3(grid_for(ng, 256)), dim3(256), 0, s->stream, (const double2 *)sums->p,
                     (const unsigned long long *)L.cnt->p, ng, (double2 *)mean->p);
  KERNEL_CHECK();
  fs_pass(s, L, av, (const double2 *)mean->p, 0, nullptr, nullptr, (double2 *)m2->p);
  hipLaunchKernelGGL(k_stdev_final, dim3(grid_for(ng, 256)), dim3(256), 0, s->stream, (const double2 *)m2->p,
                     (const unsigned long long *)L.cnt->p, ng, samp ? 1 : 0, (double *)o->data->p,
                     (uint8_t *)o->valid->p);
  KERNEL_CHECK();
}

// ------------------------------------------------------- percentiles
// PercentileCont / PercentileDisc (Expr.scala:1096-1118) with the semantics of
// the Spark backend's UDAFs (morpheus-spark-cypher/.../impl/expressions/
// PercentileUdafs.scala:59-96; the Flink mapper has no case for them): the
// group's non-NULL values sorted ascending (stable radix sorts: by value, then
// by group, NULL arguments last), then per group one thread picks
//   disc: v[pos − 1] (v[0] when pos = 0), pos = Math.round(n · p)
//   cont: x = 1 + (n − 1) · p, v[x − 1] when x is integral, else
//         (1 − w) · v[⌈x⌉ − 1] + w · v[⌊x⌋ − 1] with w = ⌈x⌉ − x
// in IEEE double arithmetic without contraction (as the JVM computes it).
__global__ void k_pct_keys(const int64_t *gid, ColView arg, int64_t n, int64_t ng, uint64_t *gkey,
                           uint64_t *vkey, unsigned long long *cnt) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid ? gid[r] : 0;
    if (g < 0 || (arg.valid && !arg.valid[r])) g = ng;
    else atomicAdd(&cnt[g], 1ull);
    gkey[r] = (uint64_t)g;
    uint64_t k;
    if (arg.type == CAPF_TYPE_FLOAT64) {
      uint64_t b = ((const uint64_t *)arg.data)[r];
      if (b == 0x8000000000000000ull) b = 0;
      k = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    } else {
      k = (uint64_t)ld_int(arg, r) ^ 0x8000000000000000ull;
    }
    vkey[r] = k;
  }
}

__device__ inline double pct_round(double x) {  // Scala Double.round (Math.round) for x >= 0
  double r = floor(x);
  if (x - r >= 0.5) r += 1.0;
  return r;
}

__global__ void k_pct_final(const int64_t *perm, const int64_t *off, const unsigned long long *cnt, int64_t ng,
                            ColView arg, int cont, double p, int out_int, void *out, uint8_t *valid) {
#pragma clang fp contract(off)  // the JVM's separately rounded * and + (no FMA)
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = (int64_t)cnt[g];
    valid[g] = c > 0 ? 1 : 0;
    if (c == 0) {
      if (out_int) ((int64_t *)out)[g] = 0;
      else ((double *)out)[g] = 0.0;
      continue;
    }
    const int64_t *v = perm + off[g];
    if (!cont) {
      const int64_t pos = (int64_t)pct_round((double)c * p);
      const int64_t row = v[pos == 0 ? 0 : pos - 1];
      if (out_int) ((int64_t *)out)[g] = ld_int(arg, row);
      else ((double *)out)[g] = load_num<double>(arg, row);
      continue;
    }
    const double x = 1.0 + (double)(c - 1) * p;
    const double fl = floor(x), ce = ceil(x);
    const int64_t prec = (int64_t)fl, succ = (int64_t)ce;
    const double w = ce - x;
    double res;
    if (x == ce) {
      res = load_num<double>(arg, v[prec - 1]);
    } else {
      const double a = load_num<double>(arg, v[succ - 1]), b = load_num<double>(arg, v[prec - 1]);
      res = (1.0 - w) * a + w * b;
    }
    ((double *)out)[g] = res;
  }
}

static void radix_pass(Session *s, const uint64_t *keys_in, BufPtr &perm, int64_t n, int bits);

static void percentile_groups(Session *s, const Grouping &g, int64_t nrows, const ColPtr &arg, bool cont,
                              double p, const ColPtr &o) {
  force(arg);
  const ColView av = view_of(arg);
  const int64_t ng = g.ngroups;
  BufPtr cnt = s->alloc(8 * (ng + 1));
  HIP_CHECK(hipMemsetAsync(cnt->p, 0, 8 * (ng + 1), s->stream));
  const int64_t n1 = std::max<int64_t>(nrows, 1);
  BufPtr gkey = s->alloc(8 * n1), vkey = s->alloc(8 * n1);
  BufPtr perm = iota_index(s, 0, nrows);
  if (nrows > 0) {
    hipLaunchKernelGGL(k_pct_keys, dim3(grid_for(nrows, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.group_of_row->p, av, nrows, ng, (uint64_t *)gkey->p, (uint64_t *)vkey->p,
                       (unsigned long long *)cnt->p);
    KERNEL_CHECK();
    int bits = 1;
    while (bits < 64 && (uint64_t(1) << bits) <= (uint64_t)ng) ++bits;
    radix_pass(s, (const uint64_t *)vkey->p, perm, nrows, 64);
    radix_pass(s, (const uint64_t *)gkey->p, perm, nrows, bits);
  }
  BufPtr off = s->alloc(8 * (ng + 1));
  exclusive_scan_i64(s, (const int64_t *)cnt->p, (int64_t *)off->p, ng + 1);
  const bool out_int = o->type == Type::Int64;
  hipLaunchKernelGGL(k_pct_final, dim3(grid_for(ng, 256)), dim3(256), 0, s->stream, (const int64_t *)perm->p,
                     (const int64_t *)off->p, (const unsigned long long *)cnt->p, ng, av, cont ? 1 : 0, p,
                     out_int ? 1 : 0, o->data->p, (uint8_t *)o->valid->p);
  KERNEL_CHECK();
}

ColPtr aggregate(Session *s, const Grouping &g, const Data &d, int64_t nrows, int32_t kind,
                 const ColPtr &arg, Type out_type, double param) {
  (void)d;
  int64_t ng = g.ngroups;
  ColPtr o = make_column(s, out_type, ng, true);
  if (ng == 0) return o;
  if (kind == CAPF_AGG_STDEV || kind == CAPF_AGG_STDEV_POP || kind == CAPF_AGG_PERCENTILE_CONT ||
      kind == CAPF_AGG_PERCENTILE_DISC) {
    if (!arg || arg->type == Type::Null || nrows == 0) {  // no values anywhere: NULL per group
      HIP_CHECK(hipMemsetAsync(o->data->p, 0, type_width(out_type) * ng, s->stream));
      HIP_CHECK(hipMemsetAsync(o->valid->p, 0, ng, s->stream));
      return o;
    }
    if (kind == CAPF_AGG_STDEV || kind == CAPF_AGG_STDEV_POP)
      stdev_groups(s, g, nrows, arg, kind == CAPF_AGG_STDEV, o);
    else
      percentile_groups(s, g, nrows, arg, kind == CAPF_AGG_PERCENTILE_CONT, param, o);
    return o;
  }
  bool fl = arg && arg->type == Type::Float64;
  if (fl && out_type == Type::Float64 && (kind == CAPF_AGG_SUM || kind == CAPF_AGG_AVG)) {
    fp64_sum_groups(s, g, nrows, arg, kind == CAPF_AGG_AVG, o);
    return o;
  }
  BufPtr acc = s->alloc(8 * ng);
  BufPtr cnt = s->alloc(8 * ng);
  HIP_CHECK(hipMemsetAsync(cnt->p, 0, 8 * ng, s->stream));
  // identity element of the accumulator
  int64_t init_bits = 0;
  if (kind == CAPF_AGG_MIN) {
    if (fl) { double x = INFINITY; memcpy(&init_bits, &x, 8); } else init_bits = INT64_MAX;
  } else if (kind == CAPF_AGG_MAX) {
    if (fl) { double x = -INFINITY; memcpy(&init_bits, &x, 8); } else init_bits = INT64_MIN;
  }
  hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(ng, 256)), dim3(256), 0, s->stream,
                     (int64_t *)acc->p, init_bits, ng);
  KERNEL_CHECK();
  ColView av = arg ? view_of(arg) : ColView{nullptr, nullptr, CAPF_TYPE_NULL, 0};
  if (nrows > 0) {
    KernelTimer kt(s, "group_aggregate", 16.0 * nrows);
    hipLaunchKernelGGL(k_agg, dim3(grid_for(nrows, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)g.group_of_row->p, nrows, av, kind, fl ? 1 : 0, acc->p,
                       (unsigned long long *)cnt->p);
    KERNEL_CHECK();
  }
  hipLaunchKernelGGL(k_agg_final, dim3(grid_for(ng, 256)), dim3(256), 0, s->stream, ng, kind,
                     fl ? 1 : 0, (int32_t)out_type, acc->p, (const unsigned long long *)cnt->p,
                     o->data ? o->data->p : nullptr, (uint8_t *)o->valid->p);
  KERNEL_CHECK();
  return o;
}

// ------------------------------------------------------------- ORDER BY
// Order-preserving uint64 image of a key; NULL handled by a separate pass.
__global__ void k_sort_key(ColView c, int64_t n, int desc, uint64_t *key, uint64_t *nullkey) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    bool nul = c.type == CAPF_TYPE_NULL || !c.data || (c.valid && !c.valid[r]);
    uint64_t k = 0;
    if (!nul) {
      if (c.type == CAPF_TYPE_BOOL) {
        k = ((const uint8_t *)c.data)[r] ? 1 : 0;
      } else if (c.type == CAPF_TYPE_FLOAT64) {
        uint64_t b = ((const uint64_t *)c.data)[r];
        if (b == 0x8000000000000000ull) b = 0;
        k = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
      } else {
        k = (uint64_t)ld_int(c, r) ^ 0x8000000000000000ull;
      }
    }
    key[r] = desc ? ~k : k;
    // Cypher/Calcite: NULL is the largest value — last ascending, first descending
    nullkey[r] = desc ? (nul ? 0 : 1) : (nul ? 1 : 0);
  }
}

__global__ void k_gather_u64(const uint64_t *src, const int64_t *idx, uint64_t *dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

static void radix_pass(Session *s, const uint64_t *keys_in, BufPtr &perm, int64_t n, int bits) {
  // stable sort of perm by keys_in[perm[i]]
  BufPtr kin = s->alloc(8 * n), kout = s->alloc(8 * n), pout = s->alloc(8 * n);
  hipLaunchKernelGGL(k_gather_u64, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, keys_in,
                     (const int64_t *)perm->p, (uint64_t *)kin->p, n);
  KERNEL_CHECK();
  size_t tmp = 0;
  HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp, (const uint64_t *)kin->p,
                                      (uint64_t *)kout->p, (const int64_t *)perm->p,
                                      (int64_t *)pout->p, (size_t)n, 0, bits, s->stream));
  BufPtr tbuf = s->alloc(std::max<size_t>(tmp, 16));
  HIP_CHECK(rocprim::radix_sort_pairs(tbuf->p, tmp, (const uint64_t *)kin->p,
                                      (uint64_t *)kout->p, (const int64_t *)perm->p,
                                      (int64_t *)pout->p, (size_t)n, 0, bits, s->stream));
  perm = pout;
}

BufPtr sort_permutation(Session *s, const std::vector<ColPtr> &keys,
                        const std::vector<int32_t> &desc, int64_t n) {
  BufPtr perm = iota_index(s, 0, n);
  if (n <= 1) return perm;
  BufPtr key = s->alloc(8 * n), nk = s->alloc(8 * n);
  // LSD over the sort items: least significant item first, each stable.
  for (int k = (int)keys.size() - 1; k >= 0; --k) {
    hipLaunchKernelGGL(k_sort_key, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                       view_of(keys[k]), n, desc[k] ? 1 : 0, (uint64_t *)key->p,
                       (uint64_t *)nk->p);
    KERNEL_CHECK();
    radix_pass(s, (const uint64_t *)key->p, perm, n, 64);
    radix_pass(s, (const uint64_t *)nk->p, perm, n, 1);
  }
  s->sync();
  return perm;
}

}  // namespace capf
