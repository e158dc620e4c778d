// dense_join.hip — the Expand join when one side's key is a dense unique id
// column (FlinkTable.join, FlinkTable.scala:171-187, in the shape the Expand
// of RelationalPlanner.scala:130-165 produces: node.id = start(r) / end(r),
// node ids of an element table being unique by construction).
//
// When the build key column holds exactly {min..max}, each value once and no
// NULL (the column statistics, computed once per column), the hash table of a
// hash join degenerates into a direct-address table: slot[v − min] = row.
// It is built once per column and cached on it, like the statistics (the
// ingest-time index of a node table); when row r holds min + r for every r
// (ids stored in order, the usual node table) no table is needed at all:
// row = v − min.  The probe is then one streaming pass:
//
//   k_dense_probe   per probe row: key → (in range? slot : miss), the build
//                   row written as int64 (−1 = no match), one match count per
//                   block (fixed grid, one atomic per block)
//   inner join      all probe rows matched (every rel's endpoints exist, the
//                   Expand case): the probe side's index is the identity —
//                   its columns pass through untouched, zero copy; otherwise
//                   the matched rows are compacted (wave ballot / scan)
//   probe-side outer (LEFT OUTER with the probe on the left, RIGHT OUTER with
//                   it on the right): identity + the −1 rows null-extended
//
// Build-side outer and FULL OUTER joins go to the radix join.  Bytes per
// probe row: the key (3/4/8 B by encoding) read, 8 B written; the slot
// table (4 B per build row) is L2/MALL-resident for node tables of up to
// ~2^25 rows.
#include <algorithm>
#include <cstring>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

struct DenseIndex {
  int64_t min = 0, n = 0;
  bool ident = false;  // row r holds min + r
  BufPtr slot;         // int32 row of value min + k (null when ident)
  // unique but not dense (sparse ids): an open-addressing table of 16-B slots
  // (int64 key, int32 row, pad) — one 16-B load per probe, linear probing from
  // fmix64(key) & (cap − 1), load ≤ 1/2.  `none`: the column has duplicate or
  // unsupported values (cached too, so the check runs once per column).
  bool hashed = false, none = false;
  int64_t cap = 0;
  BufPtr hslots;
};

constexpr int64_t HIDX_EMPTY = INT64_MIN;  // empty slot (a key equal to it: no index)

struct HSlot {
  int64_t key;
  int32_t row, pad;
};

__global__ void k_hidx_clear(HSlot *t, int64_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
    t[i] = HSlot{HIDX_EMPTY, -1, 0};
}

// flags: bit 0 = duplicate key, bit 1 = a key equal to the empty marker
__global__ void k_hidx_insert(ColView c, int64_t n, HSlot *t, int64_t cap, int *flags) {
  int f = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    if (c.valid && !c.valid[r]) continue;  // NULL keys never match: not indexed
    const int64_t k = ld_int(c, r);
    if (k == HIDX_EMPTY) {
      f |= 2;
      continue;
    }
    uint64_t h = fmix64((uint64_t)k) & (uint64_t)(cap - 1);
    for (;;) {
      const unsigned long long prev = atomicCAS((unsigned long long *)&t[h].key,
                                                (unsigned long long)HIDX_EMPTY, (unsigned long long)k);
      if (prev == (unsigned long long)HIDX_EMPTY) {
        t[h].row = (int32_t)r;
        break;
      }
      if ((int64_t)prev == k) {
        f |= 1;
        break;
      }
      h = (h + 1) & (uint64_t)(cap - 1);
    }
  }
  if (f) atomicOr(flags, f);
}

__global__ void k_dense_index(ColView c, int64_t n, int64_t mn, int32_t *slot, int *not_ident) {
  bool off = false;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = ld_int(c, r) - mn;
    slot[k] = (int32_t)r;
    off |= k != r;
  }
  if (__ballot(off) && lane_id() == 0) atomicOr(not_ident, 1);
}

// The hashed index of a unique (non-dense) INTEGER column: built once and
// cached on the column; nullptr (cached as `none`) when a value repeats.
static std::shared_ptr<DenseIndex> hashed_index(Session *s, const ColPtr &c, int64_t nrows) {
  auto di = std::make_shared<DenseIndex>();
  int64_t cap = 1024;
  while (cap < 2 * nrows) cap <<= 1;
  BufPtr t = s->alloc(sizeof(HSlot) * cap), flag = s->alloc(4);
  HIP_CHECK(hipMemsetAsync(flag->p, 0, 4, s->stream));
  hipLaunchKernelGGL(k_hidx_clear, dim3(grid_for(cap, 256)), dim3(256), 0, s->stream, (HSlot *)t->p, cap);
  KERNEL_CHECK();
  hipLaunchKernelGGL(k_hidx_insert, dim3(grid_for(nrows, 256)), dim3(256), 0, s->stream, view_of(c), nrows,
                     (HSlot *)t->p, cap, (int *)flag->p);
  KERNEL_CHECK();
  int nf = 0;
  HIP_CHECK(hipMemcpyAsync(&nf, flag->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  if (nf) {
    di->none = true;
  } else {
    di->hashed = true;
    di->cap = cap;
    di->n = nrows;
    di->hslots = t;
  }
  return di;
}

// The index of column c of a table of `nrows` rows: direct-address when the
// column is a non-null dense unique INTEGER column, hashed when it is unique
// but sparse; nullptr when neither applies.
static std::shared_ptr<DenseIndex> dense_index(Session *s, const ColPtr &c, int64_t nrows) {
  force(c);
  if (c->type != Type::Int64 || c->lazy || nrows == 0 || nrows >= (int64_t(1) << 31)) return nullptr;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->dense) {
      auto d = std::static_pointer_cast<DenseIndex>(c->dense);
      return d->none ? nullptr : d;
    }
  }
  const ColStats &st = column_stats(s, c);
  if (!st.dense_unique || st.non_null != nrows) {
    const char *hm = getenv("CAPF_HASH_INDEX");  // 0 (tuning): no hashed index
    if ((hm && atoi(hm) == 0) || c->unique_flag == 0 || nrows > (int64_t(1) << 27)) return nullptr;
    auto hi = hashed_index(s, c, nrows);
    std::lock_guard<std::mutex> lk(c->mu);
    c->dense = hi;
    c->unique_flag = hi->none ? 0 : 1;
    return hi->none ? nullptr : hi;
  }
  auto di = std::make_shared<DenseIndex>();
  di->min = st.min;
  di->n = nrows;
  BufPtr slot = s->alloc(4 * nrows), flag = s->alloc(4);
  HIP_CHECK(hipMemsetAsync(flag->p, 0, 4, s->stream));
  hipLaunchKernelGGL(k_dense_index, dim3(grid_for(nrows, 256)), dim3(256), 0, s->stream, view_of(c),
                     nrows, st.min, (int32_t *)slot->p, (int *)flag->p);
  KERNEL_CHECK();
  int nf = 0;
  HIP_CHECK(hipMemcpyAsync(&nf, flag->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  di->ident = nf == 0;
  if (!di->ident) di->slot = slot;
  std::lock_guard<std::mutex> lk(c->mu);
  c->dense = di;
  return di;
}

template <bool IDENT>
__global__ __launch_bounds__(256) void k_dense_probe(ColView key, int64_t n, int64_t mn, int64_t range,
                                                     const int32_t *slot, int64_t *brow,
                                                     unsigned long long *matched) {
  __shared__ unsigned long long red[256 / WAVE];
  unsigned long long cnt = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t b = -1;
    if (!key.valid || key.valid[r]) {
      const int64_t k = ld_int(key, r) - mn;
      if ((uint64_t)k < (uint64_t)range) b = IDENT ? k : (int64_t)slot[k];
    }
    brow[r] = b;
    cnt += b >= 0 ? 1u : 0u;
  }
  cnt = wave_reduce_sum(cnt);
  if (lane_id() == 0) red[threadIdx.x / WAVE] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < 256 / WAVE; ++w) t += red[w];
    if (t) atomicAdd(matched, t);
  }
}

// Probe of the hashed index: one 16-B slot load per step of the linear probe.
// WRITE = false: the match count only (no build row per probe row).
template <bool WRITE>
__global__ __launch_bounds__(256) void k_hidx_probe(ColView key, int64_t n, const HSlot *t, int64_t cap,
                                                    int64_t *brow, unsigned long long *matched) {
  __shared__ unsigned long long red[256 / WAVE];
  unsigned long long cnt = 0;
  const uint64_t mask = (uint64_t)(cap - 1);
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t b = -1;
    if (!key.valid || key.valid[r]) {
      const int64_t k = ld_int(key, r);
      uint64_t h = fmix64((uint64_t)k) & mask;
      for (;;) {
        const HSlot e = t[h];
        if (e.key == k) {
          b = e.row;
          break;
        }
        if (e.key == HIDX_EMPTY) break;
        h = (h + 1) & mask;
      }
    }
    if (WRITE) brow[r] = b;
    cnt += b >= 0 ? 1u : 0u;
  }
  cnt = wave_reduce_sum(cnt);
  if (lane_id() == 0) red[threadIdx.x / WAVE] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tt = 0;
    for (int w = 0; w < 256 / WAVE; ++w) tt += red[w];
    if (tt) atomicAdd(matched, tt);
  }
}

__global__ void k_dense_flags(const int64_t *brow, int64_t n, uint8_t *flags) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x)
    flags[r] = brow[r] >= 0 ? 1 : 0;
}

__global__ void k_dense_pick(const int64_t *rows, int64_t m, const int64_t *brow, int64_t *out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = brow[rows[i]];
}

// Whether dense_join would take (l, r) — the same tests, the indexes built and
// cached as dense_join builds them (a column without one caches "no index").
bool dense_join_possible(Session *s, const Data &l, const Data &r, const std::vector<std::pair<int, int>> &keys,
                         int32_t join_type) {
  if (keys.size() != 1 || join_type == CAPF_JOIN_CROSS || join_type == CAPF_JOIN_FULL_OUTER) return false;
  const char *mode = getenv("CAPF_JOIN");
  if (mode && (strcmp(mode, "radix") == 0 || strcmp(mode, "hash") == 0)) return false;
  const bool l_ok = join_type != CAPF_JOIN_LEFT_OUTER, r_ok = join_type != CAPF_JOIN_RIGHT_OUTER;
  std::shared_ptr<DenseIndex> di;
  bool build_left = false;
  if (r_ok && r.nrows <= l.nrows) di = dense_index(s, r.cols[keys[0].second], r.nrows);
  if (!di && l_ok) {
    di = dense_index(s, l.cols[keys[0].first], l.nrows);
    build_left = di != nullptr;
  }
  if (!di && r_ok && r.nrows > l.nrows) di = dense_index(s, r.cols[keys[0].second], r.nrows);
  if (!di) return false;
  const ColPtr &pk = (build_left ? r : l).cols[build_left ? keys[0].second : keys[0].first];
  return pk->type == Type::Int64;  // (a lazy column carries its type: no gather here)
}

bool dense_join(Session *s, const Data &l, const Data &r, const std::vector<std::pair<int, int>> &keys,
                int32_t join_type, JoinPairs &out) {
  if (keys.size() != 1 || join_type == CAPF_JOIN_CROSS || join_type == CAPF_JOIN_FULL_OUTER) return false;
  const char *mode = getenv("CAPF_JOIN");  // "radix" | "hash" force the general joins
  if (mode && (strcmp(mode, "radix") == 0 || strcmp(mode, "hash") == 0)) return false;
  // the build side is the dense one; an outer join must keep the probe side
  // (the build side's unmatched rows would need a second pass)
  const bool l_ok = join_type != CAPF_JOIN_LEFT_OUTER, r_ok = join_type != CAPF_JOIN_RIGHT_OUTER;
  std::shared_ptr<DenseIndex> di;
  bool build_left = false;
  if (r_ok && r.nrows <= l.nrows) di = dense_index(s, r.cols[keys[0].second], r.nrows);
  if (!di && l_ok) {
    di = dense_index(s, l.cols[keys[0].first], l.nrows);
    build_left = di != nullptr;
  }
  if (!di && r_ok && r.nrows > l.nrows) di = dense_index(s, r.cols[keys[0].second], r.nrows);
  if (!di) return false;
  const Data &Pr = build_left ? r : l;
  const ColPtr &pk = Pr.cols[build_left ? keys[0].second : keys[0].first];
  // not forced: a lazy probe key (a join's output column) may be provably
  // matching from its source's statistics, and then it is never gathered
  if (pk->type != Type::Int64) return false;
  const int64_t n = Pr.nrows;
  const bool probe_outer = join_type != CAPF_JOIN_INNER;
  // every probe key provably matches (no NULL, the key's range inside the dense
  // build range): from the probe column's cached statistics, or — a lazy gather
  // without NULL rows — from its source column's (computed once when the
  // source is far shorter than the probe side: the rel column behind a 2-path
  // join's end node)
  const bool all_match = [&] {
    if (n == 0 || di->hashed) return false;
    auto inside = [&](const ColStats &st, int64_t rows) {
      return st.non_null == rows && st.min >= di->min && st.max < di->min + di->n;
    };
    if (pk->stats) return inside(*pk->stats, n);
    if (pk->lazy && !pk->lazy->nullable) {
      const ColPtr &src = pk->lazy->src;
      if (src->stats || 4 * src->n <= n) return inside(column_stats(s, src), src->n);
    }
    return false;
  }();
  // ... and the build side carries nothing but its key and constant columns:
  // its row index would never be read — no probe at all, the probe rows pass
  // through (inner join: the build key is the probe key)
  const Data &B = build_left ? l : r;
  const int bk = build_left ? keys[0].first : keys[0].second;
  bool b_key_only = join_type == CAPF_JOIN_INNER;
  for (int j = 0; b_key_only && j < (int)B.cols.size(); ++j) {
    const ColPtr &c = B.cols[j];
    b_key_only = j == bk || (c->is_const && c->n > 0) ||
                 (c->lazy && !c->lazy->nullable && c->lazy->src->is_const && c->lazy->src->n > 0);
  }
  bool unread = all_match && b_key_only;
  // a hashed (sparse-id) index cannot prove every probe key present from
  // statistics: when the build side's rows would never be read, count the
  // matches first (no build row written per probe row) — the Expand case, where
  // every rel endpoint is a node, then passes the probe rows through as the
  // dense index does; a probe key without a node falls back to the full probe
  if (!unread && b_key_only && di->hashed && n > 0) {
    BufPtr cacc = s->alloc(8);
    HIP_CHECK(hipMemsetAsync(cacc->p, 0, 8, s->stream));
    {
      const double kw = pk->enc == ENC_FOR24 ? 3.0 : pk->enc == ENC_FOR32 ? 4.0 : 8.0;
      KernelTimer kt(s, "hidx_probe", (kw + 16.0) * n);
      const unsigned grid = grid_for(n, 256, (int64_t)s->num_cus * 8);
      hipLaunchKernelGGL(k_hidx_probe<false>, dim3(grid), dim3(256), 0, s->stream, view_of(pk), n,
                         (const HSlot *)di->hslots->p, di->cap, (int64_t *)nullptr, (unsigned long long *)cacc->p);
      KERNEL_CHECK();
    }
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, cacc->p, 8, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    unread = s->h_scalars[0] == n;
  }
  if (unread) {
    out.left = out.right = BufPtr();
    out.n = n;
    out.key_alias = build_left ? 1 : 2;
    out.build_unread = build_left ? 1 : 2;
    return true;
  }
  BufPtr brow = s->alloc(8 * std::max<int64_t>(n, 1));
  BufPtr acc = s->alloc(8);
  HIP_CHECK(hipMemsetAsync(acc->p, 0, 8, s->stream));
  if (n > 0) {
    const double kw = pk->enc == ENC_FOR24 ? 3.0 : pk->enc == ENC_FOR32 ? 4.0 : 8.0;
    KernelTimer kt(s, di->hashed ? "hidx_probe" : "dense_probe", (kw + 8.0 + (di->hashed ? 16.0 : 0.0)) * n);
    const unsigned grid = grid_for(n, 256, (int64_t)s->num_cus * 8);
    if (di->hashed)
      hipLaunchKernelGGL(k_hidx_probe<true>, dim3(grid), dim3(256), 0, s->stream, view_of(pk), n,
                         (const HSlot *)di->hslots->p, di->cap, (int64_t *)brow->p, (unsigned long long *)acc->p);
    else if (di->ident)
      hipLaunchKernelGGL(k_dense_probe<true>, dim3(grid), dim3(256), 0, s->stream, view_of(pk), n, di->min,
                         di->n, (const int32_t *)nullptr, (int64_t *)brow->p, (unsigned long long *)acc->p);
    else
      hipLaunchKernelGGL(k_dense_probe<false>, dim3(grid), dim3(256), 0, s->stream, view_of(pk), n, di->min,
                         di->n, (const int32_t *)di->slot->p, (int64_t *)brow->p,
                         (unsigned long long *)acc->p);
    KERNEL_CHECK();
  }
  // all_match: no match count to read back, so the join stays asynchronous;
  // otherwise one host read of the count
  int64_t matched = 0;
  if (all_match) {
    matched = n;
  } else {
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, acc->p, 8, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    matched = s->h_scalars[0];
  }
  BufPtr pidx, bidx = brow;  // pidx null = identity over the probe rows
  int64_t m = n;
  if (!probe_outer && matched < n) {
    BufPtr flags = s->alloc(std::max<int64_t>(n, 1));
    hipLaunchKernelGGL(k_dense_flags, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)brow->p, n, (uint8_t *)flags->p);
    KERNEL_CHECK();
    int64_t k = 0;
    pidx = compact_flags(s, (const uint8_t *)flags->p, n, &k);
    m = k;
    bidx = s->alloc(8 * std::max<int64_t>(k, 1));
    if (k > 0) {
      hipLaunchKernelGGL(k_dense_pick, dim3(grid_for(k, 256)), dim3(256), 0, s->stream,
                         (const int64_t *)pidx->p, k, (const int64_t *)brow->p, (int64_t *)bidx->p);
      KERNEL_CHECK();
    }
  }
  out.left = build_left ? bidx : pidx;
  out.right = build_left ? pidx : bidx;
  out.n = m;
  // inner join: the build key equals the probe key on every output row
  out.key_alias = join_type == CAPF_JOIN_INNER ? (build_left ? 1 : 2) : 0;
  return true;
}

}  // namespace capf
