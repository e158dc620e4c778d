// kernels_basic.hip — scans, compaction, gathers and the per-row expression
// interpreter behind Table.filter / withColumns / orderBy keys.
//
// Expression semantics follow FlinkSQLExprMapper
// (flink-cypher/.../impl/FlinkSQLExprMapper.scala:48-294) with Cypher
// three-valued logic: comparisons with NULL are NULL, Ands/Ors fold with
// SQL semantics (FlinkSQLExprMapper.scala:87-88), filter keeps TRUE rows only
// (FlinkTable.filter, FlinkTable.scala:76-78).
#include <algorithm>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

// ------------------------------------------------------------------ scan
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

template <typename T>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_tiles(const T *in, T *out, T *tile_sums,
                                                           int64_t n) {
  __shared__ T lds[17];
  int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  T v[SCAN_ITEMS];
  T local = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = base + k < n ? in[base + k] : T(0);
    local += v[k];
  }
  T total;
  T ex = block_exclusive_scan(local, lds, total);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (base + k < n) out[base + k] = ex;
    ex += v[k];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

template <typename T>
__global__ void k_add_tile_offsets(T *out, const T *tile_off, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += tile_off[i / SCAN_TILE];
}

template <typename T>
static void scan_rec(Session *s, const T *in, T *out, int64_t n, T *total_dev) {
  int64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles == 1) {  // one tile: its sum is the total (no copy launch)
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3(1), dim3(SCAN_BLOCK), 0, s->stream, in, out, total_dev, n);
    KERNEL_CHECK();
    return;
  }
  BufPtr sums = s->alloc(sizeof(T) * (tiles + 1));
  hipLaunchKernelGGL(k_scan_tiles<T>, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, s->stream, in,
                     out, (T *)sums->p, n);
  KERNEL_CHECK();
  BufPtr offs = s->alloc(sizeof(T) * tiles);
  scan_rec<T>(s, (const T *)sums->p, (T *)offs->p, tiles, total_dev);
  hipLaunchKernelGGL(k_add_tile_offsets<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     s->stream, out, (const T *)offs->p, n);
  KERNEL_CHECK();
}

int64_t exclusive_scan_i64(Session *s, const int64_t *d_in, int64_t *d_out, int64_t n) {
  if (n <= 0) return 0;
  scan_rec<int64_t>(s, d_in, d_out, n, s->d_scalars);
  HIP_CHECK(hipMemcpyAsync(s->h_scalars, s->d_scalars, 8, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  return s->h_scalars[0];
}

// The same without the host read: the total goes to the device int64 d_total.
void exclusive_scan_i64_async(Session *s, const int64_t *d_in, int64_t *d_out, int64_t n, int64_t *d_total) {
  if (n <= 0) {
    HIP_CHECK(hipMemsetAsync(d_total, 0, 8, s->stream));
    return;
  }
  scan_rec<int64_t>(s, d_in, d_out, n, d_total);
}

// uint32 variant (totals < 2^32), asynchronous: the total stays on the device.
void exclusive_scan_u32_async(Session *s, const uint32_t *d_in, uint32_t *d_out, int64_t n,
                              uint32_t *d_total) {
  if (n <= 0) {
    HIP_CHECK(hipMemsetAsync(d_total, 0, 4, s->stream));
    return;
  }
  scan_rec<uint32_t>(s, d_in, d_out, n, d_total);
}

// ------------------------------------------------------------ compaction
__global__ __launch_bounds__(SCAN_BLOCK) void k_count_flags(const uint8_t *flags, int64_t n,
                                                            int64_t *tile_counts) {
  __shared__ int64_t lds[17];
  int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) c += (base + k < n && flags[base + k]) ? 1 : 0;
  int64_t r = block_reduce_sum(c, lds);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = r;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scatter_flags(const uint8_t *flags, int64_t n,
                                                              const int64_t *tile_off,
                                                              int64_t *out) {
  __shared__ int64_t lds[17];
  int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  uint8_t f[SCAN_ITEMS];
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    f[k] = (base + k < n) ? flags[base + k] : 0;
    c += f[k] ? 1 : 0;
  }
  int64_t total;
  int64_t pos = block_exclusive_scan(c, lds, total) + tile_off[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (f[k]) out[pos++] = base + k;
}

BufPtr compact_flags(Session *s, const uint8_t *d_flags, int64_t n, int64_t *out_count) {
  if (n == 0) {
    *out_count = 0;
    return s->alloc(0);
  }
  int64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  BufPtr counts = s->alloc(8 * tiles), offs = s->alloc(8 * tiles);
  hipLaunchKernelGGL(k_count_flags, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, s->stream,
                     d_flags, n, (int64_t *)counts->p);
  KERNEL_CHECK();
  int64_t total = exclusive_scan_i64(s, (const int64_t *)counts->p, (int64_t *)offs->p, tiles);
  BufPtr idx = s->alloc(8 * std::max<int64_t>(total, 1));
  hipLaunchKernelGGL(k_scatter_flags, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, s->stream,
                     d_flags, n, (const int64_t *)offs->p, (int64_t *)idx->p);
  KERNEL_CHECK();
  *out_count = total;
  return idx;
}

// Selection of the rows whose flag is set, written through up to SEL_MAX
// sources at once: out_k[pos] = src_k ? src_k[r] : r.  A filter over a join's
// output writes the join's composed row indexes directly (li[r], ri[r] of the
// passing rows) instead of a selection index that each side then composes.
// Within a tile, rows go round by round (row tile0 + k·SCAN_BLOCK + t): flag
// reads and output writes coalesce (ballot + wave offsets per round).
constexpr int SEL_MAX = 4;
struct SelSrcs {
  const void *src[SEL_MAX];  // int64 (w 8) or int32 (w 4) row indexes, or null (the row itself, int64)
  void *out[SEL_MAX];        // written at the source's width
  int w[SEL_MAX];
  int ns;
};
__global__ __launch_bounds__(SCAN_BLOCK) void k_select_multi(const uint8_t *flags, int64_t n,
                                                             const int64_t *tile_off, SelSrcs ss) {
  __shared__ uint32_t wcnt[SCAN_BLOCK / WAVE];
  const int wv = threadIdx.x / WAVE, lane = lane_id();
  const int64_t t0 = (int64_t)blockIdx.x * SCAN_TILE;
  int64_t pos0 = tile_off[blockIdx.x];
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t r = t0 + (int64_t)k * SCAN_BLOCK + threadIdx.x;
    const bool f = r < n && flags[r];
    const unsigned long long m = __ballot(f);
    if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < SCAN_BLOCK / WAVE; ++w) {
      before += w < wv ? wcnt[w] : 0u;
      all += wcnt[w];
    }
    if (f) {
      const int64_t pos = pos0 + before + (uint32_t)__popcll(m & ((1ull << lane) - 1));
      for (int q = 0; q < ss.ns; ++q) {
        if (!ss.src[q]) ((int64_t *)ss.out[q])[pos] = r;
        else if (ss.w[q] == 4) ((int32_t *)ss.out[q])[pos] = ((const int32_t *)ss.src[q])[r];
        else ((int64_t *)ss.out[q])[pos] = ((const int64_t *)ss.src[q])[r];
      }
    }
    pos0 += all;
    __syncthreads();
  }
}

// ------------------------------------------------------------ index helpers
__global__ void k_iota(int64_t *out, int64_t start, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = start + i;
}

BufPtr iota_index(Session *s, int64_t start, int64_t m) {
  BufPtr b = s->alloc(8 * std::max<int64_t>(m, 1));
  if (m > 0) {
    hipLaunchKernelGGL(k_iota, dim3(grid_for(m, 256)), dim3(256), 0, s->stream, (int64_t *)b->p,
                       start, m);
    KERNEL_CHECK();
  }
  return b;
}

__global__ void k_cross(int64_t *li, int64_t *ri, int64_t nr, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    li[i] = i / nr;
    ri[i] = i % nr;
  }
}

void cross_index(Session *s, int64_t nl, int64_t nr, BufPtr &li, BufPtr &ri) {
  int64_t m = nl * nr;
  li = s->alloc(8 * std::max<int64_t>(m, 1));
  ri = s->alloc(8 * std::max<int64_t>(m, 1));
  if (m > 0) {
    hipLaunchKernelGGL(k_cross, dim3(grid_for(m, 256)), dim3(256), 0, s->stream,
                       (int64_t *)li->p, (int64_t *)ri->p, nr, m);
    KERNEL_CHECK();
  }
}

// ------------------------------------------------------------ gather / concat
template <typename T>
__global__ void k_gather(const T *src, const uint8_t *sval, const int64_t *idx, T *dst,
                         uint8_t *dval, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t j = idx[i];
    bool ok = j >= 0;
    if (dst) dst[i] = ok ? src[j] : T(0);
    if (dval) dval[i] = ok ? (sval ? sval[j] : 1) : 0;
  }
}

// Four consecutive rows per thread: 2 × 16-B index loads, the gathered
// values stored as one 4·sizeof(T) vector and the validity as one u32 (a
// 1-B store per row leaves the byte columns at ~1 TB/s).
template <typename T>
__device__ inline void gather_quad_store(T *dst, uint8_t *dval, int64_t q, const T (&v)[4], uint32_t vm) {
  if (dst) {
    if (sizeof(T) == 1) {
      ((uint32_t *)dst)[q] = (uint32_t)(uint8_t)v[0] | (uint32_t)(uint8_t)v[1] << 8 |
                             (uint32_t)(uint8_t)v[2] << 16 | (uint32_t)(uint8_t)v[3] << 24;
    } else if (sizeof(T) == 4) {
      ((uint4 *)dst)[q] = make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
    } else {
      ((longlong2 *)dst)[2 * q] = make_longlong2((long long)v[0], (long long)v[1]);
      ((longlong2 *)dst)[2 * q + 1] = make_longlong2((long long)v[2], (long long)v[3]);
    }
  }
  if (dval) ((uint32_t *)dval)[q] = vm;
}

// Two quads per thread per step: both quads' index loads, then all eight
// value loads, are in flight together (one quad at a time left the gather
// latency bound: 0.48 ms for 119 M FOR32 rows).
// the 4 index entries of quad q (int64: two 16-B loads, int32: one)
template <typename I>
__device__ inline void idx_quad(const I *idx, int64_t q, int64_t j[4]) {
  if constexpr (sizeof(I) == 8) {
    const longlong2 a = ((const longlong2 *)idx)[2 * q], b = ((const longlong2 *)idx)[2 * q + 1];
    j[0] = a.x;
    j[1] = a.y;
    j[2] = b.x;
    j[3] = b.y;
  } else {
    const int4 a = ((const int4 *)idx)[q];
    j[0] = a.x;
    j[1] = a.y;
    j[2] = a.z;
    j[3] = a.w;
  }
}

template <typename T, typename I>
__global__ void k_gather4(const T *src, const uint8_t *sval, const I *idx, T *dst,
                          uint8_t *dval, int64_t m) {
  const int64_t m4 = m / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; q + stride < m4; q += 2 * stride) {
    const int64_t qq[2] = {q, q + stride};
    int64_t j[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) idx_quad(idx, qq[h], j[h]);
    T v[2][4];
    uint32_t vm[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = j[h][k] >= 0;
        v[h][k] = ok && dst ? src[j[h][k]] : T(0);
        vm[h] |= (uint32_t)(ok ? (sval ? sval[j[h][k]] : 1) : 0) << (8 * k);
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) gather_quad_store(dst, dval, qq[h], v[h], vm[h]);
  }
  for (; q < m4; q += stride) {
    int64_t j[4];
    idx_quad(idx, q, j);
    T v[4];
    uint32_t vm = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = j[k] >= 0;
      v[k] = ok && dst ? src[j[k]] : T(0);
      vm |= (uint32_t)(ok ? (sval ? sval[j[k]] : 1) : 0) << (8 * k);
    }
    gather_quad_store(dst, dval, q, v, vm);
  }
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(m - 4 * m4)) {
    const int64_t i = 4 * m4 + threadIdx.x;
    const int64_t j = (int64_t)idx[i];
    const bool ok = j >= 0;
    if (dst) dst[i] = ok ? src[j] : T(0);
    if (dval) dval[i] = ok ? (sval ? sval[j] : 1) : 0;
  }
}

__global__ void k_fill_u64(uint64_t *p, uint64_t v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// m rows of a constant column's value (no validity: no NULLs)
ColPtr const_column(Session *s, const Column &c, int64_t m) {
  ColPtr o = make_column(s, c.type, m, false);
  o->is_const = true;
  o->const_bits = c.const_bits;
  if (m == 0) return o;
  if (c.type == Type::Bool) {
    HIP_CHECK(hipMemsetAsync(o->data->p, (int)(c.const_bits & 1), m, s->stream));
  } else {
    hipLaunchKernelGGL(k_fill_u64, dim3(grid_for(m, 256)), dim3(256), 0, s->stream, (uint64_t *)o->data->p,
                       c.const_bits, m);
    KERNEL_CHECK();
  }
  return o;
}

// FOR24 rows gathered into FOR32 (same base): the gathered rows are no
// longer a scan-order stream, 4-B rows keep every later access aligned
template <typename I>
__global__ void k_gather_u24(const void *src, const uint8_t *sval, const I *idx,
                             uint32_t *dst, uint8_t *dval, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t j = (int64_t)idx[i];
    bool ok = j >= 0;
    if (dst) dst[i] = ok ? ld_u24(src, j) : 0u;
    if (dval) dval[i] = ok ? (sval ? sval[j] : 1) : 0;
  }
}

// ------------------------------------------------------ late materialisation
// out = inner ∘ outer, written at the inner index's width (its values)
template <typename IO, typename II>
__global__ void k_compose_idx(const IO *outer, const II *inner, II *out, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = (int64_t)outer[i];
    out[i] = j < 0 ? II(-1) : inner[j];
  }
}

// int32 row indexes widened to int64 (for the few consumers that take int64 only)
__global__ void k_widen_idx(const int32_t *in, int64_t *out, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

static void launch_compose(Session *s, const void *outer, int ow, const void *inner, int iw, void *out, int64_t m) {
  const dim3 g(grid_for(m, 256)), b(256);
  if (ow == 8 && iw == 8)
    hipLaunchKernelGGL((k_compose_idx<int64_t, int64_t>), g, b, 0, s->stream, (const int64_t *)outer,
                       (const int64_t *)inner, (int64_t *)out, m);
  else if (ow == 8)
    hipLaunchKernelGGL((k_compose_idx<int64_t, int32_t>), g, b, 0, s->stream, (const int64_t *)outer,
                       (const int32_t *)inner, (int32_t *)out, m);
  else if (iw == 8)
    hipLaunchKernelGGL((k_compose_idx<int32_t, int64_t>), g, b, 0, s->stream, (const int32_t *)outer,
                       (const int64_t *)inner, (int64_t *)out, m);
  else
    hipLaunchKernelGGL((k_compose_idx<int32_t, int32_t>), g, b, 0, s->stream, (const int32_t *)outer,
                       (const int32_t *)inner, (int32_t *)out, m);
  KERNEL_CHECK();
}

static bool lazy_enabled() {
  static const bool on = !(getenv("CAPF_LAZY") && atoi(getenv("CAPF_LAZY")) == 0);
  return on;
}

void force(const ColPtr &c) {
  if (!c || !c->lazy) return;
  const std::shared_ptr<LazyGather> lz = c->lazy;
  ColPtr g = gather_column_w(lz->s, lz->src, lz->idx->p, lz->iw, lz->m, lz->nullable);
  c->data = g->data;
  c->valid = g->valid;
  c->enc = g->enc;
  c->base = g->base;
  c->lazy.reset();
}

ColPtr gather_lazy(Session *s, const ColPtr &c, const BufPtr &idx, int64_t m, bool nullable,
                   IdxCache *cache, int iw) {
  if (!idx && m == c->n) return c;  // identity: the column passes through, lazy or not
  if (!idx || !lazy_enabled() || c->type == Type::Null || c->type == Type::List || m == 0)
    return gather_column_w(s, c, idx ? idx->p : nullptr, iw, m, nullable);
  ColPtr src = c;
  BufPtr id = idx;
  int id_w = iw;
  if (c->lazy && c->lazy->src->is_const && !nullable && !c->lazy->nullable) {
    src = c->lazy->src;  // a constant gathers to a fill: the composed index is never read
  } else if (c->lazy) {
    const std::pair<const void *, const void *> key(c->lazy->idx.get(), idx.get());
    BufPtr composed;
    if (cache)
      for (auto &e : cache->entries)
        if (e.first == key) composed = e.second;
    if (!composed) {
      composed = s->alloc((int64_t)c->lazy->iw * m);
      launch_compose(s, idx->p, iw, c->lazy->idx->p, c->lazy->iw, composed->p, m);
      if (cache) cache->entries.emplace_back(key, composed);
    }
    id = composed;
    id_w = c->lazy->iw;  // the composed entries are the inner index's values
    nullable = nullable || c->lazy->nullable;
    src = c->lazy->src;
  }
  auto o = std::make_shared<Column>();
  o->type = src->type;
  o->n = m;
  o->lazy = std::make_shared<LazyGather>();
  o->lazy->s = s;
  o->lazy->src = src;
  o->lazy->idx = id;
  o->lazy->m = m;
  o->lazy->nullable = nullable;
  o->lazy->iw = id_w;
  return o;
}

ColPtr gather_column(Session *s, const ColPtr &c, const int64_t *d_idx, int64_t m,
                     bool idx_may_be_null) {
  return gather_column_w(s, c, d_idx, 8, m, idx_may_be_null);
}

ColPtr gather_column_w(Session *s, const ColPtr &c, const void *d_idx, int iw, int64_t m, bool idx_may_be_null) {
  force(c);
  if (!d_idx) {
    if (m == c->n) return c;
    illegal("internal: identity gather with mismatched length");
  }
  if (iw != 4 && iw != 8) illegal("internal: row index width");
  if (c->type == Type::Null) return null_column(s, Type::Null, m);
  if (c->type == Type::List) {
    if (iw == 8) return gather_list(s, c, (const int64_t *)d_idx, m);
    BufPtr w = s->alloc(8 * std::max<int64_t>(m, 1));
    if (m > 0) {
      hipLaunchKernelGGL(k_widen_idx, dim3(grid_for(m, 256)), dim3(256), 0, s->stream, (const int32_t *)d_idx,
                         (int64_t *)w->p, m);
      KERNEL_CHECK();
    }
    return gather_list(s, c, (const int64_t *)w->p, m);  // (w returns to the stream-ordered pool)
  }
  if (c->is_const && !idx_may_be_null && c->n > 0) return const_column(s, *c, m);
  if (!c->data || c->n == 0) {
    // empty source (outer join against an empty side): every index is the
    // null index, so the result is all NULL of the column's type
    if (m > 0 && !idx_may_be_null) illegal("internal: gather from an empty column");
    ColPtr o = make_column(s, c->type, m, true);
    if (m > 0) {
      HIP_CHECK(hipMemsetAsync(o->data->p, 0, m * type_width(c->type), s->stream));
      HIP_CHECK(hipMemsetAsync(o->valid->p, 0, m, s->stream));
    }
    return o;
  }
  bool with_valid = c->valid != nullptr || idx_may_be_null;
  ColPtr o;
  if (c->enc == ENC_FOR32 || c->enc == ENC_FOR24) {  // gathered rows keep the frame of reference
    o = std::make_shared<Column>();
    o->type = c->type;
    o->n = m;
    o->enc = ENC_FOR32;
    o->base = c->base;
    if (m > 0) o->data = s->alloc(4 * m);
    if (with_valid && m > 0) o->valid = s->alloc(m);
  } else {
    o = make_column(s, c->type, m, with_valid);
  }
  if (m == 0) return o;
  const uint8_t *sval = c->valid ? (const uint8_t *)c->valid->p : nullptr;
  uint8_t *dval = o->valid ? (uint8_t *)o->valid->p : nullptr;
  unsigned g = grid_for(m, 256);
  const unsigned g4 = grid_for((m + 3) / 4, 256);
  auto launch = [&](auto ityp) {
    using I = decltype(ityp);
    const I *ix = (const I *)d_idx;
    if (c->type == Type::Bool)
      hipLaunchKernelGGL((k_gather4<uint8_t, I>), dim3(g4), dim3(256), 0, s->stream,
                         (const uint8_t *)c->data->p, sval, ix, (uint8_t *)o->data->p, dval, m);
    else if (c->enc == ENC_FOR24)
      hipLaunchKernelGGL((k_gather_u24<I>), dim3(g), dim3(256), 0, s->stream, (const void *)c->data->p, sval,
                         ix, (uint32_t *)o->data->p, dval, m);
    else if (c->enc == ENC_FOR32)
      hipLaunchKernelGGL((k_gather4<uint32_t, I>), dim3(g4), dim3(256), 0, s->stream,
                         (const uint32_t *)c->data->p, sval, ix, (uint32_t *)o->data->p, dval, m);
    else
      hipLaunchKernelGGL((k_gather4<int64_t, I>), dim3(g4), dim3(256), 0, s->stream,
                         (const int64_t *)c->data->p, sval, ix, (int64_t *)o->data->p, dval, m);
    KERNEL_CHECK();
  };
  if (iw == 4) launch(int32_t{});
  else launch(int64_t{});
  return o;
}

template <typename T>
__global__ void k_copy_part(const T *src, const uint8_t *sval, T *dst, uint8_t *dval, int64_t n,
                            int64_t off) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (dst) dst[off + i] = src ? src[i] : T(0);
    if (dval) dval[off + i] = src ? (sval ? sval[i] : 1) : 0;
  }
}

// integer column of any encoding → plain int64 slice of the output
__global__ void k_copy_part_int(ColView src, int64_t *dst, uint8_t *dval, int64_t n, int64_t off) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool has = src.type != CAPF_TYPE_NULL && src.data;
    dst[off + i] = has ? ld_int(src, i) : 0;
    if (dval) dval[off + i] = has ? (src.valid ? src.valid[i] : 1) : 0;
  }
}

// LIST a ⊕ b: the offsets [na + nb + 1] with b's shifted by a's element
// count, and the row flags (a NULL-typed side is all NULL lists: no offsets)
__global__ void k_concat_list_offsets(const int64_t *ao, const uint8_t *av, int64_t na, const int64_t *bo,
                                      const uint8_t *bv, int64_t nb, int64_t *o, uint8_t *ov) {
  const int64_t atot = ao ? ao[na] : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= na + nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    o[i] = i <= na ? (ao ? ao[i] : 0) : atot + (bo ? bo[i - na] : 0);
    if (i < na) ov[i] = ao ? (av ? av[i] : 1) : 0;
    else if (i < na + nb) ov[i] = bo ? (bv ? bv[i - na] : 1) : 0;
  }
}

static ColPtr concat_lists(Session *s, const ColPtr &a, const ColPtr &b) {
  const ColPtr ca = a->type == Type::List ? a->child : nullptr, cb = b->type == Type::List ? b->child : nullptr;
  ColPtr child;
  if (ca && cb) {  // the element columns one after the other
    const Type et = ca->type == Type::Null ? cb->type : ca->type;
    if (cb->type != Type::Null && cb->type != et)
      illegal(std::string("Equal column types for union all: LIST(") + type_name(ca->type) + ") vs LIST(" +
              type_name(cb->type) + ")");
    child = concat_columns(s, ca, cb, et);
  } else {  // one side holds no elements: the other's element column as is
    child = ca ? ca : cb ? cb : null_column(s, Type::Null, 0);
  }
  const int64_t m = a->n + b->n;
  auto o = std::make_shared<Column>();
  o->type = Type::List;
  o->n = m;
  o->data = s->alloc(8 * (m + 1));
  o->valid = s->alloc(std::max<int64_t>(m, 1));
  o->child = child;
  const bool al = a->type == Type::List && a->data, bl = b->type == Type::List && b->data;
  hipLaunchKernelGGL(k_concat_list_offsets, dim3(grid_for(m + 1, 256)), dim3(256), 0, s->stream,
                     al ? (const int64_t *)a->data->p : nullptr, al && a->valid ? (const uint8_t *)a->valid->p : nullptr,
                     a->n, bl ? (const int64_t *)b->data->p : nullptr,
                     bl && b->valid ? (const uint8_t *)b->valid->p : nullptr, b->n, (int64_t *)o->data->p,
                     (uint8_t *)o->valid->p);
  KERNEL_CHECK();
  return o;
}

__global__ void k_rank_codes(ColView r, const int64_t *order, int64_t n, int64_t *out, uint8_t *ok) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool v = r.type != CAPF_TYPE_NULL && r.data && !(r.valid && !r.valid[i]);
    out[i] = v ? order[ld_int(r, i)] : 0;
    ok[i] = v ? 1 : 0;
  }
}

ColPtr ranks_to_codes(Session *s, const ColPtr &ranks) {
  force(ranks);
  size_t ns = 0;
  const int64_t *order = string_order_table(s, &ns);
  const int64_t n = ranks->n;
  ColPtr o = make_column(s, Type::String, n, true);
  if (n > 0) {
    const ColView v = ranks->type == Type::Null ? ColView{nullptr, nullptr, CAPF_TYPE_NULL, ENC_PLAIN, 0}
                                                : view_of(ranks);
    hipLaunchKernelGGL(k_rank_codes, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, v, order, n,
                       (int64_t *)o->data->p, (uint8_t *)o->valid->p);
    KERNEL_CHECK();
  }
  return o;
}

ColPtr concat_columns(Session *s, const ColPtr &a, const ColPtr &b, Type t) {
  force(a);
  force(b);
  if (t == Type::List) return concat_lists(s, a, b);
  int64_t m = a->n + b->n;
  if (t == Type::Null) return null_column(s, t, m);
  bool with_valid = a->valid || b->valid || a->type == Type::Null || b->type == Type::Null;
  ColPtr o = make_column(s, t, m, with_valid);
  uint8_t *dval = o->valid ? (uint8_t *)o->valid->p : nullptr;
  int64_t off = 0;
  for (const ColPtr &c : {a, b}) {
    if (c->n > 0) {
      const void *src = c->type == Type::Null ? nullptr : c->data->p;
      const uint8_t *sval = c->valid ? (const uint8_t *)c->valid->p : nullptr;
      unsigned g = grid_for(c->n, 256);
      if (t == Type::Bool)
        hipLaunchKernelGGL(k_copy_part<uint8_t>, dim3(g), dim3(256), 0, s->stream,
                           (const uint8_t *)src, sval, (uint8_t *)o->data->p, dval, c->n, off);
      else if (c->enc != ENC_PLAIN)
        hipLaunchKernelGGL(k_copy_part_int, dim3(g), dim3(256), 0, s->stream, view_of(c),
                           (int64_t *)o->data->p, dval, c->n, off);
      else
        hipLaunchKernelGGL(k_copy_part<int64_t>, dim3(g), dim3(256), 0, s->stream,
                           (const int64_t *)src, sval, (int64_t *)o->data->p, dval, c->n, off);
      KERNEL_CHECK();
    }
    off += c->n;
  }
  return o;
}

// ------------------------------------------------------------ encodings
__global__ void k_decode_for32(const uint32_t *src, int64_t base, int64_t *dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = base + (int64_t)src[i];
}

__global__ void k_encode_for32(const int64_t *src, const uint8_t *valid, int64_t base,
                               uint32_t *dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (valid && !valid[i]) ? 0u : (uint32_t)(src[i] - base);
}

__global__ void k_decode_for24(const void *src, int64_t base, int64_t *dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = base + (int64_t)ld_u24(src, i);
}

// Thread per 4 rows: 12 bytes = 3 aligned dwords (rows past n encode 0; the
// 16-B tail pad is zeroed by the last thread).
__global__ void k_encode_for24(const int64_t *src, const uint8_t *valid, int64_t base,
                               uint32_t *dst, int64_t n) {
  const int64_t groups = (n + 3) / 4;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups;
       g += (int64_t)gridDim.x * blockDim.x) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t r = 4 * g + k;
      v[k] = (r < n && !(valid && !valid[r])) ? (uint32_t)(src[r] - base) & 0xFFFFFFu : 0u;
    }
    dst[3 * g] = v[0] | v[1] << 24;
    dst[3 * g + 1] = v[1] >> 8 | v[2] << 16;
    dst[3 * g + 2] = v[2] >> 16 | v[3] << 8;
    if (g == groups - 1)
      for (int k = 0; k < 4; ++k) dst[3 * groups + k] = 0u;
  }
}

ColPtr decode_column(Session *s, const ColPtr &c) {
  force(c);
  if (c->enc == ENC_PLAIN) return c;
  auto o = std::make_shared<Column>();
  o->type = c->type;
  o->n = c->n;
  o->valid = c->valid;
  if (c->n > 0) {
    o->data = s->alloc(8 * c->n);
    if (c->enc == ENC_FOR24)
      hipLaunchKernelGGL(k_decode_for24, dim3(grid_for(c->n, 256)), dim3(256), 0, s->stream,
                         (const void *)c->data->p, c->base, (int64_t *)o->data->p, c->n);
    else
      hipLaunchKernelGGL(k_decode_for32, dim3(grid_for(c->n, 256)), dim3(256), 0, s->stream,
                         (const uint32_t *)c->data->p, c->base, (int64_t *)o->data->p, c->n);
    KERNEL_CHECK();
  }
  return o;
}

// width 4: FOR32 where the range fits 32 bits; width 3: FOR24 where it fits
// 24 bits, else FOR32 where it fits 32.  Already-encoded columns unchanged.
ColPtr encode_column(Session *s, const ColPtr &c, int width) {
  force(c);
  if (c->enc != ENC_PLAIN || (c->type != Type::Int64 && c->type != Type::String) || c->n == 0)
    return c;
  const ColStats &st = column_stats(s, c);
  if (st.non_null == 0 || (uint64_t)(st.max - st.min) > 0xFFFFFFFFull) return c;
  if (width == 3 && (uint64_t)(st.max - st.min) <= 0xFFFFFFull) {
    auto o = std::make_shared<Column>();
    o->type = c->type;
    o->n = c->n;
    o->enc = ENC_FOR24;
    o->base = st.min;
    o->valid = c->valid;
    const int64_t groups = (c->n + 3) / 4;
    o->data = s->alloc(12 * groups + 16);
    hipLaunchKernelGGL(k_encode_for24, dim3(grid_for(groups, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)c->data->p, c->valid ? (const uint8_t *)c->valid->p : nullptr,
                       st.min, (uint32_t *)o->data->p, c->n);
    KERNEL_CHECK();
    o->stats = st;
    std::copy(c->owner, c->owner + 4, o->owner);
    return o;
  }
  auto o = std::make_shared<Column>();
  o->type = c->type;
  o->n = c->n;
  o->enc = ENC_FOR32;
  o->base = st.min;
  o->valid = c->valid;
  o->data = s->alloc(4 * c->n);
  hipLaunchKernelGGL(k_encode_for32, dim3(grid_for(c->n, 256)), dim3(256), 0, s->stream,
                     (const int64_t *)c->data->p, c->valid ? (const uint8_t *)c->valid->p : nullptr,
                     st.min, (uint32_t *)o->data->p, c->n);
  KERNEL_CHECK();
  o->stats = st;  // the values are unchanged
  std::copy(c->owner, c->owner + 4, o->owner);
  return o;
}

// ------------------------------------------------------------ statistics
__global__ __launch_bounds__(256) void k_minmax(ColView v, int64_t n, int64_t *acc) {
  __shared__ int64_t red[3][4];
  int64_t mn = INT64_MAX, mx = INT64_MIN, cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (v.valid && !v.valid[i]) continue;
    int64_t x = ld_int(v, i);
    mn = x < mn ? x : mn;
    mx = x > mx ? x : mx;
    ++cnt;
  }
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) {
    int64_t a = __shfl_xor(mn, d, WAVE), b = __shfl_xor(mx, d, WAVE);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    cnt += __shfl_xor(cnt, d, WAVE);
  }
  // one set of atomics per block (not per wave): they serialise on 3 words
  const int w = threadIdx.x / WAVE;
  if (lane_id() == 0) {
    red[0][w] = mn;
    red[1][w] = mx;
    red[2][w] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x / WAVE); ++k) {
      mn = red[0][k] < mn ? red[0][k] : mn;
      mx = red[1][k] > mx ? red[1][k] : mx;
      cnt += red[2][k];
    }
    if (cnt) {
      atomicMin((long long *)&acc[0], (long long)mn);
      atomicMax((long long *)&acc[1], (long long)mx);
      atomicAdd((unsigned long long *)&acc[2], (unsigned long long)cnt);
    }
  }
}

// Duplicate test of a column whose values fill [base, base + n): one bit per
// value.  Each thread takes DUP_RUN consecutive rows and ORs the bits of one
// 32-value word in a register, flushing with one atomic when the word changes
// — sequential ids (node tables) cost one uncontended atomic per 32 rows
// instead of 32 lanes serialising on the same word.
constexpr int DUP_RUN = 32;

__global__ __launch_bounds__(256) void k_dup_check(ColView v, int64_t n, int64_t base,
                                                   uint32_t *bits, int64_t *dup) {
  bool found = false;
  for (int64_t c0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * DUP_RUN; c0 < n;
       c0 += (int64_t)gridDim.x * blockDim.x * DUP_RUN) {
    const int64_t c1 = c0 + DUP_RUN < n ? c0 + DUP_RUN : n;
    uint64_t cw = ~0ull;
    uint32_t acc = 0;
    for (int64_t i = c0; i < c1; ++i) {
      if (v.valid && !v.valid[i]) continue;
      const uint64_t k = (uint64_t)(ld_int(v, i) - base);
      const uint64_t w = k >> 5;
      const uint32_t m = 1u << (k & 31);
      if (w != cw) {
        if (acc) found |= (atomicOr(&bits[cw], acc) & acc) != 0;
        cw = w;
        acc = 0;
      }
      found |= (acc & m) != 0;
      acc |= m;
    }
    if (acc) found |= (atomicOr(&bits[cw], acc) & acc) != 0;
  }
  if (found) *dup = 1;
}

ColStats compute_stats(Session *s, const Column &c) {
  ColStats st;
  if (c.type != Type::Int64 && c.type != Type::String) {
    st.non_null = c.type == Type::Null ? 0 : c.n;
    return st;
  }
  if (c.n == 0) return st;
  ColView v;
  v.data = c.data->p;
  v.valid = c.valid ? (const uint8_t *)c.valid->p : nullptr;
  v.type = (int32_t)c.type;
  v.enc = c.enc;
  v.base = c.base;
  int64_t init[3] = {INT64_MAX, INT64_MIN, 0};
  HIP_CHECK(hipMemcpyAsync(s->d_scalars, init, sizeof(init), hipMemcpyHostToDevice, s->stream));
  hipLaunchKernelGGL(k_minmax, dim3(grid_for(c.n, 256, 2048)), dim3(256), 0, s->stream, v, c.n,
                     s->d_scalars);
  KERNEL_CHECK();
  HIP_CHECK(hipMemcpyAsync(s->h_scalars, s->d_scalars, sizeof(init), hipMemcpyDeviceToHost, s->stream));
  s->sync();
  st.min = s->h_scalars[0];
  st.max = s->h_scalars[1];
  st.non_null = s->h_scalars[2];
  if (st.non_null > 0 && (uint64_t)(st.max - st.min) + 1 == (uint64_t)st.non_null &&
      st.non_null <= (int64_t(1) << 34)) {
    int64_t words = (st.non_null + 31) / 32;
    BufPtr bits = s->alloc(4 * words);
    HIP_CHECK(hipMemsetAsync(bits->p, 0, 4 * words, s->stream));
    HIP_CHECK(hipMemsetAsync(s->d_scalars + 3, 0, 8, s->stream));
    hipLaunchKernelGGL(k_dup_check, dim3(grid_for((c.n + DUP_RUN - 1) / DUP_RUN, 256, 4096)),
                       dim3(256), 0, s->stream, v,
                       c.n, st.min, (uint32_t *)bits->p, s->d_scalars + 3);
    KERNEL_CHECK();
    HIP_CHECK(hipMemcpyAsync(s->h_scalars + 3, s->d_scalars + 3, 8, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    st.dense_unique = s->h_scalars[3] == 0;
  }
  return st;
}

// ------------------------------------------------------------ interpreter
struct Val {
  int64_t b;   // int64 value, bool (0/1), string code or double bits
  int32_t t;   // capf type
  int32_t nul; // 1 = NULL
};

__device__ inline double vf(const Val &v) {
  return v.t == CAPF_TYPE_FLOAT64 ? __longlong_as_double(v.b) : (double)v.b;
}
__device__ inline Val mk(int64_t b, int32_t t, int32_t nul) {
  Val v;
  v.b = b;
  v.t = t;
  v.nul = nul;
  return v;
}
__device__ inline Val mkf(double f) { return mk(__double_as_longlong(f), CAPF_TYPE_FLOAT64, 0); }
__device__ inline Val mkb(bool x) { return mk(x ? 1 : 0, CAPF_TYPE_BOOL, 0); }
__device__ inline Val mknull(int32_t t) { return mk(0, t, 1); }

__device__ inline Val load_col(const ColView &c, int64_t r) {
  if (c.type == CAPF_TYPE_NULL || !c.data) return mknull(CAPF_TYPE_NULL);
  if (c.valid && !c.valid[r]) return mknull(c.type);
  if (c.type == CAPF_TYPE_BOOL) return mk(((const uint8_t *)c.data)[r] ? 1 : 0, c.type, 0);
  return mk(ld_int(c, r), c.type, 0);
}

// -1 less, 0 equal, 1 greater (non-null operands)
__device__ inline int cmp_vals(const Val &a, const Val &b) {
  if (a.t == CAPF_TYPE_FLOAT64 || b.t == CAPF_TYPE_FLOAT64) {
    double x = vf(a), y = vf(b);
    return x < y ? -1 : (x > y ? 1 : 0);
  }
  return a.b < b.b ? -1 : (a.b > b.b ? 1 : 0);
}

// Unary math functions (FlinkSQLExprMapper.scala:199-221), NULL in NULL out.
// FP contraction is off here: no FMA changes the Java double arithmetic
// they restate.
__device__ inline Val math1(int32_t op, const Val &a) {
#pragma clang fp contract(off)
  const bool isint = a.t == CAPF_TYPE_INT64;
  if (a.nul) {
    const bool keeps = op == OP_ABS || op == OP_CEIL || op == OP_FLOOR || op == OP_SIGN;
    return mknull(keeps && isint ? CAPF_TYPE_INT64 : CAPF_TYPE_FLOAT64);
  }
  const double x = vf(a);
  switch (op) {
    case OP_ROUND: {  // half away from zero (Spark round → BigDecimal HALF_UP), a FLOAT
      if (isint) return mkf(x);
      double r = trunc(x);
      const double f = x - r;  // exact
      if (f >= 0.5) r += 1.0;
      else if (f <= -0.5) r -= 1.0;
      return mkf(r);
    }
    case OP_ABS:
      if (isint) return mk(a.b < 0 ? (int64_t)(0 - (uint64_t)a.b) : a.b, CAPF_TYPE_INT64, 0);
      return mkf(fabs(x));
    case OP_CEIL: return isint ? a : mkf(ceil(x));
    case OP_FLOOR: return isint ? a : mkf(floor(x));
    case OP_SIGN:  // Calcite SIGN keeps the operand's type
      if (isint) return mk(a.b > 0 ? 1 : (a.b < 0 ? -1 : 0), CAPF_TYPE_INT64, 0);
      return mkf(x > 0 ? 1.0 : (x < 0 ? -1.0 : x));
    case OP_SQRT: return mkf(sqrt(x));
    case OP_LOG: return mkf(log(x));
    case OP_LOG10: return mkf(log10(x));
    case OP_EXP: return mkf(exp(x));
    case OP_SIN: return mkf(sin(x));
    case OP_COS: return mkf(cos(x));
    case OP_TAN: return mkf(tan(x));
    case OP_ASIN: return mkf(asin(x));
    case OP_ACOS: return mkf(acos(x));
    case OP_ATAN: return mkf(atan(x));
    // Java 8 Math.toDegrees / toRadians: angrad * 180.0 / PI, angdeg / 180.0 * PI
    case OP_DEGREES: return mkf(x * 180.0 / 3.141592653589793);
    case OP_RADIANS: return mkf(x / 180.0 * 3.141592653589793);
    default: return mknull(CAPF_TYPE_FLOAT64);
  }
}

constexpr int MAX_STACK = 24;
constexpr int MAX_LDS_CODE = 96;

__device__ Val run_program(const Instr *code, int ncode, const ColView *cols, int64_t r) {
  Val st[MAX_STACK];
  int sp = 0;
  for (int pc = 0; pc < ncode; ++pc) {
    const Instr in = code[pc];
    switch (in.op) {
      case OP_COL: st[sp++] = load_col(cols[in.i], r); break;
      case OP_LIT_INT: st[sp++] = mk(in.i, CAPF_TYPE_INT64, 0); break;
      case OP_LIT_FLOAT: st[sp++] = mkf(in.f); break;
      case OP_LIT_BOOL: st[sp++] = mkb(in.i != 0); break;
      case OP_LIT_STRING: st[sp++] = mk(in.i, CAPF_TYPE_STRING, 0); break;
      case OP_LIT_NULL: st[sp++] = mknull((int32_t)in.i); break;
      case OP_EQ: case OP_NEQ: case OP_LT: case OP_LE: case OP_GT: case OP_GE: {
        Val b = st[--sp], a = st[--sp];
        if (a.nul || b.nul) {
          st[sp++] = mknull(CAPF_TYPE_BOOL);
          break;
        }
        int c = cmp_vals(a, b);
        bool res;
        switch (in.op) {
          case OP_EQ: res = c == 0; break;
          case OP_NEQ: res = c != 0; break;
          case OP_LT: res = c < 0; break;
          case OP_LE: res = c <= 0; break;
          case OP_GT: res = c > 0; break;
          default: res = c >= 0; break;
        }
        st[sp++] = mkb(res);
        break;
      }
      case OP_NOT: {
        Val a = st[--sp];
        st[sp++] = a.nul ? mknull(CAPF_TYPE_BOOL) : mkb(a.b == 0);
        break;
      }
      case OP_AND: case OP_OR: {
        int k = (int)in.i;
        bool any_dom = false, any_null = false;  // dominant = false for AND, true for OR
        for (int j = 0; j < k; ++j) {
          Val a = st[--sp];
          if (a.nul)
            any_null = true;
          else if ((in.op == OP_AND) == (a.b == 0))
            any_dom = true;
        }
        if (any_dom)
          st[sp++] = mkb(in.op == OP_OR);
        else if (any_null)
          st[sp++] = mknull(CAPF_TYPE_BOOL);
        else
          st[sp++] = mkb(in.op == OP_AND);
        break;
      }
      case OP_IS_NULL: {
        Val a = st[--sp];
        st[sp++] = mkb(a.nul != 0);
        break;
      }
      case OP_IS_NOT_NULL: {
        Val a = st[--sp];
        st[sp++] = mkb(a.nul == 0);
        break;
      }
      case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_MOD: {
        Val b = st[--sp], a = st[--sp];
        bool fl = a.t == CAPF_TYPE_FLOAT64 || b.t == CAPF_TYPE_FLOAT64;
        if (a.nul || b.nul) {
          st[sp++] = mknull(fl ? CAPF_TYPE_FLOAT64 : CAPF_TYPE_INT64);
          break;
        }
        if (fl) {
          double x = vf(a), y = vf(b), z;
          switch (in.op) {
            case OP_ADD: z = x + y; break;
            case OP_SUB: z = x - y; break;
            case OP_MUL: z = x * y; break;
            case OP_DIV: z = x / y; break;
            default: z = fmod(x, y); break;
          }
          st[sp++] = mkf(z);
        } else {
          int64_t x = a.b, y = b.b, z = 0;
          bool nul = false;
          switch (in.op) {
            case OP_ADD: z = (int64_t)((uint64_t)x + (uint64_t)y); break;
            case OP_SUB: z = (int64_t)((uint64_t)x - (uint64_t)y); break;
            case OP_MUL: z = (int64_t)((uint64_t)x * (uint64_t)y); break;
            case OP_DIV:
              if (y == 0) nul = true; else z = (y == -1) ? (int64_t)(0 - (uint64_t)x) : x / y;
              break;
            default:
              if (y == 0) nul = true; else z = (y == -1) ? 0 : x % y;
              break;
          }
          st[sp++] = mk(z, CAPF_TYPE_INT64, nul ? 1 : 0);
        }
        break;
      }
      case OP_NEG: {
        Val a = st[--sp];
        if (!a.nul) {
          if (a.t == CAPF_TYPE_FLOAT64)
            a = mkf(-vf(a));
          else
            a.b = (int64_t)(0 - (uint64_t)a.b);
        }
        st[sp++] = a;
        break;
      }
      case OP_TO_FLOAT: {
        Val a = st[--sp];
        if (a.nul || a.t == CAPF_TYPE_BOOL)
          st[sp++] = mknull(CAPF_TYPE_FLOAT64);
        else
          st[sp++] = mkf(vf(a));
        break;
      }
      case OP_TO_INTEGER: {
        // Flink lowers ToInteger to a cast to INT (32 bit),
        // FlinkSQLExprMapper.scala:183.  Java (int) semantics.
        Val a = st[--sp];
        if (a.nul || a.t == CAPF_TYPE_BOOL) {
          st[sp++] = mknull(CAPF_TYPE_INT64);
        } else if (a.t == CAPF_TYPE_FLOAT64) {
          double x = vf(a);
          int32_t y;
          if (x != x) y = 0;
          else if (x >= 2147483647.0) y = 2147483647;
          else if (x <= -2147483648.0) y = (-2147483647 - 1);
          else y = (int32_t)x;
          st[sp++] = mk((int64_t)y, CAPF_TYPE_INT64, 0);
        } else {
          st[sp++] = mk((int64_t)(int32_t)(uint32_t)(uint64_t)a.b, CAPF_TYPE_INT64, 0);
        }
        break;
      }
      case OP_COALESCE: {
        int k = (int)in.i;
        Val res = mknull(CAPF_TYPE_NULL);
        // operands were pushed first..last; pick the first non-null
        for (int j = 0; j < k; ++j) {
          Val a = st[sp - k + j];
          if (!a.nul) {
            res = a;
            break;
          }
        }
        sp -= k;
        st[sp++] = res;
        break;
      }
      case OP_STR_LEN: {  // cols[in.i] = the session's string lengths by code
        Val a = st[--sp];
        st[sp++] = a.nul ? mknull(CAPF_TYPE_INT64)
                         : mk(((const int64_t *)cols[in.i].data)[a.b], CAPF_TYPE_INT64, 0);
        break;
      }
      case OP_STR_RANK: {  // cols[in.i] = the session's string ranks by code
        Val a = st[--sp];
        st[sp++] = a.nul ? mknull(CAPF_TYPE_INT64)
                         : mk(((const int64_t *)cols[in.i].data)[a.b], CAPF_TYPE_INT64, 0);
        break;
      }
      case OP_LIST_SIZE: {  // cols[in.i]: LIST offsets [n + 1]
        const ColView &c = cols[in.i];
        if (!c.data || (c.valid && !c.valid[r]))
          st[sp++] = mknull(CAPF_TYPE_INT64);
        else
          st[sp++] = mk(((const int64_t *)c.data)[r + 1] - ((const int64_t *)c.data)[r], CAPF_TYPE_INT64, 0);
        break;
      }
      case OP_IF: {
        Val v = st[--sp], c = st[--sp], e = st[--sp];
        Val r = (!c.nul && c.b != 0) ? v : e;
        // an INTEGER and a FLOAT branch: the CASE is a FLOAT (Calcite's CASE
        // type; the compiler types it so) — widen the chosen value here, not
        // only at the final store, so an enclosing Divide / Modulo sees a FLOAT
        const bool mixed = (v.t == CAPF_TYPE_FLOAT64 && e.t == CAPF_TYPE_INT64) ||
                           (v.t == CAPF_TYPE_INT64 && e.t == CAPF_TYPE_FLOAT64);
        if (mixed && r.t == CAPF_TYPE_INT64) r = r.nul ? mknull(CAPF_TYPE_FLOAT64) : mkf(vf(r));
        st[sp++] = r;
        break;
      }
      case OP_ROUND: case OP_ABS: case OP_CEIL: case OP_FLOOR: case OP_SIGN: case OP_SQRT:
      case OP_LOG: case OP_LOG10: case OP_EXP: case OP_SIN: case OP_COS: case OP_TAN:
      case OP_ASIN: case OP_ACOS: case OP_ATAN: case OP_DEGREES: case OP_RADIANS: {
        Val a = st[--sp];
        st[sp++] = math1(in.op, a);
        break;
      }
      case OP_ATAN2: {  // atan2(y, x): y pushed first (FlinkSQLExprMapper.scala:212)
        Val x = st[--sp], y = st[--sp];
        st[sp++] = (x.nul || y.nul) ? mknull(CAPF_TYPE_FLOAT64) : mkf(atan2(vf(y), vf(x)));
        break;
      }
      case OP_IN_SET: {  // cols[in.i] = sorted set values, base = their count
        Val a = st[--sp];
        if (a.nul) {
          st[sp++] = mknull(CAPF_TYPE_BOOL);
          break;
        }
        const int64_t *v = (const int64_t *)cols[in.i].data;
        int64_t lo = 0, hi = cols[in.i].base;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (v[mid] < a.b) lo = mid + 1;
          else hi = mid;
        }
        const bool hit = lo < cols[in.i].base && v[lo] == a.b;
        st[sp++] = hit ? mkb(true) : in.f != 0.0 ? mknull(CAPF_TYPE_BOOL) : mkb(false);
        break;
      }
      case OP_VALUE_MAP: {  // cols[in.i]: [keys][keys2 (enc = 1)][codes], base = n
        Val y = in.f != 0.0 ? st[--sp] : Val{};
        Val a = st[--sp];
        const ColView &m = cols[in.i];
        const int64_t n = m.base;
        const int64_t *k1 = (const int64_t *)m.data, *k2 = k1 + n, *cd = k1 + (m.enc ? 2 : 1) * n;
        int64_t r = -1;
        if (!a.nul && !(in.f != 0.0 && y.nul)) {
          int64_t lo = 0, hi = n;
          while (lo < hi) {  // first entry ≥ (a, y)
            const int64_t mid = (lo + hi) >> 1;
            const bool less = k1[mid] < a.b || (m.enc && k1[mid] == a.b && k2[mid] < y.b);
            if (less) lo = mid + 1;
            else hi = mid;
          }
          if (lo < n && k1[lo] == a.b && (!m.enc || k2[lo] == y.b)) r = cd[lo];
        }
        st[sp++] = r < 0 ? mknull(CAPF_TYPE_STRING) : mk(r, CAPF_TYPE_STRING, 0);
        break;
      }
      case OP_STR_MAP: {  // cols[in.i] = a code map (base = its length)
        Val a = st[--sp];
        const int64_t c = a.nul ? -1 : a.b;
        const int64_t m = c >= 0 && c < cols[in.i].base ? ((const int64_t *)cols[in.i].data)[c] : -1;
        st[sp++] = m < 0 ? mknull(CAPF_TYPE_STRING) : mk(m, CAPF_TYPE_STRING, 0);
        break;
      }
      case OP_STR_TO_NUM: {  // cols[in.i] = [double n][int64 n][flags n], n in base; f: 1 DOUBLE, 0 INTEGER
        Val a = st[--sp];
        const bool fl = in.f != 0.0;
        const int64_t n = cols[in.i].base;
        if (a.nul || a.b < 0 || a.b >= n) {
          st[sp++] = mknull(fl ? CAPF_TYPE_FLOAT64 : CAPF_TYPE_INT64);
        } else {
          const uint8_t *base = (const uint8_t *)cols[in.i].data;
          const uint8_t f = base[16 * n + a.b];
          if (fl)
            st[sp++] = (f & 1) ? mkf(((const double *)base)[a.b]) : mknull(CAPF_TYPE_FLOAT64);
          else
            st[sp++] = (f & 2) ? mk(((const int64_t *)(base + 8 * n))[a.b], CAPF_TYPE_INT64, 0)
                               : mknull(CAPF_TYPE_INT64);
        }
        break;
      }
      case OP_RAND: {  // uniform in [0, 1): 53 bits of splitmix64(seed, row)
        const uint64_t h = splitmix64((uint64_t)in.i ^ splitmix64((uint64_t)r + 0x9E3779B97F4A7C15ull));
        st[sp++] = mkf((double)(h >> 11) * 0x1.0p-53);
        break;
      }
      case OP_LIST_INDEX: {  // cols[in.i] LIST offsets [n + 1]; cols[(int)in.f] the element column
        Val ix = st[--sp];
        const ColView &c = cols[in.i];
        const int ev = (int)in.f;
        if (ev < 0 || ix.nul || !c.data || (c.valid && !c.valid[r])) {
          st[sp++] = mknull(ev < 0 ? CAPF_TYPE_NULL : cols[ev].type);
          break;
        }
        const int64_t o0 = ((const int64_t *)c.data)[r], len = ((const int64_t *)c.data)[r + 1] - o0;
        int64_t k = ix.b < 0 ? ix.b + len : ix.b;
        st[sp++] = (k < 0 || k >= len) ? mknull(cols[ev].type) : load_col(cols[ev], o0 + k);
        break;
      }
      case OP_TO_BOOLEAN: {  // cols[in.i] = the session's strings parsed as booleans
        Val a = st[--sp];
        if (a.nul || a.t == CAPF_TYPE_BOOL) {
          st[sp++] = a.nul ? mknull(CAPF_TYPE_BOOL) : a;
        } else {
          const uint8_t b = ((const uint8_t *)cols[in.i].data)[a.b];
          st[sp++] = b == 2 ? mknull(CAPF_TYPE_BOOL) : mkb(b == 1);
        }
        break;
      }
      default: st[sp++] = mknull(CAPF_TYPE_NULL); break;
    }
  }
  return st[0];
}

__global__ void k_eval(const Instr *code, int ncode, const ColView *cols, int ncols, int64_t n,
                       void *out, uint8_t *out_valid, int32_t out_type, uint8_t *pred) {
  __shared__ Instr s_code[MAX_LDS_CODE];
  __shared__ ColView s_cols[32];
  const bool lds_code = ncode <= MAX_LDS_CODE;
  if (lds_code)
    for (int i = threadIdx.x; i < ncode; i += blockDim.x) s_code[i] = code[i];
  const bool lds_cols = ncols <= 32;
  if (lds_cols)
    for (int i = threadIdx.x; i < ncols; i += blockDim.x) s_cols[i] = cols[i];
  __syncthreads();
  const Instr *cp = lds_code ? s_code : code;
  const ColView *cv = lds_cols ? s_cols : cols;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    Val v = run_program(cp, ncode, cv, r);
    if (pred) {
      pred[r] = (!v.nul && v.b != 0) ? 1 : 0;
      continue;
    }
    if (out_valid) out_valid[r] = v.nul ? 0 : 1;
    if (out_type == CAPF_TYPE_NULL) continue;
    if (out_type == CAPF_TYPE_BOOL) {
      ((uint8_t *)out)[r] = (!v.nul && v.b != 0) ? 1 : 0;
    } else if (out_type == CAPF_TYPE_FLOAT64) {
      ((double *)out)[r] = v.nul ? 0.0 : vf(v);
    } else {
      ((int64_t *)out)[r] = v.nul ? 0 : v.b;
    }
  }
}

struct DeviceProgram {
  BufPtr code, cols;
  int ncode, ncols;
  // session tables the views point into, held until the launches that read
  // them are enqueued (a code map grown meanwhile returns its old table to the
  // stream-ordered cache only after these)
  std::vector<BufPtr> keep;
};

static DeviceProgram upload_program(Session *s, const Program &p,
                                    const std::vector<std::string> &names, const Data &d) {
  DeviceProgram dp;
  std::vector<ColView> views;
  std::vector<char> scalar_use(p.names.size(), 0);  // read by OP_COL (not only by OP_LIST_SIZE)
  for (auto &in : p.code)
    if (in.op == OP_COL && in.i >= 0 && (size_t)in.i < p.names.size()) scalar_use[(size_t)in.i] = 1;
  for (size_t j = 0; j < p.names.size(); ++j) {
    const std::string &nm = p.names[j];
    if (is_literal_set_name(nm)) {  // sorted set values, count in `base`
      const long id = atol(nm.c_str() + 5);
      std::lock_guard<std::mutex> g(s->user_mu);
      if (id < 0 || (size_t)id >= s->literal_sets.size()) illegal("unknown literal set '" + nm.substr(1) + "'");
      const auto &ls = s->literal_sets[(size_t)id];
      views.push_back(ColView{ls.first->p, nullptr, (int32_t)Type::Int64, ENC_PLAIN, ls.second});
      dp.keep.push_back(ls.first);
      continue;
    }
    if (is_value_map_name(nm)) {  // [keys][keys2][codes], n in `base`, pairs in `enc`
      const long id = atol(nm.c_str() + 6);
      std::lock_guard<std::mutex> g(s->user_mu);
      if (id < 0 || (size_t)id >= s->value_maps.size()) illegal("unknown value map '" + nm.substr(1) + "'");
      const auto &vm = s->value_maps[(size_t)id];
      views.push_back(ColView{vm.buf->p, nullptr, (int32_t)Type::Int64, vm.pairs ? 1 : 0, vm.n});
      dp.keep.push_back(vm.buf);
      continue;
    }
    if (is_code_map_name(nm)) {  // code → code table, its length in `base`
      const long id = atol(nm.c_str() + 5);
      std::lock_guard<std::mutex> g(s->user_mu);
      if (id < 0 || (size_t)id >= s->code_maps.size()) illegal("unknown code map '" + nm.substr(1) + "'");
      const auto &cm = s->code_maps[(size_t)id];
      views.push_back(ColView{cm.first->p, nullptr, (int32_t)Type::Int64, ENC_PLAIN, cm.second});
      dp.keep.push_back(cm.first);
      continue;
    }
    int idx = -1;
    for (size_t k = 0; k < names.size(); ++k)
      if (names[k] == nm) idx = (int)k;
    if (idx < 0) illegal("expression references unknown column '" + nm + "'");
    const ColPtr &c = d.cols[idx];
    if (c->type == Type::List && !scalar_use[j]) {  // size(list): the offsets [n + 1]
      force(c);
      if (c->is_const) illegal("internal: constant LIST column");
      ColView v{c->data ? c->data->p : nullptr, c->valid ? (const uint8_t *)c->valid->p : nullptr,
                (int32_t)Type::List, ENC_PLAIN, 0};
      views.push_back(v);
    } else {
      views.push_back(view_of(c));
    }
  }
  std::vector<Instr> code = p.code;
  for (auto &in : code)
    if (in.op == OP_STR_LEN) {  // the session's string lengths as one more column view
      size_t nstr = 0;
      const int64_t *len = string_length_table(s, &nstr);
      in.i = (int64_t)views.size();
      views.push_back(ColView{len, nullptr, (int32_t)Type::Int64, ENC_PLAIN, 0});
      for (auto &x : code)
        if (x.op == OP_STR_LEN) x.i = in.i;
      break;
    }
  for (auto &in : code)
    if (in.op == OP_STR_RANK) {  // the session's string sort ranks as one more column view
      size_t nstr = 0;
      const int64_t *rk = string_rank_table(s, &nstr);
      in.i = (int64_t)views.size();
      views.push_back(ColView{rk, nullptr, (int32_t)Type::Int64, ENC_PLAIN, 0});
      dp.keep.push_back(s->d_str_rank);
      for (auto &x : code)
        if (x.op == OP_STR_RANK) x.i = in.i;
      break;
    }
  for (auto &in : code)
    if (in.op == OP_STR_TO_NUM) {  // the session's strings as numbers, one more view
      size_t nstr = 0;
      const void *tn = string_num_table(s, &nstr);
      const int64_t vi = (int64_t)views.size();
      views.push_back(ColView{tn, nullptr, (int32_t)Type::Float64, ENC_PLAIN, (int64_t)std::max<size_t>(nstr, 1)});
      for (auto &x : code)
        if (x.op == OP_STR_TO_NUM) {
          x.f = (double)x.i;  // 1 DOUBLE, 0 INTEGER
          x.i = vi;
        }
      break;
    }
  for (auto &in : code)
    if (in.op == OP_LIST_INDEX) {  // the element column of the list as one more view (index in f)
      int idx = -1;
      for (size_t k = 0; k < names.size(); ++k)
        if (names[k] == p.names[(size_t)in.i]) idx = (int)k;
      if (idx < 0) illegal("expression references unknown column '" + p.names[(size_t)in.i] + "'");
      const ColPtr &c = d.cols[idx];
      if (c->type != Type::List || !c->child) {
        in.f = -1.0;  // a NULL-typed column: every row NULL
        continue;
      }
      force(c->child);
      in.f = (double)views.size();
      views.push_back(view_of(c->child));
    }
  for (auto &in : code)
    if (in.op == OP_TO_BOOLEAN) {  // the session's strings as booleans, one more view
      size_t nstr = 0;
      const uint8_t *tb = string_bool_table(s, &nstr);
      in.i = (int64_t)views.size();
      views.push_back(ColView{tb, nullptr, (int32_t)Type::Bool, ENC_PLAIN, 0});
      for (auto &x : code)
        if (x.op == OP_TO_BOOLEAN) x.i = in.i;
      break;
    }
  dp.ncode = (int)code.size();
  dp.ncols = (int)views.size();
  // stack depth check (host) — the device stack is fixed size
  int depth = 0, maxd = 0;
  for (auto &in : code) {
    switch (in.op) {
      case OP_COL: case OP_LIT_INT: case OP_LIT_FLOAT: case OP_LIT_BOOL: case OP_LIT_STRING:
      case OP_LIT_NULL: case OP_LIST_SIZE: case OP_RAND: depth++; break;
      case OP_AND: case OP_OR: case OP_COALESCE: depth -= (int)in.i - 1; break;
      case OP_NOT: case OP_IS_NULL: case OP_IS_NOT_NULL: case OP_NEG: case OP_TO_FLOAT:
      case OP_TO_INTEGER: case OP_STR_LEN: case OP_TO_BOOLEAN: case OP_IN_SET: case OP_STR_MAP:
      case OP_STR_TO_NUM: case OP_LIST_INDEX: case OP_STR_RANK: break;
      case OP_IF: depth -= 2; break;
      case OP_VALUE_MAP: depth -= in.f != 0.0 ? 1 : 0; break;
      default:
        if (!is_math1(in.op)) depth -= 1;  // binary operators; unary math keeps the depth
        break;
    }
    maxd = std::max(maxd, depth);
  }
  if (maxd > MAX_STACK) not_impl("expression too deep for the GPU interpreter");
  dp.code = s->alloc(sizeof(Instr) * code.size());
  HIP_CHECK(hipMemcpyAsync(dp.code->p, code.data(), sizeof(Instr) * code.size(),
                           hipMemcpyHostToDevice, s->stream));
  dp.cols = s->alloc(sizeof(ColView) * std::max<size_t>(views.size(), 1));
  if (!views.empty())
    HIP_CHECK(hipMemcpyAsync(dp.cols->p, views.data(), sizeof(ColView) * views.size(),
                             hipMemcpyHostToDevice, s->stream));
  // pageable host sources: make sure the copies have consumed them
  s->sync();
  return dp;
}

ColPtr eval_program(Session *s, const Program &p, const std::vector<std::string> &names,
                    const Data &d, Type out_type) {
  int64_t n = d.nrows;
  // a bare column reference of the same type (a projection `x AS y`): the
  // column is shared, not copied (columns are immutable)
  if (p.code.size() == 1 && p.code[0].op == OP_COL && p.code[0].i >= 0 &&
      (size_t)p.code[0].i < p.names.size()) {
    const auto it = std::find(names.begin(), names.end(), p.names[(size_t)p.code[0].i]);
    if (it != names.end()) {
      const ColPtr &c = d.cols[(size_t)(it - names.begin())];
      if (c->type == out_type) return c;
    }
  }
  if (p.code.size() == 1) {  // a literal of the column's type: every row holds it
    const Instr &in = p.code[0];
    const bool lit = (in.op == OP_LIT_BOOL && out_type == Type::Bool) ||
                     (in.op == OP_LIT_INT && out_type == Type::Int64) ||
                     (in.op == OP_LIT_FLOAT && out_type == Type::Float64) ||
                     (in.op == OP_LIT_STRING && out_type == Type::String);
    if (lit) {
      Column proto;
      proto.type = out_type;
      proto.const_bits = in.op == OP_LIT_BOOL ? (uint64_t)(in.i != 0)
                         : in.op == OP_LIT_FLOAT ? (uint64_t)__builtin_bit_cast(uint64_t, in.f)
                                                 : (uint64_t)in.i;
      return const_column(s, proto, n);
    }
  }
  ColPtr o = make_column(s, out_type, n, true);
  if (n == 0) return o;
  DeviceProgram dp = upload_program(s, p, names, d);
  hipLaunchKernelGGL(k_eval, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                     (const Instr *)dp.code->p, dp.ncode, (const ColView *)dp.cols->p, dp.ncols, n,
                     o->data ? o->data->p : nullptr, (uint8_t *)o->valid->p, (int32_t)out_type,
                     (uint8_t *)nullptr);
  KERNEL_CHECK();
  return o;
}

// ------------------------------------------------ conjunctive filter fast path
// A WHERE that is a conjunction of comparisons — the relational planner's
// uniqueness filters NOT(r_i = r_j) (RelationalPlanner / VarLengthExpandPlanner
// isomorphism), key checks, `x < 5` — runs without the stack interpreter (whose
// dynamically indexed Val stack lives in scratch): each term is [NOT] (a op b),
// a a column, b a column or an integer literal.  A row passes iff every term is
// TRUE (a NULL operand makes the term NULL: the row is dropped, as the 3-valued
// AND under WHERE).  An operand still held as a lazy gather (a join output's
// column) is read through its index (src[idx[r]], idx −1 = NULL row) instead of
// being materialised first.
// 4 consecutive rows per thread: each term's index and value loads for the 4
// rows are independent (in flight together), the flags go out as one word.
__device__ inline void ft_load4(const FtOperand &o, int64_t r0, int64_t val[4], bool ok[4]) {
  if (o.is_lit) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      val[k] = o.lit;
      ok[k] = true;
    }
    return;
  }
  int64_t row[4];
  if (o.idx) {
    if (o.iw == 4) idx_quad((const int32_t *)o.idx, r0 / 4, row);
    else idx_quad((const int64_t *)o.idx, r0 / 4, row);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) row[k] = r0 + k;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t rr = row[k] < 0 ? 0 : row[k];
    ok[k] = row[k] >= 0 && !(o.v.valid && !o.v.valid[rr]);
    val[k] = o.v.type == CAPF_TYPE_BOOL ? (((const uint8_t *)o.v.data)[rr] ? 1 : 0) : ld_int(o.v, rr);
  }
}

__global__ __launch_bounds__(256) void k_filter_terms4(FtProgram fp, int64_t n4, uint32_t *flags4) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    bool pass[4] = {true, true, true, true};
    for (int k = 0; k < fp.nt; ++k) {
      const FtTerm &t = fp.t[k];
      int64_t x[4], y[4];
      bool oa[4], ob[4];
      ft_load4(t.a, 4 * q, x, oa);
      ft_load4(t.b, 4 * q, y, ob);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bool res = t.op == OP_EQ   ? x[e] == y[e]
                   : t.op == OP_NEQ ? x[e] != y[e]
                   : t.op == OP_LT  ? x[e] < y[e]
                   : t.op == OP_LE  ? x[e] <= y[e]
                   : t.op == OP_GT  ? x[e] > y[e]
                                    : x[e] >= y[e];
        if (t.neg) res = !res;
        pass[e] = pass[e] && oa[e] && ob[e] && res;
      }
    }
    flags4[q] = (pass[0] ? 1u : 0u) | (pass[1] ? 1u : 0u) << 8 | (pass[2] ? 1u : 0u) << 16 |
                (pass[3] ? 1u : 0u) << 24;
  }
}

__global__ __launch_bounds__(256) void k_filter_terms(FtProgram fp, int64_t r_start, int64_t n, uint8_t *flags) {
  for (int64_t r = r_start + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    bool pass = true;
    for (int k = 0; k < fp.nt; ++k) {
      const FtTerm &t = fp.t[k];
      int64_t x = 0, y = 0;
      const bool oa = ft_load(t.a, r, x), ob = ft_load(t.b, r, y);
      const bool ok = oa && ob;
      bool res = t.op == OP_EQ   ? x == y
                 : t.op == OP_NEQ ? x != y
                 : t.op == OP_LT  ? x < y
                 : t.op == OP_LE  ? x <= y
                 : t.op == OP_GT  ? x > y
                                  : x >= y;
      if (t.neg) res = !res;
      pass = pass && ok && res;
    }
    flags[r] = pass ? 1 : 0;
  }
}

static bool ft_operand(const Instr &in, const std::vector<std::string> &pnames,
                       const std::vector<std::string> &names, const Data &d, FtOperand &o, Type &t) {
  o = FtOperand{};
  if (in.op == OP_LIT_INT) {
    o.is_lit = 1;
    o.lit = in.i;
    t = Type::Int64;
    return true;
  }
  if (in.op != OP_COL || in.i < 0 || (size_t)in.i >= pnames.size()) return false;
  int idx = -1;
  for (size_t k = 0; k < names.size(); ++k)
    if (names[k] == pnames[(size_t)in.i]) idx = (int)k;
  if (idx < 0) return false;
  const ColPtr &c = d.cols[(size_t)idx];
  t = c->type;
  if (t != Type::Int64 && t != Type::String && t != Type::Bool) return false;
  std::shared_ptr<LazyGather> lz;
  {
    std::lock_guard<std::mutex> g(c->mu);
    lz = c->lazy;
  }
  if (lz && !lz->src->is_const && !lz->src->lazy) {
    o.v = view_of(lz->src);
    o.idx = lz->idx->p;
    o.iw = lz->iw;
  } else {
    if (c->is_const) return false;  // (a fill: the interpreter handles it)
    o.v = view_of(c);
  }
  return o.v.data != nullptr;
}

// Postfix program → terms, or false (the interpreter runs it).
bool ft_compile(const Program &p, const std::vector<std::string> &names, const Data &d,
                       FtProgram &fp) {
  fp.nt = 0;
  const auto &c = p.code;
  size_t end = c.size();
  int want = 1;
  if (end > 0 && c[end - 1].op == OP_AND) {
    want = (int)c[end - 1].i;
    end -= 1;
  }
  if (want < 1 || want > FT_MAX) return false;
  size_t pc = 0;
  for (int k = 0; k < want; ++k) {
    if (pc + 3 > end) return false;
    FtTerm &t = fp.t[fp.nt++];
    Type ta, tb;
    if (!ft_operand(c[pc], p.names, names, d, t.a, ta) || !ft_operand(c[pc + 1], p.names, names, d, t.b, tb))
      return false;
    const int32_t op = c[pc + 2].op;
    if (op < OP_EQ || op > OP_GE || !(op == OP_EQ || op == OP_NEQ || op == OP_LT || op == OP_LE ||
                                      op == OP_GT || op == OP_GE))
      return false;
    if (ta != tb) return false;  // mixed types: the interpreter's rules
    if (ta != Type::Int64 && op != OP_EQ && op != OP_NEQ) return false;
    t.op = op;
    pc += 3;
    t.neg = 0;
    if (pc < end && c[pc].op == OP_NOT) {
      t.neg = 1;
      pc += 1;
    }
  }
  return pc == end;
}

// Per-row pass flags of a WHERE program (n > 0).
static BufPtr filter_flags(Session *s, const Program &p, const std::vector<std::string> &names,
                           const Data &d) {
  const int64_t n = d.nrows;
  BufPtr flags = s->alloc(n);
  const char *ft_env = getenv("CAPF_FILTER_TERMS");  // 0 (tuning/tests): always the interpreter
  FtProgram fp{};
  if (!(ft_env && atoi(ft_env) == 0) && ft_compile(p, names, d, fp)) {
    KernelTimer kt(s, "filter_terms", (double)n);
    const int64_t n4 = n / 4;  // (device buffers are hipMalloc blocks: the int64 index pairs load as 16 B)
    if (n4 > 0) {
      hipLaunchKernelGGL(k_filter_terms4, dim3(grid_for(n4, 256, 8192)), dim3(256), 0, s->stream, fp, n4,
                         (uint32_t *)flags->p);
      KERNEL_CHECK();
    }
    if (4 * n4 < n) {
      hipLaunchKernelGGL(k_filter_terms, dim3(1), dim3(64), 0, s->stream, fp, 4 * n4, n, (uint8_t *)flags->p);
      KERNEL_CHECK();
    }
    return flags;
  }
  DeviceProgram dp = upload_program(s, p, names, d);
  {
    KernelTimer kt(s, "filter_eval", (double)n);
    hipLaunchKernelGGL(k_eval, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                       (const Instr *)dp.code->p, dp.ncode, (const ColView *)dp.cols->p, dp.ncols,
                       n, (void *)nullptr, (uint8_t *)nullptr, 0, (uint8_t *)flags->p);
    KERNEL_CHECK();
  }
  return flags;
}

BufPtr eval_filter(Session *s, const Program &p, const std::vector<std::string> &names,
                   const Data &d, int64_t *out_count) {
  int64_t n = d.nrows;
  if (n == 0) {
    *out_count = 0;
    return s->alloc(0);
  }
  BufPtr flags = filter_flags(s, p, names, d);
  return compact_flags(s, (const uint8_t *)flags->p, n, out_count);
}

DataPtr filter_select(Session *s, const Program &p, const std::vector<std::string> &names, const Data &d) {
  const int64_t n = d.nrows;
  auto out = std::make_shared<Data>();
  if (n == 0) {
    *out = d;
    return out;
  }
  BufPtr flags = filter_flags(s, p, names, d);
  // the distinct lazy-gather indexes of the columns (their composed indexes are
  // written by the selection itself) and whether a plain column needs the
  // selection index
  std::vector<BufPtr> lazy_idx;
  std::vector<int> lazy_w;
  bool plain = false;
  for (auto &c : d.cols) {
    std::shared_ptr<LazyGather> lz;
    {
      std::lock_guard<std::mutex> g(c->mu);
      lz = c->lazy;
    }
    // a lazy column over a constant is a fill in gather_lazy only when no row can
    // be NULL; a nullable one (an outer join's constant side) composes its index
    if (lz && !(lz->src->is_const && !lz->nullable)) {
      bool seen = false;
      for (auto &b : lazy_idx) seen |= b.get() == lz->idx.get();
      if (!seen) {
        lazy_idx.push_back(lz->idx);
        lazy_w.push_back(lz->iw);
      }
    } else if (!lz) {
      plain = true;
    }
  }
  const char *fs_env = getenv("CAPF_FILTER_SELECT");  // 0 (tuning/tests): selection index + composes
  const int ns = (int)lazy_idx.size() + 1;
  if ((fs_env && atoi(fs_env) == 0) || !lazy_enabled() || lazy_idx.empty() || ns > SEL_MAX) {
    int64_t m = 0;
    BufPtr idx = compact_flags(s, (const uint8_t *)flags->p, n, &m);
    out->nrows = m;
    IdxCache cache;
    for (auto &c : d.cols) out->cols.push_back(gather_lazy(s, c, idx, m, false, &cache));
    return out;
  }
  const int64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  BufPtr counts = s->alloc(8 * tiles), offs = s->alloc(8 * tiles);
  hipLaunchKernelGGL(k_count_flags, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, s->stream,
                     (const uint8_t *)flags->p, n, (int64_t *)counts->p);
  KERNEL_CHECK();
  const int64_t m = exclusive_scan_i64(s, (const int64_t *)counts->p, (int64_t *)offs->p, tiles);
  out->nrows = m;
  // the selection index itself (source 0) is written only when a plain column
  // reads it; otherwise it is a key of the compose cache and never read
  BufPtr sel = s->alloc(plain ? 8 * std::max<int64_t>(m, 1) : 8);
  SelSrcs ss{};
  ss.ns = 0;
  if (plain) {
    ss.src[ss.ns] = nullptr;
    ss.w[ss.ns] = 8;
    ss.out[ss.ns++] = sel->p;
  }
  IdxCache cache;
  for (size_t k = 0; k < lazy_idx.size(); ++k) {
    const BufPtr &b = lazy_idx[k];
    BufPtr o = s->alloc((int64_t)lazy_w[k] * std::max<int64_t>(m, 1));
    ss.src[ss.ns] = b->p;
    ss.w[ss.ns] = lazy_w[k];
    ss.out[ss.ns++] = o->p;
    cache.entries.emplace_back(std::make_pair((const void *)b.get(), (const void *)sel.get()), o);
  }
  if (m > 0) {
    KernelTimer kt(s, "filter_select", 9.0 * (double)n);
    hipLaunchKernelGGL(k_select_multi, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, s->stream,
                       (const uint8_t *)flags->p, n, (const int64_t *)offs->p, ss);
    KERNEL_CHECK();
  }
  for (auto &c : d.cols) out->cols.push_back(gather_lazy(s, c, sel, m, false, &cache));
  return out;
}

}  // namespace capf
