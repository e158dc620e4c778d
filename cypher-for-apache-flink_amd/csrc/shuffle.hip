// shuffle.hip — hash routing of table rows to ranks: the exchange step of
// the distributed Table layer (dist_table.py, SURVEY §8(e): "each hop's
// frontier rows are shuffled by join key"; GROUP BY / DISTINCT rows by
// h(key)).  Flink does the same inside its DataSet join / groupBy: a hash
// repartition of both inputs before the local hash join / group-reduce
// (FlinkTable.scala:171-187, 123-150 lower onto those operators).
//
//   k_route       dest(row) = owner of h(key values): splitmix64 of each key
//                 (decoded int64 / canonical fp64 bits / bool byte / NULL
//                 sentinel), combined; owner = (h >> 32) · parts >> 32.  Equal
//                 key tuples get equal owners (collisions only co-locate more
//                 rows), all NULLs of a key go to one owner, −0.0 routes like
//                 0.0 and every NaN alike.
//   radix sort    (dest, row) pairs, rocprim, only the ⌈log2 parts⌉ dest bits:
//                 a stable counting sort of the rows by owner
//   k_bounds      first row of every owner in the sorted keys (binary search)
//
// The caller gathers every column by the permutation (gather_column), so the
// rows for rank p are the contiguous slice [off[p], off[p+1]) of each column:
// one all-to-all per column moves them (RCCL, dist_table.py).
// Bytes per row: keys read once, 8 B dest + 8 B row written and sorted.
#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr int ROUTE_MAXK = 8;

struct RouteKeys {
  ColView k[ROUTE_MAXK];
  int nk;
};

__device__ inline uint64_t route_mix(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

// 64-bit routing image of row i of key column c (type-specific canonical form).
__device__ inline uint64_t route_bits(const ColView &c, int64_t i) {
  if (c.valid && !c.valid[i]) return 0x6E756C6C6E756C6Cull;  // NULL sentinel
  switch (c.type) {
    case CAPF_TYPE_BOOL:
      return ((const uint8_t *)c.data)[i] ? 1ull : 0ull;
    case CAPF_TYPE_FLOAT64: {
      double v = ((const double *)c.data)[i];
      if (v == 0.0) v = 0.0;                           // −0.0 → 0.0
      if (v != v) return 0x7FF8000000000000ull;        // one NaN
      return (uint64_t)__double_as_longlong(v);
    }
    case CAPF_TYPE_NULL:
      return 0x6E756C6C6E756C6Cull;
    default:  // INT64 / STRING codes, any encoding
      return (uint64_t)ld_int(c, i);
  }
}

__global__ void k_route(RouteKeys rk, int64_t n, uint32_t parts, uint32_t *dest, int64_t *row) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x243F6A8885A308D3ull;
    for (int j = 0; j < rk.nk; ++j) h = route_mix(h ^ route_bits(rk.k[j], i)) + 0x9E3779B97F4A7C15ull;
    dest[i] = (uint32_t)(((h >> 32) * (uint64_t)parts) >> 32);
    row[i] = i;
  }
}

// off[p] = first index of the sorted dest array holding a value ≥ p (p ≤ parts).
__global__ void k_bounds(const uint32_t *sorted, int64_t n, int parts, int64_t *off) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > parts) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (sorted[mid] < (uint32_t)p) lo = mid + 1;
    else hi = mid;
  }
  off[p] = lo;
}

template <class F>
static void route_rocprim(Session *s, F &&f) {
  size_t tmp = 0;
  HIP_CHECK(f(nullptr, tmp));
  BufPtr t = s->alloc(std::max<size_t>(tmp, 16));
  HIP_CHECK(f(t->p, tmp));
}

// Permutation (int64 row indexes, rows grouped by owner in owner order, stable
// within an owner) and per-owner counts of the rows of `keys` over `parts`.
BufPtr route_permutation(Session *s, const std::vector<ColView> &keys, int64_t n, int parts,
                         std::vector<int64_t> &counts) {
  if (keys.empty() || keys.size() > (size_t)ROUTE_MAXK) illegal("1..8 routing keys");
  if (parts <= 0 || parts > (1 << 20)) illegal("parts out of range");
  counts.assign(parts, 0);
  const int64_t n1 = std::max<int64_t>(n, 1);
  BufPtr perm = s->alloc(8 * n1);
  if (n == 0) return perm;
  RouteKeys rk;
  rk.nk = (int)keys.size();
  for (int j = 0; j < rk.nk; ++j) rk.k[j] = keys[j];
  BufPtr dest = s->alloc(4 * n1), dsort = s->alloc(4 * n1), rows = s->alloc(8 * n1);
  {
    KernelTimer kt(s, "route", (8.0 * rk.nk + 12.0) * n);
    hipLaunchKernelGGL(k_route, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, rk, n, (uint32_t)parts,
                       (uint32_t *)dest->p, (int64_t *)rows->p);
    KERNEL_CHECK();
  }
  int bits = 0;
  while ((1 << bits) < parts) ++bits;
  if (bits == 0) {
    HIP_CHECK(hipMemcpyAsync(perm->p, rows->p, 8 * n, hipMemcpyDeviceToDevice, s->stream));
    counts[0] = n;
    return perm;
  }
  {
    KernelTimer kt(s, "route_sort", 24.0 * n);
    route_rocprim(s, [&](void *t, size_t &sz) {
      return rocprim::radix_sort_pairs(t, sz, (const uint32_t *)dest->p, (uint32_t *)dsort->p,
                                       (const int64_t *)rows->p, (int64_t *)perm->p, (size_t)n, 0, bits,
                                       s->stream);
    });
  }
  BufPtr off = s->alloc(8 * (parts + 1));
  hipLaunchKernelGGL(k_bounds, dim3((parts + 256) / 256), dim3(256), 0, s->stream, (const uint32_t *)dsort->p,
                     n, parts, (int64_t *)off->p);
  KERNEL_CHECK();
  std::vector<int64_t> h(parts + 1);
  HIP_CHECK(hipMemcpyAsync(h.data(), off->p, 8 * (parts + 1), hipMemcpyDeviceToHost, s->stream));
  s->sync();
  for (int p = 0; p < parts; ++p) counts[p] = h[p + 1] - h[p];
  return perm;
}

// ------------------------------------------------------------ row packing
// The exchange's wire format (dist_table.py GpuExchange.send): each row is W
// bytes, row-major — per column `width` bytes of (value − base) little-endian
// (width 3 / 4 for INTEGER / STRING-code columns whose range over ALL ranks
// fits 24 / 32 bits, the FOR24 / FOR32 encodings; 8 otherwise and for floats;
// 1 for BOOL), then one validity byte when the column is nullable on some
// rank.  One all_to_all_single moves the packed rows; the receiver's columns
// keep the narrow encodings (no re-encode).  One thread per row, the row
// assembled in registers and written as whole dwords when W is a multiple of 4.
struct PackCol {
  ColView v;
  int32_t width, off, voff;  // voff < 0: no validity byte
  int64_t base;
};

__device__ inline uint64_t pack_value(const PackCol &c, int64_t r, bool valid) {
  if (!valid || c.v.type == CAPF_TYPE_NULL) return 0;
  if (c.v.type == CAPF_TYPE_BOOL) return ((const uint8_t *)c.v.data)[r] ? 1u : 0u;
  if (c.v.type == CAPF_TYPE_FLOAT64) return ((const uint64_t *)c.v.data)[r];
  return (uint64_t)(ld_int(c.v, r) - c.base);
}

__global__ void k_pack_rows(const PackCol *cols, int nc, int W, int64_t n, uint8_t *out) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    uint8_t *row = out + r * W;
    for (int j = 0; j < nc; ++j) {
      const PackCol c = cols[j];
      const bool valid = !c.v.valid || c.v.valid[r];
      const uint64_t x = pack_value(c, r, valid);
      for (int b = 0; b < c.width; ++b) row[c.off + b] = (uint8_t)(x >> (8 * b));
      if (c.voff >= 0) row[c.voff] = valid ? 1 : 0;
    }
  }
}

// One column out of packed rows: width 3 → FOR24 buffer, 4 → FOR32 words,
// 8 → int64 / float64 bits, 1 → bool bytes; validity bytes when voff ≥ 0.
__global__ void k_unpack_col(const uint8_t *rows, int64_t n, int W, int off, int width, int voff,
                             uint8_t *data, uint8_t *valid) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t *row = rows + r * W;
    for (int b = 0; b < width; ++b) data[r * width + b] = row[off + b];
    if (voff >= 0) valid[r] = row[voff];
  }
}

void pack_rows(Session *s, const std::vector<ColPtr> &cols, const int32_t *width, const int64_t *base,
               const int32_t *nullable, int64_t n, int *W_out, void *d_out) {
  std::vector<PackCol> pc(cols.size());
  int W = 0;
  for (size_t j = 0; j < cols.size(); ++j) {
    pc[j].v = view_of(cols[j]);
    pc[j].width = width[j];
    pc[j].off = W;
    pc[j].base = base[j];
    W += width[j];
    pc[j].voff = nullable[j] ? W++ : -1;
  }
  *W_out = W;
  if (!d_out || n == 0 || W == 0) return;
  BufPtr dc = s->alloc(sizeof(PackCol) * std::max<size_t>(pc.size(), 1));
  HIP_CHECK(hipMemcpyAsync(dc->p, pc.data(), sizeof(PackCol) * pc.size(), hipMemcpyHostToDevice, s->stream));
  {
    KernelTimer kt(s, "pack_rows", (double)W * n);
    hipLaunchKernelGGL(k_pack_rows, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, (const PackCol *)dc->p,
                       (int)pc.size(), W, n, (uint8_t *)d_out);
    KERNEL_CHECK();
  }
  s->sync();  // the host copy of the column table is released on return
}

ColPtr unpack_column(Session *s, const void *rows, int64_t n, int W, int off, int width, int voff, int64_t base,
                     Type t) {
  auto c = std::make_shared<Column>();
  c->type = t;
  c->n = n;
  if (t == Type::Null) return c;
  c->enc = width == 3 ? ENC_FOR24 : width == 4 ? ENC_FOR32 : ENC_PLAIN;
  c->base = width == 3 || width == 4 ? base : 0;
  // FOR24 buffers carry 16 zero bytes past 3·n (4-B / 12-B loads at any row)
  const int64_t bytes = (int64_t)width * n + (width == 3 ? 16 : 0);
  c->data = s->alloc(std::max<int64_t>(bytes, 16));
  if (width == 3) HIP_CHECK(hipMemsetAsync((uint8_t *)c->data->p + 3 * n, 0, 16, s->stream));
  if (voff >= 0) c->valid = s->alloc(std::max<int64_t>(n, 1));
  if (n > 0) {
    hipLaunchKernelGGL(k_unpack_col, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, (const uint8_t *)rows, n,
                       W, off, width, voff, (uint8_t *)c->data->p, voff >= 0 ? (uint8_t *)c->valid->p : nullptr);
    KERNEL_CHECK();
  }
  return c;
}

}  // namespace capf
