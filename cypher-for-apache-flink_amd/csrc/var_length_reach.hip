// var_length_reach.hip — fused VarLengthExpand → DISTINCT (a, b) → GROUP BY a
// count(*) (config 5: MATCH (a:Person)-[:KNOWS*1..3]->(b:Person)
//                     WITH DISTINCT a, b WITH a, count(*) AS reach ...).
//
// The relational plan (VarLengthExpandPlanner.scala:82-259: one join per hop,
// isomorphism filter e_i ∉ {e_1..e_{i-1}} (:178-179), target join (:218-229),
// null padding + UNION ALL (:145-170)) materialises every path — ≈1e10 rows
// of 40 B at LDBC SF10 — and DISTINCT / GROUP BY (FlinkTable.scala:123-150,
// 189-196) then reduce them to one count per source.  With lower bound 1 and a
// directed pattern the DISTINCT pairs are exactly the pairs joined by a WALK
// of length 1..u (a walk repeating rel e contains the closed sub-walk between
// the two uses; cutting it keeps e once, so a walk of length ≥ 1 with the same
// endpoints and no repeated rel exists — isomorphism never changes the DISTINCT
// pairs).  So reach(a) = |{b ∈ targets : min walk length a→b ∈ [1, u]}|, the
// classic level-synchronous BFS from a with a itself NOT pre-visited.
//
// Bit-parallel multi-source BFS (MS-BFS), pull form, no atomics:
//   dict   all ids (rel endpoints, sources, targets) → sorted distinct keys
//          (rocprim radix sort + run-length encode); dense index = rank
//   CSR    in-edges by target (count, scan, fill)
//   state  visited / frontier / next: D nodes × K words of 64 source bits,
//          node-major (a node's K words are contiguous) in HBM
//   push1  level 1: rels of the batch's sources set their bits (M atomics)
//   level  levels 2..u, thread per (node y, word k): next = OR_{x ∈ in(y)} frontier[x][k]
//          & ~visited[y][k]; visited |= next  — K consecutive threads share
//          y's CSR row and read x's frontier words as one coalesced run
//   count  block per word k: wave ballots of (visited bit j ∧ target(y)),
//          popcount → reach of source 64k + j
// Sources are processed in batches of 64·K so the three state arrays stay
// within a fixed HBM budget.  Bytes per level ≈ 8·K·(M + 3·D).
#include <algorithm>
#include <cstring>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

template <class F>
static void vr_rocprim(Session *s, F &&f) {
  size_t tmp = 0;
  HIP_CHECK(f(nullptr, tmp));
  BufPtr t = s->alloc(std::max<size_t>(tmp, 16));
  HIP_CHECK(f(t->p, tmp));
}

// order-preserving uint64 key of an int64 id
__device__ inline uint64_t vr_key(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }

__global__ void k_vr_keys(ColView c, int64_t n, uint64_t *out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = vr_key(ld_int(c, i));
}

// dense index of each id: lower_bound in the sorted distinct keys
__global__ void k_vr_map(ColView c, int64_t n, const uint64_t *dict, uint32_t nd, uint32_t *out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = vr_key(ld_int(c, i));
    uint32_t lo = 0, hi = nd;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (dict[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    out[i] = lo;
  }
}

__global__ void k_vr_flag(const uint32_t *idx, int64_t n, uint8_t *flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    flag[idx[i]] = 1;
}

__global__ void k_vr_indeg(const uint32_t *dst, int64_t m, uint32_t *deg) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&deg[dst[i]], 1u);
}

__global__ void k_vr_fill(const uint32_t *src, const uint32_t *dst, int64_t m, uint32_t *cursor,
                          uint32_t *cols) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    cols[atomicAdd(&cursor[dst[i]], 1u)] = src[i];
}

// Level 1 by push (the frontier is only the batch's sources): every rel
// (x → y) whose x is source j of the batch sets bit j of y in visited and in
// the level-2 frontier — M atomics instead of a pull over M·K words.
__global__ void k_vr_srcpos(const int64_t *src_nodes, int64_t ns, int32_t *srcpos) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ns;
       j += (int64_t)gridDim.x * blockDim.x)
    srcpos[src_nodes[j]] = (int32_t)j;
}

__global__ void k_vr_push1(const uint32_t *si, const uint32_t *di, int64_t m, const int32_t *srcpos,
                           int64_t s0, int64_t nb, int64_t K, unsigned long long *visited,
                           unsigned long long *frontier) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = (int64_t)srcpos[si[i]] - s0;
    if (j < 0 || j >= nb) continue;
    const int64_t w = (int64_t)di[i] * K + (j >> 6);
    const unsigned long long bit = 1ull << (j & 63);
    atomicOr(&visited[w], bit);
    atomicOr(&frontier[w], bit);
  }
}

constexpr int VR_ILP = 16;

// rows by decreasing in-degree: the hub rows (long dependent load chains)
// start first and overlap with the bulk instead of forming the tail
__global__ void k_vr_degkey(const uint32_t *rowptr, uint32_t D, uint64_t *key) {
  for (uint32_t y = blockIdx.x * blockDim.x + threadIdx.x; y < D; y += gridDim.x * blockDim.x)
    key[y] = ((uint64_t)(0xFFFFFFFFu - (rowptr[y + 1] - rowptr[y])) << 32) | y;
}

__global__ __launch_bounds__(256) void k_vr_level(const uint32_t *rowptr, const uint32_t *cols,
                                                  const uint64_t *order,
                                                  const unsigned long long *frontier,
                                                  unsigned long long *next,
                                                  unsigned long long *visited, int64_t D,
                                                  int64_t K, int last) {
  const int64_t total = D * K;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / K, k = t - r * K;
    const int64_t y = (int64_t)(uint32_t)order[r];
    const int64_t ty = y * K + k;
    unsigned long long acc = 0;
    const uint32_t e1 = rowptr[y + 1];
    uint32_t e = rowptr[y];
    // VR_ILP independent (col, frontier) load pairs in flight per lane: a
    // row is a chain of dependent loads otherwise, and hub rows (in-degree
    // 10^4+) would run at one HBM latency per rel
    for (; e + VR_ILP <= e1; e += VR_ILP) {
      uint32_t c[VR_ILP];
#pragma unroll
      for (int i = 0; i < VR_ILP; ++i) c[i] = cols[e + i];
      unsigned long long f[VR_ILP];
#pragma unroll
      for (int i = 0; i < VR_ILP; ++i) f[i] = frontier[(int64_t)c[i] * K + k];
#pragma unroll
      for (int i = 0; i < VR_ILP; ++i) acc |= f[i];
    }
    for (; e < e1; ++e) acc |= frontier[(int64_t)cols[e] * K + k];
    const unsigned long long v = visited[ty];
    const unsigned long long nv = acc & ~v;
    if (!last) next[ty] = nv;
    if (nv) visited[ty] = v | nv;
  }
}

// reach[s0 + 64k + j] = #{y : target(y) ∧ bit j of visited[y][k]}
__global__ __launch_bounds__(256) void k_vr_count(const unsigned long long *visited,
                                                  const uint8_t *target, int64_t D, int64_t K,
                                                  int64_t s0, int64_t ns, int64_t *reach) {
  __shared__ uint32_t part[4][WAVE];
  const int64_t k = blockIdx.x;
  const int lane = lane_id(), w = threadIdx.x / WAVE;
  uint32_t cnt = 0;
  for (int64_t y0 = (int64_t)w * WAVE; y0 < D; y0 += 4 * WAVE) {
    const int64_t y = y0 + lane;
    const unsigned long long v = (y < D && target[y]) ? visited[y * K + k] : 0ull;
#pragma unroll 8
    for (int j = 0; j < WAVE; ++j) {
      const uint32_t c = (uint32_t)__popcll(__ballot((v >> j) & 1ull));
      cnt += lane == j ? c : 0u;
    }
  }
  part[w][lane] = cnt;
  __syncthreads();
  if (threadIdx.x < WAVE) {
    const int64_t j = k * WAVE + threadIdx.x;
    if (j < ns)
      reach[s0 + j] = (int64_t)part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] +
                      part[3][threadIdx.x];
  }
}

// The same counts from coalesced loads (CAPF_VR_COUNT=0 keeps k_vr_count):
// block (kc, cg) = source words [64·kc, 64·kc + 64) × row chunks cg·16 + w
// of VR_CR rows, one per wave; lane = source word, reading visited[y][k] as
// 512-B rows.  Each lane adds its words into a bit-sliced counter (level i
// holds bit i of the 64 per-source counts), the wave then hands out the
// counts (lane j: bit j of every level of lane l's counter) into an LDS
// table, and the block adds that table to reach[] with one coalesced atomic
// pass.  Zero reach[s0, s0 + ns) first.
constexpr int VR_CR = 256;   // rows per wave (< 2^VR_CL)
constexpr int VR_CL = 9;

__global__ __launch_bounds__(1024) void k_vr_count_bs(const unsigned long long *visited,
                                                      const uint8_t *target, int64_t D, int64_t K,
                                                      int64_t s0, int64_t ns, unsigned long long *reach) {
  __shared__ uint32_t tab[WAVE * WAVE];
  for (int i = threadIdx.x; i < WAVE * WAVE; i += 1024) tab[i] = 0;
  __syncthreads();
  const int lane = lane_id(), w = threadIdx.x / WAVE;
  const int64_t kc = blockIdx.x, k = kc * WAVE + lane;
  const int64_t y0 = ((int64_t)blockIdx.y * (1024 / WAVE) + w) * VR_CR, y1 = min(y0 + (int64_t)VR_CR, D);
  unsigned long long c[VR_CL];
#pragma unroll
  for (int i = 0; i < VR_CL; ++i) c[i] = 0ull;
  if (y0 < D) {
    const bool kin = k < K;
#pragma unroll 4
    for (int64_t y = y0; y < y1; ++y) {
      const unsigned long long v = (kin && target[y]) ? visited[y * K + k] : 0ull;
      unsigned long long carry = v;
#pragma unroll
      for (int i = 0; i < VR_CL; ++i) {
        const unsigned long long t = c[i] & carry;
        c[i] ^= carry;
        carry = t;
      }
    }
    for (int l = 0; l < WAVE; ++l) {
      uint32_t cnt = 0;
#pragma unroll
      for (int i = 0; i < VR_CL; ++i) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)c[i], l);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(c[i] >> 32), l);
        const uint32_t word = lane < 32 ? lo : hi;
        cnt += ((word >> (lane & 31)) & 1u) << i;
      }
      if (cnt) atomicAdd(&tab[l * WAVE + lane], cnt);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < WAVE * WAVE; i += 1024) {
    const int64_t src = kc * WAVE * WAVE + i;  // word kc·64 + i/64, bit i%64
    if (tab[i] && src < ns) atomicAdd(&reach[s0 + src], (unsigned long long)tab[i]);
  }
}

__global__ void k_vr_out(const int64_t *rows, int64_t n, const int64_t *src_nodes,
                         const uint64_t *dict, const int64_t *reach, int64_t *a, int64_t *r) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = rows[i];
    a[i] = (int64_t)(dict[src_nodes[j]] ^ 0x8000000000000000ull);
    r[i] = reach[j];
  }
}

// lower bound 0 (the copyElement branch, VarLengthExpandPlanner.scala:180-205):
// every source also pairs with itself — once, so +1 unless a walk of the
// batch already reached the source as a target
__global__ void k_vr_self(const unsigned long long *vis, const uint8_t *tflag, const int64_t *src_nodes,
                          int64_t K, int64_t s0, int64_t nb, int64_t *reach) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = src_nodes[s0 + i];
    const bool hit = tflag[p] && ((vis[p * K + (i >> 6)] >> (i & 63)) & 1ull);
    if (!hit) reach[s0 + i] += 1;
  }
}

__global__ void k_vr_ones(int64_t *r, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    r[i] = 1;
}

__global__ void k_vr_pos(const int64_t *reach, int64_t n, uint8_t *flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = reach[i] > 0;
}

// HBM budget of the three MS-BFS state arrays (sources are batched to fit)
constexpr double VR_STATE_BUDGET = 24e9;

// The reach index of (rels, sources, targets): id dictionary, dense endpoint
// indices, in-CSR by target, the degree order of its rows, source positions
// and target flags.  Everything here is a function of four immutable columns,
// so it is built by the first query and cached on the rel source column (an
// ingest-time adjacency index, like the triangle's oriented CSR); a query with
// other node columns (e.g. a filtered scan) builds its own.
struct VrIndex {
  uint32_t D = 0;
  int64_t ns = 0;
  BufPtr dict, si, di, tflag, src_nodes, rowptr, cols, order, srcpos;
};

static std::shared_ptr<VrIndex> vr_build(Session *s, const ColPtr &rsrc, const ColPtr &rdst, int64_t m,
                                         const ColPtr &sid, int64_t ns_in, const ColPtr &tid, int64_t nt) {
  auto ix = std::make_shared<VrIndex>();
  const int64_t nk = 2 * m + ns_in + nt;
  if (nk >= (int64_t(1) << 32)) not_impl("var-length reach: more than 2^32 ids");
  const unsigned g = grid_for(nk, 256, 256 * 64);
  // 1. dictionary of every id
  BufPtr keys = s->alloc(8 * nk), sorted = s->alloc(8 * nk);
  {
    KernelTimer kt(s, "vr_dict", 24.0 * nk);
    uint64_t *k = (uint64_t *)keys->p;
    hipLaunchKernelGGL(k_vr_keys, dim3(g), dim3(256), 0, s->stream, view_of(rsrc), m, k);
    hipLaunchKernelGGL(k_vr_keys, dim3(g), dim3(256), 0, s->stream, view_of(rdst), m, k + m);
    hipLaunchKernelGGL(k_vr_keys, dim3(g), dim3(256), 0, s->stream, view_of(sid), ns_in, k + 2 * m);
    hipLaunchKernelGGL(k_vr_keys, dim3(g), dim3(256), 0, s->stream, view_of(tid), nt,
                       k + 2 * m + ns_in);
    KERNEL_CHECK();
    vr_rocprim(s, [&](void *t, size_t &n) {
      return rocprim::radix_sort_keys(t, n, (const uint64_t *)keys->p, (uint64_t *)sorted->p,
                                      (size_t)nk, 0, 64, s->stream);
    });
  }
  BufPtr dict = s->alloc(8 * nk), runs = s->alloc(4 * nk), nruns = s->alloc(16);
  vr_rocprim(s, [&](void *t, size_t &n) {
    return rocprim::run_length_encode(t, n, (const uint64_t *)sorted->p, (unsigned int)nk,
                                      (uint64_t *)dict->p, (uint32_t *)runs->p,
                                      (uint32_t *)nruns->p, s->stream);
  });
  uint32_t D = 0;
  HIP_CHECK(hipMemcpyAsync(&D, nruns->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  keys.reset();
  sorted.reset();
  runs.reset();
  const uint64_t *dk = (const uint64_t *)dict->p;
  // 2. dense indices
  BufPtr si = s->alloc(4 * m), di = s->alloc(4 * m), xi = s->alloc(4 * std::max(ns_in, nt));
  BufPtr tflag = s->alloc(D), sflag = s->alloc(D);
  HIP_CHECK(hipMemsetAsync(tflag->p, 0, D, s->stream));
  HIP_CHECK(hipMemsetAsync(sflag->p, 0, D, s->stream));
  hipLaunchKernelGGL(k_vr_map, dim3(g), dim3(256), 0, s->stream, view_of(rsrc), m, dk, D,
                     (uint32_t *)si->p);
  hipLaunchKernelGGL(k_vr_map, dim3(g), dim3(256), 0, s->stream, view_of(rdst), m, dk, D,
                     (uint32_t *)di->p);
  hipLaunchKernelGGL(k_vr_map, dim3(g), dim3(256), 0, s->stream, view_of(tid), nt, dk, D,
                     (uint32_t *)xi->p);
  hipLaunchKernelGGL(k_vr_flag, dim3(g), dim3(256), 0, s->stream, (const uint32_t *)xi->p, nt,
                     (uint8_t *)tflag->p);
  hipLaunchKernelGGL(k_vr_map, dim3(g), dim3(256), 0, s->stream, view_of(sid), ns_in, dk, D,
                     (uint32_t *)xi->p);
  hipLaunchKernelGGL(k_vr_flag, dim3(g), dim3(256), 0, s->stream, (const uint32_t *)xi->p, ns_in,
                     (uint8_t *)sflag->p);
  KERNEL_CHECK();
  // distinct sources in dictionary order (a node scan holds each node once;
  // duplicates would be merged by the DISTINCT anyway)
  int64_t ns = 0;
  BufPtr src_nodes = compact_flags(s, (const uint8_t *)sflag->p, D, &ns);
  // 3. in-CSR by target
  BufPtr deg = s->alloc(4 * ((int64_t)D + 1)), rowptr = s->alloc(4 * ((int64_t)D + 1));
  BufPtr cursor = s->alloc(4 * ((int64_t)D + 1)), cols = s->alloc(4 * m);
  HIP_CHECK(hipMemsetAsync(deg->p, 0, 4 * ((int64_t)D + 1), s->stream));
  {
    KernelTimer kt(s, "vr_csr", 16.0 * m);
    hipLaunchKernelGGL(k_vr_indeg, dim3(g), dim3(256), 0, s->stream, (const uint32_t *)di->p, m,
                       (uint32_t *)deg->p);
    BufPtr tot = s->alloc(16);
    exclusive_scan_u32_async(s, (const uint32_t *)deg->p, (uint32_t *)rowptr->p, (int64_t)D + 1,
                             (uint32_t *)tot->p);
    HIP_CHECK(hipMemcpyAsync(cursor->p, rowptr->p, 4 * ((int64_t)D + 1), hipMemcpyDeviceToDevice,
                             s->stream));
    hipLaunchKernelGGL(k_vr_fill, dim3(g), dim3(256), 0, s->stream, (const uint32_t *)si->p,
                       (const uint32_t *)di->p, m, (uint32_t *)cursor->p, (uint32_t *)cols->p);
    KERNEL_CHECK();
  }
  cursor.reset();
  BufPtr order;
  {
    BufPtr dkey = s->alloc(8 * (int64_t)D);
    order = s->alloc(8 * (int64_t)D);
    hipLaunchKernelGGL(k_vr_degkey, dim3(grid_for(D, 256)), dim3(256), 0, s->stream,
                       (const uint32_t *)rowptr->p, D, (uint64_t *)dkey->p);
    KERNEL_CHECK();
    vr_rocprim(s, [&](void *t, size_t &n) {
      return rocprim::radix_sort_keys(t, n, (const uint64_t *)dkey->p, (uint64_t *)order->p,
                                      (size_t)D, 0, 64, s->stream);
    });
  }
  BufPtr srcpos = s->alloc(4 * (int64_t)D);
  HIP_CHECK(hipMemsetAsync(srcpos->p, 0xFF, 4 * (size_t)D, s->stream));
  hipLaunchKernelGGL(k_vr_srcpos, dim3(grid_for(ns, 256)), dim3(256), 0, s->stream,
                     (const int64_t *)src_nodes->p, ns, (int32_t *)srcpos->p);
  KERNEL_CHECK();
  ix->D = D;
  ix->ns = ns;
  ix->dict = dict;
  ix->si = si;
  ix->di = di;
  ix->tflag = tflag;
  ix->src_nodes = src_nodes;
  ix->rowptr = rowptr;
  ix->cols = cols;
  ix->order = order;
  ix->srcpos = srcpos;
  return ix;
}

struct VrCache {
  std::weak_ptr<Column> rdst, sid, tid;
  int64_t m = 0, ns_in = 0, nt = 0;
  std::shared_ptr<VrIndex> ix;
};

DataPtr var_length_reach_rows(Session *s, const ColPtr &rsrc, const ColPtr &rdst, int64_t m,
                                const ColPtr &sid, int64_t ns_in, const ColPtr &tid, int64_t nt,
                                int upper, bool include_self) {
  auto out = std::make_shared<Data>();
  out->cols = {make_column(s, Type::Int64, 0, false), make_column(s, Type::Int64, 0, false)};
  if (include_self && ns_in > 0 && (m == 0 || nt == 0)) {  // no walks: every (a, a) alone (unique ids: the caller's)
    ColPtr a = decode_column(s, sid), r = make_column(s, Type::Int64, ns_in, false);
    hipLaunchKernelGGL(k_vr_ones, dim3(grid_for(ns_in, 256)), dim3(256), 0, s->stream, (int64_t *)r->data->p,
                       ns_in);
    KERNEL_CHECK();
    out->nrows = ns_in;
    out->cols = {a, r};
    return out;
  }
  if (m == 0 || ns_in == 0 || nt == 0) return out;
  if (m >= (int64_t(1) << 32)) not_impl("var-length reach: more than 2^32 rels");
  std::shared_ptr<VrIndex> ix;
  {
    std::lock_guard<std::mutex> lk(rsrc->mu);
    if (rsrc->vr_index) {
      auto vc = std::static_pointer_cast<VrCache>(rsrc->vr_index);
      if (vc->rdst.lock() == rdst && vc->sid.lock() == sid && vc->tid.lock() == tid && vc->m == m &&
          vc->ns_in == ns_in && vc->nt == nt)
        ix = vc->ix;
    }
  }
  if (!ix) {
    ix = vr_build(s, rsrc, rdst, m, sid, ns_in, tid, nt);
    auto vc = std::make_shared<VrCache>();
    vc->rdst = rdst;
    vc->sid = sid;
    vc->tid = tid;
    vc->m = m;
    vc->ns_in = ns_in;
    vc->nt = nt;
    vc->ix = ix;
    std::lock_guard<std::mutex> lk(rsrc->mu);
    rsrc->vr_index = vc;
  }
  const uint32_t D = ix->D;
  const int64_t ns = ix->ns;
  const uint64_t *dk = (const uint64_t *)ix->dict->p;
  const BufPtr &si = ix->si, &di = ix->di, &tflag = ix->tflag, &src_nodes = ix->src_nodes;
  const BufPtr &rowptr = ix->rowptr, &cols = ix->cols, &order = ix->order, &srcpos = ix->srcpos;
  const unsigned g = grid_for(m, 256, 256 * 64);
  // 4. MS-BFS in batches of 64·K sources
  BufPtr reach = s->alloc(8 * std::max<int64_t>(ns, 1));
  // CAPF_VR_BUDGET (tests): a smaller state budget in bytes → more source batches
  const char *vb = getenv("CAPF_VR_BUDGET");
  const double budget = vb && atof(vb) > 0 ? atof(vb) : (double)VR_STATE_BUDGET;
  const int64_t kmax = std::max<int64_t>(1, (int64_t)(budget / (24.0 * D)));
  const int64_t K = std::min<int64_t>((ns + 63) / 64, kmax);
  BufPtr fa = s->alloc(8 * (int64_t)D * K), fb = s->alloc(8 * (int64_t)D * K);
  BufPtr vis = s->alloc(8 * (int64_t)D * K);
  const unsigned glev = grid_for((int64_t)D * K, 256, (int64_t)s->num_cus * 32);
  const char *vce = getenv("CAPF_VR_COUNT");  // 0 (tuning): the ballot-transpose count
  // the bit-sliced count takes row chunks on gridDim.y (≤ 65535): beyond that
  // (D > 2^26 nodes) the ballot-transpose count, whose grid is 1-D over sources
  const bool bs_count = !(vce && atoi(vce) == 0) &&
                        (int64_t)D <= (int64_t)65535 * (1024 / WAVE) * VR_CR;
  for (int64_t s0 = 0; s0 < ns; s0 += 64 * K) {
    const int64_t nb = std::min<int64_t>(64 * K, ns - s0);
    HIP_CHECK(hipMemsetAsync(fb->p, 0, 8 * (size_t)D * K, s->stream));
    HIP_CHECK(hipMemsetAsync(vis->p, 0, 8 * (size_t)D * K, s->stream));
    {
      KernelTimer kt(s, "vr_push1", 12.0 * m);
      hipLaunchKernelGGL(k_vr_push1, dim3(g), dim3(256), 0, s->stream, (const uint32_t *)si->p,
                         (const uint32_t *)di->p, m, (const int32_t *)srcpos->p, s0, nb, K,
                         (unsigned long long *)vis->p, (unsigned long long *)fb->p);
      KERNEL_CHECK();
    }
    unsigned long long *cur = (unsigned long long *)fb->p, *nxt = (unsigned long long *)fa->p;
    for (int l = 2; l <= upper; ++l) {
      KernelTimer kt(s, "vr_level", 8.0 * K * ((double)m + 3.0 * D));
      hipLaunchKernelGGL(k_vr_level, dim3(glev), dim3(256), 0, s->stream,
                         (const uint32_t *)rowptr->p, (const uint32_t *)cols->p,
                         (const uint64_t *)order->p, cur, nxt,
                         (unsigned long long *)vis->p, (int64_t)D, K, l == upper ? 1 : 0);
      KERNEL_CHECK();
      std::swap(cur, nxt);
    }
    {
      KernelTimer kt(s, "vr_count", 8.0 * K * D);
      if (bs_count) {
        HIP_CHECK(hipMemsetAsync((int64_t *)reach->p + s0, 0, 8 * (size_t)nb, s->stream));
        const int64_t kw = (nb + 63) / 64;  // source words of this batch
        const int64_t cg = (D + (int64_t)(1024 / WAVE) * VR_CR - 1) / ((int64_t)(1024 / WAVE) * VR_CR);
        hipLaunchKernelGGL(k_vr_count_bs, dim3((unsigned)((kw + 63) / 64), (unsigned)cg), dim3(1024), 0,
                           s->stream, (const unsigned long long *)vis->p, (const uint8_t *)tflag->p,
                           (int64_t)D, K, s0, nb, (unsigned long long *)reach->p);
      } else {
        hipLaunchKernelGGL(k_vr_count, dim3((unsigned)((nb + 63) / 64)), dim3(256), 0, s->stream,
                           (const unsigned long long *)vis->p, (const uint8_t *)tflag->p, (int64_t)D,
                           K, s0, nb, (int64_t *)reach->p);
      }
      KERNEL_CHECK();
      if (include_self) {
        hipLaunchKernelGGL(k_vr_self, dim3(grid_for(nb, 256)), dim3(256), 0, s->stream,
                           (const unsigned long long *)vis->p, (const uint8_t *)tflag->p,
                           (const int64_t *)src_nodes->p, K, s0, nb, (int64_t *)reach->p);
        KERNEL_CHECK();
      }
    }
  }
  // 5. rows (a, reach) for the sources that reach at least one target (every
  // source from lower bound 0)
  BufPtr pos = s->alloc(std::max<int64_t>(ns, 1));
  hipLaunchKernelGGL(k_vr_pos, dim3(grid_for(ns, 256)), dim3(256), 0, s->stream,
                     (const int64_t *)reach->p, ns, (uint8_t *)pos->p);
  KERNEL_CHECK();
  int64_t nr = 0;
  BufPtr rows = compact_flags(s, (const uint8_t *)pos->p, ns, &nr);
  ColPtr a = make_column(s, Type::Int64, nr, false), r = make_column(s, Type::Int64, nr, false);
  if (nr > 0) {
    hipLaunchKernelGGL(k_vr_out, dim3(grid_for(nr, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)rows->p, nr, (const int64_t *)src_nodes->p, dk,
                       (const int64_t *)reach->p, (int64_t *)a->data->p, (int64_t *)r->data->p);
    KERNEL_CHECK();
  }
  s->sync();
  out->nrows = nr;
  out->cols = {a, r};
  return out;
}

static ColPtr int_column_of(const NodePtr &nd, const DataPtr &d, const char *name) {
  const ColPtr &c = d->cols[nd->col_index_or_throw(name)];
  force(c);
  if (c->type != Type::Int64) illegal(std::string("column ") + name + " is not INTEGER");
  if (c->valid) not_impl(std::string("var-length reach: nullable id column ") + name);
  return c;
}

}  // namespace capf

using namespace capf;

extern "C" capf_status capf_var_length_reach(capf_session *cs, capf_table *rels, const char *src_col,
                                             const char *dst_col, capf_table *sources,
                                             const char *source_id_col, capf_table *targets,
                                             const char *target_id_col, int32_t lower, int32_t upper,
                                             const char *out_source_col, const char *out_reach_col,
                                             capf_table **out) {
  try {
    if (!cs || !rels || !src_col || !dst_col || !sources || !source_id_col || !targets ||
        !target_id_col || !out_source_col || !out_reach_col || !out)
      illegal("null argument");
    if (lower != 1 && lower != 0) not_impl("var-length reach: only lower bounds 0 and 1 are fused");
    if (upper < 1 || upper > 64) illegal("var-length reach: upper bound out of range");
    if (!strcmp(out_source_col, out_reach_col)) illegal("output column names must differ");
    Session *s = &cs->impl;
    DataPtr dr = materialize(rels->node), ds = materialize(sources->node),
            dt = materialize(targets->node);
    ColPtr rs = int_column_of(rels->node, dr, src_col), rd = int_column_of(rels->node, dr, dst_col);
    ColPtr si = int_column_of(sources->node, ds, source_id_col);
    ColPtr ti = int_column_of(targets->node, dt, target_id_col);
    DataPtr d = var_length_reach_rows(s, rs, rd, dr->nrows, si, ds->nrows, ti, dt->nrows, upper, lower == 0);
    auto n = std::make_shared<Node>();
    n->s = s;
    n->kind = Kind::Source;
    n->names = {out_source_col, out_reach_col};
    n->types = {Type::Int64, Type::Int64};
    n->result = d;
    auto *t = new capf_table;
    t->node = n;
    *out = t;
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}
