// fused_count.hip — factorised count(*) over lazy inner-join trees.
//
// This is the hot path of the north star: the relational plan of
//   MATCH (a)-->(b)-->(c) RETURN count(*)
// as lowered by RelationalPlanner (okapi-relational/.../impl/planning/
// RelationalPlanner.scala:130-165, Aggregate :111, Filter :113) is
//   S_a ⋈[a=start(r1)] R1 ⋈[end(r1)=b] S_b ⋈[b=start(r2)] R2 ⋈[end(r2)=c] S_c
//   → Filter(NOT(r1 = r2))  (front-end uniqueness rewrite, CypherParser.scala:72)
//   → Aggregate(∅, count(*)) (RelationalOperator.scala:334-346 → Table.group)
// Flink executes it as four materialising hash joins (FlinkTable.join,
// FlinkTable.scala:171-187) over ~1e12 rows at R-MAT s24.  Here the same
// result is computed exactly without materialising any joined row:
//
//  * the join tree is collected from the lazy plan DAG (Select/Alias are
//    transparent, single-table predicates are pushed into their leaf);
//  * count(*) of an acyclic equi-join is evaluated by message passing: every
//    leaf sends its parent a histogram key → Σ weight (GROUP BY on the join
//    key with a weighted count), the root sums its row weights;
//  * relationship-uniqueness filters NOT(r_i = r_j) are removed by
//    inclusion–exclusion: the r_i = r_j term merges both scans of the same
//    rel table into one leaf (ids are unique), which turns the b-join into
//    the intra-row predicate start = end (self-loops);
//  * the exact 2-hop shape runs as ONE pass over the rel table
//    (k_chain2_*): both histograms and the self-loop correction, followed by
//    a dot product over the node range.
#include <chrono>
#include <algorithm>
#include <cstring>
#include <functional>
#include <numeric>
#include <map>
#include <set>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

// ============================================================ device maps
enum MapKind : int32_t { MAP_ONES = 0, MAP_DENSE = 1, MAP_HASH = 2, MAP_DENSE32 = 3, MAP_BITS = 4 };

struct DMap {
  int32_t kind;
  int32_t pad;
  int64_t lo, hi;                 // dense / ones: key range [lo, hi]
  unsigned long long *vals;       // dense: hi-lo+1 entries; hash: capacity entries
  int64_t *keys;                  // hash keys (HASH_EMPTY = free)
  uint64_t mask;                  // hash capacity - 1
};

constexpr int64_t HASH_EMPTY = INT64_MIN;

__device__ inline unsigned long long map_get(const DMap &m, int64_t k) {
  if (m.kind == MAP_ONES) return (k >= m.lo && k <= m.hi) ? 1ull : 0ull;
  if (m.kind == MAP_DENSE) return (k >= m.lo && k <= m.hi) ? m.vals[k - m.lo] : 0ull;
  if (m.kind == MAP_DENSE32)
    return (k >= m.lo && k <= m.hi) ? (unsigned long long)((const uint32_t *)m.vals)[k - m.lo] : 0ull;
  if (m.kind == MAP_BITS) {  // 0/1 membership: 1 bit per key of [lo, hi] (L2-resident)
    if (k < m.lo || k > m.hi) return 0ull;
    const uint64_t o = (uint64_t)(k - m.lo);
    return (unsigned long long)((((const uint32_t *)m.vals)[o >> 5] >> (o & 31)) & 1u);
  }
  uint64_t slot = fmix64((uint64_t)k) & m.mask;
  while (true) {
    int64_t cur = m.keys[slot];
    if (cur == k) return m.vals[slot];
    if (cur == HASH_EMPTY) return 0ull;
    slot = (slot + 1) & m.mask;
  }
}

__device__ inline void map_add(const DMap &m, int64_t k, unsigned long long w) {
  if (m.kind == MAP_DENSE) {
    if (k >= m.lo && k <= m.hi) atomicAdd(&m.vals[k - m.lo], w);
    return;
  }
  if (m.kind != MAP_HASH) return;  // only dense and hash maps have storage
  uint64_t slot = fmix64((uint64_t)k) & m.mask;
  while (true) {
    int64_t cur = m.keys[slot];
    if (cur == HASH_EMPTY) {
      unsigned long long old = atomicCAS((unsigned long long *)&m.keys[slot],
                                         (unsigned long long)HASH_EMPTY, (unsigned long long)k);
      cur = (int64_t)old;
      if (cur == HASH_EMPTY) cur = k;
    }
    if (cur == k) {
      atomicAdd(&m.vals[slot], w);
      return;
    }
    slot = (slot + 1) & m.mask;
  }
}

constexpr int MAX_CHILD = 6;

struct MsgJob {
  ColView cols[MAX_CHILD + 1];  // child key columns, then the parent key column
  DMap child[MAX_CHILD];
  int32_t nchild;
  int32_t has_parent;
  DMap out;
};

__device__ inline bool load_key(const ColView &c, int64_t r, int64_t &k) {
  if (c.type == CAPF_TYPE_NULL || !c.data || (c.valid && !c.valid[r])) return false;
  k = ld_int(c, r);
  return true;
}

// One message (or the root sum) of the message-passing count.
__global__ void k_message(const MsgJob j, int64_t n, unsigned long long *root_acc) {
  unsigned long long local = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long w = 1;
    for (int c = 0; c < j.nchild && w; ++c) {
      int64_t k;
      w = load_key(j.cols[c], r, k) ? w * map_get(j.child[c], k) : 0ull;
    }
    if (!w) continue;
    if (j.has_parent) {
      int64_t k;
      if (load_key(j.cols[j.nchild], r, k)) map_add(j.out, k, w);
    } else {
      local += w;
    }
  }
  if (!j.has_parent) {
    local = wave_reduce_sum(local);
    if (lane_id() == 0 && local) atomicAdd(root_acc, local);
  }
}

// The root sum over a leaf with two children and non-null key columns (the
// 1-hop count of config 2: rels with the source and target scans' messages):
// MSG_U rows per thread with all key loads, then all message lookups, issued
// before any is used — the generic loop is one dependent chain per row.
constexpr int MSG_U = 8;

__global__ __launch_bounds__(256) void k_message_root2(const MsgJob j, int64_t n,
                                                       unsigned long long *root_acc) {
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  unsigned long long local = 0;
  for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r0 < n; r0 += MSG_U * T) {
    int64_t k0[MSG_U], k1[MSG_U];
#pragma unroll
    for (int u = 0; u < MSG_U; ++u) {
      const int64_t r = min(r0 + u * T, n - 1);
      k0[u] = ld_int(j.cols[0], r);
      k1[u] = ld_int(j.cols[1], r);
    }
    unsigned long long w0[MSG_U], w1[MSG_U];
#pragma unroll
    for (int u = 0; u < MSG_U; ++u) {
      w0[u] = map_get(j.child[0], k0[u]);
      w1[u] = map_get(j.child[1], k1[u]);
    }
#pragma unroll
    for (int u = 0; u < MSG_U; ++u) local += r0 + u * T < n ? w0[u] * w1[u] : 0ull;
  }
  local = wave_reduce_sum(local);
  if (lane_id() == 0 && local) atomicAdd(root_acc, local);
}

// FOR32 specialisation (both key columns uint32 + base, the compacted
// layout): 16-B loads of 4 rows per column, message kinds as template
// parameters (no per-row kind dispatch), 2 groups of 4 rows in flight.
template <int KA, int KB>
__device__ inline unsigned long long map_get_t(const DMap &m, int64_t k) {
  (void)KB;
  if (KA == MAP_ONES) return (k >= m.lo && k <= m.hi) ? 1ull : 0ull;
  if (KA == MAP_BITS) {
    if (k < m.lo || k > m.hi) return 0ull;
    const uint64_t o = (uint64_t)(k - m.lo);
    return (unsigned long long)((((const uint32_t *)m.vals)[o >> 5] >> (o & 31)) & 1u);
  }
  return map_get(m, k);
}

template <int KA, int KB>
__global__ __launch_bounds__(256) void k_message_root2_f32(const MsgJob j, int64_t n,
                                                           unsigned long long *root_acc) {
  const uint4 *c0 = (const uint4 *)j.cols[0].data, *c1 = (const uint4 *)j.cols[1].data;
  const int64_t b0 = j.cols[0].base, b1 = j.cols[1].base;
  const DMap ma = j.child[0], mb = j.child[1];
  const int64_t groups = n / 4, T = (int64_t)gridDim.x * blockDim.x;
  unsigned long long local = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += 2 * T) {
    const int64_t g2 = g + T < groups ? g + T : g;
    const uint4 a0 = c0[g], a1 = c1[g], e0 = c0[g2], e1 = c1[g2];
    const uint32_t ka[8] = {a0.x, a0.y, a0.z, a0.w, e0.x, e0.y, e0.z, e0.w};
    const uint32_t kb[8] = {a1.x, a1.y, a1.z, a1.w, e1.x, e1.y, e1.z, e1.w};
    unsigned long long w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      w[u] = map_get_t<KA, 0>(ma, b0 + (int64_t)ka[u]) * map_get_t<KB, 0>(mb, b1 + (int64_t)kb[u]);
    unsigned long long sum = w[0] + w[1] + w[2] + w[3];
    if (g2 != g) sum += w[4] + w[5] + w[6] + w[7];
    local += sum;
  }
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(n - 4 * groups)) {  // ragged tail
    const int64_t r = 4 * groups + threadIdx.x;
    local += map_get(ma, ld_int(j.cols[0], r)) * map_get(mb, ld_int(j.cols[1], r));
  }
  local = wave_reduce_sum(local);
  if (lane_id() == 0 && local) atomicAdd(root_acc, local);
}

// Root with ONE remaining child message (the others were all-ones over a
// range the root's key column provably lies in — column statistics — and are
// dropped, their column is never read): Σ_rows map(key), 4 rows per 12/16-B
// load (FOR24 / FOR32) or 2 per 16-B load (int64), 8 rows in flight per lane.
struct U3w {
  uint32_t x, y, z;
};

template <int KA, int W>
__global__ __launch_bounds__(256) void k_message_root1(const ColView c, const DMap m, int64_t n,
                                                       unsigned long long *root_acc) {
  const int64_t base = c.base;
  const int64_t groups = n / 4, T = (int64_t)gridDim.x * blockDim.x;
  unsigned long long local = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += 2 * T) {
    const int64_t g2 = g + T < groups ? g + T : g;
    int64_t k[8];
    if (W == 4) {
      const uint4 a = ((const uint4 *)c.data)[g], e = ((const uint4 *)c.data)[g2];
      const uint32_t v[8] = {a.x, a.y, a.z, a.w, e.x, e.y, e.z, e.w};
#pragma unroll
      for (int u = 0; u < 8; ++u) k[u] = base + (int64_t)v[u];
    } else if (W == 3) {
      const U3w a = *(const U3w *)((const uint8_t *)c.data + 12 * g);
      const U3w e = *(const U3w *)((const uint8_t *)c.data + 12 * g2);
      const uint32_t v[8] = {a.x & 0xFFFFFFu, __builtin_amdgcn_alignbit(a.y, a.x, 24) & 0xFFFFFFu,
                             __builtin_amdgcn_alignbit(a.z, a.y, 16) & 0xFFFFFFu, a.z >> 8,
                             e.x & 0xFFFFFFu, __builtin_amdgcn_alignbit(e.y, e.x, 24) & 0xFFFFFFu,
                             __builtin_amdgcn_alignbit(e.z, e.y, 16) & 0xFFFFFFu, e.z >> 8};
#pragma unroll
      for (int u = 0; u < 8; ++u) k[u] = base + (int64_t)v[u];
    } else {
      const longlong2 *p = (const longlong2 *)c.data;
      const longlong2 a0 = p[2 * g], a1 = p[2 * g + 1], e0 = p[2 * g2], e1 = p[2 * g2 + 1];
      const int64_t v[8] = {a0.x, a0.y, a1.x, a1.y, e0.x, e0.y, e1.x, e1.y};
#pragma unroll
      for (int u = 0; u < 8; ++u) k[u] = v[u];
    }
    unsigned long long w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = map_get_t<KA, 0>(m, k[u]);
    unsigned long long sum = w[0] + w[1] + w[2] + w[3];
    if (g2 != g) sum += w[4] + w[5] + w[6] + w[7];
    local += sum;
  }
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(n - 4 * groups)) {  // ragged tail
    const int64_t r = 4 * groups + threadIdx.x;
    local += map_get(m, ld_int(c, r));
  }
  local = wave_reduce_sum(local);
  if (lane_id() == 0 && local) atomicAdd(root_acc, local);
}

__global__ void k_add_u64(unsigned long long *acc, unsigned long long v) {
  if (threadIdx.x == 0) atomicAdd(acc, v);
}

// ============================================================ 2-hop fast path
// One pass over the rel table computes, for the Sb key range [lo, hi]:
//   h1[b] += Wa(u1)        for rels with v1 = b      (hop 1, message R1 → S_b)
//   h2[b] += Wc(v2)        for rels with u2 = b      (hop 2, message R2 → S_b)
//   loops += Wa(u1)·Wb(v1)·Wc(v2) for rels with v1 = u2 (the r1 = r2 term)
// Node weights are 1 on a dense id range (MAP_ONES) or a per-id count array.
struct Chain2Args {
  ColView u1, v1, u2, v2;  // non-null rel id columns (u2/v2 may alias u1/v1)
  int64_t n;
  DMap wa, wb, wc;
  int64_t lo, hi;
  uint32_t *h1, *h2;
  unsigned long long *loops;
  int mixed;    // 1: index the histograms by node_mix(id − lo) (the partitioned layout)
  NodeMix mix;
};

template <bool ONES>
__device__ inline unsigned long long w_of(const DMap &m, int64_t k) {
  if (ONES) return (k >= m.lo && k <= m.hi) ? 1ull : 0ull;
  return map_get(m, k);
}

template <bool ONES>
__global__ __launch_bounds__(256) void k_chain2_hist(Chain2Args a) {
  unsigned long long loops = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.n; e += stride) {
    const int64_t x1 = ld_int(a.u1, e), y1 = ld_int(a.v1, e);
    const int64_t x2 = ld_int(a.u2, e), y2 = ld_int(a.v2, e);
    const unsigned long long wa = w_of<ONES>(a.wa, x1);
    const unsigned long long wc = w_of<ONES>(a.wc, y2);
    if (wa && y1 >= a.lo && y1 <= a.hi) {
      const uint32_t i = (uint32_t)(y1 - a.lo);
      atomicAdd(&a.h1[a.mixed ? node_mix(i, a.mix) : i], (uint32_t)wa);
    }
    if (wc && x2 >= a.lo && x2 <= a.hi) {
      const uint32_t i = (uint32_t)(x2 - a.lo);
      atomicAdd(&a.h2[a.mixed ? node_mix(i, a.mix) : i], (uint32_t)wc);
    }
    if (y1 == x2 && wa && wc) loops += wa * wc * w_of<ONES>(a.wb, y1);
  }
  loops = wave_reduce_sum(loops);
  if (lane_id() == 0 && loops) atomicAdd(a.loops, loops);
}

// fin != null (capf_table_count_async): the workgroup whose `done` add comes
// last writes *fin = acc[0] − acc[1] (Σ in·out − self-loops) — the count on the
// device without a separate one-thread kernel.
// Σ over the hand-off log of (Σ(x+X)(y+Y) − Σxy) = Σ_in Δ·(y + Y) + Σ_out Δ·x
// (x, y: the stored counters, X, Y: their hand-offs).  One workgroup: the
// out-side deltas Y are summed per counter in an LDS open-addressing map, then
// every entry reads its counters once (independent loads).
// Counter `bin` of one side (h) as stored: one uint32, or (split layout given
// and the bin's run unsplit) the half of the bucket's packed pair word.
// `split_l`: the split flags staged in LDS (null: read sp.split).
constexpr int64_t C2P_BW = int64_t(1) << 16;  // bins per bucket (chain2_partitioned.hip C2_BW)
constexpr int C2_HO_BLOCKS = 8;               // workgroups computing the hand-off terms (the
                                              // FIRST ones of the grid: dispatched at once)
constexpr int C2_HO_MAXNB = 2048;             // split flags staged in LDS (2·nb ≤ this)
__device__ inline uint32_t c2_stored(const uint32_t *h, const C2Spill &sp, int side, int64_t bin,
                                     const uint8_t *split_l) {
  if (!sp.split) return h[bin];
  const int64_t b = bin / C2P_BW, k = bin % C2P_BW;
  const bool sp_run = split_l ? split_l[side * sp.nb + b] != 0 : sp.split[side * sp.nb + b] != 0;
  if (sp_run) return h[bin];
  return (h[b * C2P_BW + (k & (C2P_BW / 2 - 1))] >> ((k >> 15) * 16)) & 0xFFFFu;
}

// Σ over the hand-off log of (Σ(x+X)(y+Y) − Σxy) = Σ_in Δ·(y + Y) + Σ_out Δ·x
// (x, y: the stored counters, X, Y: their hand-offs), workgroup `part` of
// `parts` taking every parts-th entry.  Each workgroup sums ALL out-side deltas
// per counter in an LDS open-addressing map (the log is short: ~700 entries at
// s24), stages the split flags in LDS, then reads one stored counter per entry
// — dependent global loads are the cost, so the entries are spread over
// several workgroups running beside the dot.
__device__ unsigned long long c2_handoff_terms(const uint32_t *h1, const uint32_t *h2, const C2Spill &sp,
                                               unsigned long long *lds, int part, int parts) {
  constexpr uint32_t MAPN = 2048;  // slots; up to MAPN / 2 distinct out-side counters
  __shared__ uint32_t mk[MAPN];
  __shared__ unsigned long long mv[MAPN];
  __shared__ uint8_t spl[C2_HO_MAXNB];
  __shared__ int map_full;
  unsigned long long corr = 0;
  const uint32_t ne = min(*sp.n, sp.cap);
  if (ne > 0) {
    const bool stage = sp.split && 2 * sp.nb <= C2_HO_MAXNB;
    for (uint32_t i = threadIdx.x; i < MAPN; i += blockDim.x) {
      mk[i] = 0xFFFFFFFFu;
      mv[i] = 0;
    }
    if (stage)
      for (int i = threadIdx.x; i < 2 * sp.nb; i += blockDim.x) spl[i] = sp.split[i] ? 1 : 0;
    if (threadIdx.x == 0) map_full = 0;
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < ne; e += blockDim.x) {
      const uint2 y = sp.log[e];
      if (!(y.y & 1u)) continue;
      const uint32_t b = (uint32_t)((int64_t)y.x % sp.hl);
      uint32_t h = (b * 0x9E3779B1u) & (MAPN - 1), probes = 0;
      for (;;) {
        const uint32_t prev = atomicCAS(&mk[h], 0xFFFFFFFFu, b);
        if (prev == 0xFFFFFFFFu || prev == b) {
          atomicAdd(&mv[h], (unsigned long long)(y.y >> 1));
          break;
        }
        h = (h + 1) & (MAPN - 1);
        if (++probes > MAPN / 2) {
          map_full = 1;
          break;
        }
      }
    }
    __syncthreads();
    const uint8_t *sl = stage ? spl : nullptr;
    for (uint32_t e = part * blockDim.x + threadIdx.x; e < ne; e += parts * blockDim.x) {
      const uint2 x = sp.log[e];
      const int64_t b = (int64_t)x.x % sp.hl;
      const unsigned long long d = x.y >> 1;
      if (x.y & 1u) {
        corr += d * c2_stored(h1, sp, 0, b, sl);
      } else {
        unsigned long long Y = 0;
        if (!map_full) {
          uint32_t h = ((uint32_t)b * 0x9E3779B1u) & (MAPN - 1);
          for (uint32_t k = 0; k < MAPN; ++k) {
            const uint32_t c = mk[h];
            if (c == (uint32_t)b) {
              Y = mv[h];
              break;
            }
            if (c == 0xFFFFFFFFu) break;
            h = (h + 1) & (MAPN - 1);
          }
        } else {  // (pathological: > MAPN/2 distinct out-side counters) scan the log
          for (uint32_t f = 0; f < ne; ++f) {
            const uint2 y = sp.log[f];
            if ((y.y & 1u) && (int64_t)y.x % sp.hl == b) Y += y.y >> 1;
          }
        }
        corr += d * (c2_stored(h2, sp, 1, b, sl) + Y);
      }
    }
  }
  return block_reduce_sum(corr, lds);
}

// fin != null (the fused count): the workgroup whose `done` add comes last
// writes *fin = acc[0] − acc[1] (Σ in·out − self-loops) — into the async slot
// or the pinned host scalar, without a separate kernel or copy.  sp.n != null
// (the partitioned pipeline): the first C2_HO_BLOCKS workgroups compute the
// hand-off terms (beside the others' dot, not after it: dispatched first, their
// chains of dependent loads overlap the streaming) and add them to acc[0].
template <bool ONES>
__global__ __launch_bounds__(256) void k_chain2_dot(const uint32_t *h1, const uint32_t *h2,
                                                    DMap wb, int64_t lo, int64_t len,
                                                    unsigned long long *acc, int64_t *fin = nullptr,
                                                    unsigned int *done = nullptr, C2Spill sp = C2Spill()) {
  __shared__ unsigned long long lds[17];
  unsigned long long s = 0;
  const unsigned ho = sp.n ? (unsigned)C2_HO_BLOCKS : 0u;
  const unsigned nblk = gridDim.x - ho;  // dot workgroups
  if (blockIdx.x < ho) {
    s = c2_handoff_terms(h1, h2, sp, lds, (int)blockIdx.x, C2_HO_BLOCKS);
  } else {
    const unsigned bid = blockIdx.x - ho;
    const int64_t stride = (int64_t)nblk * blockDim.x;
    // 4 counters per thread per step: dwordx4 loads of both histograms
    const int64_t n4 = len / 4;
    const uint4 *a4 = (const uint4 *)h1;
    const uint4 *b4 = (const uint4 *)h2;
    int64_t i0 = (int64_t)bid * blockDim.x + threadIdx.x;
    if (ONES) {
      // 4 independent dwordx4 pairs in flight per thread before the first use
      for (; i0 + 3 * stride < n4; i0 += 4 * stride) {
        uint4 x[4], y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          x[k] = a4[i0 + k * stride];
          y[k] = b4[i0 + k * stride];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          s += (unsigned long long)x[k].x * y[k].x + (unsigned long long)x[k].y * y[k].y +
               (unsigned long long)x[k].z * y[k].z + (unsigned long long)x[k].w * y[k].w;
      }
    }
    for (int64_t i = i0; i < n4; i += stride) {
      uint4 x = a4[i], y = b4[i];
      if (ONES) {
        s += (unsigned long long)x.x * y.x + (unsigned long long)x.y * y.y +
             (unsigned long long)x.z * y.z + (unsigned long long)x.w * y.w;
      } else {
        int64_t k = lo + 4 * i;
        s += (unsigned long long)x.x * y.x * w_of<false>(wb, k) +
             (unsigned long long)x.y * y.y * w_of<false>(wb, k + 1) +
             (unsigned long long)x.z * y.z * w_of<false>(wb, k + 2) +
             (unsigned long long)x.w * y.w * w_of<false>(wb, k + 3);
      }
    }
    for (int64_t i = 4 * n4 + (int64_t)bid * blockDim.x + threadIdx.x; i < len; i += stride)
      s += (unsigned long long)h1[i] * h2[i] * (ONES ? 1ull : w_of<false>(wb, lo + i));
    s = block_reduce_sum(s, lds);
  }
  if (threadIdx.x == 0 && s) atomicAdd(acc, s);
  if (!fin) return;
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(done, 1u) == gridDim.x - 1) {  // every other block's add has landed
      __threadfence();
      const unsigned long long a0 = atomicAdd(acc, 0ull), a1 = atomicAdd(acc + 1, 0ull);
      // fin may be pinned host memory: a system-scope store
      __hip_atomic_store(fin, (int64_t)(a0 - a1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
    }
  }
}

// Σ in·out over the partitioned pipeline's bucket layout (sp.split given): an
// unsplit run's bucket holds packed uint16 pairs in its first half (half the
// bytes of one uint32 per bin), a split run's bucket one uint32 per bin.  The
// grid strides over quads (4 words of the half-range, both halves of a split
// bucket): a wave's 64 quads lie in one bucket, so the format is wave-uniform,
// and each thread keeps 4 quads' loads in flight before the first use (the
// per-bucket flags come from LDS).  Packed buckets issue their "high" load at
// the same address (an L1/L2 hit, no HBM bytes) so the loads stay branch-free.
// First C2_HO_BLOCKS workgroups: the hand-off terms; last to finish: *fin.
__device__ __forceinline__ void c2p_quad(const uint32_t *h, int64_t q, bool split, uint4 &lo, uint4 &hi) {
  constexpr int64_t HALF = C2P_BW / 2;
  const int64_t b = q >> 13, w = (q & 8191) * 4;  // HALF / 4 = 8192 quads per bucket
  const uint32_t *p = h + b * C2P_BW + w;
  lo = *(const uint4 *)p;
  hi = *(const uint4 *)(p + (split ? HALF : 0));
}
__device__ __forceinline__ unsigned long long c2p_mul(uint4 alo, uint4 ahi, bool sa, uint4 clo, uint4 chi, bool sc) {
  if (!sa) {
    ahi = make_uint4(alo.x >> 16, alo.y >> 16, alo.z >> 16, alo.w >> 16);
    alo = make_uint4(alo.x & 0xFFFF, alo.y & 0xFFFF, alo.z & 0xFFFF, alo.w & 0xFFFF);
  }
  if (!sc) {
    chi = make_uint4(clo.x >> 16, clo.y >> 16, clo.z >> 16, clo.w >> 16);
    clo = make_uint4(clo.x & 0xFFFF, clo.y & 0xFFFF, clo.z & 0xFFFF, clo.w & 0xFFFF);
  }
  return (unsigned long long)alo.x * clo.x + (unsigned long long)alo.y * clo.y +
         (unsigned long long)alo.z * clo.z + (unsigned long long)alo.w * clo.w +
         (unsigned long long)ahi.x * chi.x + (unsigned long long)ahi.y * chi.y +
         (unsigned long long)ahi.z * chi.z + (unsigned long long)ahi.w * chi.w;
}
__global__ __launch_bounds__(1024) void k_chain2_dot_pairs(const uint32_t *h1, const uint32_t *h2, C2Spill sp,
                                                          unsigned long long *acc, int64_t *fin,
                                                          unsigned int *done) {
  __shared__ unsigned long long lds[17];
  unsigned long long s = 0;
  const unsigned nblk = gridDim.x - C2_HO_BLOCKS;
  if (blockIdx.x < (unsigned)C2_HO_BLOCKS) {
    s = c2_handoff_terms(h1, h2, sp, lds, (int)blockIdx.x, C2_HO_BLOCKS);
  } else {
    const unsigned bid = blockIdx.x - C2_HO_BLOCKS;
    __shared__ uint8_t fl[C2_HO_MAXNB];
    const bool stage = 2 * sp.nb <= C2_HO_MAXNB;
    if (stage) {
      for (int i = threadIdx.x; i < 2 * sp.nb; i += blockDim.x) fl[i] = sp.split[i] ? 1 : 0;
      __syncthreads();
    }
    auto sa = [&](int64_t q) { return stage ? fl[q >> 13] != 0 : sp.split[q >> 13] != 0; };
    auto sc = [&](int64_t q) { return stage ? fl[sp.nb + (q >> 13)] != 0 : sp.split[sp.nb + (q >> 13)] != 0; };
    const int64_t nq = (int64_t)sp.nb * 8192, stride = (int64_t)nblk * blockDim.x;
    int64_t q = (int64_t)bid * blockDim.x + threadIdx.x;
    for (; q + 3 * stride < nq; q += 4 * stride) {
      uint4 alo[4], ahi[4], clo[4], chi[4];
      bool fa[4], fc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        fa[k] = sa(q + k * stride);
        fc[k] = sc(q + k * stride);
        c2p_quad(h1, q + k * stride, fa[k], alo[k], ahi[k]);
        c2p_quad(h2, q + k * stride, fc[k], clo[k], chi[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) s += c2p_mul(alo[k], ahi[k], fa[k], clo[k], chi[k], fc[k]);
    }
    for (; q < nq; q += stride) {
      uint4 alo, ahi, clo, chi;
      const bool fa = sa(q), fc = sc(q);
      c2p_quad(h1, q, fa, alo, ahi);
      c2p_quad(h2, q, fc, clo, chi);
      s += c2p_mul(alo, ahi, fa, clo, chi, fc);
    }
    s = block_reduce_sum(s, lds);
  }
  if (threadIdx.x == 0 && s) atomicAdd(acc, s);
  if (sp.tile_loops) {  // the self-loops (no transpose summed P1's per-tile counts)
    unsigned long long l = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < sp.ntiles; i += (int64_t)gridDim.x * blockDim.x)
      l += sp.tile_loops[i];
    __syncthreads();  // lds reused
    l = block_reduce_sum(l, lds);
    if (threadIdx.x == 0 && l) atomicAdd(acc + 1, l);
  }
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(done, 1u) == gridDim.x - 1) {
      __threadfence();
      const unsigned long long a0 = atomicAdd(acc, 0ull), a1 = atomicAdd(acc + 1, 0ull);
      __hip_atomic_store(fin, (int64_t)(a0 - a1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
    }
  }
}

// per-id count array of a node table's id column over [lo, hi]
__global__ void k_count_ids(ColView ids, int64_t n, int64_t lo, int64_t hi, uint32_t *cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (ids.valid && !ids.valid[i]) continue;
    int64_t k = ld_int(ids, i);
    if (k >= lo && k <= hi) atomicAdd(&cnt[k - lo], 1u);
  }
}

// ============================================================ plan analysis
struct ColRef {
  int leaf = -1;
  int col = -1;
  bool operator==(const ColRef &o) const { return leaf == o.leaf && col == o.col; }
};

struct Leaf {
  NodePtr node;                   // base plan node (materialisable)
  std::vector<Program> filters;   // single-leaf predicates pushed down (leaf column names)
  std::vector<std::pair<int, int>> col_eqs;  // intra-row equalities (after merges)
};

struct JoinGraph {
  std::vector<Leaf> leaves;
  std::vector<std::pair<ColRef, ColRef>> eqs;
  std::vector<std::pair<ColRef, ColRef>> neqs;
  // literal columns met on the way (withColumns of literals): ColRef{-2, k}
  // refers to lits[k]
  std::vector<Program> lits;
};

static bool collect(const NodePtr &n, JoinGraph &g, std::vector<ColRef> &out);

static bool program_is_uniqueness(const Program &p, std::vector<std::pair<int, int>> &pairs) {
  // [COL a, COL b, EQ, NOT] | [COL a, COL b, NEQ], possibly combined by AND(k)
  const auto &c = p.code;
  size_t i = 0;
  int terms = 0;
  while (i < c.size()) {
    if (i + 2 < c.size() && c[i].op == OP_COL && c[i + 1].op == OP_COL) {
      if (c[i + 2].op == OP_NEQ) {
        pairs.emplace_back((int)c[i].i, (int)c[i + 1].i);
        i += 3;
        ++terms;
        continue;
      }
      if (i + 3 < c.size() && c[i + 2].op == OP_EQ && c[i + 3].op == OP_NOT) {
        pairs.emplace_back((int)c[i].i, (int)c[i + 1].i);
        i += 4;
        ++terms;
        continue;
      }
    }
    if (c[i].op == OP_AND && i + 1 == c.size() && c[i].i == terms) {
      ++i;
      continue;
    }
    return false;
  }
  return terms > 0;
}

static bool collect(const NodePtr &n, JoinGraph &g, std::vector<ColRef> &out) {
  out.clear();
  {
    std::lock_guard<std::mutex> lk(n->mu);
    if (n->result) {  // already materialised: a leaf
      int id = (int)g.leaves.size();
      g.leaves.push_back(Leaf{n, {}, {}});
      for (size_t i = 0; i < n->names.size(); ++i) out.push_back(ColRef{id, (int)i});
      return true;
    }
  }
  switch (n->kind) {
    case Kind::Select: {
      std::vector<ColRef> c;
      if (!collect(n->kids[0], g, c)) return false;
      for (int i : n->sel_index) out.push_back(c[i]);
      return true;
    }
    case Kind::Join: {
      if (n->join_type != CAPF_JOIN_INNER) break;
      std::vector<ColRef> l, r;
      if (!collect(n->kids[0], g, l)) return false;
      if (!collect(n->kids[1], g, r)) return false;
      for (auto &kp : n->join_keys) {
        if (n->kids[0]->types[kp.first] != Type::Int64) return false;
        if (l[kp.first].leaf < 0 || r[kp.second].leaf < 0) return false;
        g.eqs.emplace_back(l[kp.first], r[kp.second]);
      }
      out = l;
      out.insert(out.end(), r.begin(), r.end());
      return true;
    }
    case Kind::WithColumns: {
      // transparent when it only adds/replaces columns by literals (the
      // constant label / NULL property columns of scan alignment,
      // RelationalPlanner.scala:447-515); the literal columns themselves can
      // not take part in a join or predicate of the fused count
      bool literal_only = true;
      for (auto &p : n->exprs)
        literal_only &= p.code.size() == 1 && p.code[0].op != OP_COL;
      if (!literal_only) break;
      std::vector<ColRef> c;
      if (!collect(n->kids[0], g, c)) return false;
      out = c;
      out.resize(n->names.size(), ColRef{-2, -1});
      for (size_t k = 0; k < n->exprs.size(); ++k) {
        out[n->target_index[k]] = ColRef{-2, (int)g.lits.size()};
        g.lits.push_back(n->exprs[k]);
      }
      return true;
    }
    case Kind::Filter: {
      std::vector<ColRef> c;
      if (!collect(n->kids[0], g, c)) return false;
      out = c;
      const NodePtr &kid = n->kids[0];
      std::vector<int> refs;
      for (auto &nm : n->pred.names) refs.push_back(is_session_table_name(nm) ? -1 : kid->col_index(nm));
      std::set<int> leaves;
      for (size_t k = 0; k < refs.size(); ++k) {
        if (is_session_table_name(n->pred.names[k])) continue;
        const int r = refs[k];
        if (r < 0 || c[r].leaf < 0) return false;
        leaves.insert(c[r].leaf);
      }
      if (leaves.size() == 1) {
        // single-table predicate: push into the leaf with leaf column names
        int lf = *leaves.begin();
        Program p = n->pred;
        for (size_t k = 0; k < p.names.size(); ++k)
          if (!is_session_table_name(p.names[k])) p.names[k] = g.leaves[lf].node->names[c[refs[k]].col];
        g.leaves[lf].filters.push_back(std::move(p));
        return true;
      }
      std::vector<std::pair<int, int>> pairs;
      if (!program_is_uniqueness(n->pred, pairs)) return false;
      for (auto &pr : pairs) {
        int a = refs[pr.first], b = refs[pr.second];
        if (kid->types[a] != Type::Int64 || kid->types[b] != Type::Int64) return false;
        g.neqs.emplace_back(c[a], c[b]);
      }
      return true;
    }
    default: break;
  }
  // any other operator is an opaque leaf
  int id = (int)g.leaves.size();
  g.leaves.push_back(Leaf{n, {}, {}});
  for (size_t i = 0; i < n->names.size(); ++i) out.push_back(ColRef{id, (int)i});
  return true;
}

// ============================================================ leaf data
struct LeafData {
  DataPtr data;
  bool plain = false;  // unfiltered base data (eligible for column stats / merges)
};

static NodePtr filter_node(const NodePtr &base, const Program &p) {
  auto f = std::make_shared<Node>();
  f->s = base->s;
  f->kind = Kind::Filter;
  f->kids = {base};
  f->pred = p;
  f->names = base->names;
  f->types = base->types;
  return f;
}

static Program eq_program(const std::string &a, const std::string &b) {
  Program p;
  p.names = {a, b};
  p.code = {Instr{OP_COL, 0, 0, 0}, Instr{OP_COL, 0, 1, 0}, Instr{OP_EQ, 0, 0, 0}};
  return p;
}

static LeafData leaf_data(const Leaf &lf) {
  LeafData ld;
  NodePtr cur = lf.node;
  for (auto &p : lf.filters) cur = filter_node(cur, p);
  for (auto &e : lf.col_eqs)
    cur = filter_node(cur, eq_program(lf.node->names[e.first], lf.node->names[e.second]));
  ld.data = materialize(cur);
  ld.plain = lf.filters.empty() && lf.col_eqs.empty();
  return ld;
}

// ============================================================ message passing
// A membership bitmap cached on its key column, with its node_mix-ordered copy
// (built by the first partitioned probe, bits_count_partitioned).
struct BitsCache {
  BufPtr bits, mixed;
};

struct HostMap {
  DMap m;
  BufPtr vals, keys;
  std::shared_ptr<BitsCache> bc;  // MAP_BITS from a column's cache
};

__global__ void k_fill_hash_empty(int64_t *k, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    k[i] = HASH_EMPTY;
}

static HostMap ones_map(int64_t lo, int64_t hi) {
  HostMap h;
  memset(&h.m, 0, sizeof(h.m));
  h.m.kind = MAP_ONES;
  h.m.lo = lo;
  h.m.hi = hi;
  return h;
}

// Membership bitmap of a childless leaf's key column over the parent key's
// range [lo, hi]: the leaf's message when every key occurs at most once
// (node scans) — 1 bit per key instead of an 8-B count, so the parent's
// lookups hit L2.  *dup is set when a key repeats (then counts are needed).
__global__ void k_bits_set(ColView c, int64_t n, int64_t lo, int64_t hi, uint32_t *words,
                           uint32_t *dup) {
  // whole waves per step; lanes whose keys share a 32-bit word (consecutive
  // ids: every lane of a sorted node scan) OR their bits together first and
  // the last lane of each run issues ONE atomic (32 lanes of a device atomic
  // on one word serialise at the memory side: 132 -> few µs for 2 Mi ids)
  const int lane = lane_id();
  for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~(WAVE - 1)); r0 < n;
       r0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = r0 + lane;
    bool live = r < n && (!c.valid || c.valid[r]);
    const int64_t k = live ? ld_int(c, r) : lo;
    live = live && k >= lo && k <= hi;
    const uint64_t o = (uint64_t)(k - lo);
    const uint32_t w = live ? (uint32_t)(o >> 5) : 0xFFFFFFFFu;
    uint32_t bits = live ? 1u << (o & 31) : 0u, dupb = 0;
    // segmented inclusive OR over lanes with equal words (disjoint coverage,
    // so a bit seen twice is a duplicate key)
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const uint32_t wo = __shfl_up(w, d, WAVE), bo = __shfl_up(bits, d, WAVE), dbo = __shfl_up(dupb, d, WAVE);
      if (lane >= d && wo == w) {
        dupb |= dbo | (bo & bits);
        bits |= bo;
      }
    }
    const uint32_t wn = __shfl_down(w, 1, WAVE);
    if (live && (lane == WAVE - 1 || wn != w)) {
      if ((atomicOr(&words[w], bits) & bits) || dupb) *dup = 1u;
    }
  }
}

// The membership bitmap of `mykey` over the parent key's range: built once per
// (column, range) and cached on the column (an ingest-time bitmap index of an
// immutable id column, like the statistics), then reused by every query.
static bool bits_map_for(Session *s, const ColPtr &parent_key, const ColPtr &mykey, HostMap &h) {
  const ColStats &st = column_stats(s, parent_key);
  if (st.non_null == 0 || mykey->type != Type::Int64) return false;
  const uint64_t range = (uint64_t)(st.max - st.min) + 1;
  if (range > (uint64_t(1) << 34)) return false;
  if (mykey->unique_flag == 0) return false;
  bool cached = false;
  {
    std::lock_guard<std::mutex> lk(mykey->mu);
    if (mykey->bits && mykey->bits_key[0] == st.min && mykey->bits_key[1] == st.max) {
      h.bc = std::static_pointer_cast<BitsCache>(mykey->bits);
      h.vals = h.bc->bits;
      cached = true;
    }
  }
  const int64_t nw = (int64_t)((range + 31) / 32);
  if (!cached) {
    h.vals = s->alloc(4 * nw + 4);
    HIP_CHECK(hipMemsetAsync(h.vals->p, 0, 4 * nw + 4, s->stream));
    uint32_t *words = (uint32_t *)h.vals->p, *dup = words + nw;
    if (mykey->n > 0) {
      hipLaunchKernelGGL(k_bits_set, dim3(grid_for(mykey->n, 256)), dim3(256), 0, s->stream,
                         view_of(mykey), mykey->n, st.min, st.max, words, dup);
      KERNEL_CHECK();
    }
    // duplicates → not a membership map.  Uniqueness is a property of the
    // (immutable) key column: read back once, cached on the column
    if (mykey->unique_flag < 0) {
      uint32_t d = 0;
      HIP_CHECK(hipMemcpyAsync(&d, dup, 4, hipMemcpyDeviceToHost, s->stream));
      s->sync();
      mykey->unique_flag = d ? 0 : 1;
    }
    if (!mykey->unique_flag) return false;
    std::lock_guard<std::mutex> lk(mykey->mu);
    h.bc = std::make_shared<BitsCache>();
    h.bc->bits = h.vals;
    mykey->bits = h.bc;
    mykey->bits_key[0] = st.min;
    mykey->bits_key[1] = st.max;
  }
  memset(&h.m, 0, sizeof(h.m));
  h.m.kind = MAP_BITS;
  h.m.lo = st.min;
  h.m.hi = st.max;
  h.m.vals = (unsigned long long *)h.vals->p;
  return true;
}

static HostMap new_map_for(Session *s, const ColPtr &parent_key, int64_t sender_rows) {
  HostMap h;
  memset(&h.m, 0, sizeof(h.m));
  const ColStats &st = column_stats(s, parent_key);
  int64_t prow = parent_key->n;
  uint64_t range = st.non_null > 0 ? (uint64_t)(st.max - st.min) + 1 : 0;
  if (st.non_null > 0 && range <= (uint64_t(1) << 28) &&
      range <= 16 * (uint64_t)std::max<int64_t>(std::max(prow, sender_rows), 1024)) {
    h.m.kind = MAP_DENSE;
    h.m.lo = st.min;
    h.m.hi = st.max;
    h.vals = s->alloc(8 * range);
    HIP_CHECK(hipMemsetAsync(h.vals->p, 0, 8 * range, s->stream));
    h.m.vals = (unsigned long long *)h.vals->p;
  } else if (st.non_null == 0) {
    h.m.kind = MAP_ONES;  // empty range: everything maps to 0
    h.m.lo = 1;
    h.m.hi = 0;
  } else {
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)std::max<int64_t>(sender_rows, 1)) cap <<= 1;
    h.m.kind = MAP_HASH;
    h.m.mask = cap - 1;
    h.keys = s->alloc(8 * cap);
    h.vals = s->alloc(8 * cap);
    HIP_CHECK(hipMemsetAsync(h.vals->p, 0, 8 * cap, s->stream));
    hipLaunchKernelGGL(k_fill_hash_empty, dim3(grid_for((int64_t)cap, 256)), dim3(256), 0,
                       s->stream, (int64_t *)h.keys->p, cap);
    KERNEL_CHECK();
    h.m.keys = (int64_t *)h.keys->p;
    h.m.vals = (unsigned long long *)h.vals->p;
  }
  return h;
}

// Count of the acyclic equi-join described by `g` (no inequalities).
// Adds the join tree's count to the device counter *d_acc (no host wait).
static bool tree_count(Session *s, JoinGraph &g, unsigned long long *d_acc) {
  const int L = (int)g.leaves.size();
  if (L == 0) return false;
  // adjacency; reject cycles / multi-edges / disconnected graphs
  std::vector<std::vector<std::pair<int, int>>> adj(L);  // (neighbour, eq index)
  for (size_t e = 0; e < g.eqs.size(); ++e) {
    int a = g.eqs[e].first.leaf, b = g.eqs[e].second.leaf;
    if (a == b) return false;
    adj[a].emplace_back(b, (int)e);
    adj[b].emplace_back(a, (int)e);
  }
  if ((int)g.eqs.size() != L - 1) return false;
  // choose the tree centre as root (shortest longest path)
  auto ecc = [&](int r) {
    std::vector<int> d(L, -1);
    std::vector<int> q{r};
    d[r] = 0;
    for (size_t i = 0; i < q.size(); ++i)
      for (auto &nb : adj[q[i]])
        if (d[nb.first] < 0) {
          d[nb.first] = d[q[i]] + 1;
          q.push_back(nb.first);
        }
    int m = 0;
    for (int x : d) {
      if (x < 0) return -1;
      m = std::max(m, x);
    }
    return m;
  };
  int root = 0, best = 1 << 30;
  for (int r = 0; r < L; ++r) {
    int e = ecc(r);
    if (e < 0) return false;
    if (e < best) {
      best = e;
      root = r;
    }
  }
  std::vector<LeafData> data(L);
  for (int i = 0; i < L; ++i) data[i] = leaf_data(g.leaves[i]);
  for (int i = 0; i < L; ++i)
    if (data[i].data->nrows >= (int64_t(1) << 40)) return false;

  std::vector<HostMap> msg(L);
  std::function<void(int, int, int)> visit = [&](int v, int parent, int via_eq) {
    MsgJob j;
    memset(&j, 0, sizeof(j));
    int root_cols[MAX_CHILD + 1] = {0};
    int child_leaf[MAX_CHILD + 1] = {0};
    for (auto &nb : adj[v]) {
      if (nb.first == parent) continue;
      visit(nb.first, v, nb.second);
      if (j.nchild >= MAX_CHILD) not_impl("join tree node with too many children");
      const auto &eq = g.eqs[nb.second];
      int mycol = eq.first.leaf == v ? eq.first.col : eq.second.col;
      j.cols[j.nchild] = view_of(data[v].data->cols[mycol]);
      j.child[j.nchild] = msg[nb.first].m;
      root_cols[j.nchild] = mycol;
      child_leaf[j.nchild] = nb.first;
      j.nchild++;
    }
    const int64_t n = data[v].data->nrows;
    if (parent < 0 && data[v].plain) {
      // root: a child message that is all-ones over [lo, hi] while this key
      // column's values all lie in [lo, hi] (no NULLs) weighs every row 1
      int keep = 0;
      for (int c = 0; c < j.nchild; ++c) {
        bool one = false;
        if (j.child[c].kind == MAP_ONES && !j.cols[c].valid) {
          const ColPtr &kc = data[v].data->cols[root_cols[c]];
          const ColStats &st = column_stats(s, kc);
          one = st.non_null == n && (n == 0 || (st.min >= j.child[c].lo && st.max <= j.child[c].hi));
        }
        if (!one) {
          j.cols[keep] = j.cols[c];
          j.child[keep] = j.child[c];
          root_cols[keep] = root_cols[c];
          child_leaf[keep] = child_leaf[c];
          ++keep;
        }
      }
      j.nchild = keep;
      if (keep == 0) {  // every row counts once
        if (n > 0) hipLaunchKernelGGL(k_add_u64, dim3(1), dim3(64), 0, s->stream, d_acc, (unsigned long long)n);
        return;
      }
      const ColView &c0 = j.cols[0];
      const int cw = c0.enc == ENC_FOR32 ? 4 : c0.enc == ENC_FOR24 ? 3 : 8;
      const bool aligned = ((uintptr_t)c0.data & 15) == 0;
      // a membership bitmap probed by a large FOR key column: radix-partitioned
      // probes against LDS slices (chain2_partitioned.hip)
      if (keep == 1 && j.child[0].kind == MAP_BITS && msg[child_leaf[0]].bc &&
          bits_count_partitioned(s, c0, n, j.child[0].lo, j.child[0].hi, (const uint32_t *)j.child[0].vals,
                                 msg[child_leaf[0]].bc->mixed, d_acc))
        return;
      if (keep == 1 && n > 0 && c0.data && !c0.valid && aligned &&
          (j.child[0].kind == MAP_BITS || j.child[0].kind == MAP_ONES)) {
        KernelTimer kt(s, "message_pass", (double)cw * n);
        auto pick = [&](auto ka) {
          constexpr int KA = decltype(ka)::value;
          return cw == 4 ? k_message_root1<KA, 4> : cw == 3 ? k_message_root1<KA, 3> : k_message_root1<KA, 8>;
        };
        auto kern = j.child[0].kind == MAP_BITS ? pick(std::integral_constant<int, MAP_BITS>())
                                                : pick(std::integral_constant<int, MAP_ONES>());
        hipLaunchKernelGGL(kern, dim3(grid_for(n / 8 + 1, 256, (int64_t)s->num_cus * 16)), dim3(256), 0,
                           s->stream, c0, j.child[0], n, d_acc);
        KERNEL_CHECK();
        return;
      }
    }
    if (parent >= 0) {
      const auto &eq = g.eqs[via_eq];
      int mycol = eq.first.leaf == v ? eq.first.col : eq.second.col;
      int pcol = eq.first.leaf == v ? eq.second.col : eq.first.col;
      const ColPtr &mykey = data[v].data->cols[mycol];
      // leaf without children whose key is a dense unique id range: all ones
      if (j.nchild == 0 && data[v].plain) {
        const ColStats &st = column_stats(s, mykey);
        if (st.dense_unique && st.non_null == n) {
          msg[v] = ones_map(st.min, st.max);
          return;
        }
      }
      // childless leaf with unique keys: a membership bitmap (no pass, no atomics on counts)
      if (j.nchild == 0 && bits_map_for(s, data[parent].data->cols[pcol], mykey, msg[v])) return;
      msg[v] = new_map_for(s, data[parent].data->cols[pcol], n);
      // the parent's key column has no value: the empty all-ones map already
      // weighs every key 0 — nothing to add (the map has no storage)
      if (msg[v].m.kind == MAP_ONES) return;
      j.cols[j.nchild] = view_of(mykey);
      j.has_parent = 1;
      j.out = msg[v].m;
    }
    if (n == 0) return;
    {
      KernelTimer kt(s, "message_pass", 8.0 * n * (j.nchild + j.has_parent));
      const bool root2 = !j.has_parent && j.nchild == 2 && !j.cols[0].valid && !j.cols[1].valid &&
                         j.cols[0].data && j.cols[1].data;
      const bool f32 = root2 && j.cols[0].enc == ENC_FOR32 && j.cols[1].enc == ENC_FOR32;
      auto simple = [](int k) { return k == MAP_ONES || k == MAP_BITS; };
      if (f32 && simple(j.child[0].kind) && simple(j.child[1].kind)) {
        auto kern = j.child[0].kind == MAP_BITS
                        ? (j.child[1].kind == MAP_BITS ? k_message_root2_f32<MAP_BITS, MAP_BITS>
                                                       : k_message_root2_f32<MAP_BITS, MAP_ONES>)
                        : (j.child[1].kind == MAP_BITS ? k_message_root2_f32<MAP_ONES, MAP_BITS>
                                                       : k_message_root2_f32<MAP_ONES, MAP_ONES>);
        hipLaunchKernelGGL(kern, dim3(grid_for(n / 8 + 1, 256, (int64_t)s->num_cus * 16)), dim3(256),
                           0, s->stream, j, n, d_acc);
      } else if (root2)
        hipLaunchKernelGGL(k_message_root2, dim3(grid_for(n, 256 * MSG_U, (int64_t)s->num_cus * 16)),
                           dim3(256), 0, s->stream, j, n, d_acc);
      else
        hipLaunchKernelGGL(k_message, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, j, n, d_acc);
      KERNEL_CHECK();
    }
    // the job travels as a kernel argument (copied at launch): no host wait
    // between messages (buffers are recycled in stream order)
  };
  visit(root, -1, -1);
  return true;
}

// Union-find merge of leaves for one inclusion–exclusion term.
// Are the values of column `col` of a (materialisable) base node non-null and
// pairwise distinct?  Dense statistics answer at once; otherwise uniqueness is
// verified by grouping ONCE and cached on the (immutable) column.
static bool column_unique(const NodePtr &node, int col) {
  DataPtr d = materialize(node);
  const ColStats &st = column_stats(node->s, d->cols[col]);
  if (st.non_null != d->nrows) return false;
  if (st.dense_unique) return true;
  const ColPtr &idc = d->cols[col];
  if (idc->unique_flag < 0) {
    Grouping gr = group_rows(node->s, *d, {col});
    idc->unique_flag = gr.ngroups == d->nrows ? 1 : 0;
  }
  return idc->unique_flag == 1;
}

static bool apply_equalities(const JoinGraph &g, const std::vector<int> &subset, JoinGraph &out) {
  const int L = (int)g.leaves.size();
  std::vector<int> rep(L);
  std::iota(rep.begin(), rep.end(), 0);
  std::function<int(int)> find = [&](int x) { return rep[x] == x ? x : rep[x] = find(rep[x]); };
  std::vector<std::pair<int, int>> intra_by_leaf;  // (leaf, col a, col b) gathered below
  std::vector<std::tuple<int, int, int>> intra;
  for (int k : subset) {
    ColRef a = g.neqs[k].first, b = g.neqs[k].second;
    if (a.leaf == b.leaf) {
      if (a.col == b.col) continue;  // x = x: always true
      intra.emplace_back(a.leaf, a.col, b.col);
      continue;
    }
    // merging two scans requires the same base data and a unique id column
    const Leaf &la = g.leaves[a.leaf], &lb = g.leaves[b.leaf];
    if (la.node != lb.node || !la.filters.empty() || !lb.filters.empty() || a.col != b.col)
      return false;
    if (!column_unique(la.node, a.col)) return false;
    int ra = find(a.leaf), rb = find(b.leaf);
    if (ra != rb) rep[rb] = ra;
  }
  // new leaves
  std::vector<int> newid(L, -1);
  out = JoinGraph();
  for (int i = 0; i < L; ++i)
    if (find(i) == i) {
      newid[i] = (int)out.leaves.size();
      out.leaves.push_back(g.leaves[i]);
    }
  for (auto &t : intra) out.leaves[newid[find(std::get<0>(t))]].col_eqs.emplace_back(std::get<1>(t), std::get<2>(t));
  // re-express equalities; same-leaf equalities become intra-row predicates,
  // parallel edges sharing one side collapse (x=y ∧ x'=y → x=x' intra-row)
  for (auto &e : g.eqs) {
    ColRef a{newid[find(e.first.leaf)], e.first.col};
    ColRef b{newid[find(e.second.leaf)], e.second.col};
    if (a.leaf == b.leaf) {
      if (a.col != b.col) out.leaves[a.leaf].col_eqs.emplace_back(a.col, b.col);
      continue;
    }
    bool merged = false;
    for (auto &f : out.eqs) {
      ColRef &x = f.first, &y = f.second;
      ColRef xa = x.leaf == a.leaf ? x : y, yb = x.leaf == a.leaf ? y : x;
      bool same_pair = (x.leaf == a.leaf && y.leaf == b.leaf) || (x.leaf == b.leaf && y.leaf == a.leaf);
      if (!same_pair) continue;
      if (xa.col == a.col && yb.col == b.col) { merged = true; break; }  // duplicate
      if (yb.col == b.col) {
        out.leaves[a.leaf].col_eqs.emplace_back(xa.col, a.col);
        merged = true;
        break;
      }
      if (xa.col == a.col) {
        out.leaves[b.leaf].col_eqs.emplace_back(yb.col, b.col);
        merged = true;
        break;
      }
      return false;  // genuine two-key join: not a tree
    }
    if (!merged) out.eqs.emplace_back(a, b);
  }
  return true;
}

// ------------------------------------------------------------ 2-hop matcher
struct Chain2 {
  int ra, rb;        // the two rel leaves (same base node)
  int sa, sb, sc;    // node leaves
  int u1, v1, u2, v2;
  int ya, yb, yc;    // node id columns
};

static bool match_chain2(const JoinGraph &g, Chain2 &c) {
  if (g.leaves.size() != 5 || g.eqs.size() != 4 || g.neqs.size() != 1) return false;
  ColRef x = g.neqs[0].first, y = g.neqs[0].second;
  if (x.leaf == y.leaf || x.col != y.col) return false;
  const Leaf &lx = g.leaves[x.leaf], &ly = g.leaves[y.leaf];
  if (lx.node != ly.node || !lx.filters.empty() || !ly.filters.empty()) return false;
  // each rel leaf joins exactly two eqs; find its neighbours
  auto edges_of = [&](int leaf) {
    std::vector<std::pair<int, ColRef>> r;  // (my col, other)
    for (auto &e : g.eqs) {
      if (e.first.leaf == leaf) r.emplace_back(e.first.col, e.second);
      if (e.second.leaf == leaf) r.emplace_back(e.second.col, e.first);
    }
    return r;
  };
  auto e1 = edges_of(x.leaf), e2 = edges_of(y.leaf);
  if (e1.size() != 2 || e2.size() != 2) return false;
  // the shared node leaf S_b is the one adjacent to both
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 2; ++k) {
      if (e1[i].second.leaf != e2[k].second.leaf) continue;
      if (e1[i].second.col != e2[k].second.col) continue;
      const auto &to_a = e1[1 - i], &to_c = e2[1 - k];
      int sa = to_a.second.leaf, sb = e1[i].second.leaf, sc = to_c.second.leaf;
      if (sa == sb || sc == sb || sa == x.leaf || sc == y.leaf) return false;
      std::set<int> all{x.leaf, y.leaf, sa, sb, sc};
      if (all.size() != 5) return false;
      if (edges_of(sa).size() != 1 || edges_of(sc).size() != 1 || edges_of(sb).size() != 2)
        return false;
      for (int nl : {sa, sb, sc})
        if (!g.leaves[nl].col_eqs.empty()) return false;
      c.ra = x.leaf;
      c.rb = y.leaf;
      c.sa = sa;
      c.sb = sb;
      c.sc = sc;
      c.u1 = to_a.first;
      c.v1 = e1[i].first;
      c.u2 = e2[k].first;
      c.v2 = to_c.first;
      c.ya = to_a.second.col;
      c.yb = e1[i].second.col;
      c.yc = to_c.second.col;
      return true;
    }
  return false;
}

// ---------------------------------------------------------- triangle matcher
// (a)-[r1]->(b)-[r2]->(c)-[r3]->(a): Expand, Expand, ExpandInto
// (RelationalPlanner.scala:130-189) — three scans of one rel table, three node
// scans, six equalities forming a 6-cycle, pairwise r_i <> r_j.
struct Tri {
  int rel;         // one of the rel leaves (all scan the same base)
  int src, dst;    // its start / end columns
  int nodes[3];    // node leaves
  int ycol[3];     // their id columns
  int idcol;       // the uniqueness column of the rel leaves
};

static bool match_triangle(const JoinGraph &g, Tri &t) {
  if (g.leaves.size() != 6 || g.eqs.size() != 6 || g.neqs.size() != 3) return false;
  std::set<int> rels;
  int idcol = -1;
  for (auto &ne : g.neqs) {
    if (ne.first.leaf == ne.second.leaf || ne.first.col != ne.second.col) return false;
    if (idcol >= 0 && ne.first.col != idcol) return false;
    idcol = ne.first.col;
    rels.insert(ne.first.leaf);
    rels.insert(ne.second.leaf);
  }
  if (rels.size() != 3) return false;
  const int r0 = *rels.begin();
  for (int r : rels) {
    const Leaf &l = g.leaves[r];
    if (l.node != g.leaves[r0].node || !l.filters.empty() || !l.col_eqs.empty()) return false;
  }
  auto edges_of = [&](int leaf) {
    std::vector<std::pair<int, ColRef>> r;  // (my col, other)
    for (auto &e : g.eqs) {
      if (e.first.leaf == leaf) r.emplace_back(e.first.col, e.second);
      if (e.second.leaf == leaf) r.emplace_back(e.second.col, e.first);
    }
    return r;
  };
  auto e0 = edges_of(r0);
  if (e0.size() != 2 || e0[0].first == e0[1].first) return false;
  const int cs = e0[0].first, cd = e0[1].first;  // orientation: any consistent one
  std::map<int, std::pair<int, int>> node_ends;  // node leaf → (#cs ends, #cd ends)
  std::map<int, int> node_col;
  for (int r : rels) {
    auto e = edges_of(r);
    if (e.size() != 2 || e[0].first == e[1].first) return false;
    for (auto &x : e) {
      const int nl = x.second.leaf;
      if (rels.count(nl)) return false;
      if (x.first != cs && x.first != cd) return false;
      auto it = node_col.find(nl);
      if (it != node_col.end() && it->second != x.second.col) return false;
      node_col[nl] = x.second.col;
      (x.first == cs ? node_ends[nl].first : node_ends[nl].second)++;
    }
  }
  if (node_ends.size() != 3) return false;
  int k = 0;
  for (auto &ne : node_ends) {
    if (ne.second.first != 1 || ne.second.second != 1) return false;  // a directed cycle
    if (!g.leaves[ne.first].col_eqs.empty()) return false;
    t.nodes[k] = ne.first;
    t.ycol[k] = node_col[ne.first];
    ++k;
  }
  t.rel = r0;
  t.src = cs;
  t.dst = cd;
  t.idcol = idcol;
  return true;
}

struct NodeWeights {
  HostMap map;
  bool ones = false;
  BufPtr cnt;
};

// Per-id weights of a node leaf: MAP_ONES for a dense unique id range,
// otherwise a uint32 count array over [min, max] (returns false if sparse).
static bool node_weights(Session *s, const LeafData &ld, int col, NodeWeights &w) {
  const ColPtr &c = ld.data->cols[col];
  if (c->type != Type::Int64) return false;
  const ColStats &st = column_stats(s, c);
  if (st.non_null == 0) {
    w.map = ones_map(1, 0);
    w.ones = true;
    return true;
  }
  if (st.dense_unique && st.non_null == c->n) {
    w.map = ones_map(st.min, st.max);
    w.ones = true;
    return true;
  }
  uint64_t range = (uint64_t)(st.max - st.min) + 1;
  if (range > (uint64_t(1) << 31) || range > 64 * (uint64_t)std::max<int64_t>(c->n, 1024))
    return false;
  w.cnt = s->alloc(4 * range);
  HIP_CHECK(hipMemsetAsync(w.cnt->p, 0, 4 * range, s->stream));
  hipLaunchKernelGGL(k_count_ids, dim3(grid_for(c->n, 256)), dim3(256), 0, s->stream,
                     view_of(c), c->n, st.min, st.max, (uint32_t *)w.cnt->p);
  KERNEL_CHECK();
  memset(&w.map.m, 0, sizeof(w.map.m));
  w.map.m.kind = MAP_DENSE32;
  w.map.m.lo = st.min;
  w.map.m.hi = st.max;
  w.map.m.vals = (unsigned long long *)w.cnt->p;
  w.ones = false;
  return true;
}

// CAPF_HOST_TRACE=1: host-side timestamps of the fused count (diagnostics)
static double host_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
static bool host_trace() {
  static const bool on = getenv("CAPF_HOST_TRACE") != nullptr;
  return on;
}
static double g_trace_t0 = 0;

// acc = (Σ in·out, self-loop term) → the count, on the device
__global__ void k_partial_minus_loops(const unsigned long long *acc, int64_t *out) {
  if (threadIdx.x == 0) *out = (int64_t)(acc[0] - acc[1]);
}

static bool run_chain2(Session *s, const JoinGraph &g, const Chain2 &c, uint64_t *out) {
  const double ta = host_trace() ? host_us() : 0;
  double tb = ta;
  LeafData rel = leaf_data(g.leaves[c.ra]);
  LeafData na = leaf_data(g.leaves[c.sa]), nb = leaf_data(g.leaves[c.sb]),
           nc = leaf_data(g.leaves[c.sc]);
  const Data &R = *rel.data;
  for (int col : {c.u1, c.v1, c.u2, c.v2}) {
    force(R.cols[col]);
    if (R.cols[col]->type != Type::Int64 || R.cols[col]->valid) return false;
  }
  NodeWeights wa, wb, wc;
  if (!node_weights(s, na, c.ya, wa) || !node_weights(s, nb, c.yb, wb) ||
      !node_weights(s, nc, c.yc, wc))
    return false;
  const int64_t lo = wb.map.m.lo, hi = wb.map.m.hi;
  const int64_t len = hi >= lo ? hi - lo + 1 : 0;
  const int64_t n = R.nrows;
  if (len > (int64_t(1) << 31)) return false;
  // per-bin counts must fit uint32: rels × max node multiplicity
  if (!(wa.ones && wc.ones) && n >= (int64_t(1) << 26)) return false;
  if (n >= (int64_t(1) << 32)) return false;
  const bool all_ones = wa.ones && wb.ones && wc.ones;

  // partitioned histograms are indexed by node_mix(b − lo) over 2^k ≥ len counters
  const int64_t hlen = len > 0 ? std::max(len, chain2_hist_len(len)) : 0;
  BufPtr h = s->alloc(8 * std::max<int64_t>(hlen, 1) + 64);
  BufPtr acc = s->alloc(24);  // Σ in·out, self-loops, the dot's done counter
  bool fin_done = false;  // the dot kernel wrote the async count
  C2Spill spill;          // hand-offs P3 left for the dot (partitioned pipeline)
  bool acc_zeroed = false;  // the partitioned pipeline clears acc itself
  uint32_t *h1 = (uint32_t *)h->p;
  uint32_t *h2 = h1 + ((hlen + 15) & ~int64_t(15));  // keep dwordx4 alignment
  int64_t dot_len = len;
  if (len > 0) {
    Chain2Args a;
    a.u1 = view_of(R.cols[c.u1]);
    a.v1 = view_of(R.cols[c.v1]);
    a.u2 = view_of(R.cols[c.u2]);
    a.v2 = view_of(R.cols[c.v2]);
    const ColView pc[4] = {a.u1, a.v1, a.u2, a.v2};
    a.n = n;
    a.wa = wa.map.m;
    a.wb = wb.map.m;
    a.wc = wc.map.m;
    a.lo = lo;
    a.hi = hi;
    a.h1 = h1;
    a.h2 = h2;
    a.loops = (unsigned long long *)acc->p + 1;
    a.mixed = 0;
    a.mix = node_mix_for(0);
    const char *mode = getenv("CAPF_CHAIN2");  // "atomic" | "partitioned" (default: by size)
    const bool want_part = all_ones && wa.map.m.lo == lo && wc.map.m.lo == lo &&
                           wa.map.m.hi == hi && wc.map.m.hi == hi &&
                           (mode ? strcmp(mode, "partitioned") == 0 : n >= (int64_t(1) << 22));
    bool in_range = true;  // column statistics (cached): all endpoint ids inside [lo, hi]
    for (int col : {c.u1, c.v1, c.u2, c.v2}) {
      const ColStats &st = column_stats(s, R.cols[col]);
      in_range = in_range && st.min >= lo && st.max <= hi;
    }
    tb = host_trace() ? host_us() : 0;
    // the count (Σ − loops) straight into the async slot or the pinned host
    // scalar (no D2H copy; polling that word instead of the stream wait
    // measured no gain at s24: 1.111 vs 1.107 ms)
    int64_t *fin = s->async_out ? s->async_out : s->h_scalars;
    spill.fin = fin;
    if (n > 0 && want_part &&
        chain2_partitioned(s, pc, n, lo, hi, in_range, h1, h2, (unsigned long long *)acc->p, &spill)) {
      dot_len = chain2_hist_len(len);  // every counter written; loops accumulated on the device
      acc_zeroed = true;
    } else {
      HIP_CHECK(hipMemsetAsync(acc->p, 0, 24, s->stream));
      acc_zeroed = true;
      HIP_CHECK(hipMemsetAsync(h->p, 0, 8 * std::max<int64_t>(hlen, 1) + 64, s->stream));
      if (n > 0) {
        KernelTimer kt(s, "chain2_hist", 16.0 * n);
        unsigned grid = grid_for(n, 256, 256 * 32);
        if (all_ones)
          hipLaunchKernelGGL(k_chain2_hist<true>, dim3(grid), dim3(256), 0, s->stream, a);
        else
          hipLaunchKernelGGL(k_chain2_hist<false>, dim3(grid), dim3(256), 0, s->stream, a);
        KERNEL_CHECK();
      }
    }
    {
      KernelTimer kt(s, "chain2_dot", 8.0 * dot_len);
      // one block per CU (s24: 256 blocks 24 µs, 2048 37 µs — same-address atomics)
      unsigned grid = grid_for(dot_len / 4 + 1, 256, dot_grid(s->num_cus));
      unsigned int *done = (unsigned int *)((unsigned long long *)acc->p + 2);
      if (spill.split)  // the bucket layout of the partitioned pipeline (+1 block: hand-offs)
        // 256-lane groups: 4 quads in flight per lane, ~4 waves per CU (512 / 1024: no gain)
        hipLaunchKernelGGL(k_chain2_dot_pairs, dim3(dot_grid(s->num_cus) + C2_HO_BLOCKS), dim3(256), 0, s->stream, h1,
                           h2, spill, (unsigned long long *)acc->p, fin, done);
      else if (wb.ones)  // ONES: Σ in·out is invariant under the node_mix bijection (+1 block: hand-offs)
        hipLaunchKernelGGL(k_chain2_dot<true>, dim3(grid + (spill.n ? C2_HO_BLOCKS : 0)), dim3(256), 0, s->stream, h1, h2,
                           wb.map.m, lo, dot_len, (unsigned long long *)acc->p, fin, done, spill);
      else
        hipLaunchKernelGGL(k_chain2_dot<false>, dim3(grid), dim3(256), 0, s->stream, h1, h2,
                           wb.map.m, lo, dot_len, (unsigned long long *)acc->p, fin, done);
      KERNEL_CHECK();
      fin_done = true;
    }
  }
  if (!acc_zeroed) HIP_CHECK(hipMemsetAsync(acc->p, 0, 24, s->stream));  // empty node range
  const double tc = host_trace() ? host_us() : 0;
  if (s->async_out) {  // capf_table_count_async: total − loops on the device, no wait
    if (!fin_done) {
      hipLaunchKernelGGL(k_partial_minus_loops, dim3(1), dim3(64), 0, s->stream,
                         (const unsigned long long *)acc->p, s->async_out);
      KERNEL_CHECK();
    }
    *out = 0;
    return true;
  }
  if (s->profiling && spill.n) {  // diagnostics (profiling mode only): hand-off log entries
    uint32_t ne = 0;
    HIP_CHECK(hipMemcpyAsync(&ne, spill.n, 4, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    s->profile["c3_handoffs"].bytes += (double)ne;
  }
  if (fin_done) {
    s->sync();
    *out = (uint64_t)s->h_scalars[0];
  } else {
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, acc->p, 16, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    *out = (uint64_t)s->h_scalars[0] - (uint64_t)s->h_scalars[1];
  }
  if (host_trace())
    fprintf(stderr, "[capf host] analyse %.1f us, weights+stats %.1f us, launches %.1f us, wait %.1f us\n",
            ta - g_trace_t0, tb - ta, tc - tb, host_us() - tc);
  return true;
}

// The triangle on the GPU (triangle.hip) when the three node scans are one
// dense unique id range and the rel ids are unique (r_i = r_j ⇔ same row).
static bool run_triangle(Session *s, const JoinGraph &g, const Tri &t, uint64_t *out) {
  LeafData rel = leaf_data(g.leaves[t.rel]);
  const Data &R = *rel.data;
  for (int col : {t.src, t.dst, t.idcol}) {
    force(R.cols[col]);
    if (R.cols[col]->type != Type::Int64 || R.cols[col]->valid) return false;
  }
  const ColStats &ids = column_stats(s, R.cols[t.idcol]);
  if (!(ids.dense_unique && ids.non_null == R.nrows) && R.nrows > 1) return false;
  NodeWeights w[3];
  for (int k = 0; k < 3; ++k) {
    LeafData nd = leaf_data(g.leaves[t.nodes[k]]);
    if (!node_weights(s, nd, t.ycol[k], w[k]) || !w[k].ones) return false;
    if (w[k].map.m.lo != w[0].map.m.lo || w[k].map.m.hi != w[0].map.m.hi) return false;
  }
  const int64_t lo = w[0].map.m.lo, hi = w[0].map.m.hi;
  const int64_t len = hi >= lo ? hi - lo + 1 : 0;
  if (len > (int64_t(1) << 31) || R.nrows >= (int64_t(1) << 32)) return false;
  BufPtr acc = s->alloc(16);
  int64_t *dst = s->async_out ? s->async_out : (int64_t *)acc->p;
  if (len > 0 && R.nrows > 0) {
    triangle_count_async(s, R.cols[t.src], R.cols[t.dst], R.nrows, lo,
                         (uint64_t)len, 1, 0, dst);
  } else {
    HIP_CHECK(hipMemsetAsync(dst, 0, 8, s->stream));
  }
  if (s->async_out) {
    *out = 0;
    return true;
  }
  HIP_CHECK(hipMemcpyAsync(s->h_scalars, acc->p, 8, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  *out = (uint64_t)s->h_scalars[0];
  return true;
}

// *dst = Σ_mask (−1)^|mask| · term[mask] (inclusion–exclusion, exact in
// two's complement)
__global__ void k_signed_terms(const unsigned long long *term, int k, int64_t *dst) {
  if (threadIdx.x != 0) return;
  unsigned long long t = 0;
  for (int mask = 0; mask < (1 << k); ++mask)
    t += (__popc(mask) & 1) ? (0ull - term[mask]) : term[mask];
  *dst = (int64_t)t;
}

bool try_fused_count(const NodePtr &n, int64_t *out) {
  if (host_trace()) g_trace_t0 = host_us();
  Session *s = n->s;
  {
    std::lock_guard<std::mutex> lk(n->mu);
    if (n->result) return false;
  }
  if (n->kind != Kind::Join && n->kind != Kind::Filter && n->kind != Kind::Select) return false;
  JoinGraph g;
  std::vector<ColRef> cols;
  if (!collect(n, g, cols)) return false;
  if (g.eqs.empty()) return false;  // no join: nothing to fuse
  if (g.neqs.size() > 4) return false;
  Chain2 c2;
  if (match_chain2(g, c2)) {
    uint64_t r;
    if (run_chain2(s, g, c2, &r)) {
      s->last_plan = "fused_chain2";
      *out = (int64_t)r;
      return true;
    }
  }
  Tri tri;
  if (match_triangle(g, tri)) {
    uint64_t r;
    if (run_triangle(s, g, tri, &r)) {
      s->last_plan = "fused_triangle";
      *out = (int64_t)r;
      return true;
    }
  }
  // general: inclusion–exclusion over the uniqueness predicates.  Every term
  // is counted into its own device slot; one kernel forms Σ ±term on the
  // device (into the async slot, or one download at the end)
  const int k = (int)g.neqs.size();
  std::vector<JoinGraph> terms(1 << k);
  for (int mask = 0; mask < (1 << k); ++mask) {
    std::vector<int> subset;
    for (int b = 0; b < k; ++b)
      if (mask >> b & 1) subset.push_back(b);
    if (!apply_equalities(g, subset, terms[mask])) return false;
  }
  BufPtr slots = s->alloc(8 * (1 << k) + 8);
  HIP_CHECK(hipMemsetAsync(slots->p, 0, 8 * (1 << k) + 8, s->stream));
  unsigned long long *d_slots = (unsigned long long *)slots->p;
  for (int mask = 0; mask < (1 << k); ++mask)
    if (!tree_count(s, terms[mask], d_slots + mask)) {
      s->sync();  // kernels of earlier terms may still read their maps
      return false;
    }
  int64_t *dst = s->async_out ? s->async_out : (int64_t *)(d_slots + (1 << k));
  hipLaunchKernelGGL(k_signed_terms, dim3(1), dim3(64), 0, s->stream,
                     (const unsigned long long *)d_slots, k, dst);
  KERNEL_CHECK();
  s->last_plan = "message_passing";
  if (s->async_out) {
    *out = 0;
    return true;
  }
  HIP_CHECK(hipMemcpyAsync(s->h_scalars, dst, 8, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  *out = (int64_t)s->h_scalars[0];
  return true;
}


// ============================================================ fused reach
// Config 5 below the Table SPI.  The unchanged okapi front end lowers
//   MATCH (a)-[:T*1..u]->(b) WITH DISTINCT a, b WITH a, count(*) AS reach
// into (DirectedVarLengthExpandPlanner, VarLengthExpandPlanner.scala:82-259;
// Distinct RelationalOperator.scala:325-332; Aggregate :334-346)
//   Group(a-columns; count(*))
//     ← [column copies] ← Distinct(a-columns, b-columns) ← [column copies]
//     ← UNION ALL over k = 1..u of
//         S_a ⋈[a = start(e1)] E ⋈[end(e1) = start(e2)] E … E ⋈[end(ek) = b] S_b
//         → Filter(NOT(e_i = e_j)) → withColumns(NULL padding)
// which would materialise every path (~1e10 rows at SF10).  When the DAG has
// exactly this shape, the Group is evaluated by the multi-source BFS of
// var_length_reach.hip instead — CAPF's Calcite rule set plays the same
// physical-choice role (flink-cypher/.../api/CAPFSession.scala:83-91).
// Exact for lower bound 1 (directed): the DISTINCT (a, b) pairs of
// relationship-isomorphic paths of length 1..u are exactly the pairs joined by
// a walk of length 1..u (cutting the closed sub-walk between two uses of a rel
// leaves a shorter walk with the same endpoints), so the isomorphism filters
// do not change the answer.  Group keys other than a's id must be columns of
// S_a (functions of the unique id) or literals; DISTINCT columns columns of
// S_a / S_b or literals.  Any other shape returns false (relational path).

static bool prog_eq(const Program &a, const Program &b) {
  if (a.code.size() != b.code.size() || a.names != b.names) return false;
  for (size_t i = 0; i < a.code.size(); ++i)
    if (a.code[i].op != b.code[i].op || a.code[i].i != b.code[i].i ||
        __builtin_bit_cast(uint64_t, a.code[i].f) != __builtin_bit_cast(uint64_t, b.code[i].f))
      return false;
  return true;
}

static bool progs_eq(const std::vector<Program> &a, const std::vector<Program> &b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!prog_eq(a[i], b[i])) return false;
  return true;
}

// A tracked column: index in the current node, or a literal.
struct TCol {
  int col = -1;
  const Program *lit = nullptr;
};

static bool reach_reject(const char *why) {
  static const bool trace = getenv("CAPF_TRACE_FUSE") && atoi(getenv("CAPF_TRACE_FUSE")) == 1;
  if (trace) fprintf(stderr, "[capf] fused reach not applied: %s\n", why);
  return false;
}

static bool is_literal_program(const Program &p) { return p.code.size() == 1 && p.code[0].op != OP_COL; }

// Descends through column-mapping operators (Select; withColumns whose
// expressions are column copies or literals), re-expressing the tracked
// columns; returns the first other node.
static NodePtr through_mappings(NodePtr n, std::vector<TCol> &cols) {
  for (;;) {
    if (n->kind == Kind::Select) {
      for (auto &c : cols)
        if (!c.lit) c.col = n->sel_index[c.col];
      n = n->kids[0];
      continue;
    }
    if (n->kind == Kind::WithColumns) {
      for (auto &p : n->exprs)
        if (p.code.size() != 1) return n;
      const NodePtr &kid = n->kids[0];
      for (auto &c : cols) {
        if (c.lit) continue;
        int k = -1;
        for (size_t t = 0; t < n->target_index.size(); ++t)
          if (n->target_index[t] == c.col) k = (int)t;
        if (k < 0) continue;  // passes through at the same index
        const Program &p = n->exprs[k];
        if (is_literal_program(p)) {
          c.lit = &p;
          c.col = -1;
        } else {
          const int64_t ni = p.code[0].i;
          if (ni < 0 || (size_t)ni >= p.names.size()) return n;
          c.col = kid->col_index(p.names[(size_t)ni]);
          if (c.col < 0) return n;
        }
      }
      n = kid;
      continue;
    }
    return n;
  }
}

struct ReachBranch {
  NodePtr base;
  std::vector<TCol> cols;
};

static bool union_branches(NodePtr n, std::vector<TCol> cols, std::vector<ReachBranch> &out) {
  n = through_mappings(n, cols);
  if (n->kind != Kind::Union) {
    out.push_back(ReachBranch{n, cols});
    return out.size() <= 64;
  }
  std::vector<TCol> rc = cols;
  for (auto &c : rc)
    if (!c.lit) {
      c.col = n->kids[1]->col_index(n->names[c.col]);
      if (c.col < 0) return false;
    }
  return union_branches(n->kids[0], cols, out) && union_branches(n->kids[1], rc, out);
}

// One branch's role of a tracked column.
struct RCol {
  int role = -1;  // 0: S_a column, 1: S_b column, 2: literal
  int col = -1;
  Program lit;     // role 2 (a copy: the branch's join graph is temporary)
};

struct ReachShape {
  Leaf sa, sb, rel;
  int x = -1, y = -1, cs = -1, cd = -1;  // S_a / S_b id columns, rel start / end columns
  int k = 0;                              // rel leaves in the chain
  std::vector<RCol> roles;                // per tracked column
};

static bool leaf_eq(const Leaf &a, const Leaf &b) {
  return a.node == b.node && progs_eq(a.filters, b.filters) && a.col_eqs == b.col_eqs;
}

// The chain S_a ⋈ E ⋈ … ⋈ E ⋈ S_b of one branch; `a_cols` are tracked columns
// that must lie on S_a (the group keys).
static bool reach_branch(const ReachBranch &br, const std::vector<int> &a_cols, ReachShape &sh) {
  JoinGraph g;
  std::vector<ColRef> refs;
  if (br.base->kind != Kind::Join && br.base->kind != Kind::Filter) return reach_reject("branch check 1");
  if (!collect(br.base, g, refs)) return reach_reject("branch check 2");
  const int L = (int)g.leaves.size();
  if (L < 3 || (int)g.eqs.size() != L - 1) return reach_reject("branch check 3");
  // tracked column → (leaf, col) or literal
  std::vector<ColRef> tr(br.cols.size());
  std::vector<const Program *> tl(br.cols.size(), nullptr);
  for (size_t i = 0; i < br.cols.size(); ++i) {
    if (br.cols[i].lit) {
      tl[i] = br.cols[i].lit;
      continue;
    }
    tr[i] = refs[br.cols[i].col];
    if (tr[i].leaf == -2 && tr[i].col >= 0) tl[i] = &g.lits[tr[i].col];  // copied into the roles
    else if (tr[i].leaf < 0) return reach_reject("branch check 4");
  }
  int la = -1;
  for (int i : a_cols)
    if (!tl[i]) {
      if (la >= 0 && tr[i].leaf != la) return reach_reject("branch check 5");
      la = tr[i].leaf;
    }
  if (la < 0) return reach_reject("branch check 6");
  auto edges_of = [&](int leaf) {
    std::vector<std::pair<int, ColRef>> r;  // (my col, other)
    for (auto &e : g.eqs) {
      if (e.first.leaf == leaf) r.emplace_back(e.first.col, e.second);
      if (e.second.leaf == leaf) r.emplace_back(e.second.col, e.first);
    }
    return r;
  };
  auto ea = edges_of(la);
  if (ea.size() != 1) return reach_reject("branch check 7");
  sh.sa = g.leaves[la];
  sh.x = ea[0].first;
  int cur = ea[0].second.leaf, entry = ea[0].second.col, prev = la, lb = -1;
  std::vector<char> seen(L, 0);
  seen[la] = 1;
  sh.k = 0;
  sh.cs = entry;
  for (;;) {
    if (cur < 0 || seen[cur]) return reach_reject("branch check 8");
    seen[cur] = 1;
    auto e = edges_of(cur);
    if (e.size() == 1) {  // the far end: S_b
      lb = cur;
      sh.y = entry;
      break;
    }
    if (e.size() != 2) return reach_reject("branch check 9");
    const Leaf &lr = g.leaves[cur];
    if (sh.k == 0) sh.rel = lr;
    else if (!leaf_eq(lr, sh.rel)) return reach_reject("branch check 10");
    if (entry != sh.cs) return reach_reject("branch check 11");
    const auto &out = e[0].second.leaf == prev && e[0].first == entry ? e[1] : e[0];
    if (out.first == entry) return reach_reject("branch check 12");
    if (sh.k == 0) sh.cd = out.first;
    else if (out.first != sh.cd) return reach_reject("branch check 13");
    ++sh.k;
    prev = cur;
    cur = out.second.leaf;
    entry = out.second.col;
  }
  for (int i = 0; i < L; ++i)
    if (!seen[i]) return reach_reject("branch check 14");
  if (sh.k < 1 || lb < 0) return reach_reject("branch check 15");
  sh.sb = g.leaves[lb];
  if (sh.sa.node == sh.rel.node || sh.sb.node == sh.rel.node) return reach_reject("branch check 16");
  if (!sh.rel.col_eqs.empty() || !sh.sa.col_eqs.empty() || !sh.sb.col_eqs.empty()) return reach_reject("branch check 17");
  // isomorphism filters: NOT(e_i = e_j) on one unique rel column
  for (auto &ne : g.neqs) {
    if (ne.first.leaf == ne.second.leaf || ne.first.col != ne.second.col) return reach_reject("branch check 18");
    if (ne.first.leaf == la || ne.first.leaf == lb || ne.second.leaf == la || ne.second.leaf == lb)
      return reach_reject("branch check 19");
    if (!column_unique(sh.rel.node, ne.first.col)) return reach_reject("branch check 20");
  }
  // roles of the tracked columns
  sh.roles.assign(br.cols.size(), RCol{});
  for (size_t i = 0; i < br.cols.size(); ++i) {
    RCol &r = sh.roles[i];
    if (tl[i]) {
      r.role = 2;
      r.lit = *tl[i];
    } else if (tr[i].leaf == la) {
      r.role = 0;
      r.col = tr[i].col;
    } else if (tr[i].leaf == lb) {
      r.role = 1;
      r.col = tr[i].col;
    } else {
      return reach_reject("branch check 21");
    }
  }
  return true;
}

bool try_fused_reach(const NodePtr &grp, DataPtr &result) {
  const char *fe = getenv("CAPF_FUSED_REACH");  // 0: always the relational plan
  if (fe && atoi(fe) == 0) return false;
  if (grp->kind != Kind::Group || grp->key_index.empty() || grp->aggs.empty()) return false;
  for (auto &a : grp->aggs)
    if (a.kind != CAPF_AGG_COUNT_STAR) return false;
  Session *s = grp->s;
  // group keys → columns of the Distinct
  std::vector<TCol> gk;
  for (int k : grp->key_index) gk.push_back(TCol{k, nullptr});
  NodePtr d = through_mappings(grp->kids[0], gk);
  if (d->kind != Kind::Distinct || d->key_index.empty()) return reach_reject("group input is not a DISTINCT");
  {
    std::lock_guard<std::mutex> lk(d->mu);
    if (d->result) return false;  // already materialised: the plain group is cheap
  }
  // tracked columns below the Distinct: its keys, then the group keys
  std::vector<TCol> tracked;
  for (int k : d->key_index) tracked.push_back(TCol{k, nullptr});
  const size_t nd = tracked.size();
  std::vector<int> gk_at(gk.size(), -1);  // group key → tracked index (−1: literal)
  for (size_t i = 0; i < gk.size(); ++i) {
    if (gk[i].lit) continue;
    gk_at[i] = (int)tracked.size();
    tracked.push_back(TCol{gk[i].col, nullptr});
  }
  std::vector<int> a_cols;
  for (int t : gk_at)
    if (t >= 0) a_cols.push_back(t);
  if (a_cols.empty()) return reach_reject("no group key column");
  std::vector<ReachBranch> brs;
  if (!union_branches(d->kids[0], tracked, brs)) return reach_reject("union branches");
  // lower bound 0: one branch is the copyElement branch (VarLengthExpandPlanner.scala:180-205),
  // S_a itself with b's columns copied from a's — no join below the mappings
  int zero = -1;
  for (size_t b = 0; b < brs.size(); ++b)
    if (brs[b].base->kind != Kind::Join) {
      JoinGraph g0;
      std::vector<ColRef> r0;
      if (collect(brs[b].base, g0, r0) && g0.leaves.size() == 1 && g0.eqs.empty()) {
        if (zero >= 0) return reach_reject("two zero-length branches");
        zero = (int)b;
      }
    }
  const ReachBranch zbr = zero >= 0 ? brs[(size_t)zero] : ReachBranch{};
  if (zero >= 0) brs.erase(brs.begin() + zero);
  if (brs.empty()) return reach_reject("no var-length chain");
  std::vector<ReachShape> shapes(brs.size());
  uint64_t lengths = 0;
  for (size_t b = 0; b < brs.size(); ++b) {
    if (!reach_branch(brs[b], a_cols, shapes[b])) return reach_reject("a branch is not a var-length chain");
    const ReachShape &sh = shapes[b], &s0 = shapes[0];
    if (sh.k > 64 || (lengths >> (sh.k - 1) & 1)) return reach_reject("branch lengths");
    lengths |= uint64_t(1) << (sh.k - 1);
    if (!leaf_eq(sh.sa, s0.sa) || !leaf_eq(sh.sb, s0.sb) || !leaf_eq(sh.rel, s0.rel))
      return reach_reject("branches scan different tables");
    if (sh.x != s0.x || sh.y != s0.y || sh.cs != s0.cs || sh.cd != s0.cd)
      return reach_reject("branches join different columns");
    for (size_t i = 0; i < tracked.size(); ++i) {
      const RCol &r = sh.roles[i], &r0 = s0.roles[i];
      if (r.role != r0.role || r.col != r0.col) return reach_reject("column roles differ across branches");
      if (r.role == 2 && !prog_eq(r.lit, r0.lit)) return reach_reject("literals differ across branches");
    }
  }
  const int upper = 64 - __builtin_clzll(lengths);
  if (lengths != (upper == 64 ? ~uint64_t(0) : (uint64_t(1) << upper) - 1))
    return reach_reject("lengths are not 1..u");
  const ReachShape &sh = shapes[0];
  // DISTINCT over (a, b): both ids among its keys, every key a column of S_a /
  // S_b or a literal; group keys: S_a columns (with the id) or literals
  bool has_x = false, has_y = false;
  for (size_t i = 0; i < nd; ++i) {
    const RCol &r = sh.roles[i];
    has_x |= r.role == 0 && r.col == sh.x;
    has_y |= r.role == 1 && r.col == sh.y;
  }
  bool gx = false;
  for (int t : a_cols) {
    if (sh.roles[t].role == 1) return reach_reject("a group key is a target column");
    gx |= sh.roles[t].role == 0 && sh.roles[t].col == sh.x;
  }
  if (!has_x || !has_y || !gx) return reach_reject("DISTINCT / group keys lack the endpoint ids");
  if (zero >= 0) {  // the copy branch: S_a's leaf, a's columns where the chains have a's / b's
    JoinGraph g0;
    std::vector<ColRef> r0;
    if (!collect(zbr.base, g0, r0) || g0.leaves.size() != 1 || !g0.neqs.empty() || !leaf_eq(g0.leaves[0], sh.sa))
      return reach_reject("the zero-length branch is not the source scan");
    const bool same_scan = leaf_eq(sh.sa, sh.sb);
    for (size_t i = 0; i < tracked.size(); ++i) {
      const RCol &r = sh.roles[i];
      const TCol &z = zbr.cols[i];
      const Program *zl = z.lit;
      ColRef zr{-1, -1};
      if (!zl) {
        zr = r0[(size_t)z.col];
        if (zr.leaf == -2 && zr.col >= 0) zl = &g0.lits[(size_t)zr.col];
      }
      if (r.role == 2) {
        if (!zl || !prog_eq(*zl, r.lit)) return reach_reject("zero-length branch: a literal differs");
        continue;
      }
      if (zl || zr.leaf != 0) return reach_reject("zero-length branch: a column is not the source's");
      const int want = r.role == 0 ? r.col : r.col == sh.y ? sh.x : same_scan ? r.col : -1;
      if (want < 0 || zr.col != want) return reach_reject("zero-length branch: b's column is not a's");
    }
  }
  if (!column_unique(sh.sa.node, sh.x) || !column_unique(sh.sb.node, sh.y))
    return reach_reject("endpoint ids not unique");
  // rel endpoint columns: non-null INTEGER
  LeafData lr = leaf_data(sh.rel), la = leaf_data(sh.sa), lb = leaf_data(sh.sb);
  const ColPtr &rs = lr.data->cols[sh.cs], &rd = lr.data->cols[sh.cd];
  const ColPtr &xa = la.data->cols[sh.x], &yb = lb.data->cols[sh.y];
  for (const ColPtr *c : {&rs, &rd, &xa, &yb}) {
    force(*c);
    if ((*c)->type != Type::Int64 || (*c)->valid) return reach_reject("nullable or non-INTEGER ids");
  }
  if (lr.data->nrows >= (int64_t(1) << 32)) return reach_reject("more than 2^32 rels");
  DataPtr res = var_length_reach_rows(s, rs, rd, lr.data->nrows, xa, la.data->nrows, yb,
                                      lb.data->nrows, upper, zero >= 0);
  s->last_plan = "fused_var_length_reach";
  // output: group keys (a's id, other S_a columns gathered by a's row, literals)
  // then one reach column per count(*)
  const int64_t nr = res->nrows;
  auto out = std::make_shared<Data>();
  out->nrows = nr;
  bool need_rows = false;
  for (int t : a_cols) need_rows |= sh.roles[t].role == 0 && sh.roles[t].col != sh.x;
  DataPtr a_rows;  // S_a's columns at each result row
  std::vector<ColPtr> rcols = res->cols;
  if (need_rows && nr > 0) {
    Data l;
    l.nrows = nr;
    l.cols = {res->cols[0]};
    JoinPairs jp;
    const std::vector<std::pair<int, int>> keys = {{0, sh.x}};
    if (!dense_join(s, l, *la.data, keys, CAPF_JOIN_INNER, jp))
      jp = hash_join(s, l, *la.data, keys, CAPF_JOIN_INNER);
    if (jp.n != nr) fail(CAPF_ERR_INTERNAL, "fused reach: source rows lost");
    IdxCache cache;
    if (jp.left)
      for (auto &c : rcols) c = gather_lazy(s, c, jp.left, nr, false, &cache, jp.iw);
    a_rows = std::make_shared<Data>();
    a_rows->nrows = nr;
    for (size_t j = 0; j < la.data->cols.size(); ++j) {
      const ColPtr &c = la.data->cols[j];
      if (jp.build_unread == 2)  // S_a holds its key and constants only: no row index
        a_rows->cols.push_back((int)j == sh.x ? rcols[0] : const_column(s, c->is_const ? *c : *c->lazy->src, nr));
      else
        a_rows->cols.push_back(jp.right ? gather_lazy(s, c, jp.right, nr, false, &cache, jp.iw) : c);
    }
  }
  for (size_t i = 0; i < gk.size(); ++i) {
    const Type t = grp->types[i];
    if (gk_at[i] < 0) {
      Data e;
      e.nrows = nr;
      out->cols.push_back(eval_program(s, *gk[i].lit, {}, e, t));
      continue;
    }
    const RCol &r = sh.roles[gk_at[i]];
    if (r.role == 2) {  // a literal in every branch (a constant label column)
      Data e;
      e.nrows = nr;
      out->cols.push_back(eval_program(s, r.lit, {}, e, t));
      continue;
    }
    out->cols.push_back(r.col == sh.x ? rcols[0] : a_rows->cols[r.col]);
  }
  for (size_t k = 0; k < grp->aggs.size(); ++k) out->cols.push_back(rcols[1]);
  result = out;
  return true;
}
}  // namespace capf

// ===================================================================== C-ABI
using namespace capf;

extern "C" int64_t capf_chain2_hist_len(int64_t n_nodes) {
  return n_nodes > 0 && n_nodes <= (int64_t(1) << 31) ? chain2_hist_len(n_nodes) : 0;
}

extern "C" capf_status capf_chain2_local_hists(capf_session *cs, capf_table *rels,
                                               const char *src_col, const char *dst_col,
                                               int64_t node_base, int64_t n_nodes,
                                               uint32_t *d_in_hist, uint32_t *d_out_hist,
                                               int64_t *self_loops) {
  try {
    if (!cs || !rels || !src_col || !dst_col || !d_in_hist || !d_out_hist || !self_loops)
      illegal("null argument");
    if (n_nodes <= 0 || n_nodes > (int64_t(1) << 31)) illegal("node count out of range");
    Session *s = &cs->impl;
    const NodePtr &nd = rels->node;
    int si = nd->col_index_or_throw(src_col), di = nd->col_index_or_throw(dst_col);
    DataPtr d = materialize(nd);
    const ColPtr &src = d->cols[si], &dst = d->cols[di];
    force(src);
    force(dst);
    if (src->type != Type::Int64 || dst->type != Type::Int64 || src->valid || dst->valid)
      illegal("chain2_local_hists needs non-null INTEGER endpoint columns");
    if (d->nrows >= (int64_t(1) << 32)) not_impl("more than 2^32 rels per rank");
    const int64_t hlen = chain2_hist_len(n_nodes);
    BufPtr acc = s->alloc(24);  // [Σ (unused), self-loops, done]
    HIP_CHECK(hipMemsetAsync(acc->p, 0, 24, s->stream));
    Chain2Args a;
    a.u1 = a.u2 = view_of(src);
    a.v1 = a.v2 = view_of(dst);
    a.n = d->nrows;
    a.wa = a.wb = a.wc = ones_map(node_base, node_base + n_nodes - 1).m;
    a.lo = node_base;
    a.hi = node_base + n_nodes - 1;
    a.h1 = d_in_hist;
    a.h2 = d_out_hist;
    a.loops = (unsigned long long *)acc->p + 1;
    a.mixed = 1;
    a.mix = node_mix_for(chain2_hist_bits(n_nodes));
    const char *mode = getenv("CAPF_CHAIN2");
    const bool want_part = mode ? strcmp(mode, "partitioned") == 0 : a.n >= (int64_t(1) << 22);
    const ColView pc[4] = {a.u1, a.v1, a.u2, a.v2};
    const ColStats &ss = column_stats(s, src), &sd = column_stats(s, dst);
    const bool in_range = ss.min >= a.lo && ss.max <= a.hi && sd.min >= a.lo && sd.max <= a.hi;
    const bool done = want_part && chain2_partitioned(s, pc, a.n, a.lo, a.hi, in_range, a.h1,
                                                      a.h2, (unsigned long long *)acc->p);
    if (!done) {
      HIP_CHECK(hipMemsetAsync(d_in_hist, 0, 4 * hlen, s->stream));
      HIP_CHECK(hipMemsetAsync(d_out_hist, 0, 4 * hlen, s->stream));
      if (a.n > 0) {
        KernelTimer kt(s, "chain2_hist", 16.0 * a.n);
        hipLaunchKernelGGL(k_chain2_hist<true>, dim3(grid_for(a.n, 256, 256 * 32)), dim3(256), 0,
                           s->stream, a);
        KERNEL_CHECK();
      }
    }
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, acc->p, 16, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    *self_loops = s->h_scalars[1];
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}

extern "C" capf_status capf_chain2_sharded_count(capf_session *cs, capf_table *in_copy,
                                                 const char *in_dst, capf_table *out_copy,
                                                 const char *out_src, const char *out_dst,
                                                 int64_t node_base, int64_t n_nodes,
                                                 int32_t parts, int32_t part, int64_t *d_partial) {
  return capf_chain2_sharded_count_diag(cs, in_copy, in_dst, out_copy, out_src, out_dst, -1, 0, nullptr,
                                        node_base, n_nodes, parts, part, d_partial);
}

extern "C" capf_status capf_chain2_sharded_count_diag(capf_session *cs, capf_table *in_copy,
                                                      const char *in_dst, capf_table *out_copy,
                                                      const char *out_src, const char *out_dst,
                                                      int64_t n_diag, int32_t n_hot,
                                                      const int64_t *hot_ids, int64_t node_base,
                                                      int64_t n_nodes, int32_t parts, int32_t part,
                                                      int64_t *d_partial) {
  try {
    if (!cs || !in_copy || !out_copy || !in_dst || !out_src || !out_dst || !d_partial)
      illegal("null argument");
    if (n_nodes <= 0 || n_nodes > (int64_t(1) << 31)) illegal("node count out of range");
    if (parts <= 0 || part < 0 || part >= parts) illegal("part out of range");
    Session *s = &cs->impl;
    DataPtr di = materialize(in_copy->node), dout = materialize(out_copy->node);
    const ColPtr &a = di->cols[in_copy->node->col_index_or_throw(in_dst)];
    const ColPtr &b = dout->cols[out_copy->node->col_index_or_throw(out_src)];
    const ColPtr &c = dout->cols[out_copy->node->col_index_or_throw(out_dst)];
    for (const ColPtr *x : {&a, &b, &c})
      if (force(*x), (*x)->type != Type::Int64 || (*x)->valid)
        illegal("sharded 2-hop count needs non-null INTEGER endpoint columns");
    const ColView cols[3] = {view_of(a), view_of(b), view_of(c)};
    // both key columns came out of capf_table_node_partition for this very
    // (range, parts, part): every key is an owned node — no per-key tests
    auto owned = [&](const ColPtr &x) {
      return x->owner[3] == part && x->owner[0] == node_base && x->owner[1] == n_nodes && x->owner[2] == parts;
    };
    const bool trusted = owned(a) && owned(b);
    if (!chain2_sharded(s, cols, di->nrows, dout->nrows, node_base, n_nodes, parts, part,
                        d_partial, n_diag, n_hot, hot_ids, trusted))
      not_impl("sharded 2-hop count: shape outside the kernel's limits (buckets per rank, "
               "rows per copy < 2^31, mixed encodings)");
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}

extern "C" capf_status capf_triangle_count_part(capf_session *cs, capf_table *rels,
                                                const char *src_col, const char *dst_col,
                                                int64_t node_base, int64_t n_nodes, int32_t parts,
                                                int32_t part, int64_t *d_count) {
  try {
    if (!cs || !rels || !src_col || !dst_col || !d_count) illegal("null argument");
    if (n_nodes <= 0 || n_nodes > (int64_t(1) << 31)) illegal("node count out of range");
    if (parts <= 0 || part < 0 || part >= parts) illegal("part out of range");
    Session *s = &cs->impl;
    const NodePtr &nd = rels->node;
    DataPtr d = materialize(nd);
    const ColPtr &a = d->cols[nd->col_index_or_throw(src_col)];
    const ColPtr &b = d->cols[nd->col_index_or_throw(dst_col)];
    force(a);
    force(b);
    if (a->type != Type::Int64 || b->type != Type::Int64 || a->valid || b->valid)
      illegal("triangle count needs non-null INTEGER endpoint columns");
    if (d->nrows >= (int64_t(1) << 32)) not_impl("more than 2^32 rels");
    if (d->nrows == 0) {
      HIP_CHECK(hipMemsetAsync(d_count, 0, 8, s->stream));
      return CAPF_OK;
    }
    triangle_count_async(s, a, b, d->nrows, node_base, (uint64_t)n_nodes, parts,
                         part, d_count);
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}

extern "C" capf_status capf_dot_u32(capf_session *cs, const uint32_t *d_a, const uint32_t *d_b,
                                    int64_t n, uint64_t *out) {
  try {
    if (!cs || !d_a || !d_b || !out) illegal("null argument");
    Session *s = &cs->impl;
    BufPtr acc = s->alloc(8);
    HIP_CHECK(hipMemsetAsync(acc->p, 0, 8, s->stream));
    if (n > 0) {
      if (((uintptr_t)d_a | (uintptr_t)d_b) & 15) illegal("dot operands must be 16-B aligned");
      KernelTimer kt(s, "chain2_dot", 8.0 * n);
      hipLaunchKernelGGL(k_chain2_dot<true>, dim3(grid_for(n / 4 + 1, 256, 256 * 8)), dim3(256),
                         0, s->stream, d_a, d_b, ones_map(0, n - 1).m, (int64_t)0, n,
                         (unsigned long long *)acc->p);
      KERNEL_CHECK();
    }
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, acc->p, 8, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    *out = (uint64_t)s->h_scalars[0];
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}
