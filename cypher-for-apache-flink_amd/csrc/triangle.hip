// triangle.hip — fused count of the directed triangle
//   MATCH (a)-->(b)-->(c)-->(a) RETURN count(*)
// i.e. the okapi plan Expand, Expand, ExpandInto (RelationalPlanner.scala:
// 130-189: the closing edge is a join on TWO keys, start = c and end = a)
// followed by the pairwise uniqueness filter r1 <> r2, r1 <> r3, r2 <> r3.
//
// The relational plan materialises the wedge table (~1.3e12 rows at R-MAT
// s24) before the closing join.  Here the count comes from the multiplicity
// matrix A (A[x][y] = #rels x -> y) without any wedge row:
//
//   count = 3·T + 3·Σ_{pairs {x,y}, x≠y} (L[x] + L[y])·A[x][y]·A[y][x]
//           + Σ_x L[x](L[x]−1)(L[x]−2)
//
// T  = Σ over node triples {p, q, w}, all distinct, of the directed 3-cycles
//      p→q→w→p and p→w→q→p weighted by multiplicities (each triple once; the
//      factor 3 = the rotations (a, b, c) of one cycle);
// L  = self-loops per node: a walk with exactly one self-loop (a→a→c→a and its
//      rotations) has distinct rels automatically; three self-loops at one
//      node need three distinct rels.
// oracle/cmodel.py restates the same count as trace(A³) − Σ_x (L³ − L(L−1)(L−2))
// and by brute force over rels.
//
// T uses the degree-ordered "forward" algorithm: every distinct node pair
// {u, v} becomes ONE oriented edge p→q from the lower to the higher (degree,
// id) rank, carrying f = A[p][q] and b = A[q][p]; every triangle is found once,
// at its lowest-rank vertex p, as q, w ∈ N+(p) with w ∈ N+(q).
//
// Kernels:
//   keys   (min, max, dir) 63-bit key per non-loop rel, loops counted per node
//   sort   rocprim radix sort + run-length encode → distinct (pair, dir) runs
//   pairs  merge the two directions of a pair, degrees (atomics)
//   orient (p << 32 | q) key, (f, b) value, loop term; radix sort → CSR
//          (binary-search row pointers)
//   count  one wave per row p (rows handed out in chunks by an atomic
//          cursor): N+(p) staged in LDS, lanes walk N+(q) for each q ∈ N+(p)
//          and binary-search each w in the LDS copy
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr uint64_t TRI_NONE = ~0ull;

// (u, v, dir) key of a non-loop rel inside [lo, lo + len); loops → L[x]++.
__global__ void k_tri_keys(ColView s, ColView d, int64_t m, int64_t lo, uint64_t len,
                           uint64_t *keys, uint32_t *loops) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t x = (uint64_t)(ld_int(s, i) - lo), y = (uint64_t)(ld_int(d, i) - lo);
    uint64_t k = TRI_NONE;
    if (x < len && y < len) {
      if (x == y) {
        atomicAdd(&loops[x], 1u);
      } else {
        const uint64_t u = min(x, y), v = max(x, y);
        k = (u << 32) | (v << 1) | (x > y ? 1u : 0u);
      }
    }
    keys[i] = k;
  }
}

// Runs of equal (pair, dir) keys → one entry per distinct pair.  Run j emits
// its pair if it is the pair's first run; the pair's other direction, if
// present, is run j + 1.  Degrees count distinct neighbours.
__global__ void k_tri_pairs(const uint64_t *ukeys, const uint32_t *cnt, const uint32_t *nruns,
                            uint32_t *deg, uint64_t *pair_uv, uint2 *pair_fb) {
  const uint32_t nr = *nruns;
  const int lane = lane_id();
  const uint32_t stride = gridDim.x * blockDim.x;
  // whole waves per step: the degree of u is aggregated over the wave (a hub's
  // pairs are consecutive in the sorted order and would serialise on deg[u])
  for (uint32_t j0 = blockIdx.x * blockDim.x + (threadIdx.x & ~(WAVE - 1)); j0 < nr; j0 += stride) {
    const uint32_t j = j0 + lane;
    bool emit = false;
    uint32_t u = 0xFFFFFFFFu, v = 0;
    if (j < nr) {
      const uint64_t k = ukeys[j];
      const uint64_t pr = k >> 1;
      if (k == TRI_NONE || (j > 0 && (ukeys[j - 1] >> 1) == pr)) {
        pair_uv[j] = TRI_NONE;  // dropped rels / second direction merged into run j − 1
      } else {
        uint32_t f = 0, b = 0;
        if (k & 1) {
          b = cnt[j];
        } else {
          f = cnt[j];
          if (j + 1 < nr && ukeys[j + 1] != TRI_NONE && (ukeys[j + 1] >> 1) == pr) b = cnt[j + 1];
        }
        u = (uint32_t)(pr >> 31);
        v = (uint32_t)(pr & 0x7FFFFFFFu);
        pair_uv[j] = ((uint64_t)u << 32) | v;
        pair_fb[j] = make_uint2(f, b);  // f = #(u→v), b = #(v→u)
        emit = true;
      }
    }
    const uint32_t key = emit ? u : 0xFFFFFFFFu;
    const uint32_t prev = __shfl_up(key, 1, WAVE);
    const bool head = lane == 0 || key != prev;
    const unsigned long long heads = __ballot(head);
    const unsigned long long above = lane == WAVE - 1 ? 0ull : heads & ~((2ull << lane) - 1);
    const int next = above ? __ffsll((long long)above) - 1 : WAVE;
    if (emit && head) atomicAdd(&deg[u], (uint32_t)(next - lane));
    if (emit) atomicAdd(&deg[v], 1u);
  }
}

// Orient each pair from the lower to the higher (degree, id) rank; the loop
// term Σ (L[u] + L[v])·f·b goes to acc[1].
__global__ void k_tri_orient(const uint64_t *pair_uv, const uint2 *pair_fb, const uint32_t *nruns,
                             const uint32_t *deg, const uint32_t *loops, uint64_t *okey, uint64_t *oval,
                             unsigned long long *acc) {
  __shared__ unsigned long long lds[17];
  const uint32_t nr = *nruns;
  unsigned long long lt = 0;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nr; j += gridDim.x * blockDim.x) {
    const uint64_t uv = pair_uv[j];
    if (uv == TRI_NONE) {
      okey[j] = TRI_NONE;
      oval[j] = 0;
      continue;
    }
    const uint32_t u = (uint32_t)(uv >> 32), v = (uint32_t)uv;
    const uint2 fb = pair_fb[j];
    const uint64_t ru = ((uint64_t)deg[u] << 32) | u, rv = ((uint64_t)deg[v] << 32) | v;
    const bool fwd = ru < rv;
    const uint32_t p = fwd ? u : v, q = fwd ? v : u;
    const uint32_t f = fwd ? fb.x : fb.y, b = fwd ? fb.y : fb.x;  // f = #(p→q), b = #(q→p)
    okey[j] = ((uint64_t)p << 32) | q;
    oval[j] = ((uint64_t)f << 32) | b;
    lt += (unsigned long long)(loops[u] + loops[v]) * f * b;
  }
  unsigned long long tot;
  block_exclusive_scan(lt, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[1], tot);
}

__global__ void k_tri_rowptr(const uint64_t *okey, uint32_t nr, uint64_t len, uint32_t *rowptr) {
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x <= len;
       x += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t lo = 0, hi = nr;
    const uint64_t t = x << 32;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (okey[mid] < t) lo = mid + 1;
      else hi = mid;
    }
    rowptr[x] = lo;
  }
}

__global__ void k_tri_split(const uint64_t *okey, const uint64_t *oval, uint32_t P, uint32_t *cols,
                            uint2 *vals) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x) {
    cols[i] = (uint32_t)okey[i];
    const uint64_t v = oval[i];
    vals[i] = make_uint2((uint32_t)(v >> 32), (uint32_t)v);
  }
}

// Σ_x L(L−1)(L−2) into acc[2].
__global__ void k_tri_loop3(const uint32_t *loops, uint64_t len, unsigned long long *acc) {
  __shared__ unsigned long long lds[17];
  unsigned long long t = 0;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < len;
       x += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long L = loops[x];
    if (L >= 3) t += L * (L - 1) * (L - 2);
  }
  unsigned long long tot;
  block_exclusive_scan(t, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[2], tot);
}

constexpr int TRI_BLOCK = 256;
#ifndef CAPF_TRI_CAP
#define CAPF_TRI_CAP 1024
#endif
constexpr int TRI_CAP = CAPF_TRI_CAP;  // N+(p) staged in LDS up to this many entries
constexpr int TRI_CHUNK = 16;  // rows per cursor grab
// N+(q) entries per lane in flight.  s24 at the round-4 closing kernels (5
// waves/SIMD): ILP 2 308 ms, 3 290, 4 269; before the ids-only copies and the
// pointer-form searches: 2 333, 3 314, 4 322
constexpr int TRI_ILP = 4;

// Index of w in the ascending a(0..n), or −1.
template <class A>
__device__ inline int64_t tri_find(const A &a, int64_t n, uint32_t w) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a(mid) < w) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && a(lo) == w ? lo : -1;
}

struct TriBatch {
  uint32_t pre[WAVE + 1];  // exclusive prefix of the batch's |N+(q)|, + total
  uint32_t qa[WAVE];       // N+(q) start in cols
  uint2 pq[WAVE];          // (#p→q, #q→p)
};

// One row p: its q's are taken 64 at a time and their lists N+(q) are walked
// as ONE flattened sequence (lane = position, found by a 6-step search in the
// batch's prefix table — most lists are far shorter than a wave), TRI_ILP
// positions per lane in flight, each w searched in N+(p) by `find` (the LDS
// copy of a short row, the row in global memory — L2-resident while the wave
// walks it — for a long one).  `qs(k)` = the k-th q of N+(p).
template <int ILP, class Q, class F, class M>
__device__ inline void tri_row(uint32_t a, uint32_t dp, const uint32_t *rowptr, const uint32_t *cols,
                               const uint2 *vals, TriBatch &tb, Q qs, F find, M maybe,
                               unsigned long long &t, unsigned long long &probes,
                               unsigned long long &hits) {
  const int lane = lane_id();
  for (uint32_t kb = 0; kb < dp; kb += WAVE) {
    // the batch's table: one q per lane
    const uint32_t k = kb + lane;
    uint32_t qa = 0, dq = 0;
    uint2 pq = make_uint2(0, 0);
    if (k < dp) {
      const uint32_t q = qs(k);
      qa = rowptr[q];
      dq = rowptr[q + 1] - qa;
      pq = vals[a + k];
    }
    const uint32_t inc = wave_inclusive_scan(dq);
    tb.pre[lane] = inc - dq;
    if (lane == WAVE - 1) tb.pre[WAVE] = inc;
    tb.qa[lane] = qa;
    tb.pq[lane] = pq;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane(inc, WAVE - 1);
    if (lane == 0) probes += total;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t t0 = 0; t0 < total; t0 += ILP * WAVE) {
      uint32_t w[ILP], pos[ILP], bi[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) {
        const uint32_t x = t0 + u * WAVE + lane;
        uint32_t b = 0;  // last batch entry with pre[b] <= x
#pragma unroll
        for (int st = WAVE / 2; st > 0; st >>= 1)
          if (tb.pre[b + st] <= x) b += st;
        bi[u] = b;
        pos[u] = tb.qa[b] + (x - tb.pre[b]);
        w[u] = x < total ? cols[pos[u]] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int u = 0; u < ILP; ++u) {
        if (w[u] == 0xFFFFFFFFu || !maybe(w[u])) continue;
        const int64_t i = tri_find(find, dp, w[u]);
        if (i >= 0) {
          ++hits;
          const uint2 pqv = tb.pq[bi[u]], qw = vals[pos[u]], pw = vals[a + i];
          // p→q→w→p  +  p→w→q→p
          t += (unsigned long long)pqv.x * qw.x * pw.y + (unsigned long long)pw.x * qw.y * pqv.y;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the table is rewritten by the next batch
  }
}

// T over this part's rows into acc[0]: row chunks of TRI_CHUNK are dealt
// round-robin over the parts (chunk c of the graph belongs to part c mod
// parts) and handed to waves by an atomic cursor.  N+(p) is staged in LDS when
// it has ≤ TRI_CAP entries (tri_row searches the LDS copy), else searched in
// place.  (An LDS hash table instead of the sorted row, 12 KiB per wave,
// measured 1.6× slower: the kernel waits on the N+(q) loads, so occupancy
// wins.)
template <int ILP>
__global__ __launch_bounds__(TRI_BLOCK) void k_tri_count(const uint32_t *rowptr,
                                                          const uint32_t *cols, const uint2 *vals,
                                                          uint64_t len, int parts, int part,
                                                          unsigned long long *cursor,
                                                          unsigned long long *acc) {
  __shared__ uint32_t s_cols[TRI_BLOCK / WAVE][TRI_CAP];
  __shared__ TriBatch s_tab[TRI_BLOCK / WAVE];
  __shared__ unsigned long long lds[17];
  const int wv = threadIdx.x / WAVE, lane = lane_id();
  uint32_t *sc = s_cols[wv];
  TriBatch &tb = s_tab[wv];
  unsigned long long t = 0, probes = 0, hits = 0;
  for (;;) {
    unsigned long long r0 = 0;
    if (lane == 0) r0 = atomicAdd(cursor, 1ull);
    r0 = ((unsigned long long)__shfl((long long)r0, 0, WAVE) * parts + part) * TRI_CHUNK;
    if (r0 >= len) break;
    const uint64_t r1 = min<uint64_t>(r0 + TRI_CHUNK, len);
    for (uint64_t p = r0; p < r1; ++p) {
      const uint32_t a = rowptr[p], dp = rowptr[p + 1] - a;
      if (dp < 2) continue;  // a triangle needs two out-neighbours at its lowest vertex
      if (dp > TRI_CAP) {  // rare long row: searched in global memory
        const uint32_t *row = cols + a;
        tri_row<ILP>(a, dp, rowptr, cols, vals, tb, [&](uint32_t k) { return row[k]; },
                [&](int64_t x) { return row[x]; }, [](uint32_t) { return true; }, t, probes, hits);
        continue;
      }
      for (uint32_t k = lane; k < dp; k += WAVE) sc[k] = cols[a + k];
      __builtin_amdgcn_wave_barrier();
      tri_row<ILP>(a, dp, rowptr, cols, vals, tb, [&](uint32_t k) { return sc[k]; },
              [&](int64_t x) { return sc[x]; }, [](uint32_t) { return true; }, t, probes, hits);
      __builtin_amdgcn_wave_barrier();  // sc is rewritten by the next row
    }
  }
  unsigned long long tot;
  block_exclusive_scan(t, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[0], tot);
  block_exclusive_scan(probes, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[4], tot);
  block_exclusive_scan(hits, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[5], tot);
}

// ------------------------------------------------------------ packed count
// Node ids < 2^24 (R-MAT s ≤ 24): the oriented CSR's column word carries the
// pair's multiplicities in its top byte — f = #(p→q) in bits 24..27, b =
// #(q→p) in bits 28..31, 15 = "look up vals" (rare multi-edges) — so a hit
// needs no dependent global load: p→q from the batch table, q→w from the
// streamed word itself, p→w from the LDS copy of N+(p).
constexpr uint32_t TRI_M24 = 0xFFFFFFu;

__global__ void k_tri_pack(const uint32_t *cols, const uint2 *vals, uint32_t P, uint32_t *pcols) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x) {
    const uint2 v = vals[i];
    // f = 15 sends every reader to vals, so b is then left 0: no word equals
    // 0xFFFFFFFF (id 2^24 − 1 saturated both ways), the kernels' end marker
    const uint32_t f = min(v.x, 15u), b = f == 15u ? 0u : min(v.y, 15u);
    pcols[i] = cols[i] | f << 24 | b << 28;
  }
}

struct TriBatch2 {
  uint32_t pre[WAVE + 1];  // exclusive prefix of the batch's |N+(q)|, + total
  uint32_t qa[WAVE];       // N+(q) start in pcols
  uint8_t pk[WAVE];        // multiplicity nibbles of the pair p–q (the top byte of q's word)
};

// packed word's multiplicity nibbles say "look the pair up in vals"
__device__ inline bool tri_esc(uint32_t word) { return ((word >> 24) & 15u) == 15u || (word >> 28) == 15u; }

// (f, b) of a packed word, or of vals[e] when a nibble says "look it up"
__device__ inline uint2 tri_fb(uint32_t word, const uint2 *vals, uint32_t e) {
  const uint32_t f = (word >> 24) & 15u, b = word >> 28;
  return (f == 15u || b == 15u) ? vals[e] : make_uint2(f, b);
}

// One row p (packed words).  Positions of the flattened N+(q) sequence are
// taken ILP·64 at a time and software-pipelined: the words of step i+1
// (prefix search + global loads) are issued before step i's binary searches,
// in ping-pong registers (no copy, so no early wait on the loads in flight).
// SPLIT (pass A of the two-pass schedule): the edges p→q with |N+(p)| < |N+(q)|
// belong to pass B and are skipped here.  SWAP (pass B): the staged list is
// N+(q) and the streamed lists are N+(p) of q's in-list entries — the roles
// of the two looked-up words swap in the weight.  `pqe(k)`: the vals index of
// the k-th batch entry's p–q pair (for a saturated nibble).  `qrow(k)`: the
// k-th entry's streamed list as {start in pcols, length | p–q nibbles << 24}.
// nb batch entries; the staged list of ns words is searched by `find`
// (wk → found, its packed word pw, and — when pw's nibbles say "look it up" —
// its vals index pos).
template <int ILP, bool SPLIT = false, bool SWAP = false, bool STATS = true, class Q, class F, class E>
__device__ inline void tri_row_packed(uint32_t nb, uint32_t ns, const uint32_t *pcols, const uint2 *vals,
                                      TriBatch2 &tb, Q qrow, F find,
                                      E pqe, unsigned long long &t, unsigned long long &probes,
                                      unsigned long long &hits) {
  const int lane = lane_id();
  constexpr uint32_t STEP = ILP * WAVE;
  const uint32_t dp = ns;
  for (uint32_t kb = 0; kb < nb; kb += WAVE) {
    const uint32_t k = kb + lane;
    uint32_t qa = 0, dq = 0, pk = 0;
    if (k < nb) {
      const uint2 r = qrow(k);
      qa = r.x;
      dq = r.y & TRI_M24;
      pk = r.y & 0xFF000000u;
      if (SPLIT && dp < dq) dq = 0;  // pass B counts this edge
    }
    const uint32_t inc = wave_inclusive_scan(dq);
    tb.pre[lane] = inc - dq;
    if (lane == WAVE - 1) tb.pre[WAVE] = inc;
    tb.qa[lane] = qa;
    tb.pk[lane] = (uint8_t)(pk >> 24);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane(inc, WAVE - 1);
    if (STATS) probes += total;  // (wave-uniform: the kernels take lane 0's)
    __builtin_amdgcn_wave_barrier();
    // ping-pong words and batch owners of the steps in flight; a word's pcols
    // position is recomputed from its owner on the rare escape instead of held
    // (owners are < 64: one byte each, ILP of them packed in one register)
    uint32_t w[2][ILP], bi[2];
    static_assert(ILP <= 4, "owner bytes of one register");
    auto issue = [&](uint32_t t0, uint32_t (&ww)[ILP], uint32_t &bbp) {
      uint32_t xc[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) xc[u] = min(t0 + u * WAVE + lane, total - 1);
      // the ILP searches over all 64 entries in lockstep (positions as pointers:
      // one add per step gives the probe address)
      const uint32_t *bp[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) bp[u] = tb.pre;
#pragma unroll
      for (int st = WAVE / 2; st > 0; st >>= 1) {
        const uint32_t *cand[ILP];
        uint32_t v[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) {
          cand[u] = bp[u] + st;
          v[u] = *cand[u];
        }
#pragma unroll
        for (int u = 0; u < ILP; ++u) bp[u] = v[u] <= xc[u] ? cand[u] : bp[u];
      }
      uint32_t bb[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) bb[u] = (uint32_t)(bp[u] - tb.pre);
      bbp = 0;
#pragma unroll
      for (int u = 0; u < ILP; ++u) bbp |= bb[u] << (8 * u);
#pragma unroll
      for (int u = 0; u < ILP; ++u) {
        const uint32_t pp = tb.qa[bb[u]] + (xc[u] - tb.pre[bb[u]]);
        // past the end: a clamped position, masked by `live` in probe.  (Masking
        // the word here made the compiler wait on each load before the next
        // slice's lookups, serialising the ILP loads: s24 231 → 210 ms.)
        ww[u] = pcols[pp];
      }
    };
    auto probe = [&](const uint32_t (&ww)[ILP], uint32_t bbp, uint32_t t0) {
      uint32_t wk[ILP], fp[ILP];
      bool live[ILP], hit[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) {
        live[u] = t0 + u * WAVE + lane < total;
        wk[u] = ww[u] & TRI_M24;
      }
      find.template batch<ILP>(wk, live, hit, fp);
#pragma unroll
      for (int u = 0; u < ILP; ++u) {
        if (STATS) hits += (unsigned long long)__popcll(__ballot(hit[u]));  // (wave-uniform)
        if (hit[u]) {
          const uint32_t bo = (bbp >> (8 * u)) & 0xFFu;
          const uint32_t pkw = (uint32_t)tb.pk[bo] << 24;
          const uint2 a1 = tri_esc(pkw) ? vals[pqe(kb + bo)]  // p–q
                                        : make_uint2((pkw >> 24) & 15u, pkw >> 28);
          const uint32_t x = t0 + u * WAVE + lane;
          const uint2 s2 = tri_esc(ww[u]) ? vals[tb.qa[bo] + (x - tb.pre[bo])]  // streamed: q–w (A) / p–w (B)
                                          : make_uint2((ww[u] >> 24) & 15u, ww[u] >> 28);
          const uint32_t sn = fp[u] >> 24;                             // staged:   p–w (A) / q–w (B)
          const uint2 s3 = ((sn & 15u) == 15u || (sn >> 4) == 15u) ? vals[find.a + (fp[u] & TRI_M24)]
                                                                    : make_uint2(sn & 15u, sn >> 4);
          const uint2 a2 = SWAP ? s3 : s2, a3 = SWAP ? s2 : s3;
          // p→q→w→p  +  p→w→q→p
          t += (unsigned long long)a1.x * a2.x * a3.y + (unsigned long long)a3.x * a2.y * a1.y;
        }
      }
    };
    if (total > 0) issue(0, w[0], bi[0]);
    for (uint32_t t0 = 0; t0 < total; t0 += 2 * STEP) {
      if (t0 + STEP < total) issue(t0 + STEP, w[1], bi[1]);
      probe(w[0], bi[0], t0);
      if (t0 + STEP >= total) break;
      if (t0 + 2 * STEP < total) issue(t0 + 2 * STEP, w[0], bi[0]);
      probe(w[1], bi[1], t0 + STEP);
    }
    __builtin_amdgcn_wave_barrier();  // the table is rewritten by the next batch
  }
}

// {start, length | nibbles << 24} of the list N+(q) of the packed word w (q = w's id)
__device__ inline uint2 tri_qrow(const uint32_t *rowptr, uint32_t w) {
  const uint32_t q = w & TRI_M24, qa = rowptr[q];
  return make_uint2(qa, (rowptr[q + 1] - qa) | (w & 0xFF000000u));
}

// Binary search of wk in the ascending packed words f(0..n) (vals index a + lo).
template <class F>
__device__ inline bool tri_bsearch(F f, uint32_t n, uint32_t a, uint32_t wk, uint32_t &pw, uint32_t &pos) {
  uint32_t lo = 0, m = n;
  while (m > 0) {
    const uint32_t half = m >> 1;
    if ((f(lo + half) & TRI_M24) < wk) {
      lo += half + 1;
      m -= half + 1;
    } else {
      m = half;
    }
  }
  if (lo >= n) return false;
  pw = f(lo);
  pos = a + lo;
  return (pw & TRI_M24) == wk;
}

// Finders of the staged list: batch<ILP>(wk, live → hit, fp = the found word's
// multiplicity nibbles << 24 | its index in the list — vals index a + index
// when a nibble says "look it up"; one register per search, not two).  Sorted: ILP lower-bound searches
// in lockstep by binary lifting (the list length n is wave-uniform, so every
// lane runs the same floor(log2 n) + 1 steps, and the ILP dependent chains
// interleave instead of running one after the other).
template <class A>
struct TriSorted {
  A at;
  uint32_t n, a;
  template <int ILP>
  __device__ inline void batch(const uint32_t (&wk)[ILP], const bool (&live)[ILP], bool (&hit)[ILP],
                               uint32_t (&fp)[ILP]) const {
    // n is the staged list's length, equal on every lane: the halving loop is
    // scalar and every probe index is in range (no guard), so the ILP reads of
    // a step issue back to back under one wait.  base: lower bound of wk lies
    // in [base, base + len]; at len = 1 it is base or base + 1.
    const uint32_t nu = __builtin_amdgcn_readfirstlane(n);
    if (nu == 0) {
#pragma unroll
      for (int u = 0; u < ILP; ++u) hit[u] = false;
      return;
    }
    uint32_t base[ILP];
#pragma unroll
    for (int u = 0; u < ILP; ++u) base[u] = 0;
    for (uint32_t len = nu; len > 1;) {
      const uint32_t half = len >> 1;
      uint32_t v[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) v[u] = at(base[u] + half);
#pragma unroll
      for (int u = 0; u < ILP; ++u) base[u] = (v[u] & TRI_M24) < wk[u] ? base[u] + half : base[u];
      len -= half;
    }
    uint32_t v0[ILP], v1[ILP];
#pragma unroll
    for (int u = 0; u < ILP; ++u) {
      v0[u] = at(base[u]);
      v1[u] = at(min(base[u] + 1, nu - 1));
    }
#pragma unroll
    for (int u = 0; u < ILP; ++u) {
      const bool first = (v0[u] & TRI_M24) == wk[u];
      const bool second = (v1[u] & TRI_M24) == wk[u] && base[u] + 1 < nu;
      hit[u] = live[u] && (first || second);
      fp[u] = ((first ? v0[u] : v1[u]) & 0xFF000000u) | (base[u] + (first ? 0u : 1u));
    }
  }
};
template <class A>
__device__ inline TriSorted<A> tri_sorted(A at, uint32_t n, uint32_t a) {
  return TriSorted<A>{at, n, a};
}

// The same search over an LDS copy of rotated words (id << 8 | nibbles): they
// sort as the ids do, so a step compares with wk << 8 and needs no mask, and
// the nibbles need no array of their own (the copy stays at 4 B per entry).
struct TriSortedRot {
  const uint32_t *ids;
  uint32_t n, a;
  template <int ILP>
  __device__ inline void batch(const uint32_t (&wk)[ILP], const bool (&live)[ILP], bool (&hit)[ILP],
                               uint32_t (&fp)[ILP]) const {
    const uint32_t nu = __builtin_amdgcn_readfirstlane(n);
    if (nu == 0) {
#pragma unroll
      for (int u = 0; u < ILP; ++u) hit[u] = false;
      return;
    }
    // the search position as an element pointer: one add per step gives the
    // probe address, and the select keeps it (no index → address arithmetic)
    const uint32_t *bp[ILP];
    uint32_t k8[ILP];
#pragma unroll
    for (int u = 0; u < ILP; ++u) {
      bp[u] = ids;
      k8[u] = wk[u] << 8;
    }
    for (uint32_t len = nu; len > 1;) {
      const uint32_t half = len >> 1;
      const uint32_t *cand[ILP];
      uint32_t v[ILP];
#pragma unroll
      for (int u = 0; u < ILP; ++u) {
        cand[u] = bp[u] + half;
        v[u] = *cand[u];
      }
#pragma unroll
      for (int u = 0; u < ILP; ++u) bp[u] = v[u] < k8[u] ? cand[u] : bp[u];
      len -= half;
    }
    uint32_t base[ILP], v0[ILP], v1[ILP];
#pragma unroll
    for (int u = 0; u < ILP; ++u) {
      base[u] = (uint32_t)(bp[u] - ids);
      v0[u] = *bp[u];
      v1[u] = ids[min(base[u] + 1, nu - 1)];
    }
#pragma unroll
    for (int u = 0; u < ILP; ++u) {
      const bool first = (v0[u] >> 8) == wk[u];
      const bool second = (v1[u] >> 8) == wk[u] && base[u] + 1 < nu;
      hit[u] = live[u] && (first || second);
      const uint32_t r = first ? v0[u] : v1[u];
      fp[u] = (r << 24) | (base[u] + (first ? 0u : 1u));
    }
  }
};

// stage row[0..n) as rotated words into the LDS copy
__device__ inline void tri_stage_rot(uint32_t *ids, const uint32_t *row, uint32_t n) {
  for (uint32_t k = lane_id(); k < n; k += WAVE) {
    const uint32_t w = row[k];
    ids[k] = (w << 8) | (w >> 24);
  }
}

// Pass B of the two-pass schedule (shorter list streamed): the edges p→q with
// |N+(p)| < |N+(q)| are counted at q — N+(q) staged in LDS once, the in-list
// p's (sorted by q, chunks of TRI_BCHUNK entries per work item so a hub's long
// in-list spreads over waves) stream their N+(p) and binary-search each w in
// N+(q).  Σ min(|N+(p)|, |N+(q)|) over the edges is ~2.2× below the one-pass
// Σ |N+(q)| on R-MAT (s18 / s20).
// (s24, one box: 256 217.6 ms, 1024 223.6, 4096 231.2, 16384 235.6 — pass B)
constexpr uint32_t TRI_BCHUNK = 256;
// pass-A tile size (log2 words; 0 = row by row).  s24 (profiles/r04_tri_sweep.txt):
// row by row 350 ms, 2^23 268, 2^24 220, 2^25 190, 2^26 184 ms
constexpr int TRI_QTILE_DEFAULT = 26;

// First item of the wave's next grab.  xcd = 0: one cursor, grabs in order.
// xcd = C > 0: the grabs are dealt to the 8 XCD groups (blocks b, b + 8, …
// share an XCD and its L2) in chunks of C consecutive grabs, each group with
// its own cursor (cursor[32·g], a line of its own): every XCD walks the item
// order at the same pace, its L2 seeing contiguous chunks.  Either way grab
// index g covers items [(g·parts + part)·grab, … + grab).
constexpr int TRI_XCHUNK = 64;
__device__ inline unsigned long long tri_dequeue(unsigned long long *cursor, int xcd, int parts, int part,
                                                 int grab) {
  const unsigned long long xg = xcd ? (blockIdx.x & 7u) : 0ull;
  unsigned long long c0 = 0;
  if (lane_id() == 0) c0 = atomicAdd(cursor + 32 * xg, 1ull);
  c0 = (unsigned long long)__shfl((long long)c0, 0, WAVE);
  if (xcd) {
    const unsigned long long ch = (unsigned long long)xcd;
    c0 = ((c0 / ch) * 8 + xg) * ch + c0 % ch;
  }
  const unsigned long long g = (c0 * parts + part) * grab;
  // wave-uniform: the item loads and everything derived from them stay scalar
  // (as VGPRs they pushed the 8-wave count kernels into scratch: 92 / 84 B per
  // lane of spills → 60 / 76 B)
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)g);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(g >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

struct TriPassB {
  const uint32_t *in_words;   // p | multiplicity nibbles of the pair p–q, by (p-block, q, p)
  const uint2 *in_rows;       // the same entries as {start of N+(p), |N+(p)| | nibbles << 24}, or null
  const uint32_t *in_eidx;    // out-CSR index of the edge p→q (vals escape)
  const uint4 *items;         // (q, first in-list entry, entries ≤ TRI_BCHUNK) per work item
  uint32_t nitems;
};

template <int ILP, int WPE, bool STATS, int SCAP = TRI_CAP>
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void k_tri_count_passb(const uint32_t *rowptr, const uint32_t *pcols,
                                                                const uint2 *vals, TriPassB b, int parts,
                                                                int part, int grab, int xcd,
                                                                unsigned long long *cursor,
                                                                unsigned long long *acc) {
  constexpr uint32_t CAP = SCAP;  // staged lists of ≤ SCAP words as sorted rotated copies
  __shared__ __attribute__((aligned(16))) uint32_t s_cols[TRI_BLOCK / WAVE][SCAP];

  __shared__ TriBatch2 s_tab[TRI_BLOCK / WAVE];
  __shared__ unsigned long long lds[17];
  const int wv = threadIdx.x / WAVE;
  uint32_t *sc = s_cols[wv];
  TriBatch2 &tb = s_tab[wv];
  unsigned long long t = 0, probes = 0, hits = 0;
  uint32_t staged = 0xFFFFFFFFu;  // q whose list sits in sc
  for (;;) {
    const unsigned long long c0 = tri_dequeue(cursor, xcd, parts, part, grab);
    if (c0 >= b.nitems) break;
    const uint64_t c1 = min<uint64_t>(c0 + grab, b.nitems);
    for (uint64_t it = c0; it < c1; ++it) {
      const uint4 item = b.items[it];
      const uint32_t q = item.x;
      const uint32_t a = rowptr[q], dq = rowptr[q + 1] - a;
      const uint32_t i0 = item.y, n = item.z;
      const uint32_t *inw = b.in_words + i0;
      const uint32_t *ine = b.in_eidx + i0;
      const uint32_t *row = pcols + a;
      auto qs = [&](uint32_t k) { return b.in_rows ? b.in_rows[i0 + k] : tri_qrow(rowptr, inw[k]); };
      auto pqe = [&](uint32_t k) { return ine[k]; };
      if (dq > CAP) {  // long N+(q): searched in global memory
        tri_row_packed<ILP, false, true, STATS>(n, dq, pcols, vals, tb, qs,
                                         tri_sorted([&](uint32_t x) { return row[x]; }, dq, a),
                                         pqe, t, probes, hits);
        staged = 0xFFFFFFFFu;
        continue;
      }
      if (q != staged) {
        __builtin_amdgcn_wave_barrier();  // the previous list's searches are done
        tri_stage_rot(sc, row, dq);
        __builtin_amdgcn_wave_barrier();
        staged = q;
      }
      tri_row_packed<ILP, false, true, STATS>(n, dq, pcols, vals, tb, qs, TriSortedRot{sc, dq, a}, pqe, t, probes, hits);
    }
  }
  unsigned long long tot;
  block_exclusive_scan(t, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[0], tot);
  if (STATS) {
    block_exclusive_scan(lane_id() == 0 ? probes : 0ull, lds, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&acc[4], tot);
    block_exclusive_scan(lane_id() == 0 ? hits : 0ull, lds, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&acc[5], tot);
  }
}

__global__ void k_tri_total(const unsigned long long *acc, int64_t *out) {
  if (threadIdx.x == 0) *out = (int64_t)(3ull * acc[0] + 3ull * acc[1] + acc[2]);
}

template <class F>
static void rocprim_call(Session *s, F &&f) {
  size_t tmp = 0;
  HIP_CHECK(f(nullptr, tmp));
  BufPtr t = s->alloc(std::max<size_t>(tmp, 16));
  HIP_CHECK(f(t->p, tmp));
}

// Pass-B keys: edge e = p→q (sorted oriented keys) goes to pass B when
// |N+(p)| < |N+(q)|: key (q << 32 | p), value e; otherwise TRI_NONE.
// Key (block of p << 48 | q << 24 | p): pass B's in-lists grouped by p-block
// first — blocks of 2^pshift words of N+(p) lists (block(p) = rowptr[p] >>
// pshift) — so the waves in flight stream lists from one block, a region the
// Infinity Cache holds, instead of from the whole CSR (node ids < 2^24).
__global__ void k_tri_passb_keys(const uint64_t *okey, const uint32_t *rowptr, uint32_t P, int pshift,
                                 uint64_t *keys, uint32_t *eidx) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < P; e += gridDim.x * blockDim.x) {
    const uint64_t k = okey[e];
    const uint32_t pp = (uint32_t)(k >> 32), q = (uint32_t)k;
    const uint32_t ap = rowptr[pp];
    const uint32_t dp = rowptr[pp + 1] - ap, dq = rowptr[q + 1] - rowptr[q];
    keys[e] = dp < dq ? ((uint64_t)(ap >> pshift) << 48) | ((uint64_t)q << 24) | pp : TRI_NONE;
    eidx[e] = e;
  }
}

// number of keys below TRI_NONE (sorted): one thread, binary search
__global__ void k_tri_count_below(const uint64_t *skeys, uint32_t P, uint32_t *out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t lo = 0, hi = P;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (skeys[mid] < TRI_NONE) lo = mid + 1;
    else hi = mid;
  }
  *out = lo;
}

__global__ void k_tri_segkeys(const uint64_t *skeys, uint32_t n, uint64_t *seg) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    seg[i] = skeys[i] >> 24;
}

// items of segment j (a run of equal (p-block, q)): ⌈cnt / TRI_BCHUNK⌉ chunks
__global__ void k_tri_seg_items(const uint32_t *cnt, uint32_t nseg, uint32_t bchunk, uint32_t *nitems) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nseg; j += gridDim.x * blockDim.x)
    nitems[j] = (cnt[j] + bchunk - 1) / bchunk;
}

__global__ void k_tri_seg_fill(const uint64_t *useg, const uint32_t *cnt, const uint32_t *start,
                               const uint32_t *istart, uint32_t nseg, uint32_t bchunk, uint4 *items) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nseg; j += gridDim.x * blockDim.x) {
    const uint32_t q = (uint32_t)(useg[j] & 0xFFFFFFu), c = cnt[j], s0 = start[j];
    for (uint32_t i = 0; i * bchunk < c; ++i)
      items[istart[j] + i] = make_uint4(q, s0 + i * bchunk, min(bchunk, c - i * bchunk), 0u);
  }
}

// In-list words of pass B: p with the pair's multiplicity nibbles.
__global__ void k_tri_inlist(const uint64_t *skeys, const uint32_t *seidx, const uint32_t *pcols, uint32_t nB,
                             uint32_t *in_words) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nB; i += gridDim.x * blockDim.x)
    in_words[i] = (pcols[seidx[i]] & 0xFF000000u) | ((uint32_t)skeys[i] & 0xFFFFFFu);
}

// {start, length | nibbles << 24} of the list named by each packed word:
// rows[i] = the list N+(x) of x = words[i]'s id (the batch entries of the count
// kernels then need one coalesced 8-B load instead of a dependent rowptr pair).
__global__ void k_tri_list_rows(const uint32_t *words, const uint32_t *rowptr, uint32_t n, uint2 *rows) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    rows[i] = tri_qrow(rowptr, words[i]);
}

// Oriented CSR of the distinct node pairs of (src, dst) over [lo, lo + len).
struct TriGraph {
  // acc: [0] T, [1] Σ(L+L)·f·b, [2] Σ L(L−1)(L−2), [3] cursor, [4] probes (w ∈ N+(q)
  // looked up in N+(p)), [5] hits (closed triangles found)
  BufPtr rowptr, cols, vals, loops, acc;
  BufPtr pcols;  // packed column words (node ids < 2^24), else null
  // two-pass schedule (pass B: edges with |N+(p)| < |N+(q)| counted at q)
  BufPtr in_words, in_eidx, items;
  BufPtr erow, in_rows;  // list rows of pcols / in_words (k_tri_list_rows), or null
  uint32_t nB = 0, nitems = 0;
  // q-tiled pass A: work items (p, k0, k1) sorted by (tile of N+(q)'s position, p)
  BufPtr aitems;
  uint32_t naitems = 0;
  int qshift = 0;  // log2 of the pcols words per tile (0: pass A row by row)
  uint32_t P = 0;
  uint64_t len = 0;
};

// In-lists and work items of pass B (built with the CSR, cached with it).
static void tri_build_passb(Session *s, const uint64_t *okey, TriGraph &g) {
  const uint32_t P = g.P;
  KernelTimer kt(s, "tri_passb_build", 40.0 * P);
  // log2 of the N+(p) words per p-block; ≥ 16: the pass-B key holds the p-block
  // id (ap >> pshift, ap < 2^32) in 16 bits at bit 48.
  // s24: 2^22 355 ms, 2^23 338, 2^24 333, 2^25 326 (pass B)
  constexpr int pshift = 25;
  BufPtr keys = s->alloc(8 * (int64_t)P), skeys = s->alloc(8 * (int64_t)P);
  BufPtr eidx = s->alloc(4 * (int64_t)P), seidx = s->alloc(4 * (int64_t)P);
  hipLaunchKernelGGL(k_tri_passb_keys, dim3(grid_for(P, 256, 256 * 64)), dim3(256), 0, s->stream, okey,
                     (const uint32_t *)g.rowptr->p, P, pshift, (uint64_t *)keys->p, (uint32_t *)eidx->p);
  KERNEL_CHECK();
  rocprim_call(s, [&](void *t, size_t &n) {
    return rocprim::radix_sort_pairs(t, n, (const uint64_t *)keys->p, (uint64_t *)skeys->p,
                                     (const uint32_t *)eidx->p, (uint32_t *)seidx->p, (size_t)P, 0, 64,
                                     s->stream);
  });
  BufPtr nb = s->alloc(16);
  hipLaunchKernelGGL(k_tri_count_below, dim3(1), dim3(64), 0, s->stream, (const uint64_t *)skeys->p, P,
                     (uint32_t *)nb->p);
  KERNEL_CHECK();
  HIP_CHECK(hipMemcpyAsync(&g.nB, nb->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  g.in_words = s->alloc(4 * std::max<uint32_t>(g.nB, 1));
  g.in_eidx = s->alloc(4 * std::max<uint32_t>(g.nB, 1));
  g.nitems = 0;
  if (g.nB == 0) {
    g.items = s->alloc(16);
    s->sync();
    return;
  }
  hipLaunchKernelGGL(k_tri_inlist, dim3(grid_for(g.nB, 256, 256 * 64)), dim3(256), 0, s->stream,
                     (const uint64_t *)skeys->p, (const uint32_t *)seidx->p, (const uint32_t *)g.pcols->p, g.nB,
                     (uint32_t *)g.in_words->p);
  KERNEL_CHECK();
  HIP_CHECK(hipMemcpyAsync(g.in_eidx->p, seidx->p, 4 * (size_t)g.nB, hipMemcpyDeviceToDevice, s->stream));
  g.in_rows = s->alloc(8 * (int64_t)g.nB);
  hipLaunchKernelGGL(k_tri_list_rows, dim3(grid_for(g.nB, 256, 256 * 64)), dim3(256), 0, s->stream,
                     (const uint32_t *)g.in_words->p, (const uint32_t *)g.rowptr->p, g.nB, (uint2 *)g.in_rows->p);
  KERNEL_CHECK();
  // segments = runs of equal (p-block, q) → work items of ≤ TRI_BCHUNK entries
  BufPtr seg = s->alloc(8 * (int64_t)g.nB), useg = s->alloc(8 * (int64_t)g.nB);
  BufPtr cnt = s->alloc(4 * ((int64_t)g.nB + 1)), nseg_d = s->alloc(16);
  hipLaunchKernelGGL(k_tri_segkeys, dim3(grid_for(g.nB, 256, 256 * 64)), dim3(256), 0, s->stream,
                     (const uint64_t *)skeys->p, g.nB, (uint64_t *)seg->p);
  KERNEL_CHECK();
  rocprim_call(s, [&](void *t, size_t &n) {
    return rocprim::run_length_encode(t, n, (const uint64_t *)seg->p, (unsigned int)g.nB, (uint64_t *)useg->p,
                                      (uint32_t *)cnt->p, (uint32_t *)nseg_d->p, s->stream);
  });
  uint32_t nseg = 0;
  HIP_CHECK(hipMemcpyAsync(&nseg, nseg_d->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  BufPtr start = s->alloc(4 * ((int64_t)nseg + 1)), nit = s->alloc(4 * ((int64_t)nseg + 1)),
         istart = s->alloc(4 * ((int64_t)nseg + 1));
  rocprim_call(s, [&](void *t, size_t &n) {
    return rocprim::exclusive_scan(t, n, (const uint32_t *)cnt->p, (uint32_t *)start->p, 0u, (size_t)nseg,
                                   rocprim::plus<uint32_t>(), s->stream);
  });
  const uint32_t bchunk = TRI_BCHUNK;  // in-list entries per pass-B work item
  hipLaunchKernelGGL(k_tri_seg_items, dim3(grid_for(nseg, 256, 256 * 64)), dim3(256), 0, s->stream,
                     (const uint32_t *)cnt->p, nseg, bchunk, (uint32_t *)nit->p);
  KERNEL_CHECK();
  HIP_CHECK(hipMemsetAsync((uint32_t *)nit->p + nseg, 0, 4, s->stream));
  rocprim_call(s, [&](void *t, size_t &n) {
    return rocprim::exclusive_scan(t, n, (const uint32_t *)nit->p, (uint32_t *)istart->p, 0u, (size_t)nseg + 1,
                                   rocprim::plus<uint32_t>(), s->stream);
  });
  HIP_CHECK(hipMemcpyAsync(&g.nitems, (uint32_t *)istart->p + nseg, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  g.items = s->alloc(16 * std::max<uint32_t>(g.nitems, 1));
  hipLaunchKernelGGL(k_tri_seg_fill, dim3(grid_for(nseg, 256, 256 * 64)), dim3(256), 0, s->stream,
                     (const uint64_t *)useg->p, (const uint32_t *)cnt->p, (const uint32_t *)start->p,
                     (const uint32_t *)istart->p, nseg, bchunk, (uint4 *)g.items->p);
  KERNEL_CHECK();
  s->sync();  // the temporaries go back to the pool
}

// Pass A over q-tiled work items (see tri_build_qtiles): item (p, k0, k1) probes
// the q's N+(p)[k0, k1) — N+(p) staged in LDS (≤ TRI_CAP words) or searched in
// place — with the pass-A rule (edges with |N+(p)| < |N+(q)| belong to pass B).
template <int ILP, int WPE, bool STATS, int SCAP = TRI_CAP>
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void k_tri_count_qtiled(const uint32_t *rowptr, const uint32_t *pcols,
                                                                 const uint2 *vals, const uint2 *erow,
                                                                 const uint4 *items,
                                                                 uint32_t nitems, int parts, int part, int grab,
                                                                 int xcd,
                                                                 unsigned long long *cursor,
                                                                 unsigned long long *acc) {
  constexpr uint32_t CAP = SCAP;  // staged lists of ≤ SCAP words as sorted rotated copies
  __shared__ __attribute__((aligned(16))) uint32_t s_cols[TRI_BLOCK / WAVE][SCAP];

  __shared__ TriBatch2 s_tab[TRI_BLOCK / WAVE];
  __shared__ unsigned long long lds[17];
  const int wv = threadIdx.x / WAVE;
  uint32_t *sc = s_cols[wv];
  TriBatch2 &tb = s_tab[wv];
  unsigned long long t = 0, probes = 0, hits = 0;
  uint32_t staged = 0xFFFFFFFFu;  // p whose list sits in sc
  for (;;) {
    const unsigned long long c0 = tri_dequeue(cursor, xcd, parts, part, grab);
    if (c0 >= nitems) break;
    const uint64_t c1 = min<uint64_t>(c0 + grab, nitems);
    for (uint64_t it = c0; it < c1; ++it) {
      const uint4 item = items[it];
      const uint32_t p = item.x, k0 = item.y, nb = item.z - item.y;
      const uint32_t a = rowptr[p], dp = rowptr[p + 1] - a;
      const uint32_t *row = pcols + a;
      auto pqe = [&](uint32_t k) { return a + k0 + k; };
      auto qrow = [&](uint32_t k) { return erow ? erow[a + k0 + k] : tri_qrow(rowptr, row[k0 + k]); };
      if (dp > CAP) {  // long N+(p): searched in global memory
        tri_row_packed<ILP, true, false, STATS>(nb, dp, pcols, vals, tb, qrow,
                                  tri_sorted([&](uint32_t x) { return row[x]; }, dp, a),
                                  pqe, t, probes, hits);
        staged = 0xFFFFFFFFu;
        continue;
      }
      if (p != staged) {
        __builtin_amdgcn_wave_barrier();  // the previous list's searches are done
        tri_stage_rot(sc, row, dp);
        __builtin_amdgcn_wave_barrier();
        staged = p;
      }
      tri_row_packed<ILP, true, false, STATS>(nb, dp, pcols, vals, tb, qrow, TriSortedRot{sc, dp, a}, pqe, t, probes, hits);
    }
  }
  unsigned long long tot;
  block_exclusive_scan(t, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&acc[0], tot);
  if (STATS) {
    block_exclusive_scan(lane_id() == 0 ? probes : 0ull, lds, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&acc[4], tot);
    block_exclusive_scan(lane_id() == 0 ? hits : 0ull, lds, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&acc[5], tot);
  }
}

// ------------------------------------------------------ q-tiled pass A
// Pass A streams N+(q) for the q's of each row p.  Row by row those lists lie
// anywhere in the 1 GB column array (s24), so nearly every streamed word is an
// L2 miss.  Tiled: the column array is cut into tiles of 2^qshift words; the
// work item (p, k0, k1) is the run of N+(p) whose q's lists START in one tile
// (tile(q) = rowptr[q] >> qshift is monotone along the sorted N+(p)), and the
// items are processed in (tile, p) order — all waves of the chip stream lists
// from one tile at a time, a region the caches hold, while N+(p) is staged once
// per (p, tile).

// head of an item: the first edge of a row, or the first whose q's tile differs
// from the previous edge's; key (tile << 32 | p), value = edge index
__global__ void k_tri_qtile_heads(const uint64_t *okey, const uint32_t *rowptr, uint32_t P, int qshift,
                                  uint64_t *keys, uint32_t *eidx) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < P; e += gridDim.x * blockDim.x) {
    const uint64_t k = okey[e];
    const uint32_t p = (uint32_t)(k >> 32), q = (uint32_t)k;
    const uint32_t a = rowptr[p], dp = rowptr[p + 1] - a;
    const uint32_t t = rowptr[q] >> qshift;
    bool head = dp >= 2;
    if (head && e > a) head = (rowptr[(uint32_t)okey[e - 1]] >> qshift) != t;
    keys[e] = head ? ((uint64_t)t << 32 | p) : TRI_NONE;
    eidx[e] = e;
  }
}

// items (p, k0, k1): k1 = the end of the head's tile run inside the row
// (binary search: tile(q) is monotone along the row)
__global__ void k_tri_qtile_items(const uint64_t *skeys, const uint32_t *seidx, uint32_t n,
                                  const uint64_t *okey, const uint32_t *rowptr, int qshift, uint4 *items) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t e = seidx[i];
    const uint32_t p = (uint32_t)(skeys[i] & 0xFFFFFFFFu), t = (uint32_t)(skeys[i] >> 32);
    const uint32_t a = rowptr[p], end = rowptr[p + 1];
    uint32_t lo = e + 1, hi = end;  // first edge of the row whose tile is > t
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((rowptr[(uint32_t)okey[mid]] >> qshift) <= t) lo = mid + 1;
      else hi = mid;
    }
    items[i] = make_uint4(p, e - a, lo - a, 0u);
  }
}

static void tri_build_qtiles(Session *s, const uint64_t *okey, TriGraph &g, int qshift) {
  const uint32_t P = g.P;
  KernelTimer kt(s, "tri_qtile_build", 24.0 * P);
  BufPtr keys = s->alloc(8 * (int64_t)P), skeys = s->alloc(8 * (int64_t)P);
  BufPtr eidx = s->alloc(4 * (int64_t)P), seidx = s->alloc(4 * (int64_t)P);
  hipLaunchKernelGGL(k_tri_qtile_heads, dim3(grid_for(P, 256, 256 * 64)), dim3(256), 0, s->stream, okey,
                     (const uint32_t *)g.rowptr->p, P, qshift, (uint64_t *)keys->p, (uint32_t *)eidx->p);
  KERNEL_CHECK();
  rocprim_call(s, [&](void *t, size_t &n) {
    return rocprim::radix_sort_pairs(t, n, (const uint64_t *)keys->p, (uint64_t *)skeys->p,
                                     (const uint32_t *)eidx->p, (uint32_t *)seidx->p, (size_t)P, 0, 64,
                                     s->stream);
  });
  BufPtr nb = s->alloc(16);
  hipLaunchKernelGGL(k_tri_count_below, dim3(1), dim3(64), 0, s->stream, (const uint64_t *)skeys->p, P,
                     (uint32_t *)nb->p);
  KERNEL_CHECK();
  HIP_CHECK(hipMemcpyAsync(&g.naitems, nb->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  g.aitems = s->alloc(16 * std::max<uint32_t>(g.naitems, 1));
  if (g.naitems > 0) {
    hipLaunchKernelGGL(k_tri_qtile_items, dim3(grid_for(g.naitems, 256, 256 * 64)), dim3(256), 0, s->stream,
                       (const uint64_t *)skeys->p, (const uint32_t *)seidx->p, g.naitems, okey,
                       (const uint32_t *)g.rowptr->p, qshift, (uint4 *)g.aitems->p);
    KERNEL_CHECK();
  }
  g.qshift = qshift;
  s->sync();  // the temporaries go back to the pool
}

static void tri_build(Session *s, const ColView &src, const ColView &dst, int64_t m, int64_t lo,
                      uint64_t len, TriGraph &g) {
  g.len = len;
  g.acc = s->alloc(48);
  HIP_CHECK(hipMemsetAsync(g.acc->p, 0, 48, s->stream));
  unsigned long long *acc = (unsigned long long *)g.acc->p;
  g.loops = s->alloc(4 * len);
  HIP_CHECK(hipMemsetAsync(g.loops->p, 0, 4 * len, s->stream));
  uint32_t *loops = (uint32_t *)g.loops->p;
  const int64_t m1 = std::max<int64_t>(m, 1);
  BufPtr keys = s->alloc(8 * m1), sorted = s->alloc(8 * m1);
  {
    KernelTimer kt(s, "tri_keys", 16.0 * m);
    hipLaunchKernelGGL(k_tri_keys, dim3(grid_for(m1, 256)), dim3(256), 0, s->stream, src, dst, m,
                       lo, len, (uint64_t *)keys->p, loops);
    KERNEL_CHECK();
  }
  uint64_t *kout = (uint64_t *)sorted->p;
  {
    KernelTimer kt(s, "tri_sort_keys", 32.0 * m);
    const uint64_t *kin = (const uint64_t *)keys->p;
    rocprim_call(s, [&](void *t, size_t &n) {
      return rocprim::radix_sort_keys(t, n, kin, kout, (size_t)m, 0, 64, s->stream);
    });
  }
  BufPtr ukeys = s->alloc(8 * m1), cnt = s->alloc(4 * m1), nruns = s->alloc(16);
  {
    KernelTimer kt(s, "tri_rle", 20.0 * m);
    rocprim_call(s, [&](void *t, size_t &n) {
      return rocprim::run_length_encode(t, n, (const uint64_t *)kout, (unsigned int)m,
                                        (uint64_t *)ukeys->p, (uint32_t *)cnt->p,
                                        (uint32_t *)nruns->p, s->stream);
    });
  }
  BufPtr deg = s->alloc(4 * len);
  HIP_CHECK(hipMemsetAsync(deg->p, 0, 4 * len, s->stream));
  uint64_t *pair_uv = (uint64_t *)keys->p;  // runs ≤ m: the unsorted keys are dead
  BufPtr pair_fb = s->alloc(8 * m1);
  const unsigned grid = grid_for(m1, 256, 256 * 64);
  {
    KernelTimer kt(s, "tri_pairs", 24.0 * m);
    hipLaunchKernelGGL(k_tri_pairs, dim3(grid), dim3(256), 0, s->stream, (const uint64_t *)ukeys->p,
                       (const uint32_t *)cnt->p, (const uint32_t *)nruns->p, (uint32_t *)deg->p,
                       pair_uv, (uint2 *)pair_fb->p);
    KERNEL_CHECK();
  }
  uint64_t *okey = (uint64_t *)ukeys->p;  // runs ≤ m: the run keys are dead after the merge
  uint64_t *oval = kout;
  {
    KernelTimer kt(s, "tri_orient", 32.0 * m);
    hipLaunchKernelGGL(k_tri_orient, dim3(grid), dim3(256), 0, s->stream, (const uint64_t *)pair_uv,
                       (const uint2 *)pair_fb->p, (const uint32_t *)nruns->p, (const uint32_t *)deg->p,
                       (const uint32_t *)loops, okey, oval, acc);
    KERNEL_CHECK();
  }
  uint32_t nr = 0;
  HIP_CHECK(hipMemcpyAsync(&nr, nruns->p, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  BufPtr ok2 = s->alloc(8 * std::max<uint32_t>(nr, 1)), ov2 = s->alloc(8 * std::max<uint32_t>(nr, 1));
  {
    KernelTimer kt(s, "tri_sort_pairs", 32.0 * nr);
    rocprim_call(s, [&](void *t, size_t &n) {
      return rocprim::radix_sort_pairs(t, n, (const uint64_t *)okey, (uint64_t *)ok2->p,
                                       (const uint64_t *)oval, (uint64_t *)ov2->p, (size_t)nr, 0, 64,
                                       s->stream);
    });
  }
  g.rowptr = s->alloc(4 * (len + 2));
  {
    KernelTimer kt(s, "tri_rowptr", 4.0 * len);
    hipLaunchKernelGGL(k_tri_rowptr, dim3(grid_for((int64_t)len + 1, 256, 256 * 64)), dim3(256), 0,
                       s->stream, (const uint64_t *)ok2->p, nr, len, (uint32_t *)g.rowptr->p);
    KERNEL_CHECK();
  }
  HIP_CHECK(hipMemcpyAsync(&g.P, (uint32_t *)g.rowptr->p + len, 4, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  g.cols = s->alloc(4 * std::max<uint32_t>(g.P, 1));
  g.vals = s->alloc(8 * std::max<uint32_t>(g.P, 1));
  if (g.P > 0) {
    KernelTimer kt(s, "tri_split", 20.0 * g.P);
    hipLaunchKernelGGL(k_tri_split, dim3(grid_for(g.P, 256, 256 * 64)), dim3(256), 0, s->stream,
                       (const uint64_t *)ok2->p, (const uint64_t *)ov2->p, g.P, (uint32_t *)g.cols->p,
                       (uint2 *)g.vals->p);
    KERNEL_CHECK();
  }
  if (g.P > 0 && len <= (uint64_t)TRI_M24 + 1) {
    g.pcols = s->alloc(4 * (int64_t)g.P);
    hipLaunchKernelGGL(k_tri_pack, dim3(grid_for(g.P, 256, 256 * 64)), dim3(256), 0, s->stream,
                       (const uint32_t *)g.cols->p, (const uint2 *)g.vals->p, g.P, (uint32_t *)g.pcols->p);
    KERNEL_CHECK();
    g.erow = s->alloc(8 * (int64_t)g.P);
    hipLaunchKernelGGL(k_tri_list_rows, dim3(grid_for(g.P, 256, 256 * 64)), dim3(256), 0, s->stream,
                       (const uint32_t *)g.pcols->p, (const uint32_t *)g.rowptr->p, g.P, (uint2 *)g.erow->p);
    KERNEL_CHECK();
    tri_build_passb(s, (const uint64_t *)ok2->p, g);
    // CAPF_TRI_QTILE (test hook): log2 of the words per pass-A tile (small tiles
    // cut rows into many items: the tests' way to reach the item boundaries)
    const char *qt = getenv("CAPF_TRI_QTILE");
    const int qshift = qt && atoi(qt) > 0 ? atoi(qt) : TRI_QTILE_DEFAULT;
    tri_build_qtiles(s, (const uint64_t *)ok2->p, g, std::max(12, std::min(30, qshift)));
  }
}

// Count kernels: ILP 4 positions per lane in flight, compiled for 8 waves/SIMD
// (the rotated-word LDS copies take 18.8 KB per 4-wave block, 8 blocks fit a
// CU; s24, ILP 4: 4 waves 308 ms, 5 268, 6 240, 7 226, 8 222 ms), staged
// lists of ≤ TRI_CAP words.  Pass A deals its grabs (2 items) to the 8 XCD
// groups in chunks of TRI_XCHUNK grabs (tri_dequeue: 121 → 103 ms at s24);
// pass B takes 4 items per grab from one cursor (per-XCD cursors were slower).
// Measured and removed: an LDS hash table per staged list (290 vs 222 ms),
// galloping batch-owner search, an LDS bitmap pre-filter, relabelling the CSR
// by degree rank, larger grabs (4/4 319 ms … 128/32 720 ms).
constexpr int TRI_WPE = 8, TRI_GRAB_A = 2, TRI_GRAB_B = 4;
// CAPF_TRI_ILP=3 (A/B of the spill trade-off): ILP 3 compiles the two count
// kernels with 24 / 48 B per lane of scratch against 56 / 80 B at ILP 4
// CAPF_TRI_WPE=6 / 7 (A/B): the count kernels held at 6 / 7 waves per SIMD
// (80 / 72 VGPRs: 0 / 24 B per lane of scratch in pass A, 8 / 40 B in pass B)
static int tri_wpe() {
  static const int v = [] {
    const char *e = getenv("CAPF_TRI_WPE");
    return e ? atoi(e) : TRI_WPE;
  }();
  return v;
}
static int tri_ilp() {
  static const int v = [] {
    const char *e = getenv("CAPF_TRI_ILP");
    return e && atoi(e) == 3 ? 3 : TRI_ILP;
  }();
  return v;
}

// Device count (int64 at d_out) of the directed triangle over rels (src, dst)
// with endpoints in [lo, lo + len), restricted to part `part` of `parts`
// (row chunks dealt round-robin; the loop terms belong to part 0): the sum
// over parts is the count.  The oriented CSR (and the pair-loop term) is
// built on the first query over (src, dst, lo, len) and cached on src's
// Column (the two columns are immutable): later queries run the count
// kernels only, asynchronously.
void triangle_count_async(Session *s, const ColPtr &srcc, const ColPtr &dstc, int64_t m,
                          int64_t lo, uint64_t len, int parts, int part, int64_t *d_out) {
  std::shared_ptr<TriGraph> gp;
  {
    std::lock_guard<std::mutex> lk(srcc->mu);
    if (srcc->index && srcc->index_peer.lock() == dstc && srcc->index_key[0] == lo &&
        srcc->index_key[1] == (int64_t)len)
      gp = std::static_pointer_cast<TriGraph>(srcc->index);
  }
  if (!gp) {
    gp = std::make_shared<TriGraph>();
    tri_build(s, view_of(srcc), view_of(dstc), m, lo, len, *gp);
    std::lock_guard<std::mutex> lk(srcc->mu);
    srcc->index = gp;
    srcc->index_peer = dstc;
    srcc->index_key[0] = lo;
    srcc->index_key[1] = (int64_t)len;
  }
  const TriGraph &g = *gp;
  // per-query accumulators: T, the cached pair-loop term, Σ L(L−1)(L−2), the
  // row cursor, probes, hits
  BufPtr qacc = s->alloc(64);  // + [6] the pass-B cursor
  // per-XCD-group cursors of the q-tiled pass A and of pass B (tri_dequeue)
  BufPtr xcur = s->alloc(8 * 32 * 8);  // per-XCD-group cursors of pass A (tri_dequeue)
  HIP_CHECK(hipMemsetAsync(xcur->p, 0, 8 * 32 * 8, s->stream));
  unsigned long long *xa = (unsigned long long *)xcur->p;
  HIP_CHECK(hipMemsetAsync(qacc->p, 0, 64, s->stream));
  if (part == 0)
    HIP_CHECK(hipMemcpyAsync((char *)qacc->p + 8, (const char *)g.acc->p + 8, 8,
                             hipMemcpyDeviceToDevice, s->stream));
  unsigned long long *acc = (unsigned long long *)qacc->p;
  if (part == 0) {
    KernelTimer kt(s, "tri_loop3", 4.0 * len);
    hipLaunchKernelGGL(k_tri_loop3, dim3(grid_for((int64_t)len, 256, 1024)), dim3(256), 0,
                       s->stream, (const uint32_t *)g.loops->p, len, acc);
    KERNEL_CHECK();
  }
  if (g.P > 0) {
    // timers are named after the kernels that run (bench.py matches them against the
    // kernel names of the committed PMC counters)
    if (g.pcols) {  // node ids < 2^24: packed words, pass A q-tiled + pass B
      // STATS: the probe / hit counters of the profiling diagnostics (their
      // registers push the 8-wave kernels into scratch: 44 / 48 B per lane with,
      // 20 / 32 B without), so the timed kernels run without them and a
      // profiled query counts them in an untimed second launch
      auto kq = [&](bool st) {
        const int ilp = tri_ilp(), wpe = tri_wpe();
        if (st) return ilp == 3 ? k_tri_count_qtiled<3, TRI_WPE, true>
                       : wpe == 6 ? k_tri_count_qtiled<TRI_ILP, 6, true>
                       : wpe == 7 ? k_tri_count_qtiled<TRI_ILP, 7, true> : k_tri_count_qtiled<TRI_ILP, TRI_WPE, true>;
        return ilp == 3 ? k_tri_count_qtiled<3, TRI_WPE, false>
               : wpe == 6 ? k_tri_count_qtiled<TRI_ILP, 6, false>
               : wpe == 7 ? k_tri_count_qtiled<TRI_ILP, 7, false> : k_tri_count_qtiled<TRI_ILP, TRI_WPE, false>;
      };
      auto kb = [&](bool st) {
        const int ilp = tri_ilp(), wpe = tri_wpe();
        if (st) return ilp == 3 ? k_tri_count_passb<3, TRI_WPE, true>
                       : wpe == 6 ? k_tri_count_passb<TRI_ILP, 6, true>
                       : wpe == 7 ? k_tri_count_passb<TRI_ILP, 7, true> : k_tri_count_passb<TRI_ILP, TRI_WPE, true>;
        return ilp == 3 ? k_tri_count_passb<3, TRI_WPE, false>
               : wpe == 6 ? k_tri_count_passb<TRI_ILP, 6, false>
               : wpe == 7 ? k_tri_count_passb<TRI_ILP, 7, false> : k_tri_count_passb<TRI_ILP, TRI_WPE, false>;
      };
      auto ptr = [](const BufPtr &x) { return x ? x->p : nullptr; };  // (no pass-B buffers without items)
      TriPassB b{(const uint32_t *)ptr(g.in_words), (const uint2 *)ptr(g.in_rows), (const uint32_t *)ptr(g.in_eidx),
                 (const uint4 *)ptr(g.items), g.nitems};
      auto pass_a = [&](bool st, unsigned long long *cur, unsigned long long *ac) {
        hipLaunchKernelGGL(kq(st), dim3((unsigned)(s->num_cus * 8)), dim3(TRI_BLOCK),
                           0, s->stream, (const uint32_t *)g.rowptr->p, (const uint32_t *)g.pcols->p,
                           (const uint2 *)g.vals->p, (const uint2 *)g.erow->p, (const uint4 *)g.aitems->p,
                           g.naitems, parts, part, TRI_GRAB_A, TRI_XCHUNK, cur, ac);
        KERNEL_CHECK();
      };
      auto pass_b = [&](bool st, unsigned long long *ac) {
        hipLaunchKernelGGL(kb(st), dim3((unsigned)(s->num_cus * 8)), dim3(TRI_BLOCK),
                           0, s->stream, (const uint32_t *)g.rowptr->p, (const uint32_t *)g.pcols->p,
                           (const uint2 *)g.vals->p, b, parts, part, TRI_GRAB_B, 0, ac + 6, ac);
        KERNEL_CHECK();
      };
      if (g.naitems > 0) {
        KernelTimer kt(s, "tri_count_qtiled", 4.0 * g.P);
        pass_a(false, xa, acc);
      }
      if (g.nitems > 0) {
        KernelTimer kt(s, "tri_count_passb", 4.0 * g.P);
        pass_b(false, acc);
      }
      if (s->profiling) {  // diagnostics (profiling mode only, untimed, host sync): probes and hits
        BufPtr sacc = s->alloc(64), scur = s->alloc(8 * 32 * 8);
        unsigned long long *sa = (unsigned long long *)sacc->p;
        HIP_CHECK(hipMemsetAsync(sacc->p, 0, 64, s->stream));
        HIP_CHECK(hipMemsetAsync(scur->p, 0, 8 * 32 * 8, s->stream));
        unsigned long long h[2] = {0, 0};
        if (g.naitems > 0) pass_a(true, (unsigned long long *)scur->p, sa);
        HIP_CHECK(hipMemcpyAsync(h, sa + 4, 8, hipMemcpyDeviceToHost, s->stream));
        s->sync();
        s->profile["tri_probes_pass_a"].bytes += (double)h[0];
        if (g.nitems > 0) pass_b(true, sa);
        HIP_CHECK(hipMemcpyAsync(h, sa + 4, 16, hipMemcpyDeviceToHost, s->stream));
        s->sync();
        s->profile["tri_probes"].bytes += (double)h[0];
        s->profile["tri_hits"].bytes += (double)h[1];
      }
    } else {  // wider node ranges: one pass over the unpacked CSR
      KernelTimer kt(s, "tri_count", 4.0 * g.P);
      hipLaunchKernelGGL(k_tri_count<TRI_ILP>, dim3((unsigned)(s->num_cus * 8)), dim3(TRI_BLOCK), 0, s->stream,
                         (const uint32_t *)g.rowptr->p, (const uint32_t *)g.cols->p,
                         (const uint2 *)g.vals->p, len, parts, part, acc + 3, acc);
      KERNEL_CHECK();
    }
  }
  hipLaunchKernelGGL(k_tri_total, dim3(1), dim3(64), 0, s->stream, (const unsigned long long *)acc,
                     d_out);
  KERNEL_CHECK();
  if (s->profiling && g.P > 0) {
    // diagnostics (profiling mode only, host sync): the count kernel's work —
    // probes (w ∈ N+(q) searched in N+(p)), hits, oriented edges — as
    // byte-only profile entries, for bench.py's probe-traffic roofline
    if (!g.pcols) {  // (the packed path counted them in its untimed stats launch)
      unsigned long long h[2];
      HIP_CHECK(hipMemcpyAsync(h, acc + 4, 16, hipMemcpyDeviceToHost, s->stream));
      s->sync();
      s->profile["tri_probes"].bytes += (double)h[0];
      s->profile["tri_hits"].bytes += (double)h[1];
    }
    s->profile["tri_oriented_edges"].bytes += (double)g.P;
    s->profile["tri_passb_edges"].bytes += (double)g.nB;
    s->profile["tri_passa_items"].bytes += (double)g.naitems;
  }
  // qacc returns to the stream-ordered pool: reuse is ordered after the kernels
}

}  // namespace capf
