// chain2_partitioned.hip — radix-partitioned LDS histograms for the fused
// 2-hop count (replaces the global-atomic k_chain2_hist for large rel tables).
//
// The two per-node histograms of the 2-hop message passing
//   in[b]  = |{r1 : end(r1) = b, start(r1) ∈ S_a}|
//   out[b] = |{r2 : start(r2) = b, end(r2) ∈ S_c}|
// are GROUP BY counts on a 2^24-key domain at R-MAT s24: far larger than LDS,
// and scattered device-scope atomics execute at the memory side at ~11 G/s on
// MI355X (measured: 47.7 ms for the 5.4e8 updates at s24).  This is the
// radix-partitioned hash aggregation of the north star, partitions sized to
// the 160 KiB LDS:
//
//   key   h = node_mix(id − lo)  (device_common.h: a bijection on 2^k, so the
//         runs are hash partitions — uniform whatever the id skew)
//   run   (side, h >> 16): 2 sides × 2^(k−16) buckets of 64 Ki node keys
//   P1 k_c5_partition  per tile of TILE rels (16-B loads): LDS count per run
//         (the count's return value is the key's rank), block scan of the
//         8-key-padded run sizes, LDS counting sort of the keys (uint16 =
//         h & 0xFFFF) into a stage prefilled with pad keys, ONE contiguous
//         copy-out into the tile's region, one (start/8 | count << 16) word
//         per run; self-loop term on the side
//   T  k_c3_transpose  [tile][run] → [run][tile] meta, per-run totals
//   U  k_c3_units      device work list (one unit per run; hub-heavy runs split)
//   P3 k_c5_gather     per unit: 64 Ki counters as packed uint16 pairs in
//         128 KiB LDS; each wave flattens the segments of 64 tiles into one
//         sequence of 16-B pieces (coalesced 128-B lines, every lane live, no
//         per-key predicate: pads are counted and subtracted), flushes every
//         bin with plain stores (no memset anywhere)
//   O  k_c3_overflow   adds the 2^15 carries a uint16 counter hands off (rare)
//   D  k_chain2_dot    Σ in·out (fused_count.hip)
// Bytes per rel at FOR32 width: P1 8 read + 4(+pads) written, P3 4(+pads) read.
// Both big kernels are VALU-issue bound before they are HBM bound (PMC:
// SQ_INSTS_VALU), so the per-key instruction count is what the code minimises.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <vector>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr int C2_BITS = 16;
constexpr int C2_BW = 1 << C2_BITS;  // node keys per bucket
constexpr int C2_WORDS = C2_BW / 2;  // LDS words of a P3 unit: 2 uint16 counters each (128 KiB)
constexpr int C5_BLOCK = 1024;       // P1 and P3 workgroup
constexpr int C5_CORR = 64;          // P3 bins 0..63 receive pad / dead-lane keys (subtracted)

// P1 shapes: (TILE rels, MAXR runs incl. the dummy).  The stage holds
// 2·TILE keys plus ≤ 7 pads per run; two workgroups per CU (≤ 80 KiB each).
//   small: ≤ 2^24 nodes (nb ≤ 256),  big: ≤ 2^26 nodes (nb ≤ 1023)
struct C5Small {
  static constexpr int TILE = 16384, MAXR = 520;
  static constexpr bool WIDE = false;  // k ≤ 24: 24-bit multiply in node_mix
};
struct C5Big {
  static constexpr int TILE = 8192, MAXR = 2048;
  static constexpr bool WIDE = true;
};

template <class SH>
constexpr int c5_stage_keys() { return 2 * SH::TILE + 8 * SH::MAXR; }

// P1 arguments: four id columns of W bytes per id: 8 = plain int64, 4 =
// FOR32, 3 = FOR24 (offset + base; 0 base for plain columns).
template <int W>
struct C5Cols {
  const void *u1, *v1, *u2, *v2;
  int64_t bu1, bv1, bu2, bv2;  // FOR bases (0 for plain columns)
  int64_t n;
  int64_t lo;
  uint64_t len;      // node range [lo, lo + len)
  int nb;            // buckets per side
  int64_t ntiles;
  int64_t rstride;   // keys per tile region in `part` (multiple of 8)
  NodeMix mix;
};

struct U3 {  // 12 bytes, 4-B aligned: one global_load_dwordx3
  uint32_t x, y, z;
};

// Raw offset of row r of a W-byte column (W = 4 or 3).
template <int W>
__device__ inline uint32_t c5_off(const void *p, int64_t r) {
  return W == 4 ? ((const uint32_t *)p)[r] : ld_u24(p, r);
}

// Four 32-bit node offsets (id − lo) from 12 B (FOR24), 16 B (FOR32) or 32 B
// (int64) at row e (a multiple of 4: FOR24 rows e..e+3 are 3 aligned
// dwords).  CHECK = false (the columns' min/max lie inside the node range):
// only the low word matters, offsets wrap exactly into [0, len).  With
// CHECK, `ok` says whether each id lies in the range.
template <int W, bool CHECK>
__device__ inline void c5_load4(const void *p, int64_t base, int64_t lo, uint64_t len, int64_t e,
                                int64_t e1, bool ragged, uint32_t o[4], bool ok[4]) {
  int64_t v[4];
  if (!ragged || e + 4 <= e1) {
    if (W != 8) {
      uint32_t q[4];
      if (W == 4) {
        const uint4 t = *(const uint4 *)((const uint32_t *)p + e);
        q[0] = t.x;
        q[1] = t.y;
        q[2] = t.z;
        q[3] = t.w;
      } else {
        const U3 t = *(const U3 *)((const uint8_t *)p + 3 * e);
        q[0] = t.x & 0xFFFFFFu;
        q[1] = __builtin_amdgcn_alignbit(t.y, t.x, 24) & 0xFFFFFFu;
        q[2] = __builtin_amdgcn_alignbit(t.z, t.y, 16) & 0xFFFFFFu;
        q[3] = t.z >> 8;
      }
      if (!CHECK) {
        const uint32_t d = (uint32_t)(base - lo);
        o[0] = q[0] + d;
        o[1] = q[1] + d;
        o[2] = q[2] + d;
        o[3] = q[3] + d;
        ok[0] = ok[1] = ok[2] = ok[3] = true;
        return;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = base + (int64_t)q[k];
    } else {
      const longlong2 q0 = *(const longlong2 *)((const int64_t *)p + e);
      const longlong2 q1 = *(const longlong2 *)((const int64_t *)p + e + 2);
      v[0] = q0.x;
      v[1] = q0.y;
      v[2] = q1.x;
      v[3] = q1.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = e + k < e1 ? (W != 8 ? base + (int64_t)c5_off<W>(p, e + k) : ((const int64_t *)p)[e + k])
                        : lo - 1;  // out of range → dummy
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t x = v[k] - lo;
    o[k] = (uint32_t)x;
    ok[k] = CHECK || ragged ? (uint64_t)x < len : true;
  }
}

// Σ of v over the workgroup into *out (plain store by thread 0); red: ≥ 16 words of LDS.
__device__ inline void c5_tile_sum(uint32_t v, uint32_t *red, uint32_t *out) {
  const uint32_t w = (uint32_t)wave_reduce_sum((unsigned long long)v);
  __syncthreads();  // red may still be read by an earlier scan
  if (lane_id() == 0) red[threadIdx.x / WAVE] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int i = 0; i < (int)(blockDim.x / WAVE); ++i) t += red[i];
    *out = t;
  }
}

// P1.  ALIAS: r1 and r2 scan the same (start, end) columns — the directed
// 2-hop (a)-->(b)-->(c) — so one 8-B row gives both keys.  CHECK: range
// tests needed.  RAGGED: the single last partial tile.
// (Measured floors at s24, diagnostics since removed: keys straight from
// registers to the tile region, no LDS sort — P1's streaming floor; count
// phase and scan only, no scatter.)
// Raw row data of one load group (4 rows of a FOR24 / FOR32 column) and its
// decoding to node offsets (id − lo) — the !CHECK form of c5_load4.
template <int W>
using C5Raw = typename std::conditional<W == 3, U3, uint4>::type;

template <int W>
__device__ inline void c5_decode(const C5Raw<W> &t, uint32_t d, uint32_t o[4]) {
  if constexpr (W == 3) {
    o[0] = (t.x & 0xFFFFFFu) + d;
    o[1] = (__builtin_amdgcn_alignbit(t.y, t.x, 24) & 0xFFFFFFu) + d;
    o[2] = (__builtin_amdgcn_alignbit(t.z, t.y, 16) & 0xFFFFFFu) + d;
    o[3] = (t.z >> 8) + d;
  } else {
    o[0] = t.x + d;
    o[1] = t.y + d;
    o[2] = t.z + d;
    o[3] = t.w + d;
  }
}

// Raw row data at byte address p; NT = non-temporal loads (the stream is read once)
template <int W, bool NT>
__device__ inline C5Raw<W> c5_ld_raw(const uint8_t *p) {
  if constexpr (!NT) {
    return *(const C5Raw<W> *)p;
  } else if constexpr (W == 3) {
    const uint32_t *q = (const uint32_t *)p;
    return U3{__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1), __builtin_nontemporal_load(q + 2)};
  } else {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load((const v4u *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
}

// UPF (ALIAS, in-range, full tiles, FOR24 / FOR32): every load of the tile is
// issued before the first key is counted — 2 × GROUPS raw loads in flight per
// thread (96 B at FOR24) instead of one group ahead; the raw registers of a
// group die as its keys appear, so the peak stays within 64 VGPRs.  UPF 2:
// non-temporal loads (s24 P1 0.516 vs 0.521 ms with default-policy loads);
// UPF 3: also the FOR24 fields used raw when the bases are lo (0.512 ms).
// run_major: meta goes out run-major ([run][tile], what P3 reads: no transpose
// launch) and the full tiles are dealt to the XCDs in contiguous ranges (block b
// runs on XCD b mod 8), so the 32 tiles sharing a 128-B meta line are written
// through one L2 at about the same time and leave as whole lines.
__device__ inline int64_t c5_xcd_tile(int64_t b, int64_t g) {
  const int64_t per = g / 8;
  return b < 8 * per ? (b % 8) * per + b / 8 : b;
}

template <int W, bool ALIAS, bool CHECK, bool RAGGED, class SH, int UPF = 0>
// Self-loops go out as one plain uint32 per tile (tile_loops[t], summed by
// k_c3_units); every tile's workgroup also clears its share of the `zwords` words at zbuf
// (the run totals / work-list header of the post-P1 kernels) — no memset
// launches in front of or behind P1.
__global__ __launch_bounds__(C5_BLOCK) __attribute__((amdgpu_waves_per_eu(8))) void k_c5_partition(C5Cols<W> c, uint16_t *part,
                                                            uint32_t *meta,
                                                            uint32_t *tile_loops,
                                                            int64_t t_base, uint32_t *zbuf, int64_t zwords,
                                                            unsigned long long *zacc, int run_major) {
  constexpr int TILE = SH::TILE, MAXR = SH::MAXR;
  constexpr int RPT = TILE / C5_BLOCK, GROUPS = RPT / 4;
  constexpr int STAGE = c5_stage_keys<SH>();
  constexpr int RUNS_PT = (MAXR + C5_BLOCK - 1) / C5_BLOCK;
  __shared__ uint4 stage4[STAGE / 8];
  __shared__ uint32_t cur[MAXR];
  __shared__ uint32_t lds_scan[17];
  uint16_t *stage = (uint16_t *)stage4;
  const int64_t t = t_base + (run_major && !RAGGED ? c5_xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x);
  const int nr = 2 * c.nb;
  // pad keys: 8·(t mod 8) + slot-in-piece (P3 subtracts them per bin)
  const uint32_t pb = 8u * (uint32_t)(t & 7);
  const uint4 pad = make_uint4(pb | (pb + 1) << 16, (pb + 2) | (pb + 3) << 16,
                               (pb + 4) | (pb + 5) << 16, (pb + 6) | (pb + 7) << 16);
  (void)pad;  // pads are written per run after the scan (no stage prefill)
  for (int i = threadIdx.x; i <= nr; i += C5_BLOCK) cur[i] = 0;
  if (zbuf) {  // every tile's workgroup clears its share (the hand-off log makes it ~10^5 words)
    const int64_t per = (zwords + c.ntiles - 1) / c.ntiles, z0 = t * per, z1 = min<int64_t>(zwords, z0 + per);
    for (int64_t i = z0 + threadIdx.x; i < z1; i += C5_BLOCK) zbuf[i] = 0;
  }
  if (t == 0 && zacc && threadIdx.x < 3) zacc[threadIdx.x] = 0;  // [Σ, loops, done]
  __syncthreads();
  const int64_t e0 = t * TILE;
  const int64_t e1 = RAGGED ? min(e0 + TILE, c.n) : e0 + TILE;
  const uint32_t out_run0 = (uint32_t)c.nb << C2_BITS;
  const uint32_t dummy = (uint32_t)nr << C2_BITS;
  uint32_t kin[RPT], kout[RPT];
  uint32_t lp = 0;
  constexpr bool UPFRONT = UPF != 0 && ALIAS && !CHECK && !RAGGED && (W == 3 || W == 4);
  if constexpr (UPFRONT) {
    C5Raw<W> ru[GROUPS], rv[GROUPS];
#pragma unroll
    for (int g = 0; g < GROUPS; ++g) {
      const int64_t e = e0 + 4 * ((int64_t)g * C5_BLOCK + threadIdx.x);
      ru[g] = c5_ld_raw<W, UPF >= 2>((const uint8_t *)c.u1 + W * e);
      rv[g] = c5_ld_raw<W, UPF >= 2>((const uint8_t *)c.v1 + W * e);
    }
    const uint32_t du = (uint32_t)(c.bu1 - c.lo), dv = (uint32_t)(c.bv1 - c.lo);
    // D0 (UPF 3: FOR bases = lo, 24-bit multiply): offsets are the raw fields —
    // __umul24 reads only the low 24 bits, so no mask and no add; the self-loop
    // test compares the mixed keys (node_mix is a bijection on [0, 2^k))
    constexpr bool D0 = UPF == 3 && W == 3 && !SH::WIDE;
#pragma unroll
    for (int g = 0; g < GROUPS; ++g) {
      uint32_t x1[4], y1[4];
      if constexpr (D0) {
        x1[0] = ru[g].x;
        x1[1] = __builtin_amdgcn_alignbit(ru[g].y, ru[g].x, 24);
        x1[2] = __builtin_amdgcn_alignbit(ru[g].z, ru[g].y, 16);
        x1[3] = ru[g].z >> 8;
        y1[0] = rv[g].x;
        y1[1] = __builtin_amdgcn_alignbit(rv[g].y, rv[g].x, 24);
        y1[2] = __builtin_amdgcn_alignbit(rv[g].z, rv[g].y, 16);
        y1[3] = rv[g].z >> 8;
      } else {
        c5_decode<W>(ru[g], du, x1);
        c5_decode<W>(rv[g], dv, y1);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = 4 * g + k;
        kin[j] = node_mix_t<SH::WIDE>(y1[k], c.mix);
        kout[j] = node_mix_t<SH::WIDE>(x1[k], c.mix) + out_run0;
        if constexpr (D0)
          lp += kout[j] - kin[j] == out_run0 ? 1u : 0u;
        else
          lp += y1[k] == x1[k] ? 1u : 0u;
        atomicAdd(&cur[kin[j] >> C2_BITS], 1u);
        atomicAdd(&cur[kout[j] >> C2_BITS], 1u);
      }
      asm volatile("" : "+v"(lp));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // ALIAS: the next group's two loads are issued before this group's hashing
  // and counting (double-buffered registers; the unrolled loop renames them)
  uint32_t px[2][4], py[2][4];
  bool pox[2][4], poy[2][4];
  if (ALIAS && !UPFRONT) {
    const int64_t e = e0 + 4 * (int64_t)threadIdx.x;
    c5_load4<W, CHECK>(c.u1, c.bu1, c.lo, c.len, e, e1, RAGGED, px[0], pox[0]);
    c5_load4<W, CHECK>(c.v1, c.bv1, c.lo, c.len, e, e1, RAGGED, py[0], poy[0]);
  }
#pragma unroll
  for (int g = 0; g < (UPFRONT ? 0 : GROUPS); ++g) {
    const int64_t e = e0 + 4 * ((int64_t)g * C5_BLOCK + threadIdx.x);
    uint32_t x1[4], y1[4], x2[4], y2[4];
    bool okx1[4], oky1[4], okx2[4], oky2[4];
    if (ALIAS) {
      if (g + 1 < GROUPS) {
        const int64_t en = e + 4 * C5_BLOCK;
        c5_load4<W, CHECK>(c.u1, c.bu1, c.lo, c.len, en, e1, RAGGED, px[(g + 1) & 1], pox[(g + 1) & 1]);
        c5_load4<W, CHECK>(c.v1, c.bv1, c.lo, c.len, en, e1, RAGGED, py[(g + 1) & 1], poy[(g + 1) & 1]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x1[k] = px[g & 1][k];
        y1[k] = py[g & 1][k];
        okx1[k] = pox[g & 1][k];
        oky1[k] = poy[g & 1][k];
      }
    } else {
      c5_load4<W, CHECK>(c.u1, c.bu1, c.lo, c.len, e, e1, RAGGED, x1, okx1);
      c5_load4<W, CHECK>(c.v1, c.bv1, c.lo, c.len, e, e1, RAGGED, y1, oky1);
      c5_load4<W, CHECK>(c.u2, c.bu2, c.lo, c.len, e, e1, RAGGED, x2, okx2);
      c5_load4<W, CHECK>(c.v2, c.bv2, c.lo, c.len, e, e1, RAGGED, y2, oky2);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = 4 * g + k;
      const uint32_t b = y1[k];                   // end(r1)
      const uint32_t cq = ALIAS ? x1[k] : x2[k];  // start(r2)
      const bool in_ok = okx1[k] & oky1[k];       // start(r1) ∈ S_a, end(r1) ∈ S_b
      const bool out_ok = ALIAS ? in_ok : (okx2[k] & oky2[k]);
      kin[j] = node_mix_t<SH::WIDE>(b, c.mix);
      kout[j] = node_mix_t<SH::WIDE>(cq, c.mix) + out_run0;
      if (CHECK || RAGGED) {
        kin[j] = in_ok ? kin[j] : dummy;
        kout[j] = out_ok ? kout[j] : dummy;
      }
      lp += (in_ok & out_ok & (b == cq)) ? 1u : 0u;
      // count only (no return: no wait); positions come from a second pass
      atomicAdd(&cur[kin[j] >> C2_BITS], 1u);
      atomicAdd(&cur[kout[j] >> C2_BITS], 1u);
    }
    asm volatile("" : "+v"(lp));        // keep the self-loop sum here (no raw ids kept alive)
    __builtin_amdgcn_sched_barrier(0);  // bound what the scheduler keeps in flight
  }
  // launder the keys: stops the compiler from keeping the count phase's LDS
  // addresses alive across the scan (extra VGPRs → spills)
#pragma unroll
  for (int j = 0; j < RPT; ++j) asm volatile("" : "+v"(kin[j]), "+v"(kout[j]));
  __syncthreads();
  // exclusive scan of the 8-padded run sizes (the dummy run nr last)
  uint32_t cs[RUNS_PT], sum = 0;
#pragma unroll
  for (int q = 0; q < RUNS_PT; ++q) {
    const int r = RUNS_PT * threadIdx.x + q;
    cs[q] = r <= nr ? cur[r] : 0u;
    sum += (cs[q] + 7) & ~7u;
  }
  uint32_t total;
  uint32_t ex = block_exclusive_scan(sum, lds_scan, total);
#pragma unroll
  for (int q = 0; q < RUNS_PT; ++q) {
    const int r = RUNS_PT * threadIdx.x + q;
    if (r <= nr) cur[r] = ex;
    if (r < nr) {
      meta[run_major ? (int64_t)r * c.ntiles + t : t * nr + r] = (ex >> 3) | (cs[q] << 16);  // [tile][run] or [run][tile]
      // pad slots of the run's last piece: 8·(t mod 8) + slot (P3 subtracts them per bin)
      for (uint32_t p = ex + cs[q]; p & 7u; ++p) stage[p] = (uint16_t)(pb + (p & 7u));
    }
    ex += (cs[q] + 7) & ~7u;
  }
  __syncthreads();
  // counting sort: each key claims the next slot of its run (the order inside
  // a run is free — P3 only counts)
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    stage[atomicAdd(&cur[kin[j] >> C2_BITS], 1u)] = (uint16_t)kin[j];
    stage[atomicAdd(&cur[kout[j] >> C2_BITS], 1u)] = (uint16_t)kout[j];
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  // the stage IS the region's layout: contiguous 16-B copy-out
  uint4 *dst = (uint4 *)(part + t * c.rstride);
  for (uint32_t i = threadIdx.x; i < total / 8; i += C5_BLOCK) dst[i] = stage4[i];
  c5_tile_sum(lp, lds_scan, tile_loops + t);
}

// [tile][run] → [run][tile] and per-run totals.  A block moves 32 runs ×
// tt (≤ 256) tiles through LDS in ONE round: every thread issues its tt/8
// row loads before the single barrier (the old 32-tile rounds kept 4 loads
// in flight per thread), then each run's tt words go out as one contiguous
// row.  Run totals are summed during the loads and added once per run per
// block (a per-block partial row summed by k_c3_units instead was measured
// slower: the one-block units kernel turns latency bound).
constexpr int C3_TT = 256;
// tile_loops (2-hop pipeline): the blocks of run row 0 also add their tiles'
// self-loop counts (P1's per-tile plain stores) into *loops.
__device__ __forceinline__ void c3_transpose_body(uint32_t (*tilebuf)[33], const uint32_t *meta,
                                                  uint32_t *meta_t, int64_t ntiles, int nr,
                                                  unsigned long long *run_total, int64_t tt, uint32_t *bsum,
                                                  const uint32_t *tile_loops, unsigned long long *loops) {
  __shared__ uint32_t part[8][33];
  const int r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads = 32 × 8
  const int64_t tb = (int64_t)blockIdx.x * tt;
  const int64_t tn = min<int64_t>(tt, ntiles - tb);  // tiles in this block
  const int r = r0 + tx;
  uint32_t cnt = 0;
#pragma unroll 8
  for (int k = ty; k < tt; k += 8) {
    const uint32_t v = (k < tn && r < nr) ? meta[(tb + k) * nr + r] : 0u;
    tilebuf[k][tx] = v;
    cnt += v >> 16;
  }
  part[ty][tx] = cnt;
  if (tile_loops && blockIdx.y == 0 && threadIdx.x < 64) {  // one wave: this block's tiles
    unsigned long long l = 0;
    for (int64_t k = threadIdx.x; k < tn; k += 64) l += tile_loops[tb + k];
    l = wave_reduce_sum(l);
    if (threadIdx.x == 0 && l) atomicAdd(loops, l);
  }
  __syncthreads();
  if (ty == 0) {
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) c += part[q][tx];
    if (c && r < nr) atomicAdd(&run_total[r], (unsigned long long)c);
    // per-(run, tile block) key counts: the balanced P3's split points
    if (bsum && r < nr) bsum[(int64_t)r * gridDim.x + blockIdx.x] = c;
  }
  if (!meta_t) return;  // run totals only (P3 reads meta in place)
  const int lt = __builtin_ctzll((unsigned long long)tt);  // tt is a power of two
  for (int idx = threadIdx.x; idx < 32 * tt; idx += 256) {
    const int q = idx >> lt, i = idx & (int)(tt - 1);
    if (i < tn && r0 + q < nr) meta_t[(int64_t)(r0 + q) * ntiles + tb + i] = tilebuf[i][q];
  }
}
__global__ __launch_bounds__(256) void k_c3_transpose(const uint32_t *meta, uint32_t *meta_t,
                                                       int64_t ntiles, int nr,
                                                       unsigned long long *run_total, int64_t tt,
                                                       uint32_t *bsum = nullptr,
                                                       const uint32_t *tile_loops = nullptr,
                                                       unsigned long long *loops = nullptr) {
  __shared__ uint32_t tilebuf[C3_TT][33];
  c3_transpose_body(tilebuf, meta, meta_t, ntiles, nr, run_total, tt, bsum, tile_loops, loops);
}

struct C3Unit {
  int32_t run;
  int32_t exclusive;  // the only unit writing (run, slice) → plain stores
  int64_t t0, t1;     // tile range
  int32_t slice;      // histogram slice it writes
  int32_t pad;
};

// Histogram slices: a graph with few runs (small, or one rank's share of a
// node-partitioned graph) still needs 2 full waves of P3 units on 256 CUs, so every run is cut into S tile ranges, each counted into its own
// slice of the histograms with plain stores; the dot sums the slices.
static int c5_slices(int nr) {
  // one unit per CU: G = 8 rank (64 runs) S = 4 → 0.250 ms/rank vs S = 8 0.271, S = 2 0.300
  return std::min(8, std::max(1, (256 + nr - 1) / nr));
}

constexpr int C3_UBLOCK = 1024;

// Work list of P3 on the device.  With hash-partitioned runs the run sizes
// are near-uniform (max/mean ≈ 1.3 at s24), so every run is ONE unit — an
// exclusive one, whose plain stores cover all bins of its bucket: the
// histograms need no memset, empty runs included (they store zeros).  A run
// holding more than twice the mean (a hub-heavy bucket) is split into tile
// ranges that flush with atomic adds into bins cleared by k_c3_zero.  Units
// stay in run order: P3 maps them onto XCDs in groups of consecutive runs
// (c3_unit_of).
struct C3Sides {
  int nb;              // runs per side: runs [0, nb) in, [nb, 2·nb) out
  int64_t t0[2], t1[2];  // tile range holding each side's segments
  int split_x16;       // a run is split when it holds > split_x16/16 × the mean
  int packed = 0;      // static units store their counters as packed uint16 pairs
                       // (word i of bucket b of slice k at (k·nb + b)·2^15 + i); the
                       // hand-off log then holds side bins b·2^16 + key, applied by
                       // k_c5_dot_packed (no k_c3_overflow)
  int pairs = 0;       // (fused 2-hop, one slice) exclusive units store packed uint16
                       // pairs in the first half of their bucket's 2^16 words (half
                       // the flush and dot bytes); split runs keep one uint32 per bin
  int32_t *claim = nullptr;  // the units kernel's split flags: non-null → P3's split units
                             // clear their own buckets (claim / ready bits, no k_c3_zero)
};

// CAPF_P3_SPLIT (tuning): split threshold in units of the mean run size
static int c3_split_x16() {
  const char *e = getenv("CAPF_P3_SPLIT");
  return e ? std::max(1, (int)(16.0 * atof(e))) : 32;
}

// The P1 → P3 path of the fused 2-hop count: P1's per-tile self-loops (summed
// into acc3[1] by the transpose), acc3 = [Σ in·out, self-loops, done] cleared
// by P1's tile-0 workgroup, and where the hand-off log goes.
struct C3Post {
  const uint32_t *tile_loops;
  int64_t ntiles;
  unsigned long long *acc3;
  C2Spill *spill;  // host side: non-null → the hand-off log goes to the dot kernel
};

// The work-list computation (one workgroup, RPT runs per thread, nr ≤
// RPT·blockDim.x).  (Per-(run, block) partial rows stored by the transpose
// and summed here instead of the run-total adds: T 38 vs 34 µs, U 12 vs 9 µs.)
struct C3UnitsOut {
  C3Unit *units;
  int32_t *nunits, *split;
};
template <int RPT>
__device__ void c3_units_body(const unsigned long long *run_total, int nr, const C3Sides &sd, int S,
                              const C3UnitsOut &uo) {
  __shared__ unsigned long long lds64[17];
  __shared__ uint32_t lds32[17];
  unsigned long long cnt[RPT], tot = 0;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int r = RPT * threadIdx.x + q;
    cnt[q] = r >= nr ? 0ull : run_total[r];
    tot += cnt[q];
  }
  unsigned long long total;
  block_exclusive_scan(tot, lds64, total);
  const unsigned long long target =
      max((unsigned long long)sd.split_x16 * total / (16ull * (unsigned long long)max(nr, 1)), 65536ull);
  uint32_t nu[RPT], nsum = 0;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int r = RPT * threadIdx.x + q;
    const int sdi = r >= sd.nb ? 1 : 0;
    const int64_t maxsplit = max<int64_t>(1, (sd.t1[sdi] - sd.t0[sdi]) / 256);
    const uint32_t hub = cnt[q] ? (uint32_t)min<int64_t>((int64_t)((cnt[q] + target - 1) / target), maxsplit) : 1u;
    nu[q] = r >= nr ? 0u : max(hub, (uint32_t)S);
    nsum += nu[q];
  }
  uint32_t ntot;
  uint32_t off = block_exclusive_scan(nsum, lds32, ntot);
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int r = RPT * threadIdx.x + q;
    if (!nu[q]) continue;
    const int sdi = r >= sd.nb ? 1 : 0;
    const int64_t b = sd.t0[sdi], len = sd.t1[sdi] - sd.t0[sdi];
    for (uint32_t k = 0; k < nu[q]; ++k) {
      C3Unit u;
      u.run = r;
      u.exclusive = nu[q] == (uint32_t)S;
      u.t0 = cnt[q] ? b + len * k / nu[q] : b;
      u.t1 = cnt[q] ? b + len * (k + 1) / nu[q] : b;
      u.slice = (int32_t)(k % (uint32_t)S);
      u.pad = 0;
      uo.units[off + k] = u;
    }
    off += nu[q];
    uo.split[r] = nu[q] > (uint32_t)S;
  }
  if (threadIdx.x == 0) *uo.nunits = (int32_t)ntot;
}


__global__ __launch_bounds__(C3_UBLOCK) void k_c3_units(unsigned long long *run_total, int nr, C3Sides sd,
                                                         int S, C3UnitsOut uo) {
  c3_units_body<2>(run_total, nr, sd, S, uo);
}

// XCD-aware unit placement.  Workgroup i runs on XCD i mod 8, and P3 holds
// one workgroup per CU (128 KiB LDS), 32 per XCD.  Runs r and r+1 are
// adjacent in every tile's region, so their segments share 128-B lines:
// giving each XCD 32 CONSECUTIVE units per 256-workgroup wave lets those
// blocks (sweeping the tiles in the same order at the same pace) hit the
// shared lines in their own L2 instead of fetching each line once per run.
__device__ inline int c3_unit_of(int i) {
  return (i / 256) * 256 + (i % 8) * 32 + (i % 256) / 8;
}

// P3 counters: bins are packed uint16 pairs, word w holds bin w (low half)
// and bin w + 2^15 (high half).  The add that lifts a half from below 2^15
// to 2^15 or more hands 2^15 off to the overflow log and takes it back out
// of the word, so a half never exceeds 2^15 + (sum of the adds in flight on
// the CU: ≤ 1024 lanes × 8 for the merged hub adds) < 2^16: exact, no carry.
struct C3Ovf {
  uint2 *log;  // (histogram index, side | count << 1): hand-offs (count 2^15) and hot-key totals
  uint32_t *n;
  uint32_t cap;
};

// Slow path of an overflowing add (rare: a bin reached 2^15 within the unit).
__device__ inline void c3_handoff(uint32_t *w, uint32_t inc, uint32_t hidx, uint32_t side,
                                        const C3Ovf &o) {
  atomicSub(w, inc << 15);
  const uint32_t k = atomicAdd(o.n, 1u);
  if (k < o.cap) o.log[k] = make_uint2(hidx, side | (1u << 16));
}

// P3 pieces per lane per step, double-buffered (s24: 2 → 0.49 ms; 4 spills → 0.66 ms)
constexpr int C5_PPS = 2;

struct C5WaveTab {
  uint32_t pre[WAVE + 1];  // exclusive prefix of the 64 tiles' piece counts, + total
  uint32_t qb[WAVE];       // first piece of each segment (uint4 index into part)
};

constexpr size_t C5_GATHER_LDS =
    4 * (C2_WORDS + C5_CORR) + 2 * sizeof(C5WaveTab) * (C5_BLOCK / WAVE);

__device__ inline int64_t uniform64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// P3.  The wave takes 64 tiles of its unit at a time and treats their
// segments (8-key padded, 16-B aligned pieces) as ONE sequence: lane l of
// step s handles piece s·64·PPS + l (+ 64·j), found by a 6-step binary search
// in the wave's LDS prefix table.  Consecutive lanes read consecutive pieces
// of a segment — coalesced 128-B lines (lane-per-segment reads of 64 distinct
// lines run at 3.2 TB/s, coalesced random 128-B lines at 5.7 TB/s:
// tools/bench_gather.hip) — and every lane holds a live piece.  Pad keys
// (8·(t mod 8) + slot) and the keys of past-the-end lanes (= lane) are
// counted like the others and subtracted from bins 0..63 at the flush.
//
// Software-pipelined: the wave walks ONE stream of steps across its batches;
// the pieces of step i+1 (search + 16-B loads, possibly in the next batch) are
// issued before the LDS atomics of step i.  Batch tables are double-buffered
// in LDS, the next batch's meta word is prefetched while the current table is
// built, piece buffers ping-pong (no register copies → no early vmcnt wait).
//
// What bounds it (s24, measured): 0.49 ms; loads + search alone 0.29 ms; with
// the keys spread so no two lanes of an atomic share a word 0.30 ms.
// R-MAT's skew puts ~2.4 lanes of a typical 64-lane ds_add on one word
// (tools: simulated per run), and same-word lanes serialise in the LDS atomic
// unit.  Voting out lane 0's key, half-wave atomics and non-returning atomics
// were measured and do not help (the duplicates are spread over many
// moderately hot keys); so were a per-wave hot-key register, rotating and
// fully deduplicating each piece's 8 keys, and a third piece buffer depth vs two
// (no gain at s24).
template <int PPS>
__global__ __launch_bounds__(C5_BLOCK) void k_c5_gather(const C3Unit *units,
                                                            const int32_t *nunits,
                                                            const uint16_t *part,
                                                            const uint32_t *meta_t, int64_t ntiles,
                                                            int nb, int64_t rstride, uint32_t *h_in,
                                                            uint32_t *h_out, int64_t slice_stride,
                                                            C3Ovf ovf,
                                                            C3Sides sd, int S, int64_t mstride) {
  // units == null: the static work list of a node-partitioned rank — unit
  // (run, k) counts tile range k of S of the run's side into slice k
  const int nu = units ? *nunits : 2 * sd.nb * S;
  const int ui = c3_unit_of((int)blockIdx.x);
  if (ui >= nu) return;
  extern __shared__ __attribute__((aligned(16))) uint32_t words[];
  constexpr int NW = C5_BLOCK / WAVE;
  constexpr uint32_t STEP = WAVE * PPS;
  uint32_t *corr = words + C2_WORDS;
  C5WaveTab *tabs = (C5WaveTab *)(corr + C5_CORR);  // 2 per wave
  C3Unit u;
  if (units) {
    u = units[ui];
  } else {
    const int k = ui % S, sdi = ui / S >= sd.nb ? 1 : 0;
    const int64_t len = sd.t1[sdi] - sd.t0[sdi];
    u.run = ui / S;
    u.exclusive = 1;
    u.t0 = sd.t0[sdi] + len * k / S;
    u.t1 = sd.t0[sdi] + len * (k + 1) / S;
    u.slice = k;
  }
  const uint32_t side = u.run >= nb ? 1u : 0u;
  uint32_t *hist = side ? h_out : h_in;
  const uint32_t log_base = (uint32_t)((int64_t)(u.run % nb) * C2_BW);  // packed: side bin of key 0
  const uint32_t hist_base = (uint32_t)(u.slice * slice_stride + (int64_t)(u.run % nb) * C2_BW);
  for (int i = threadIdx.x; i < C2_WORDS + C5_CORR; i += C5_BLOCK) words[i] = 0;
  // A split run's units flush with atomic adds into bins that must start at
  // zero: the first unit of (run, slice) to start sets its claim bit and clears
  // the bucket in HBM, then its ready bit; the others wait for the ready bit
  // before flushing.  A waiter only ever waits on a workgroup already running
  // (the claimer), so the wait ends — and k_c3_zero plus a kernel boundary go.
  const bool zsplit = sd.claim && !u.exclusive;
  if (zsplit) {
    __shared__ int zown;
    if (threadIdx.x == 0) zown = !(atomicOr(&sd.claim[u.run], 2 << u.slice) & (2 << u.slice));
    __syncthreads();
    if (zown) {
      uint4 *z = (uint4 *)(hist + hist_base);
      for (int i = threadIdx.x; i < C2_BW / 4; i += C5_BLOCK) z[i] = make_uint4(0, 0, 0, 0);
      __threadfence();
      __syncthreads();
      if (threadIdx.x == 0) atomicOr(&sd.claim[u.run], 512 << u.slice);
    }
  }
  __syncthreads();
  // wave-uniform values live in SGPRs: uniform loop control, no exec masking
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = lane_id();
  C5WaveTab *tab2 = tabs + 2 * wave;
  const uint4 *part4 = (const uint4 *)part;
  // run-major meta_t (mstride 1) or P1's tile-major meta read in place (mstride nr)
  const uint32_t *m = meta_t + (mstride == 1 ? (int64_t)u.run * ntiles : (int64_t)u.run);
  const int64_t ut = u.t1 - u.t0;
  const int64_t w0 = uniform64(u.t0 + ut * wave / NW), w1 = uniform64(u.t0 + ut * (wave + 1) / NW);
  const uint32_t rs8 = (uint32_t)(rstride / 8);
  uint32_t padc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t dead = 0;
  const uint4 dead_keys = make_uint4(lane | lane << 16, lane | lane << 16, lane | lane << 16,
                                     lane | lane << 16);
  // batch setup: table of tiles [tb, tb + 64) into tab2[buf]; returns the piece total
  uint32_t wpre = w0 + lane < w1 ? m[(w0 + lane) * mstride] : 0u;  // meta word of the next batch
  auto setup = [&](int64_t tb, int buf) -> uint32_t {
    const int64_t t = tb + lane;
    const uint32_t w = wpre;
    const uint32_t len = w >> 16, nq = (len + 7) >> 3, r = len & 7;
#pragma unroll
    for (int e = 1; e < 8; ++e) padc[e] += (r != 0 && r <= (uint32_t)e) ? 1u : 0u;
    const uint32_t inc = wave_inclusive_scan(nq);
    tab2[buf].pre[lane] = inc - nq;
    if (lane == WAVE - 1) tab2[buf].pre[WAVE] = inc;
    tab2[buf].qb[lane] = (uint32_t)t * rs8 + (w & 0xFFFF);
    // prefetch the next batch's meta word only now that `w` is dead, so the
    // load lands in the same register (no copy → no early wait)
    __builtin_amdgcn_sched_barrier(0);
    const int64_t tn = tb + WAVE + lane;
    wpre = tn < w1 ? m[tn * mstride] : 0u;
    __builtin_amdgcn_wave_barrier();
    return (uint32_t)__builtin_amdgcn_readlane(inc, WAVE - 1);
  };
  // total > 0.  Past-the-end lanes load a valid piece (the last one) and
  // replace it with their dead keys: every load is unconditional, so the
  // wait before the counting only covers the step being counted.
  auto fetch = [&](int buf, uint32_t p0, uint32_t total, uint4 *v) {
    const C5WaveTab &tab = tab2[buf];
#pragma unroll
    for (int j = 0; j < PPS; ++j) {
      const uint32_t p = p0 + j * WAVE + lane;
      const uint32_t pc = min(p, total - 1);
      uint32_t k = 0;
#pragma unroll
      for (int b = WAVE / 2; b > 0; b >>= 1)
        if (tab.pre[k + b] <= pc) k += b;
      v[j] = part4[tab.qb[k] + (pc - tab.pre[k])];
    }
  };
  // Counting one step: 8 keys per piece, PPS pieces per lane (hub-key merge
  // below).  `acc` ORs every post-add word: bit 15 of a half set ⇒ some add
  // may have lifted that half to 2^15 → the exact (rare) hand-off check.
  auto count = [&](const uint4 *v, uint32_t p0, uint32_t total) {
    uint32_t acc = 0;
    uint32_t old[PPS][8];
    uint32_t n0[PPS], n1[PPS];
    bool dup[PPS][8];
#pragma unroll
    for (int j = 0; j < PPS; ++j) {
      const bool live = p0 + j * WAVE + lane < total;
      dead += live ? 0u : 1u;
      const uint32_t wd[4] = {live ? v[j].x : dead_keys.x, live ? v[j].y : dead_keys.y,
                              live ? v[j].z : dead_keys.z, live ? v[j].w : dead_keys.w};
      {
        // hub keys: the keys of the piece equal to its first (second) key
        // are added once, as a count ≤ 8, by slot 0 (1) (R-MAT skew puts a hub's key in
        // many slots of its run's pieces, and same-word lanes of one ds_add
        // serialise); the other slots add 1 each, lanes holding a duplicate
        // sit that atomic out
        const uint32_t k0 = wd[0] & 0xFFFF, k1 = wd[0] >> 16;
        dup[j][0] = false;
        dup[j][1] = k1 == k0;
        n0[j] = dup[j][1] ? 2u : 1u;
        n1[j] = 1;
#pragma unroll
        for (int e = 2; e < 8; ++e) {
          const uint32_t key = (e & 1) ? wd[e >> 1] >> 16 : wd[e >> 1] & 0xFFFF;
          const bool d0 = key == k0, d1 = !d0 && key == k1;  // k1 == k0 ⇒ d0 already
          dup[j][e] = d0 || d1;
          n0[j] += d0 ? 1u : 0u;
          n1[j] += d1 ? 1u : 0u;
        }
        const uint32_t inc0 = n0[j] << ((k0 >> 15) << 4);
        old[j][0] = atomicAdd(&words[k0 & (C2_WORDS - 1)], inc0);
        acc |= old[j][0] + inc0;
        const uint32_t inc1 = n1[j] << ((k1 >> 15) << 4);
        old[j][1] = 0;
        if (!dup[j][1]) old[j][1] = atomicAdd(&words[k1 & (C2_WORDS - 1)], inc1);
        acc |= old[j][1] + inc1;
#pragma unroll
        for (int e = 2; e < 8; ++e) {
          const uint32_t key = (e & 1) ? wd[e >> 1] >> 16 : wd[e >> 1] & 0xFFFF;
          const uint32_t unit = (key >> 15) * 0xFFFFu + 1u;
          old[j][e] = 0;
          if (!dup[j][e]) old[j][e] = atomicAdd(&words[key & (C2_WORDS - 1)], unit);
          acc |= old[j][e] + unit;
        }
      }
    }
    if (acc & 0x80008000u) {
      // rare: some half reached 2^15 — find the add(s) that crossed it (the
      // half before the add was < 2^15 and the add took it to ≥ 2^15)
#pragma unroll
      for (int j = 0; j < PPS; ++j) {
        const bool live = p0 + j * WAVE + lane < total;
        const uint32_t wd[4] = {live ? v[j].x : dead_keys.x, live ? v[j].y : dead_keys.y,
                                live ? v[j].z : dead_keys.z, live ? v[j].w : dead_keys.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t key = (e & 1) ? wd[e >> 1] >> 16 : wd[e >> 1] & 0xFFFF;
          const uint32_t inc = e == 0 ? n0[j] : e == 1 ? n1[j] : 1u;
          if (e > 0 && dup[j][e]) continue;
          const uint32_t sh = (key >> 15) << 4;
          const uint32_t oh = (old[j][e] >> sh) & 0xFFFFu;
          if (oh < 0x8000u && oh + inc >= 0x8000u)
            c3_handoff(&words[key & (C2_WORDS - 1)], 1u << sh, (sd.packed ? log_base : hist_base) + key,
                       side, ovf);
        }
      }
    }
  };
  if (w0 < w1) {
    int64_t tb = uniform64(w0);
    int buf = 0;
    uint32_t total = setup(tb, buf), p0 = 0;
    while (total == 0) {  // first non-empty batch
      tb += WAVE;
      if (tb >= w1) break;
      buf ^= 1;
      total = setup(tb, buf);
    }
    if (total) {
      // the next step: the same batch, or the next non-empty one
      // scalar (wave-uniform) loop state: readfirstlane keeps it in SGPRs
      auto advance = [&]() -> bool {
        if (p0 + STEP < total) {
          p0 = (uint32_t)__builtin_amdgcn_readfirstlane(p0 + STEP);
          return true;
        }
        do {
          tb = uniform64(tb + WAVE);
          if (tb >= w1) return false;
          buf ^= 1;
          total = setup(tb, buf);
          p0 = 0;
        } while (total == 0);
        return true;
      };
      {
        // three rotating piece buffers: the loads of steps i+1 and i+2 are in
        // flight while step i counts (unrolled by 3, no register copies)
        uint4 va[PPS], vb[PPS], vc[PPS];
        uint32_t pa, ta, pb, tb2, pc, tc;
        pa = p0;
        ta = total;
        fetch(buf, p0, total, va);
        if (!advance()) {
          count(va, pa, ta);
        } else {
          pb = p0;
          tb2 = total;
          fetch(buf, p0, total, vb);
          for (;;) {
            if (!advance()) {
              count(va, pa, ta);
              count(vb, pb, tb2);
              break;
            }
            pc = p0;
            tc = total;
            fetch(buf, p0, total, vc);
            count(va, pa, ta);
            if (!advance()) {
              count(vb, pb, tb2);
              count(vc, pc, tc);
              break;
            }
            pa = p0;
            ta = total;
            fetch(buf, p0, total, va);
            count(vb, pb, tb2);
            if (!advance()) {
              count(vc, pc, tc);
              count(va, pa, ta);
              break;
            }
            pb = p0;
            tb2 = total;
            fetch(buf, p0, total, vb);
            count(vc, pc, tc);
          }
        }
      }
    }
  }
  const uint32_t pcls = 8u * (uint32_t)((w0 + lane) & 7);
#pragma unroll
  for (int e = 1; e < 8; ++e)
    if (padc[e]) atomicAdd(&corr[pcls + e], padc[e]);
  if (dead) atomicAdd(&corr[lane], 8 * dead);
  if (zsplit && threadIdx.x == 0)
    while (!(__hip_atomic_load(&sd.claim[u.run], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) & (512 << u.slice)))
      __builtin_amdgcn_s_sleep(4);
  __syncthreads();
  if (sd.packed) {  // exclusive static unit: one packed word per bin pair
    uint32_t *h = hist + ((int64_t)u.slice * nb + u.run % nb) * C2_WORDS;
    for (int i = threadIdx.x; i < C2_WORDS; i += C5_BLOCK) h[i] = words[i] - (i < C5_CORR ? corr[i] : 0u);
  } else
  if (sd.pairs && u.exclusive) {  // packed pairs (lo: bin i, hi: bin i + 2^15)
    uint32_t *h = hist + hist_base;
    for (int i = threadIdx.x; i < C2_WORDS; i += C5_BLOCK) h[i] = words[i] - (i < C5_CORR ? corr[i] : 0u);
  } else
  for (int i = threadIdx.x; i < C2_WORDS; i += C5_BLOCK) {
    const uint32_t w = words[i];
    const uint32_t lo = (w & 0xFFFF) - (i < C5_CORR ? corr[i] : 0u), hi = w >> 16;
    uint32_t *h = hist + hist_base + i;
    if (u.exclusive) {
      h[0] = lo;
      h[C2_WORDS] = hi;
    } else {
      if (lo) atomicAdd(h, lo);
      if (hi) atomicAdd(h + C2_WORDS, hi);
    }
  }

}

// Adds the handed-off 2^15 units (after every P3 store has landed).
__global__ __launch_bounds__(256) void k_c3_overflow(C3Ovf o, uint32_t *h_in, uint32_t *h_out) {
  const uint32_t n = min(*o.n, o.cap);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint2 e = o.log[i];
    atomicAdd(&((e.y & 1u) ? h_out : h_in)[e.x], e.y >> 1);
  }
}

template <int W, bool ALIAS, bool CHECK, class SH>
static void launch_c5(Session *s, const C5Cols<W> &c, uint16_t *part, uint32_t *meta,
                      uint32_t *tile_loops, uint32_t *zbuf, int64_t zwords, unsigned long long *zacc,
                      int run_major = 0) {
  const int64_t nfull = c.n / SH::TILE;
  if (nfull > 0) {
    auto kern = c.bu1 == c.lo && c.bv1 == c.lo && W == 3 && !SH::WIDE
                    ? k_c5_partition<W, ALIAS, CHECK, false, SH, 3>
                    : k_c5_partition<W, ALIAS, CHECK, false, SH, 2>;
    hipLaunchKernelGGL(kern, dim3((unsigned)nfull), dim3(C5_BLOCK), 0, s->stream, c, part, meta,
                       tile_loops, (int64_t)0, zbuf, zwords, zacc, run_major);
    KERNEL_CHECK();
  }
  if (nfull < c.ntiles) {  // the ragged last tile
    hipLaunchKernelGGL((k_c5_partition<W, ALIAS, true, true, SH>), dim3(1), dim3(C5_BLOCK), 0,
                       s->stream, c, part, meta, tile_loops, nfull, zbuf, zwords, zacc, run_major);
    KERNEL_CHECK();
  }
}

// Everything after P1: meta transpose + run totals, the work list, P3, the
// overflow hand-offs.  `part`/`meta` hold ntiles tiles of nr = 2·sd.nb runs.
// Histograms: S slices (c5_slices) of sd.nb·64 Ki counters per side, slice s
// at h_in/h_out + s·slice_stride; every counter of every slice is written.
// Bytes of c5_post's work area (run totals, counters, split flags, units, the
// hand-off log) and its leading words that must start at zero.
static int64_t c5_post_acc_bytes(int nr, int S, int split_x16, int64_t nkeys, int *max_units_out,
                                 uint32_t *ovf_cap_out) {
  // runs × slices + hub splits (≤ 2 per run beyond the slices), whole XCD waves
  // Σ_runs max(S, ⌈cnt/target⌉) ≤ S·nr + nr + total/target, target ≥ split/16 × mean
  const int max_units = (S * nr + nr + 16 * nr / std::max(1, split_x16) + 2 + 255) / 256 * 256;
  // every overflow event consumes 2^15 adds of one half-counter within one unit
  const uint32_t ovf_cap = (uint32_t)(nkeys / (1 << 15) + 64 + 16 * (int64_t)max_units);
  if (max_units_out) *max_units_out = max_units;
  if (ovf_cap_out) *ovf_cap_out = ovf_cap;
  // run_total[nr] | nunits[4] | bdone[nr] | hand-off log | split[nr] | rnu[nr] | units
  return 8 * nr + 16 + 12 * nr + (int64_t)sizeof(C3Unit) * max_units + 8 * (int64_t)ovf_cap;
}
// words that start at zero: run totals, unit / event / done counters, bucket counters
// (and the hand-off log: P3's bucket-dot epilogue may read a reserved slot
// that another bucket's unit has not written yet — a zero entry adds nothing)
static int64_t c5_post_zero_words(int nr, uint32_t ovf_cap, bool with_split = false) {
  return (8 * (int64_t)nr + 16 + 4 * (int64_t)nr + 8 * (int64_t)ovf_cap + (with_split ? 4 * (int64_t)nr : 0)) / 4;
}

static void c5_post(Session *s, const uint16_t *part, const uint32_t *meta, const C3Sides &sd,
                    int64_t ntiles, int64_t rstride, int64_t nkeys, int S, uint32_t *h_in,
                    uint32_t *h_out, int64_t slice_stride, bool static_units = false,
                    C3Ovf *packed_ovf = nullptr, BufPtr *keep = nullptr, const C3Post *post = nullptr,
                    BufPtr acc_pre = BufPtr(), bool direct = false) {
  const int nr = 2 * sd.nb;
  static bool attr_set = false;
  if (!attr_set) {
    HIP_CHECK(hipFuncSetAttribute((const void *)k_c5_gather<C5_PPS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  C5_GATHER_LDS));
    attr_set = true;
  }
  int max_units = 0;
  uint32_t ovf_cap = 0;
  const int64_t acc_bytes = c5_post_acc_bytes(nr, S, sd.split_x16, nkeys, &max_units, &ovf_cap);
  // P3 reads run-major meta (transposed here); reading P1's tile-major meta in
  // place saved 7 µs of transpose and cost P3 7..20 µs at s24 (measured).  A
  // node-partitioned rank's static work list needs no run totals, and its few
  // runs (≤ 64 at G = 8) share each tile's meta lines: P3 reads them in place,
  // no transpose launch.
  // direct (2-hop pipeline, one slice): P1 wrote run-major meta and every run is
  // one exclusive unit — no transpose, no work list; the dot adds the
  // self-loops and the split flags (all 0) were cleared by P1
  const bool in_place = (static_units && !post) || direct;
  BufPtr meta_t = in_place ? BufPtr() : s->alloc(4 * nr * ntiles);
  // transpose blocks: tiles per block tt, fewer when there are few runs (≥ ~1024 blocks)
  int64_t tt = C3_TT;
  // (s24: 128 tiles per block 34 µs, 64 41 µs, 32 54 µs — fewer, longer blocks win;
  // the same launch again right after takes 19 µs: ~15 µs of T is P1's dirty
  // lines written back at the boundary, paid by whichever kernel follows P1)
  while (tt > 32 && ((ntiles + tt - 1) / tt) * ((nr + 31) / 32) < 1024) tt /= 2;
  const int nparts = (int)((ntiles + tt - 1) / tt);
  // acc_pre: allocated by the caller, its first c5_post_zero_words words
  // cleared by P1's tile-0 workgroup (no memset here)
  BufPtr acc = acc_pre ? acc_pre : s->alloc(acc_bytes);
  unsigned long long *run_total = (unsigned long long *)acc->p;
  int32_t *nunits = (int32_t *)(run_total + nr);  // [0] units, [1] overflow events
  unsigned int *bdone = (unsigned int *)(nunits + 4);  // (reserved: keeps the layout's alignment)
  uint2 *log = (uint2 *)(bdone + nr);                    // (12·nr + 16 B in: 8-B aligned, nr even)
  int32_t *split = (int32_t *)(log + ovf_cap);
  int32_t *rnu = split + nr;
  C3Unit *units = (C3Unit *)(rnu + nr);
  C3Ovf ovf{};
  ovf.n = (uint32_t *)(nunits + 1);
  ovf.log = log;
  ovf.cap = ovf_cap;
  // the hand-off log is folded in by the dot kernel (no overflow kernel) when
  // the caller takes it
  const bool log_to_dot = post && post->spill && !sd.packed;
  if (!acc_pre) HIP_CHECK(hipMemsetAsync(acc->p, 0, 4 * (size_t)c5_post_zero_words(nr, ovf_cap), s->stream));
  // units in the XCD-grouped run order (largest-first order: measured no gain)
  const C3UnitsOut uo{units, nunits, split};
  if (!in_place) {
    KernelTimer kt(s, "c3_transpose", 8.0 * nr * ntiles);
    hipLaunchKernelGGL(k_c3_transpose, dim3((unsigned)nparts, (nr + 31) / 32), dim3(256), 0, s->stream, meta,
                       (uint32_t *)meta_t->p, ntiles, nr, run_total, tt, nullptr,
                       post ? post->tile_loops : nullptr, post ? post->acc3 + 1 : nullptr);
    KERNEL_CHECK();
  }
  C3Sides sdk = sd;  // as launched: split units clear their buckets (claim bits)
  const bool stat = static_units || direct;
  if (!stat) {
    sdk.claim = split;
    // the work list in its own one-workgroup kernel (fusing it into the
    // transpose's last workgroup made T+U 55 µs against 35 + 6 µs + a 10 µs
    // boundary at s24)
    KernelTimer kt(s, "c3_units", 8.0 * nr);
    hipLaunchKernelGGL(k_c3_units, dim3(1), dim3(C3_UBLOCK), 0, s->stream, run_total, nr, sd, S, uo);
    KERNEL_CHECK();
  }
  {
    // (folding the dot into P3's epilogue measured 0.51 ms for P3 against
    // 0.44 + 0.027 ms + a ~10 µs boundary: the dot kernel runs after P3)
    KernelTimer kt(s, "c5_gather", 2.0 * nkeys);
    const int grid = stat ? (nr * S + 255) / 256 * 256 : max_units;
    hipLaunchKernelGGL(k_c5_gather<C5_PPS>, dim3((unsigned)grid), dim3(C5_BLOCK), C5_GATHER_LDS, s->stream,
                       stat ? nullptr : (const C3Unit *)units, (const int32_t *)nunits, part,
                       in_place ? meta : (const uint32_t *)meta_t->p, ntiles, sd.nb, rstride, h_in, h_out,
                       slice_stride, ovf, sdk, S, in_place && !direct ? (int64_t)nr : (int64_t)1);
    KERNEL_CHECK();
  }
  if (sd.packed) {  // the hand-offs are applied by k_c5_dot_packed
    *packed_ovf = ovf;
    *keep = acc;
  } else if (log_to_dot) {  // the dot kernel adds the hand-offs' terms
    post->spill->log = ovf.log;
    post->spill->n = ovf.n;
    post->spill->cap = ovf.cap;
    post->spill->hl = slice_stride;
    post->spill->split = sd.pairs ? split : nullptr;  // per run: 1 = uint32 bins, 0 = packed pairs
    post->spill->nb = sd.nb;
    post->spill->tile_loops = direct ? post->tile_loops : nullptr;  // (direct: no transpose summed them)
    post->spill->ntiles = direct ? post->ntiles : 0;
  } else {
    KernelTimer kt(s, "c3_overflow", 0.0);
    hipLaunchKernelGGL(k_c3_overflow, dim3(16), dim3(256), 0, s->stream, ovf, h_in, h_out);
    KERNEL_CHECK();
  }
}

// out[i] = Σ_s slices[s·stride + i] for both sides (n a multiple of 4).
__global__ __launch_bounds__(256) void k_c5_fold(const uint32_t *si, const uint32_t *so, int S,
                                                  int64_t stride, int64_t n, uint32_t *oi,
                                                  uint32_t *oo) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n / 4;
       i += (int64_t)gridDim.x * 256) {
    uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < S; ++k) {
      const uint4 x = ((const uint4 *)(si + k * stride))[i];
      const uint4 y = ((const uint4 *)(so + k * stride))[i];
      a = make_uint4(a.x + x.x, a.y + x.y, a.z + x.z, a.w + x.w);
      b = make_uint4(b.x + y.x, b.y + y.y, b.z + y.z, b.w + y.w);
    }
    ((uint4 *)oi)[i] = a;
    ((uint4 *)oo)[i] = b;
  }
}

// acc[0] += Σ_i (Σ_s in_s[i])·(Σ_s out_s[i]) (n a multiple of 4).
__global__ __launch_bounds__(1024) void k_c5_dot_slices(const uint32_t *si, const uint32_t *so,
                                                         int S, int64_t stride, int64_t n,
                                                         unsigned long long *acc) {
  __shared__ unsigned long long lds[17];
  unsigned long long t = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < S; ++k) {
      const uint4 x = ((const uint4 *)(si + k * stride))[i];
      const uint4 y = ((const uint4 *)(so + k * stride))[i];
      a = make_uint4(a.x + x.x, a.y + x.y, a.z + x.z, a.w + x.w);
      b = make_uint4(b.x + y.x, b.y + y.y, b.z + y.z, b.w + y.w);
    }
    t += (unsigned long long)a.x * b.x + (unsigned long long)a.y * b.y +
         (unsigned long long)a.z * b.z + (unsigned long long)a.w * b.w;
  }
  unsigned long long tot;
  block_exclusive_scan(t, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(acc, tot);
}

// acc[0] += Σ_b Σ_i (Σ in-slices of b)·(Σ out-slices of b) over the apportioned
// slices sl[unit][64 Ki] (table: base[2·nb], k[2·nb]; runs [0, nb) in, [nb, 2·nb) out).
__device__ inline uint32_t packed_half_sum(const uint32_t *sl, int S, int64_t stride, int64_t g) {
  const int64_t w = (g >> C2_BITS) * C2_WORDS + (g & (C2_WORDS - 1));
  const int sh = (int)((g >> 15) & 1) * 16;
  uint32_t x = 0;
  for (int k = 0; k < S; ++k) x += (sl[k * stride + w] >> sh) & 0xFFFFu;
  return x;
}

__global__ __launch_bounds__(1024) void k_c5_dot_packed(const uint32_t *si, const uint32_t *so, int S,
                                                        int64_t stride, int64_t nwords, C3Ovf ovf,
                                                        unsigned long long *acc) {
  __shared__ unsigned long long lds[17];
  unsigned long long t = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords / 4;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < S; ++k) {
      const uint4 x = ((const uint4 *)(si + k * stride))[i];
      const uint4 y = ((const uint4 *)(so + k * stride))[i];
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[2 * q] += xs[q] & 0xFFFFu;
        a[2 * q + 1] += xs[q] >> 16;
        b[2 * q] += ys[q] & 0xFFFFu;
        b[2 * q + 1] += ys[q] >> 16;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) t += (unsigned long long)a[q] * b[q];
  }
  // the log (a few entries per hub bin) staged in LDS when it fits: the
  // first-occurrence test and the per-bin sums then cost LDS reads only
  constexpr uint32_t LOG_LDS = 4096;
  __shared__ uint2 lg[LOG_LDS];
  const uint32_t n = min(*ovf.n, ovf.cap);
  const bool staged = n <= LOG_LDS;
  const uint2 *L = staged ? lg : ovf.log;
  if (staged)
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) lg[j] = ovf.log[j];
  __syncthreads();
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint32_t g = L[e].x;
    bool first = true;
    for (uint32_t j = 0; j < e && first; ++j) first = L[j].x != g;
    if (!first) continue;
    unsigned long long cin = 0, cout = 0;
    for (uint32_t j = e; j < n; ++j) {
      const uint2 f = L[j];
      if (f.x != g) continue;
      if (f.y & 1u) cout += f.y >> 1;
      else cin += f.y >> 1;
    }
    const unsigned long long bi = packed_half_sum(si, S, stride, g), bo = packed_half_sum(so, S, stride, g);
    t += (bi + cin) * (bo + cout) - bi * bo;
  }
  unsigned long long tot;
  block_exclusive_scan(t, lds, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(acc, tot);
}

// d_acc3 = [Σ in·out, self-loops, done]: the units kernel writes the self-loop
// total and clears the other two (the caller needs no memset).
template <int W, class SH>
static void chain2_c5(Session *s, C5Cols<W> c, bool in_range, uint32_t *h_in, uint32_t *h_out,
                      unsigned long long *d_acc3, C2Spill *spill) {
  c.ntiles = (c.n + SH::TILE - 1) / SH::TILE;
  const int nr = 2 * c.nb;
  c.rstride = ((int64_t)2 * SH::TILE + 8 * (nr + 1) + 7) & ~int64_t(7);
  BufPtr part = s->alloc(2 * c.rstride * c.ntiles);
  BufPtr meta = s->alloc(4 * nr * c.ntiles);
  BufPtr tl = s->alloc(4 * std::max<int64_t>(c.ntiles, 1));
  C3Sides sd;
  sd.split_x16 = c3_split_x16();
  sd.nb = c.nb;
  sd.t0[0] = sd.t0[1] = 0;
  sd.t1[0] = sd.t1[1] = c.ntiles;
  const int S = c5_slices(nr);
  uint32_t ovf_cap = 0;
  BufPtr post_acc = s->alloc(c5_post_acc_bytes(nr, S, sd.split_x16, 2 * c.n, nullptr, &ovf_cap));
  // One slice (≥ 256 runs): no transpose and no work-list kernel — P1 writes
  // run-major meta, every run is one exclusive P3 unit (hash-partitioned runs
  // are near-uniform: no hub split at s24), the dot adds the self-loops.  s24
  // (profiles/r05_ab_direct.txt): pipeline 1.000 → 0.980 ms, T 37 + U 8 µs
  // gone, P1 +8 µs (scattered meta lines), P3 +13 µs (it now pays P1's dirty-line
  // write-back that T used to).  CAPF_C5_DIRECT=0 keeps the transpose pipeline.
  const char *de = getenv("CAPF_C5_DIRECT");
  const bool direct_env = !(de && atoi(de) == 0);
  const bool direct = direct_env && S == 1 && spill != nullptr;
  {
    KernelTimer kt(s, "c5_partition", (2.0 * W + 4.0) * c.n);
    uint16_t *pp = (uint16_t *)part->p;
    uint32_t *mp = (uint32_t *)meta->p;
    uint32_t *tlp = (uint32_t *)tl->p, *zb = (uint32_t *)post_acc->p;
    const int64_t zw = c5_post_zero_words(nr, ovf_cap, direct);
    const bool alias = c.u2 == c.u1 && c.v2 == c.v1;
    const int rm = direct ? 1 : 0;
    if (alias && !in_range) launch_c5<W, true, true, SH>(s, c, pp, mp, tlp, zb, zw, d_acc3, rm);
    if (alias && in_range) launch_c5<W, true, false, SH>(s, c, pp, mp, tlp, zb, zw, d_acc3, rm);
    if (!alias && !in_range) launch_c5<W, false, true, SH>(s, c, pp, mp, tlp, zb, zw, d_acc3, rm);
    if (!alias && in_range) launch_c5<W, false, false, SH>(s, c, pp, mp, tlp, zb, zw, d_acc3, rm);
  }
  C3Post post{};
  post.tile_loops = (const uint32_t *)tl->p;
  post.ntiles = c.ntiles;
  post.acc3 = d_acc3;
  post.spill = spill;
  const int64_t hl = (int64_t)c.nb * C2_BW;
  sd.pairs = S == 1 && spill ? 1 : 0;  // packed-pair buckets (one uint32 per bin when split)
  if (S == 1) {
    c5_post(s, (const uint16_t *)part->p, (const uint32_t *)meta->p, sd, c.ntiles, c.rstride,
            2 * c.n, 1, h_in, h_out, hl, false, nullptr, nullptr, &post, post_acc, direct);
    return;
  }
  BufPtr sl = s->alloc(8 * S * hl);
  uint32_t *si = (uint32_t *)sl->p, *so = si + S * hl;
  c5_post(s, (const uint16_t *)part->p, (const uint32_t *)meta->p, sd, c.ntiles, c.rstride,
          2 * c.n, S, si, so, hl, false, nullptr, nullptr, &post, post_acc);
  hipLaunchKernelGGL(k_c5_fold, dim3(grid_for(hl / 4, 256, 1024)), dim3(256), 0, s->stream, si, so,
                     S, hl, hl, h_in, h_out);
  KERNEL_CHECK();
}

// ------------------------------------------------------------- sharded P1
// Node-partitioned multi-GPU layout: rank p owns the nodes
// whose mixed index falls in its bucket range [b0, b1), and holds every rel
// twice — the out-copy (rels whose source it owns) and the in-copy (rels whose
// target it owns).  in[b] then comes from the in-copy's target column and
// out[b] from the out-copy's source column, both for owned b only: the 2-hop
// count needs no histogram exchange, only one int64 all-reduce.  One key per
// row; tiles [0, T_in) scan the in-copy, [T_in, T_in + T_out) the out-copy
// (whose target column is read for the self-loop term).
struct C5Shard {
  const void *kin, *kout, *oth;  // in-copy key, out-copy key, out-copy other endpoint
  int64_t bin, bout, both;       // FOR32 bases (0 for plain int64 columns)
  int64_t n_in, n_out;
  int64_t t_in;                  // in-copy tiles
  int64_t lo;
  uint64_t len;
  int b0, nbl;                   // owned buckets [b0, b0 + nbl)
  int nsb;                       // runs per side: one per owned bucket (= nbl)
  int copies;                    // run counters per run (power of 2, see below)
  int gpt;                       // 4096-row groups per tile (≤ 4): tile = 4096·gpt rows
  int nhot;                      // heavy hitters (≤ C5S_MAXHOT): keys equal to hot[j] are
  uint32_t hot[2];               // counted per wave, not partitioned (node_mix(id − lo))
  int upf;                       // raw loads D groups ahead on tiles without the loop test
  int64_t n_diag;                // out-copy rows [0, n_diag) may be self-loops (2-D layout:
                                 // rows whose target is owned too come first); the
                                 // target column is read for those rows only
  NodeMix mix;
};

constexpr int C5S_TILE = 32768;  // rows (= keys) per tile (at most) at FOR24; 16384 otherwise
constexpr int C5S_MAXHOT = 1;    // heavy-hitter keys of a rank (sampled at ingest, a plan hint)
constexpr int C5S_MAXR = 520;    // runs incl. the dummy: nbl ≤ 259
// a tile scans ONE copy, so it fills only its side's ≤ nsb ≤ 259 runs + the
// dummy: the stage reserves pad slots for those, which leaves room for 2 Ki
// run counters (more copies per run: fewer same-word LDS atomics when a rank
// owns few runs) at 2 workgroups per CU
constexpr int C5S_PADRUNS = 261;
constexpr int C5S_CNT = 2048;    // LDS run counters: copies · (runs + 1) ≤ 2048

// A rank of a G-GPU node owns few buckets (2·32 + 1 runs at s24, G = 8): the
// 64 lanes of a counting atomic would pile onto a handful of words.  Each run
// then gets `copies` counters, lane l using copy l mod copies, and a run's
// slots are the concatenation of its copies' sub-ranges.
static int c5s_copies(int nr) {
  int c = 1;
  while (2 * c * (nr + 1) <= C5S_CNT && c < 8) c *= 2;
  return c;
}

// TR (trusted): both key columns are node-partitioned copies of this very
// (range, parts, part) — every key is an owned node, so the ring path's keys
// skip the 64-bit range test and the ownership test: run and key come from
// the mixed index alone, key = ((run0 − b0 + h >> 16) << 16) | (h & 0xFFFF).
template <int W, bool WIDE, int TILE, bool HOT, bool TR = false>
__global__ __launch_bounds__(C5_BLOCK) __attribute__((amdgpu_waves_per_eu(8))) void k_c5_shard_partition(
    C5Shard c, uint16_t *part, uint32_t *meta, uint32_t *tile_acc, int64_t rstride) {
  constexpr int MAXR = C5S_MAXR;
  constexpr int RPT = TILE / C5_BLOCK, GROUPS = RPT / 4;
  constexpr int STAGE = TILE + 8 * C5S_PADRUNS;
  static_assert(MAXR <= C5_BLOCK, "one run per thread in the scan");
  __shared__ uint4 stage4[STAGE / 8];
  __shared__ uint32_t cur[C5S_CNT];
  __shared__ uint32_t lds_scan[17];
  __shared__ uint32_t body_end, dummy_n;
  uint16_t *stage = (uint16_t *)stage4;
  const int64_t t = blockIdx.x;
  const int side = t >= c.t_in ? 1 : 0;  // block-uniform
  const int nr = 2 * c.nsb;
  const int C = c.copies;
  const uint32_t my_copy = (uint32_t)(lane_id() & (C - 1));
  const uint32_t pb = 8u * (uint32_t)(t & 7);
  const uint4 pad = make_uint4(pb | (pb + 1) << 16, (pb + 2) | (pb + 3) << 16,
                               (pb + 4) | (pb + 5) << 16, (pb + 6) | (pb + 7) << 16);
  for (int i = threadIdx.x; i < STAGE / 8; i += C5_BLOCK) stage4[i] = pad;
  for (int i = threadIdx.x; i < C * (nr + 1); i += C5_BLOCK) cur[i] = 0;
  __syncthreads();
  const int64_t ts = side ? t - c.t_in : t;
  const int64_t rows = (int64_t)c.gpt * 4 * C5_BLOCK;
  const int64_t e0 = ts * rows, e1 = min(e0 + rows, side ? c.n_out : c.n_in);
  const bool chk = side && e0 < c.n_diag;  // block-uniform: this tile needs the loop test
  // groups holding rows of this tile (uniform): later groups are skipped, so a
  // short tile never floods the dummy run's counter
  const int gu = (int)min<int64_t>(c.gpt, (e1 - e0 + 4 * C5_BLOCK - 1) / (4 * C5_BLOCK));
  const void *kp = side ? c.kout : c.kin;
  const int64_t kb = side ? c.bout : c.bin;
  const uint32_t dummy = (uint32_t)nr << C2_BITS;
  const uint32_t run0 = (uint32_t)(side * c.nsb);
  uint32_t key[RPT];
  uint32_t lp = 0;
  // heavy hitter (skew handling): keys whose mixed index is c.hot[0] are not
  // partitioned but counted at the end from the dummy run's stage slots — one
  // compare per key and no counter register (32 keys per thread already fill
  // the VGPR budget); no hint = 0xFFFFFFFF, never a mixed index
  // (run, key) of node offset x (ok: inside the node range), or a dummy key:
  // a heavy hitter goes to the dummy run as key 1 (past-the-end rows as key 0),
  // never copied out, counted in the dummy run's stage slots
  auto mk = [&](uint32_t x, bool okx) {
    const uint32_t h = node_mix_t<WIDE>(x, c.mix);
    const uint32_t b = (h >> C2_BITS) - (uint32_t)c.b0;  // wraps when below b0
    const bool ok = okx && b < (uint32_t)c.nbl;
    const uint32_t run = run0 + b;
    return HOT ? (ok && h != c.hot[0] ? (run << C2_BITS) | (h & 0xFFFF) : dummy | (ok ? 1u : 0u))
               : (ok ? (run << C2_BITS) | (h & 0xFFFF) : dummy);
  };
  if (W != 8 && !chk && c.upf) {
    // tiles without the loop test (FOR24 / FOR32): raw loads run D groups
    // ahead in a ring of registers (the single-GPU P1's upfront schedule,
    // bounded to stay within 64 VGPRs); a partial last group loads per row
    constexpr int D = 4;
    using Raw = C5Raw<(W == 3 ? 3 : 4)>;
    Raw raw[D];
    auto issue = [&](int g) {
      const int64_t e = e0 + 4 * ((int64_t)g * C5_BLOCK + threadIdx.x);
      if (g < gu && e + 4 <= e1)
        raw[g & (D - 1)] = c.upf == 2 ? c5_ld_raw<(W == 3 ? 3 : 4), true>((const uint8_t *)kp + W * e)
                                      : c5_ld_raw<(W == 3 ? 3 : 4), false>((const uint8_t *)kp + W * e);
    };
#pragma unroll
    for (int g = 0; g < D && g < GROUPS; ++g) issue(g);
    const int64_t dlo = kb - c.lo;
#pragma unroll
    for (int g = 0; g < GROUPS; ++g) {
      if (g < gu) {
        const int64_t e = e0 + 4 * ((int64_t)g * C5_BLOCK + threadIdx.x);
        uint32_t x[4];
        bool okx[4];
        if (TR && e + 4 <= e1) {
          uint32_t q[4];
          c5_decode<(W == 3 ? 3 : 4)>(raw[g & (D - 1)], (uint32_t)dlo, q);
          if (g + D < GROUPS) issue(g + D);
          const uint32_t run0t = run0 - (uint32_t)c.b0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t h = node_mix_t<WIDE>(q[k], c.mix);
            const uint32_t kk = ((run0t + (h >> C2_BITS)) << C2_BITS) | (h & 0xFFFF);
            key[4 * g + k] = HOT ? (h != c.hot[0] ? kk : dummy | 1u) : kk;
            atomicAdd(&cur[(key[4 * g + k] >> C2_BITS) * C + my_copy], 1u);
          }
          __builtin_amdgcn_sched_barrier(0);
          continue;
        }
        if (e + 4 <= e1) {
          uint32_t q[4];
          c5_decode<(W == 3 ? 3 : 4)>(raw[g & (D - 1)], 0u, q);
          if (g + D < GROUPS) issue(g + D);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int64_t o = dlo + (int64_t)q[k];
            x[k] = (uint32_t)o;
            okx[k] = (uint64_t)o < c.len;
          }
        } else {
          c5_load4<W, true>(kp, kb, c.lo, c.len, e, e1, true, x, okx);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          key[4 * g + k] = mk(x[k], okx[k]);
          atomicAdd(&cur[(key[4 * g + k] >> C2_BITS) * C + my_copy], 1u);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
  // the next group's loads are issued before this group's hashing/counting
  uint32_t px[2][4], py[2][4];
  bool pox[2][4], poy[2][4];
  {
    const int64_t e = e0 + 4 * (int64_t)threadIdx.x;
    c5_load4<W, true>(kp, kb, c.lo, c.len, e, e1, true, px[0], pox[0]);
    if (chk) c5_load4<W, true>(c.oth, c.both, c.lo, c.len, e, e1, true, py[0], poy[0]);
  }
#pragma unroll
  for (int g = 0; g < GROUPS; ++g) {
    if (g < gu) {  // static index per unrolled group: key[] stays in VGPRs
      if (g + 1 < gu) {
        const int64_t en = e0 + 4 * ((int64_t)(g + 1) * C5_BLOCK + threadIdx.x);
        c5_load4<W, true>(kp, kb, c.lo, c.len, en, e1, true, px[(g + 1) & 1], pox[(g + 1) & 1]);
        if (chk)
          c5_load4<W, true>(c.oth, c.both, c.lo, c.len, en, e1, true, py[(g + 1) & 1], poy[(g + 1) & 1]);
      }
      uint32_t x[4], y[4];
      bool okx[4], oky[4];
      // rows of this group's 4 that lie in the diagonal block (2-D order)
      const uint32_t dg = chk ? (uint32_t)min<int64_t>(max<int64_t>(
                                    c.n_diag - (e0 + 4 * ((int64_t)g * C5_BLOCK + threadIdx.x)), 0), 4)
                              : 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[k] = px[g & 1][k];
        y[k] = py[g & 1][k];
        okx[k] = pox[g & 1][k];
        oky[k] = poy[g & 1][k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t h = node_mix_t<WIDE>(x[k], c.mix);
        const uint32_t b = (h >> C2_BITS) - (uint32_t)c.b0;  // wraps when below b0
        const bool ok = okx[k] && b < (uint32_t)c.nbl;
        // a heavy hitter goes to the dummy run: counted here, never copied out
        // the heavy hitter (mixed index) goes to the dummy run as key 1 (past-the-end
        // rows as key 0): never copied out, counted in the dummy run's stage slots
        const uint32_t run = run0 + b;
        key[4 * g + k] = HOT ? (ok && h != c.hot[0] ? (run << C2_BITS) | (h & 0xFFFF) : dummy | (ok ? 1u : 0u))
                             : (ok ? (run << C2_BITS) | (h & 0xFFFF) : dummy);
        if (chk) lp += (ok && oky[k] && x[k] == y[k] && (uint32_t)k < dg) ? 1u : 0u;
        atomicAdd(&cur[(key[4 * g + k] >> C2_BITS) * C + my_copy], 1u);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  }
#pragma unroll
  for (int j = 0; j < RPT; ++j) asm volatile("" : "+v"(key[j]));
  __syncthreads();
  // exclusive scan of the 8-padded run sizes, one run per thread (dummy last)
  const int r = threadIdx.x;
  uint32_t cnt = 0;
  if (r <= nr)
    for (int k = 0; k < C; ++k) cnt += cur[r * C + k];
  uint32_t total;
  const uint32_t ex = block_exclusive_scan((cnt + 7) & ~7u, lds_scan, total);
  if (r <= nr) {
    uint32_t o = ex;
    for (int k = 0; k < C; ++k) {
      const uint32_t v = cur[r * C + k];
      cur[r * C + k] = o;
      o += v;
    }
  }
  if (r < nr) meta[t * nr + r] = (ex >> 3) | (cnt << 16);
  if (r == nr) {
    body_end = ex;  // the dummy run (last) is not copied out
    dummy_n = cnt;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    if (j < 4 * gu) stage[atomicAdd(&cur[(key[j] >> C2_BITS) * C + my_copy], 1u)] = (uint16_t)key[j];
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  uint4 *dst = (uint4 *)(part + t * rstride);
  for (uint32_t i = threadIdx.x; i < body_end / 8; i += C5_BLOCK) dst[i] = stage4[i];
  // the heavy hitter's keys of this tile: the 1s of the dummy run's slots
  uint32_t hn = 0;
  if (HOT)
    for (uint32_t i = threadIdx.x; i < dummy_n; i += C5_BLOCK) hn += stage[body_end + i] == 1 ? 1u : 0u;
  // per-tile (self-loops, hot keys) with plain stores, summed by k_sharded_final:
  // one same-address device atomic per wave serialises at the memory side
  // (~88 per µs on one word: 2·10^3 tiles × 16 waves ≈ 0.37 ms)
  __shared__ uint32_t red[2][C5_BLOCK / WAVE];
  const uint32_t l32 = (uint32_t)wave_reduce_sum((unsigned long long)lp);
  const uint32_t h32 = (uint32_t)wave_reduce_sum((unsigned long long)hn);
  if (lane_id() == 0) {
    red[0][threadIdx.x / WAVE] = l32;
    red[1][threadIdx.x / WAVE] = h32;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t v = 0;
    for (int w = 0; w < C5_BLOCK / WAVE; ++w) v += red[threadIdx.x][w];
    tile_acc[2 * t + threadIdx.x] = v;
  }
}

// this rank's partial: Σ in·out over the partitioned keys (acc[0]) + hot_in·hot_out −
// self-loops; tile_acc = (loops, hot keys) per P1 tile, tiles [0, t_in) in-copy
__global__ __launch_bounds__(1024) void k_sharded_final(const unsigned long long *acc, const uint32_t *tile_acc,
                                                        int64_t ntiles, int64_t t_in, int64_t *out) {
  __shared__ unsigned long long lds[3][17];
  unsigned long long lp = 0, hi = 0, ho = 0;
  for (int64_t t = threadIdx.x; t < ntiles; t += blockDim.x) {
    lp += tile_acc[2 * t];
    (t < t_in ? hi : ho) += tile_acc[2 * t + 1];
  }
  const unsigned long long L = block_reduce_sum(lp, lds[0]), I = block_reduce_sum(hi, lds[1]),
                           O = block_reduce_sum(ho, lds[2]);
  if (threadIdx.x == 0) *out = (int64_t)(acc[0] + I * O - L);
}

template <int TILE, bool TR>
static auto c5s_kernel_t(int W, bool wide, bool hot) {
  if (hot)
    return W == 3 ? (wide ? k_c5_shard_partition<3, true, TILE, true, TR> : k_c5_shard_partition<3, false, TILE, true, TR>)
           : W == 4 ? (wide ? k_c5_shard_partition<4, true, TILE, true, TR> : k_c5_shard_partition<4, false, TILE, true, TR>)
                    : (wide ? k_c5_shard_partition<8, true, TILE, true, TR> : k_c5_shard_partition<8, false, TILE, true, TR>);
  return W == 3 ? (wide ? k_c5_shard_partition<3, true, TILE, false, TR> : k_c5_shard_partition<3, false, TILE, false, TR>)
         : W == 4 ? (wide ? k_c5_shard_partition<4, true, TILE, false, TR> : k_c5_shard_partition<4, false, TILE, false, TR>)
                  : (wide ? k_c5_shard_partition<8, true, TILE, false, TR> : k_c5_shard_partition<8, false, TILE, false, TR>);
}

template <int TILE>
static auto c5s_kernel(int W, bool wide, bool hot) {
  if (hot)  // a heavy-hitter hint: one more compare per key (only ranks that hold a hub pay it)
    return W == 3 ? (wide ? k_c5_shard_partition<3, true, TILE, true> : k_c5_shard_partition<3, false, TILE, true>)
           : W == 4 ? (wide ? k_c5_shard_partition<4, true, TILE, true> : k_c5_shard_partition<4, false, TILE, true>)
                    : (wide ? k_c5_shard_partition<8, true, TILE, true> : k_c5_shard_partition<8, false, TILE, true>);
  return W == 3 ? (wide ? k_c5_shard_partition<3, true, TILE, false> : k_c5_shard_partition<3, false, TILE, false>)
         : W == 4 ? (wide ? k_c5_shard_partition<4, true, TILE, false> : k_c5_shard_partition<4, false, TILE, false>)
                  : (wide ? k_c5_shard_partition<8, true, TILE, false> : k_c5_shard_partition<8, false, TILE, false>);
}

// Buckets of 64 Ki mixed node indexes owned by `part` of `parts`.
static void owned_buckets(int kbits, int parts, int part, int *b0, int *nbl) {
  const int64_t nb = (int64_t(1) << kbits) / C2_BW;
  const int64_t lo = nb * part / parts, hi = nb * (part + 1) / parts;
  *b0 = (int)lo;
  *nbl = (int)(hi - lo);
}

int node_owner_bits(int64_t n_nodes) { return chain2_hist_bits(n_nodes); }

// Owner rank of node offset x (id − lo): the bucket of its mixed index.
__device__ inline int owner_of(uint32_t x, NodeMix mix, bool wide, int64_t nb, int parts) {
  const uint32_t h = wide ? node_mix_t<true>(x, mix) : node_mix_t<false>(x, mix);
  const int64_t b = h >> C2_BITS;
  // smallest p with b < nb·(p+1)/parts
  int p = (int)((b * parts) / nb);
  while (p > 0 && b < nb * p / parts) --p;
  while (p + 1 < parts && b >= nb * (p + 1) / parts) ++p;
  return p;
}

__global__ void k_owner_flags(ColView key, int64_t n, int64_t lo, NodeMix mix, int wide,
                              int64_t nb, int parts, int part, uint8_t *flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = ld_int(key, i);
    flags[i] = owner_of((uint32_t)(v - lo), mix, wide != 0, nb, parts) == part;
  }
}

// 2-D split of a rank's out-copy: f_diag = source and target owned by `part`,
// f_off = source owned, target not.
__global__ void k_owner_flags2(ColView src, ColView dst, int64_t n, int64_t lo, NodeMix mix, int wide,
                               int64_t nb, int parts, int part, uint8_t *f_diag, uint8_t *f_off) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool so = owner_of((uint32_t)(ld_int(src, i) - lo), mix, wide != 0, nb, parts) == part;
    const bool dw = owner_of((uint32_t)(ld_int(dst, i) - lo), mix, wide != 0, nb, parts) == part;
    f_diag[i] = so && dw;
    f_off[i] = so && !dw;
  }
}

// Gather index of the out-copy in 2-D order: the rows whose source AND target
// `part` owns first (*n_diag of them), then the rows whose source only it owns.
BufPtr node_partition_diag_index(Session *s, const ColView &src, const ColView &dst, int64_t n, int64_t lo,
                                 int64_t n_nodes, int parts, int part, int64_t *m, int64_t *n_diag) {
  const int kbits = chain2_hist_bits(n_nodes);
  const int64_t n1 = std::max<int64_t>(n, 1);
  BufPtr fl = s->alloc(2 * n1);
  uint8_t *fd = (uint8_t *)fl->p, *fo = fd + n1;
  if (n > 0) {
    hipLaunchKernelGGL(k_owner_flags2, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, src, dst, n, lo,
                       node_mix_for(kbits), (int)(kbits > 24), (int64_t(1) << kbits) / C2_BW, parts, part,
                       fd, fo);
    KERNEL_CHECK();
  }
  int64_t a = 0, b = 0;
  BufPtr ia = compact_flags(s, fd, n, &a), ib = compact_flags(s, fo, n, &b);
  BufPtr idx = s->alloc(8 * std::max<int64_t>(a + b, 1));
  if (a) HIP_CHECK(hipMemcpyAsync(idx->p, ia->p, 8 * a, hipMemcpyDeviceToDevice, s->stream));
  if (b) HIP_CHECK(hipMemcpyAsync((int64_t *)idx->p + a, ib->p, 8 * b, hipMemcpyDeviceToDevice, s->stream));
  *m = a + b;
  *n_diag = a;
  return idx;
}

uint8_t *node_owner_flags(Session *s, const ColView &key, int64_t n, int64_t lo, int64_t n_nodes,
                          int parts, int part, BufPtr &keep) {
  const int kbits = chain2_hist_bits(n_nodes);
  keep = s->alloc(std::max<int64_t>(n, 1));
  if (n > 0) {
    hipLaunchKernelGGL(k_owner_flags, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, key, n, lo,
                       node_mix_for(kbits), (int)(kbits > 24), (int64_t(1) << kbits) / C2_BW,
                       parts, part, (uint8_t *)keep->p);
    KERNEL_CHECK();
  }
  return (uint8_t *)keep->p;
}

// Local 2-hop partial of `part`: Σ_{owned b} in[b]·out[b] − owned self-loops
// into *d_partial (device, int64) — asynchronous on the session stream.
// cols = {in-copy target, out-copy source, out-copy target}; all plain or all
// FOR32, 16-B aligned, non-null.  Histograms live in session scratch.
bool chain2_sharded(Session *s, const ColView *cols, int64_t n_in, int64_t n_out, int64_t lo,
                    int64_t n_nodes, int parts, int part, int64_t *d_partial, int64_t n_diag,
                    int nhot, const int64_t *hot_ids, bool trusted) {
  const int kbits = chain2_hist_bits(n_nodes);
  int b0, nbl;
  owned_buckets(kbits, parts, part, &b0, &nbl);
  if (2 * nbl + 1 > C5S_MAXR) return false;
  if (n_in >= (int64_t(1) << 31) || n_out >= (int64_t(1) << 31)) return false;
  int nf = 0, n24 = 0;
  for (int i = 0; i < 3; ++i) {
    if (cols[i].valid || (!cols[i].data && (i == 0 ? n_in : n_out) > 0)) return false;
    if ((uintptr_t)cols[i].data & 15) return false;
    nf += cols[i].enc == ENC_FOR32;
    n24 += cols[i].enc == ENC_FOR24;
  }
  if (nf + n24 != 0 && nf != 3 && n24 != 3) return false;
  const int W = n24 == 3 ? 3 : nf == 3 ? 4 : 8;
  BufPtr acc = s->alloc(16);
  HIP_CHECK(hipMemsetAsync(acc->p, 0, 16, s->stream));
  unsigned long long *d_acc = (unsigned long long *)acc->p;  // [0] Σ in·out
  BufPtr tacc;  // P1's per-tile (self-loops, hot keys)
  uint32_t *tile_acc = nullptr;
  int64_t ntiles_all = 0, t_in_all = 0;
  // heavy hitters: distinct ids inside the node range (others could never match a key)
  uint32_t hot[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};  // mixed indexes (< 2^31: never all ones)
  int nh = 0;
  {
    const NodeMix mx = node_mix_for(kbits);
    for (int i = 0; i < nhot && hot_ids && nh < C5S_MAXHOT; ++i) {
      const int64_t x = hot_ids[i] - lo;
      if (x < 0 || x >= n_nodes) continue;
      const uint32_t ux = (uint32_t)x;
      uint32_t hh = mx.wide ? ux * NODE_MIX_A : (uint32_t)((uint64_t)(ux & 0xFFFFFFu) * NODE_MIX_A);
      hh &= mx.mask;
      hh ^= hh >> mx.sh;
      bool dup = false;
      for (int j = 0; j < nh; ++j) dup |= hot[j] == hh;
      if (!dup) hot[nh++] = hh;
    }
  }
  if (nbl > 0) {
    C5Shard c;
    c.kin = cols[0].data;
    c.kout = cols[1].data;
    c.oth = cols[2].data;
    c.bin = W != 8 ? cols[0].base : 0;
    c.bout = W != 8 ? cols[1].base : 0;
    c.both = W != 8 ? cols[2].base : 0;
    c.n_in = n_in;
    c.n_out = n_out;
    c.n_diag = n_diag < 0 ? n_out : std::min(n_diag, n_out);
    c.nhot = nh;
    c.upf = 1;  // raw loads D groups ahead on tiles without the loop test (nt loads: no change)
    c.hot[0] = hot[0];
    c.hot[1] = hot[1];
    // tile size: whole rounds of resident blocks (2 per CU), counting one
    // group of per-tile overhead (stage fill, scan, copy-out)
    // (32 Ki-row tiles need 32 keys per thread in VGPRs: no spills at FOR24 only;
    // 16 Ki / 24 Ki-row tiles at FOR24 measured no gain)
    const int tile = W != 3 ? 16384 : C5S_TILE;
    {
      const int64_t slots = 2 * (int64_t)s->num_cus;
      int64_t best = -1;
      for (int g = tile / (4 * C5_BLOCK); g >= 1; --g) {
        const int64_t rows = (int64_t)g * 4 * C5_BLOCK;
        const int64_t tiles = (n_in + rows - 1) / rows + (n_out + rows - 1) / rows;
        const int64_t cost = (tiles + slots - 1) / slots * (g + 1);
        if (best < 0 || cost < best) {
          best = cost;
          c.gpt = g;
        }
      }
    }
    const int64_t trows = (int64_t)c.gpt * 4 * C5_BLOCK;
    c.t_in = (n_in + trows - 1) / trows;
    const int64_t t_out = (n_out + trows - 1) / trows;
    const int64_t ntiles = c.t_in + t_out;
    tacc = s->alloc(8 * std::max<int64_t>(ntiles, 1));
    tile_acc = (uint32_t *)tacc->p;
    ntiles_all = ntiles;
    t_in_all = c.t_in;
    c.lo = lo;
    c.len = (uint64_t)n_nodes;
    c.b0 = b0;
    c.nbl = nbl;
    c.mix = node_mix_for(kbits);
    // one run per owned bucket and side (measured and removed: sub-bucket units
    // and balanced key ranges — 8 Ki-node sub-buckets are skewed, p99 unit 1.7×:
    // 0.296 vs 0.235 ms/rank at G = 8)
    c.nsb = nbl;
    const int nr = 2 * c.nsb;
    c.copies = c5s_copies(nr);
    const int64_t rstride = ((int64_t)tile + 8 * (nr + 1) + 7) & ~int64_t(7);
    if (ntiles > 0) {
      BufPtr partb = s->alloc(2 * rstride * ntiles);
      BufPtr meta = s->alloc(4 * nr * ntiles);
      {
        KernelTimer kt(s, "c5_partition", (double)W * (n_in + 2 * n_out));
        // the trusted ring only where the ring runs (FOR24 / FOR32 columns)
        const bool tr = trusted && W != 8 && c.upf;
        auto kern = tile == C5S_TILE ? (tr ? c5s_kernel_t<C5S_TILE, true>(W, kbits > 24, nh > 0)
                                           : c5s_kernel<C5S_TILE>(W, kbits > 24, nh > 0))
                                     : (tr ? c5s_kernel_t<16384, true>(W, kbits > 24, nh > 0)
                                           : c5s_kernel<16384>(W, kbits > 24, nh > 0));
        hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(C5_BLOCK), 0, s->stream, c,
                           (uint16_t *)partb->p, (uint32_t *)meta->p, tile_acc, rstride);
        KERNEL_CHECK();
      }
      {
        C3Sides sd;
        sd.split_x16 = c3_split_x16();
        sd.nb = nbl;
        sd.t0[0] = 0;
        sd.t1[0] = c.t_in;
        sd.t0[1] = c.t_in;
        sd.t1[1] = ntiles;
        const int S = c5_slices(nr);
        const int64_t hl = (int64_t)nbl * C2_BW;
        {
        // packed when several slices per run (G ≥ 4 at s24): with one slice the runs
        // are whole buckets whose hub bins log many hand-offs (measured G = 2:
        // packed dot 41 µs vs uint32 dot + overflow 22 µs)
        sd.packed = S >= 2;
        if (sd.packed) {
          // packed uint16 slices: half the slice bytes written by P3 and read by the dot
          const int64_t hw = (int64_t)nbl * C2_WORDS;
          BufPtr sl = s->alloc(8 * S * hw);
          uint32_t *si = (uint32_t *)sl->p, *so = si + S * hw;
          C3Ovf ovf{};
          BufPtr keep;
          c5_post(s, (const uint16_t *)partb->p, (const uint32_t *)meta->p, sd, ntiles, rstride,
                  n_in + n_out, S, si, so, hw, true, &ovf, &keep);
          KernelTimer kt(s, "chain2_dot", 8.0 * S * hw);
          hipLaunchKernelGGL(k_c5_dot_packed, dim3(grid_for(hw / 4, 1024, dot_grid(s->num_cus))), dim3(1024),
                             0, s->stream, si, so, S, hw, hw, ovf, d_acc);
          KERNEL_CHECK();
        } else {
        BufPtr sl = s->alloc(8 * S * hl);
        uint32_t *si = (uint32_t *)sl->p, *so = si + S * hl;
        // static work list (no units kernel): S tile ranges per run; a rank's
        // runs hold ≤ 1.4 × the mean at s24 (no hub splits happen)
        c5_post(s, (const uint16_t *)partb->p, (const uint32_t *)meta->p, sd, ntiles, rstride,
                n_in + n_out, S, si, so, hl, true);
        KernelTimer kt(s, "chain2_dot", 8.0 * S * hl);
        // one block per CU: every block ends in one same-address device atomic
        // (G = 8 rank: 256 blocks 18.5 µs, 1024 24.4 µs, 2048 36 µs)
        // one block per CU (each block ends in one device atomic); 16 waves per
        // block keep 8·S·… loads in flight per CU (256 threads: latency bound)
        hipLaunchKernelGGL(k_c5_dot_slices, dim3(grid_for(hl / 4, 1024, dot_grid(s->num_cus))),
                           dim3(1024), 0, s->stream, si, so, S, hl, hl, d_acc);
        KERNEL_CHECK();
        }
        }
      }
    }
  }
  hipLaunchKernelGGL(k_sharded_final, dim3(1), dim3(1024), 0, s->stream, (const unsigned long long *)d_acc,
                     tile_acc, ntiles_all, t_in_all, d_partial);
  KERNEL_CHECK();
  return true;
}

int chain2_hist_bits(int64_t len) {
  int k = C2_BITS;
  while (k < 62 && (int64_t(1) << k) < len) ++k;
  return k;
}

int64_t chain2_hist_len(int64_t len) { return int64_t(1) << chain2_hist_bits(len); }

// cols = {start(r1), end(r1), start(r2), end(r2)}: non-null INTEGER columns,
// all plain or all FOR32.  h_in / h_out hold chain2_hist_len(hi − lo + 1)
// counters each, indexed by node_mix(id − lo); every counter is written (no
// memset needed).  in_range: every id of the four columns lies in [lo, hi]
// (column statistics), so P1 skips the range tests.  The self-loop count is
// added to *d_loops (device).  Returns false — before launching anything —
// if the shape is outside this kernel's limits (the caller falls back to
// k_chain2_hist).
bool chain2_partitioned(Session *s, const ColView *cols, int64_t n, int64_t lo, int64_t hi,
                        bool in_range, uint32_t *h_in, uint32_t *h_out,
                        unsigned long long *d_acc3, C2Spill *spill) {
  const int64_t len = hi - lo + 1;
  if (len <= 0 || n <= 0) return false;
  const int kbits = chain2_hist_bits(len);
  const int64_t nb = (int64_t(1) << kbits) / C2_BW;
  if (2 * nb + 1 > C5Big::MAXR) return false;  // + the dummy run
  if (n >= (int64_t(1) << 30)) return false;   // 2·n keys: 32-bit element indices in `part`
  int nf = 0, n24 = 0;
  for (int i = 0; i < 4; ++i) {
    if (cols[i].valid || !cols[i].data) return false;
    if ((uintptr_t)cols[i].data & 15) return false;  // 16-B vector loads
    nf += cols[i].enc == ENC_FOR32;
    n24 += cols[i].enc == ENC_FOR24;
  }
  if (n24 != 0 && n24 != 4) return false;
  if (n24 == 0 && nf != 0 && nf != 4) return false;
  auto fill = [&](auto &c) {
    c.u1 = cols[0].data;
    c.v1 = cols[1].data;
    c.u2 = cols[2].data;
    c.v2 = cols[3].data;
    const bool f = nf == 4 || n24 == 4;
    c.bu1 = f ? cols[0].base : 0;
    c.bv1 = f ? cols[1].base : 0;
    c.bu2 = f ? cols[2].base : 0;
    c.bv2 = f ? cols[3].base : 0;
    c.n = n;
    c.lo = lo;
    c.len = (uint64_t)len;
    c.nb = (int)nb;
    c.mix = node_mix_for(kbits);
  };
  const bool small = 2 * nb + 1 <= C5Small::MAXR;
  if (n24 == 4) {
    C5Cols<3> c;
    fill(c);
    if (small)
      chain2_c5<3, C5Small>(s, c, in_range, h_in, h_out, d_acc3, spill);
    else
      chain2_c5<3, C5Big>(s, c, in_range, h_in, h_out, d_acc3, spill);
    return true;
  }
  if (nf == 4) {
    C5Cols<4> c;
    fill(c);
    if (small)
      chain2_c5<4, C5Small>(s, c, in_range, h_in, h_out, d_acc3, spill);
    else
      chain2_c5<4, C5Big>(s, c, in_range, h_in, h_out, d_acc3, spill);
    return true;
  }
  C5Cols<8> c;
  fill(c);
  if (small)
    chain2_c5<8, C5Small>(s, c, in_range, h_in, h_out, d_acc3, spill);
  else
    chain2_c5<8, C5Big>(s, c, in_range, h_in, h_out, d_acc3, spill);
  return true;
}

}  // namespace capf

namespace capf {

// ------------------------------------------ partitioned semi-join count
// Σ_rows bit[key − lo]: the root message of the 1-hop label count
// (MATCH (a:Person)-->(b), fused_count.hip): the Person id column's
// membership bitmap probed with every rel's source.  Probed row by row, each
// random 4-B lookup pulls a 128-B line from L2 into the CU — L2-bandwidth bound
// (≈31 TB/s of lines for 67 M lookups at s22).  Radix-partitioned instead, like
// the 2-hop P1: the keys are grouped by 64 Ki-node bucket of node_mix(key −
// lo) (the sharded P1 kernel as one rank owning every bucket), then each
// bucket's 8 KiB slice of the bitmap — in mixed order, built once per bitmap —
// sits in LDS while its keys stream past: no atomics, no random HBM/L2 access.

__global__ void k_mix_bits(const uint32_t *bits, uint64_t range, NodeMix mix, uint32_t *mbits) {
  const uint64_t nw = (range + 31) / 32;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t v = bits[w];
    while (v) {
      const uint32_t b = __builtin_ctz(v);
      v &= v - 1;
      const uint64_t o = w * 32 + b;
      if (o >= range) break;
      const uint32_t h = node_mix((uint32_t)o, mix);
      atomicOr(&mbits[h >> 5], 1u << (h & 31));
    }
  }
}

// One block per (bucket, tile chunk): the bucket's bitmap slice in LDS, the
// waves walk the chunk's tiles (P1's tile-major meta read in place), one
// 16-B piece of 8 keys per lane; the segment's last piece counts only its
// `cnt & 7` live keys (the rest are P1's pads).
constexpr int BC_BLOCK = 1024;
__global__ __launch_bounds__(BC_BLOCK) void k_c5_bits_count(const uint16_t *part, const uint32_t *meta,
                                                            int64_t ntiles, int nr, int64_t rstride,
                                                            int chunks, const uint32_t *mbits,
                                                            unsigned long long *acc) {
  __shared__ uint32_t slice[C2_BW / 32];
  __shared__ unsigned long long red[BC_BLOCK / WAVE];
  const int r = blockIdx.x / chunks, k = blockIdx.x % chunks;
  for (int i = threadIdx.x; i < C2_BW / 32; i += BC_BLOCK) slice[i] = mbits[(int64_t)r * (C2_BW / 32) + i];
  __syncthreads();
  const int64_t t0 = ntiles * k / chunks, t1 = ntiles * (k + 1) / chunks;
  const int wave = threadIdx.x / WAVE, lane = lane_id();
  const uint4 *part4 = (const uint4 *)part;
  unsigned long long sum = 0;
  for (int64_t t = t0 + wave; t < t1; t += BC_BLOCK / WAVE) {
    const uint32_t mw = meta[t * nr + r];
    const uint32_t start = mw & 0xFFFF, cnt = mw >> 16, np = (cnt + 7) >> 3;
    const int64_t base = t * (rstride / 8) + start;
    for (uint32_t p = lane; p < np; p += WAVE) {
      const uint4 v = part4[base + p];
      const uint32_t live = min(cnt - 8 * p, 8u);
      const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t key = (e & 1) ? wd[e >> 1] >> 16 : wd[e >> 1] & 0xFFFF;
        sum += ((uint32_t)e < live) ? ((slice[key >> 5] >> (key & 31)) & 1u) : 0u;
      }
    }
  }
  sum = wave_reduce_sum(sum);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (int w = 0; w < BC_BLOCK / WAVE; ++w) tot += red[w];
    if (tot) atomicAdd(acc, tot);
  }
}

bool bits_count_partitioned(Session *s, const ColView &key, int64_t n, int64_t lo, int64_t hi,
                            const uint32_t *bits, BufPtr &mixed_cache, unsigned long long *d_acc) {
  const char *e = getenv("CAPF_SEMI_PART");  // tuning: 0 = row-by-row bitmap probes
  if (e && atoi(e) == 0) return false;
  if (n < (int64_t(1) << 20) || n >= (int64_t(1) << 31) || key.valid || !key.data) return false;
  if (key.enc != ENC_FOR24 && key.enc != ENC_FOR32) return false;
  if ((uintptr_t)key.data & 15) return false;
  const int64_t range = hi - lo + 1;
  if (range <= 0 || range > (int64_t(1) << 31)) return false;
  const int kbits = chain2_hist_bits(range);
  const int nbl = (int)((int64_t(1) << kbits) / C2_BW);
  if (2 * nbl + 1 > C5S_MAXR) return false;
  const NodeMix mix = node_mix_for(kbits);
  // the bitmap in mixed order (cached by the caller with the bitmap)
  if (!mixed_cache) {
    const int64_t mw = (int64_t(1) << kbits) / 32;
    mixed_cache = s->alloc(4 * mw);
    HIP_CHECK(hipMemsetAsync(mixed_cache->p, 0, 4 * mw, s->stream));
    hipLaunchKernelGGL(k_mix_bits, dim3(grid_for((range + 31) / 32, 256)), dim3(256), 0, s->stream, bits,
                       (uint64_t)range, mix, (uint32_t *)mixed_cache->p);
    KERNEL_CHECK();
  }
  // P1: the sharded partition kernel, one "rank" owning every bucket, keys = the column
  const int W = key.enc == ENC_FOR24 ? 3 : 4;
  C5Shard c;
  memset(&c, 0, sizeof(c));
  c.kin = c.kout = c.oth = key.data;
  c.bin = c.bout = c.both = key.base;
  c.n_in = n;
  c.n_out = 0;
  c.n_diag = 0;
  c.nhot = 0;
  c.hot[0] = c.hot[1] = 0xFFFFFFFFu;
  c.lo = lo;
  c.len = (uint64_t)range;
  c.b0 = 0;
  c.nbl = nbl;
  c.nsb = nbl;
  c.mix = mix;
  const int nr = 2 * nbl;
  c.copies = c5s_copies(nr);
  c.upf = 1;
  const int tile = W == 3 ? C5S_TILE : 16384;
  c.gpt = tile / (4 * C5_BLOCK);
  c.t_in = (n + tile - 1) / tile;
  const int64_t ntiles = c.t_in;
  const int64_t rstride = ((int64_t)tile + 8 * (nr + 1) + 7) & ~int64_t(7);
  BufPtr partb = s->alloc(2 * rstride * ntiles), meta = s->alloc(4 * (int64_t)nr * ntiles),
         tacc = s->alloc(8 * ntiles);
  {
    KernelTimer kt(s, "semi_partition", (double)W * n + 2.0 * n);
    auto kern = W == 3 ? (kbits > 24 ? k_c5_shard_partition<3, true, C5S_TILE, false>
                                     : k_c5_shard_partition<3, false, C5S_TILE, false>)
                       : (kbits > 24 ? k_c5_shard_partition<4, true, 16384, false>
                                     : k_c5_shard_partition<4, false, 16384, false>);
    hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(C5_BLOCK), 0, s->stream, c, (uint16_t *)partb->p,
                       (uint32_t *)meta->p, (uint32_t *)tacc->p, rstride);
    KERNEL_CHECK();
  }
  {
    KernelTimer kt(s, "semi_count", 2.0 * n);
    // ≥ 2 blocks per CU over the buckets
    const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, (4 * s->num_cus + nbl - 1) / nbl));
    hipLaunchKernelGGL(k_c5_bits_count, dim3((unsigned)(nbl * chunks)), dim3(BC_BLOCK), 0, s->stream,
                       (const uint16_t *)partb->p, (const uint32_t *)meta->p, ntiles, nr, rstride, chunks,
                       (const uint32_t *)mixed_cache->p, d_acc);
    KERNEL_CHECK();
  }
  return true;
}

}  // namespace capf
