// device_common.h — wave64 building blocks shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace capf {

constexpr int WAVE = 64;  // CDNA wavefront width (never 32)

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 64-bit finaliser used for hash tables (murmur3 fmix64).
__host__ __device__ inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// Bijective mixer of node offsets on a 2^k domain: odd multiply mod 2^k, then
// xorshift (each step invertible).  The radix-partitioned histograms key
// their runs by the HIGH bits of node_mix(id − lo): hash partitioning, so the
// per-bit skew of R-MAT ids (bit = 0 with p = .76 at every level) cannot pile
// 8 % of all keys into run 0 (measured at s24, 256 runs: max/mean 43 raw,
// 1.27 mixed).  Σ_b in[b]·out[b] is invariant under a bijection of b, so the
// dot runs over the mixed index unchanged.  For k ≤ 24 the multiply is the
// full-rate 24-bit v_mul_u32_u24 (the 32-bit form is quarter rate).
struct NodeMix {
  uint32_t mask;  // 2^k − 1
  int sh;         // k / 2
  int wide;       // k > 24: 32-bit multiply
};

constexpr uint32_t NODE_MIX_A = 0xB5297Bu;  // odd, < 2^24

template <bool WIDE>
__device__ inline uint32_t node_mix_t(uint32_t x, NodeMix m) {
  const uint32_t h = (WIDE ? x * NODE_MIX_A : __umul24(x, NODE_MIX_A)) & m.mask;
  return h ^ (h >> m.sh);
}

__device__ inline uint32_t node_mix(uint32_t x, NodeMix m) {
  return m.wide ? node_mix_t<true>(x, m) : node_mix_t<false>(x, m);
}

inline NodeMix node_mix_for(int kbits) {
  NodeMix m;
  m.mask = kbits >= 32 ? 0xFFFFFFFFu : (uint32_t(1) << kbits) - 1;
  m.sh = kbits / 2;
  m.wide = kbits > 24;
  return m;
}

__device__ inline int lane_id() { return threadIdx.x & (WAVE - 1); }

// Inclusive wave64 prefix sum.  32-bit values scan through DPP: row_shr 1, 2,
// 4, 8 inside each 16-lane row, then row_bcast15 / row_bcast31 carry row
// totals across; out-of-range sources read the `old` operand (0).  No lane
// address registers stay live, unlike the ds_bpermute form below, which
// kept six per-lane shuffle addresses alive (spilled in the triangle loop).
template <typename T>
__device__ inline T wave_inclusive_scan(T v) {
  if constexpr (sizeof(T) == 4) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return (T)x;
  }
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    T u = __shfl_up(v, d, WAVE);
    if (lane >= d) v += u;
  }
  return v;
}

template <typename T>
__device__ inline T wave_reduce_sum(T v) {
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, WAVE);
  return v;
}

// Block-wide exclusive scan (blockDim.x multiple of 64, <= 1024); returns the
// exclusive prefix of `v` and the block total through `total`.
template <typename T>
__device__ inline T block_exclusive_scan(T v, T *lds /* >= 16 */, T &total) {
  const int lane = lane_id();
  const int wid = threadIdx.x / WAVE;
  const int nw = blockDim.x / WAVE;
  T inc = wave_inclusive_scan(v);
  if (lane == WAVE - 1) lds[wid] = inc;
  __syncthreads();
  if (wid == 0) {
    T w = lane < nw ? lds[lane] : T(0);
    T winc = wave_inclusive_scan(w);
    if (lane < nw) lds[lane] = winc - w;  // exclusive wave offsets
    if (lane == nw - 1) lds[16] = winc;
  }
  __syncthreads();
  T res = inc - v + lds[wid];
  total = lds[16];
  __syncthreads();
  return res;
}

template <typename T>
__device__ inline T block_reduce_sum(T v, T *lds /* >= 16 */) {
  const int lane = lane_id();
  const int wid = threadIdx.x / WAVE;
  const int nw = blockDim.x / WAVE;
  v = wave_reduce_sum(v);
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  T r = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < nw; ++i) r += lds[i];
  __syncthreads();
  return r;  // valid in thread 0 only
}

// Blocks of a dot-product kernel (each block ends in one same-address device
// atomic, so fewer blocks cost less): `dflt`, or CAPF_DOT_GRID (tuning).
inline int64_t dot_grid(int64_t dflt) {
  const char *e = getenv("CAPF_DOT_GRID");
  return e && atoi(e) > 0 ? atoi(e) : dflt;
}

inline unsigned grid_for(int64_t n, int block, int64_t cap = 256 * 16) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace capf
