// tilewalk.h -- wave-level building blocks of the tile walks (softtile.hip, rastertile.hip):
// the candidate-chunk sequence of a tile's bin bitmap and a 64x64 bit-matrix transpose
// across the wave.
#pragma once

#include "common.h"

namespace kl {

// Lane exchange v <- v[lane ^ S] with cross-lane VALU ops (gfx950 permlane swaps, DPP)
// where they exist and ds_swizzle (no memory access) for xor 4.
template <int S>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int lane) {
  if constexpr (S == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? r[0] : r[1];
  } else if constexpr (S == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else if constexpr (S == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  } else if constexpr (S == 4) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1f);  // bitmask mode, xor 4
  } else if constexpr (S == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  } else {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  }
}

template <int S>
__device__ __forceinline__ uint64_t transpose_stage(uint64_t x, uint64_t m, int lane) {
  const uint64_t p = ((uint64_t)xor_lane<S>((uint32_t)(x >> 32), lane) << 32) | xor_lane<S>((uint32_t)x, lane);
  return (lane & S) ? ((x & ~m) | ((p & ~m) >> S)) : ((x & m) | ((p & m) << S));
}

// 64x64 bit-matrix transpose across the wave: lane i holds row i (bit j = column j) on
// entry and column i (bit j = row j) on exit.  Six block-swap stages.
__device__ __forceinline__ uint64_t transpose64(uint64_t x, int lane) {
  x = transpose_stage<32>(x, 0x00000000ffffffffull, lane);
  x = transpose_stage<16>(x, 0x0000ffff0000ffffull, lane);
  x = transpose_stage<8>(x, 0x00ff00ff00ff00ffull, lane);
  x = transpose_stage<4>(x, 0x0f0f0f0f0f0f0f0full, lane);
  x = transpose_stage<2>(x, 0x3333333333333333ull, lane);
  x = transpose_stage<1>(x, 0x5555555555555555ull, lane);
  return x;
}

// The candidate chunks of a tile (set bits of its bitmap words, ascending) as a sequence
// with random access by ordinal: 64 words per group, one per lane, with an exclusive
// prefix of their bit counts.  Wave-uniform; every wave of the workgroup holds a copy.
// at(n) must be called with non-decreasing n.
struct ChunkSeq {
  const uint32_t *words;  // the tile's word 0; word w at words[w * stride] (binning.h bm_index)
  size_t stride;
  int nwords, grp, base, gtot, pc;
  uint32_t wv;
  __device__ __forceinline__ void load(int g, int lane) {
    grp = g;
    const int w = g * 64 + lane;
    wv = w < nwords ? words[(size_t)w * stride] : 0u;
    const int c = __popc(wv);
    int inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    pc = inc - c;
    gtot = __shfl(inc, 63);
  }
  __device__ __forceinline__ void init(const uint32_t *w, int n, size_t st, int lane) {
    words = w;
    stride = st;
    nwords = n;
    base = 0;
    load(0, lane);
  }
  __device__ __forceinline__ int at(int n, int lane) {
    while (n >= base + gtot) {
      if ((grp + 1) * 64 >= nwords) return -1;
      base += gtot;
      load(grp + 1, lane);
    }
    const int t = n - base;
    const uint64_t le = ballot(pc <= t);
    const int L = 63 - __builtin_clzll(le);
    int k = t - __builtin_amdgcn_readlane(pc, L);
    uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)wv, L);
    int bit = 0;
#pragma unroll
    for (int h = 16; h > 0; h >>= 1) {  // the k-th set bit of w
      const int c = __popc(w & ((1u << h) - 1u));
      if (k >= c) {
        k -= c;
        w >>= h;
        bit += h;
      }
    }
    return (grp * 64 + L) * 32 + bit;
  }
};

}  // namespace kl
