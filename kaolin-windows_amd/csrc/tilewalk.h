// tilewalk.h -- wave-level building blocks of the tile walks (softtile.hip, rastertile.hip):
// the candidate-chunk sequence of a tile's bin bitmap and a 64x64 bit-matrix transpose
// across the wave.
#pragma once

#include "common.h"

namespace kl {

// Lane exchange v <- v[lane ^ S] with cross-lane VALU ops (gfx950 permlane swaps, DPP).
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
    // lanes with bit 2 clear read lane + 4 (row_ror:12), the others lane - 4 (row_ror:4): two DPP
    // moves and a select, no LDS pipe (r05; ds_swizzle before)
    const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
    const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12c, 0xf, 0xf, false);  // row_ror:12
    return (lane & 4) ? dn : up;
  } else if constexpr (S == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  } else {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  }
}

// One block-swap stage of the transpose on a lane's row split in 32-bit halves (S <= 16: the
// stage's 2S-bit groups never cross the halves), branch-free: the partner's halves (lane ^ S), a
// per-lane rotate that brings the partner's other half-group into place (rotl S on lanes with bit S
// clear, rotr S on the others: one v_alignbit_b32) and a bit select (v_bfi_b32) keeping the lane's
// own half-group (m on clear lanes, ~m on set lanes).
template <int S>
__device__ __forceinline__ void transpose_stage(uint32_t &lo, uint32_t &hi, uint32_t m, int lane) {
  const uint32_t plo = xor_lane<S>(lo, lane), phi = xor_lane<S>(hi, lane);
  const uint32_t sgn = (uint32_t)((int)((uint32_t)lane << (31 - __builtin_ctz(S))) >> 31);  // lane & S ? ~0 : 0
  const uint32_t keep = m ^ sgn;
  const uint32_t amt = (32u - S) + (sgn & (uint32_t)(2 * S - 32));  // rotr amount (mod 32)
  const uint32_t qlo = __builtin_amdgcn_alignbit(plo, plo, amt), qhi = __builtin_amdgcn_alignbit(phi, phi, amt);
  lo = (keep & lo) | (~keep & qlo);
  hi = (keep & hi) | (~keep & qhi);
}

// 64x64 bit-matrix transpose across the wave: lane i holds row i (bit j = column j) on
// entry and column i (bit j = row j) on exit.  Six block-swap stages; the first (32-bit
// halves across lanes i, i ^ 32: lanes < 32 take the partner's low half as their high half, the
// others the partner's high half as their low half) is one v_permlane32_swap of (lo, hi).
__device__ __forceinline__ uint64_t transpose64(uint64_t x, int lane) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
  lo = r[0];
  hi = r[1];
  transpose_stage<16>(lo, hi, 0x0000ffffu, lane);
  transpose_stage<8>(lo, hi, 0x00ff00ffu, lane);
  transpose_stage<4>(lo, hi, 0x0f0f0f0fu, lane);
  transpose_stage<2>(lo, hi, 0x33333333u, lane);
  transpose_stage<1>(lo, hi, 0x55555555u, lane);
  return ((uint64_t)hi << 32) | lo;
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
    const int inc = wave_incl_scan(c);
    pc = inc - c;
    gtot = __builtin_amdgcn_readlane(inc, 63);
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
