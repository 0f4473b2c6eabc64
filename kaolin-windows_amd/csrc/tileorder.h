// tileorder.h -- heaviest-first order of the 64x8 tiles of a bin bitmap (binning.h), shared
// by the soft mask (softtile.hip) and the tile rasterizer (raster.hip).
#pragma once

#include "common.h"

namespace kl {

constexpr int ORD_BUCKETS = 32;

// Counting sort of the tiles on floor(log2(count + 1)) of their candidate-chunk counts
// (set bits of the tile's bitmap words), descending.  Two kernels: one wave per tile
// counts and adds to the bucket histogram `ghist` (zeroed with the bitmap); one
// workgroup then scans the histogram and scatters the order (a kernel boundary instead
// of a per-workgroup release fence).  `scratch` (optional) is zeroed here too.
static __global__ void __launch_bounds__(256) tile_bucket_kernel(const uint32_t *__restrict__ bitmap, int words, int nt,
                                                          uint8_t *__restrict__ bk, int *__restrict__ ghist,
                                                          int *__restrict__ scratch) {
  __shared__ int hist[ORD_BUCKETS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x < ORD_BUCKETS) hist[threadIdx.x] = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0 && scratch) *scratch = 0;
  __syncthreads();
  const int t = blockIdx.x * (blockDim.x >> 6) + wid;  // one wave per tile
  if (t < nt) {
    const uint32_t *w = bitmap + (size_t)t * words;
    unsigned n = 0;
    for (int k = lane; k < words; k += 64) n += __popc(w[k]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if (lane == 0) {
      const int b = 31 - __clz(n + 1u);
      bk[t] = (uint8_t)b;
      atomicAdd(&hist[b], 1);
    }
  }
  __syncthreads();
  if (threadIdx.x < ORD_BUCKETS && hist[threadIdx.x]) atomicAdd(&ghist[threadIdx.x], hist[threadIdx.x]);
}

// Work items, heaviest first: tile | part << 24 | log2(parts) << 28.  Tiles of bucket
// >= split_from become 2^split_log2 items (parts of the tile's rows), the others one.
// nitems (optional) receives the item count.  identity: grid order, no split (dev ablation).
// `base` is a workgroup-shared [ORD_BUCKETS] array.
__device__ __forceinline__ void order_items(int *base, const uint8_t *__restrict__ bk, const int *__restrict__ ghist,
                                            int nt, int32_t *__restrict__ order, int identity, int split_from,
                                            int split_log2, int *__restrict__ nitems) {
  if (identity) {
    for (int u = threadIdx.x; u < nt; u += blockDim.x) order[u] = u;
    if (nitems && threadIdx.x == 0) *nitems = nt;
    return;
  }
  if (threadIdx.x == 0) {
    int s = 0;
    for (int q = ORD_BUCKETS - 1; q >= 0; q--) {
      base[q] = s;
      s += ghist[q] << (q >= split_from ? split_log2 : 0);
    }
    if (nitems) *nitems = s;
  }
  __syncthreads();
  for (int u = threadIdx.x; u < nt; u += blockDim.x) {
    const int q = bk[u];
    if (q >= split_from) {
      const int np = 1 << split_log2;
      const int o = atomicAdd(&base[q], np);
      for (int k = 0; k < np; k++) order[o + k] = u | (k << 24) | (split_log2 << 28);
    } else {
      order[atomicAdd(&base[q], 1)] = u;
    }
  }
}

// Soft-mask work items (softtile.hip), heaviest first: tile | part << 24 | lp << 28.  A tile's
// 8 rows are cut into 2^lp parts of 8 >> lp rows, one 4-wave workgroup per part.  lp is lp_min
// (set by the LDS the slot lists need) except for the heaviest buckets: >= ST_B8 candidate-chunk
// bucket -> 8 parts (one row, 4 waves sharing its evaluation), >= ST_B4 -> 4 parts (2 rows,
// 2 waves each), at most ST_CAP8 / ST_CAP4 tiles each, so that soft_items_bound() holds.
constexpr int ST_B4 = 5, ST_B8 = 6, ST_CAP4 = 256, ST_CAP8 = 128;
inline int soft_items_bound(int nt, int lp_min) {
  auto extra = [&](int lp, int cap) { return lp > lp_min ? cap * ((1 << lp) - (1 << lp_min)) : 0; };
  return (nt << lp_min) + extra(2, ST_CAP4) + extra(3, ST_CAP8);
}
__device__ __forceinline__ void order_soft_items(int *base, int *lpb, const uint8_t *__restrict__ bk,
                                                 const int *__restrict__ ghist, int nt, int32_t *__restrict__ order,
                                                 int lp_min, int *__restrict__ nitems) {
  if (threadIdx.x == 0) {
    int s = 0, n4 = 0, n8 = 0;
    for (int q = ORD_BUCKETS - 1; q >= 0; q--) {
      const int h = ghist[q];
      int lp = lp_min;
      if (q >= ST_B8 && n8 + h <= ST_CAP8) {
        lp = lp > 3 ? lp : 3;
        n8 += h;
      } else if (q >= ST_B4 && n4 + h <= ST_CAP4) {
        lp = lp > 2 ? lp : 2;
        n4 += h;
      }
      lpb[q] = lp;
      base[q] = s;
      s += h << lp;
    }
    *nitems = s;
  }
  __syncthreads();
  for (int u = threadIdx.x; u < nt; u += blockDim.x) {
    const int q = bk[u], lp = lpb[q], np = 1 << lp;
    const int o = atomicAdd(&base[q], np);
    for (int k = 0; k < np; k++) order[o + k] = u | (k << 24) | (lp << 28);
  }
}

static __global__ void __launch_bounds__(1024) soft_order_kernel(const uint8_t *__restrict__ bk,
                                                                 const int *__restrict__ ghist, int nt,
                                                                 int32_t *__restrict__ order, int lp_min,
                                                                 int *__restrict__ nitems) {
  __shared__ int base[ORD_BUCKETS], lpb[ORD_BUCKETS];
  order_soft_items(base, lpb, bk, ghist, nt, order, lp_min, nitems);
}

static __global__ void __launch_bounds__(1024) tile_order_kernel(const uint8_t *__restrict__ bk,
                                                                 const int *__restrict__ ghist, int nt,
                                                                 int32_t *__restrict__ order, int identity,
                                                                 int split_from, int split_log2,
                                                                 int *__restrict__ nitems) {
  __shared__ int base[ORD_BUCKETS];
  order_items(base, bk, ghist, nt, order, identity, split_from, split_log2, nitems);
}

// Two bitmaps over the same tiles at once (kl_dibr_forward: the rasterizer's and the soft
// mask's bins): one wave per tile counts both; the order kernel writes the rasterizer's items
// and the soft mask's (order_soft_items).
static __global__ void __launch_bounds__(256) tile_bucket2_kernel(const uint32_t *__restrict__ bm0,
                                                                  const uint32_t *__restrict__ bm1, int words, int nt,
                                                                  uint8_t *__restrict__ bk0, uint8_t *__restrict__ bk1,
                                                                  int *__restrict__ gh0, int *__restrict__ gh1,
                                                                  int *__restrict__ scratch) {
  __shared__ int hist[2][ORD_BUCKETS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x < 2 * ORD_BUCKETS) hist[threadIdx.x / ORD_BUCKETS][threadIdx.x % ORD_BUCKETS] = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0 && scratch) *scratch = 0;
  __syncthreads();
  const int t = blockIdx.x * (blockDim.x >> 6) + wid;
  if (t < nt) {
    unsigned n0 = 0, n1 = 0;
    for (int k = lane; k < words; k += 64) {
      n0 += __popc(bm0[(size_t)t * words + k]);
      n1 += __popc(bm1[(size_t)t * words + k]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      n0 += __shfl_xor(n0, o);
      n1 += __shfl_xor(n1, o);
    }
    if (lane == 0) {
      const int b0 = 31 - __clz(n0 + 1u), b1 = 31 - __clz(n1 + 1u);
      bk0[t] = (uint8_t)b0;
      bk1[t] = (uint8_t)b1;
      atomicAdd(&hist[0][b0], 1);
      atomicAdd(&hist[1][b1], 1);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * ORD_BUCKETS) {
    const int h = hist[threadIdx.x / ORD_BUCKETS][threadIdx.x % ORD_BUCKETS];
    if (h) atomicAdd((threadIdx.x < ORD_BUCKETS ? gh0 : gh1) + threadIdx.x % ORD_BUCKETS, h);
  }
}

static __global__ void __launch_bounds__(1024) tile_order2_kernel(const uint8_t *__restrict__ bk0,
                                                                  const int *__restrict__ gh0,
                                                                  int32_t *__restrict__ order0, int split_from,
                                                                  int split_log2, int *__restrict__ nitems0,
                                                                  const uint8_t *__restrict__ bk1,
                                                                  const int *__restrict__ gh1,
                                                                  int32_t *__restrict__ order1, int nt, int lp_min1,
                                                                  int *__restrict__ nitems1) {
  __shared__ int base[2][ORD_BUCKETS], lpb[ORD_BUCKETS];
  order_items(base[0], bk0, gh0, nt, order0, 0, split_from, split_log2, nitems0);
  order_soft_items(base[1], lpb, bk1, gh1, nt, order1, lp_min1, nitems1);
}

}  // namespace kl
