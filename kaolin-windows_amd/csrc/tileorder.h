// tileorder.h -- heaviest-first order of the 64x8 tiles of a bin bitmap (binning.h), shared
// by the soft mask (softtile.hip) and the tile rasterizer (raster.hip).
#pragma once

#include "common.h"

namespace kl {

constexpr int ORD_BUCKETS = 32;
constexpr int ORD_HIST = 8 * ORD_BUCKETS;  // histogram ints: (band, bucket) tile counts (tile_band below)

// Tiles are cut into 8 bands of consecutive tiles (XCD-aware placement, see place_items).
__device__ __forceinline__ int tile_band(int u, int nt) { return (int)((int64_t)u * 8 / nt); }

// Counting sort of the tiles on floor(log2(count + 1)) of their candidate-chunk counts
// (set bits of the tile's bitmap words), descending.  Two kernels: one wave per tile
// counts and adds to the bucket histogram `ghist` (zeroed with the bitmap); one
// workgroup then scans the histogram and scatters the order (a kernel boundary instead
// of a per-workgroup release fence).  `scratch` (optional) is zeroed here too.
static __global__ void __launch_bounds__(256) tile_bucket_kernel(const uint32_t *__restrict__ bitmap, int words, int nt,
                                                          uint8_t *__restrict__ bk, int *__restrict__ ghist,
                                                          int *__restrict__ scratch) {
  __shared__ int hist[ORD_HIST];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < ORD_HIST; i += blockDim.x) hist[i] = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0 && scratch) *scratch = 0;
  __syncthreads();
  const int t = blockIdx.x * (blockDim.x >> 6) + wid;  // one wave per tile
  if (t < nt) {
    unsigned n = 0;
    for (int k = lane; k < words; k += 64) n += __popc(bitmap[bm_index(nt, t, k)]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if (lane == 0) {
      const int b = 31 - __clz(n + 1u);
      bk[t] = (uint8_t)b;
      atomicAdd(&hist[tile_band(t, nt) * ORD_BUCKETS + b], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ORD_HIST; i += blockDim.x)
    if (hist[i]) atomicAdd(&ghist[i], hist[i]);
}

// Work items: tile | part << 24 | lp << 28, a tile's rows cut into 2^lp parts.
//
// XCD-aware placement.  Workgroups are dealt round-robin over the 8 XCDs (block b and b + 8
// share one; MI355X_MICROARCH.md, "Workgroup dispatch"), and each XCD has its own L2.  A
// tile's work reads the face records / ranges of the faces over it, chunk by chunk, so tiles
// far apart on different XCDs fetch the same lines from HBM once per XCD.  The tiles are cut
// into 8 bands of consecutive tiles (tile rows of one view); band g's items go to positions
// p = 8 r + g (r = the item's rank in the band, heaviest first), so each XCD walks one
// band's faces.  Bands with more items than their share of positions (N / 8) place the
// rest, lightest last, in the other classes' free positions.  For speed only: the results do
// not depend on the placement.
// The order kernels keep the tiles' buckets in LDS (one global read) up to this many tiles.
constexpr int ORD_LDS_TILES = 16384;

// lpb[q]: parts (log2) of a tile of bucket q; ghist: tiles per (band, bucket) (bucket kernels);
// bk: the buckets, in LDS when nt <= ORD_LDS_TILES.  Shared scratch: sb[8*32], sx[32].  All
// threads of the (single) workgroup call it.
__device__ __forceinline__ void place_prefix(int *sb, int *sx, const int *lpb, const int *__restrict__ ghist,
                                             int *__restrict__ nitems) {
  __syncthreads();  // lpb / staged buckets written
  // per band, the exclusive prefix over buckets, heaviest first: one lane per (band, bucket),
  // a 32-lane segmented scan (two bands per wave)
  if (threadIdx.x < 8 * ORD_BUCKETS) {
    const int t = threadIdx.x, g = t / ORD_BUCKETS, q = ORD_BUCKETS - 1 - t % ORD_BUCKETS;
    const int v = lpb[q] < 0 ? 0 : ghist[g * ORD_BUCKETS + q] << lpb[q];  // items of (band g, bucket q)
    static_assert(ORD_BUCKETS == 32, "the segmented scan is per 32-lane half");
    const int inc = wave_incl_scan32(v);  // (threads < 256: four whole waves)
    sb[g * ORD_BUCKETS + q] = inc - v;
    if (q == 0) sx[8 + g] = inc;  // items of band g
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int n[8], N = 0;
    for (int g = 0; g < 8; g++) {
      n[g] = sx[8 + g];
      N += n[g];
    }
    int ob = 0, fp = 0;
    for (int g = 0; g < 8; g++) {
      const int cap = N / 8 + (g < N % 8 ? 1 : 0);
      sx[g] = cap;                 // positions of class g
      sx[8 + g] = n[g];            // items of band g
      sx[16 + g] = ob;             // first overflow index of band g
      sx[24 + g] = fp;             // first free-slot index of class g
      ob += n[g] > cap ? n[g] - cap : 0;
      fp += cap > n[g] ? cap - n[g] : 0;
    }
    if (nitems) *nitems = N;
  }
  __syncthreads();
}

// position of band g's item of rank r (heaviest first) after place_prefix
__device__ __forceinline__ int place_pos(const int *sx, int g, int r) {
  if (r < sx[g]) return r * 8 + g;
  const int j = sx[16 + g] + r - sx[g];  // the j-th overflow item takes the j-th free position
  int x = 0;
  while (x < 7 && sx[24 + x + 1] <= j) x++;
  return (sx[8 + x] + j - sx[24 + x]) * 8 + x;
}

__device__ __forceinline__ void place_items(int *sb, int *sx, const int *lpb, const int *__restrict__ ghist,
                                            const uint8_t *__restrict__ bk, int nt, int32_t *__restrict__ order,
                                            int *__restrict__ nitems, uint64_t *dbg = nullptr) {
  place_prefix(sb, sx, lpb, ghist, nitems);
  if (dbg && threadIdx.x == 0) dbg[2] = stamp_wall();
  // the tiles' ranks in their (band, bucket): one LDS atomic per distinct key of a wave (a wave's
  // tiles are consecutive, so they share a band and mostly a few buckets; one returning atomic per
  // tile serialised up to 64 lanes on one address)
  const int lane = threadIdx.x & 63;
  for (int u0 = threadIdx.x - lane; u0 < nt; u0 += blockDim.x) {  // wave-uniform
    const int u = u0 + lane;
    const int q = u < nt ? bk[u] : 0, g = u < nt ? tile_band(u, nt) : 0, lp = u < nt ? lpb[q] : -1;
    const int key = lp < 0 ? -1 : g * ORD_BUCKETS + q;
    uint64_t todo = ballot(key >= 0);
    int r0 = 0;
    while (todo) {
      const int kl = __builtin_ctzll(todo);
      const int kk = __builtin_amdgcn_readlane(key, kl);
      const uint64_t same = ballot(key == kk) & todo;
      todo &= ~same;
      const int npk = 1 << __builtin_amdgcn_readlane(lp < 0 ? 0 : lp, kl);
      int base = 0;
      if (lane == kl) base = atomicAdd(&sb[kk], npk * __popcll(same));
      base = __builtin_amdgcn_readlane(base, kl);
      if (key == kk)
        r0 = base + npk * (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(same >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)same, 0u));
    }
    if (key < 0) continue;
    const int np = 1 << lp;
    for (int k = 0; k < np; k++) order[place_pos(sx, g, r0 + k)] = u | (k << 24) | (lp << 28);
  }
}

// The rasterizer's items: tiles of bucket >= split_from become 2^split_log2 items (parts of
// the tile's rows), the others one.  nitems (optional) receives the item count.  identity:
// grid order, no split (dev ablation).
__device__ __forceinline__ void order_items(int *sb, int *sx, int *lpb, const int *__restrict__ ghist,
                                            const uint8_t *__restrict__ bk, int nt, int32_t *__restrict__ order,
                                            int identity, int split_from, int split_log2,
                                            int *__restrict__ nitems, uint64_t *dbg = nullptr) {
  if (identity) {
    for (int u = threadIdx.x; u < nt; u += blockDim.x) order[u] = u;
    if (nitems && threadIdx.x == 0) *nitems = nt;
    return;
  }
  if (threadIdx.x < ORD_BUCKETS) lpb[threadIdx.x] = (int)threadIdx.x >= split_from ? split_log2 : 0;
  place_items(sb, sx, lpb, ghist, bk, nt, order, nitems, dbg);
}

// Soft-mask work items (softtile.hip).  A 4-wave workgroup takes one part.  lp is lp_min (set
// by the LDS the slot lists need) except for the heaviest buckets: >= b8 candidate-chunk
// bucket -> 8 parts (one row, 4 waves sharing its walk and evaluation), >= b4 -> 4 parts
// (2 rows, 2 waves each), at most cap8 / cap4 tiles each (SoftSplit), so that soft_items_bound()
// holds.
struct SoftSplit {
  int b4, b8, cap4, cap8;
};
constexpr SoftSplit ST_SPLIT{5, 6, 256, 128};
SoftSplit soft_split();  // ST_SPLIT, or the dev parameters' override (softtile.hip)
inline int soft_items_bound(int nt, int lp_min, SoftSplit sp) {
  auto extra = [&](int lp, int cap) { return lp > lp_min ? cap * ((1 << lp) - (1 << lp_min)) : 0; };
  return (nt << lp_min) + extra(2, sp.cap4) + extra(3, sp.cap8);
}
// parts (log2) per bucket of the soft mask's tiles; ghist (band, bucket) tile counts; sx scratch
__device__ __forceinline__ void soft_parts(int *sx, int *lpb, const int *__restrict__ ghist, int lp_min, SoftSplit sp,
                                           int skip_empty) {
  // tiles per bucket summed over the bands (one lane of wave 0 per bucket); a bucket's tiles get 8
  // parts when it and every heavier bucket >= b8 fit in cap8 together, else 4 parts when it and every
  // heavier bucket >= b4 not given 8 fit in cap4 -- two suffix sums over the 32 bucket lanes (r05;
  // the r04 rule walked the buckets serially and could skip a bucket that did not fit to give a
  // lighter one the split: one lane's serial walk measured ~2 us from a cold instruction cache)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int h = 0;
    if (lane < ORD_BUCKETS) {
#pragma unroll
      for (int g = 0; g < 8; g++) h += ghist[g * ORD_BUCKETS + lane];
    }
    auto suffix = [&](int v) {  // sum over lanes lane..31: the lanes' total less the prefix before
      const int inc = wave_incl_scan32(v);  // (lanes 32..63 hold 0)
      return __builtin_amdgcn_readlane(inc, ORD_BUCKETS - 1) - inc + v;
    };
    const bool e8 = lane < ORD_BUCKETS && lane >= sp.b8;
    const int s8 = suffix(e8 ? h : 0);  // (every lane of the wave: the scans are DPP)
    const bool acc8 = e8 && s8 <= sp.cap8;
    const bool e4 = lane < ORD_BUCKETS && lane >= sp.b4 && !acc8;
    const int s4 = suffix(e4 ? h : 0);
    const bool acc4 = e4 && s4 <= sp.cap4;
    int lp = lp_min;
    if (acc8) lp = lp > 3 ? lp : 3;
    else if (acc4) lp = lp > 2 ? lp : 2;
    if (lane < ORD_BUCKETS) lpb[lane] = lane == 0 && skip_empty ? -1 : lp;  // skip_empty: no item for tiles without candidates
  }
  __syncthreads();  // sx is reused by place_prefix
}

__device__ __forceinline__ void order_soft_items(int *sb, int *sx, int *lpb, const uint8_t *__restrict__ bk,
                                                 const int *__restrict__ ghist, int nt, int32_t *__restrict__ order,
                                                 int lp_min, int *__restrict__ nitems, SoftSplit sp,
                                                 int skip_empty = 0, uint64_t *dbg = nullptr) {
  soft_parts(sx, lpb, ghist, lp_min, sp, skip_empty);
  place_items(sb, sx, lpb, ghist, bk, nt, order, nitems, dbg);
}

// the buckets of tiles [0, nt) into LDS when they fit (else the global array is used)
__device__ __forceinline__ const uint8_t *stage_buckets(uint8_t *lds, const uint8_t *__restrict__ bk, int nt) {
  if (nt > ORD_LDS_TILES) return bk;
  for (int u = threadIdx.x; u < nt; u += blockDim.x) lds[u] = bk[u];
  return lds;  // (the first barrier of place_items orders these writes)
}

static __global__ void __launch_bounds__(1024) soft_order_kernel(const uint8_t *__restrict__ bk,
                                                                 const int *__restrict__ ghist, int nt,
                                                                 int32_t *__restrict__ order, int lp_min,
                                                                 int *__restrict__ nitems, SoftSplit sp) {
  __shared__ int sb[ORD_HIST], sx[32], lpb[ORD_BUCKETS];
  __shared__ uint8_t sbk[ORD_LDS_TILES];
  const uint8_t *b = stage_buckets(sbk, bk, nt);
  order_soft_items(sb, sx, lpb, b, ghist, nt, order, lp_min, nitems, sp);
}

static __global__ void __launch_bounds__(1024) tile_order_kernel(const uint8_t *__restrict__ bk,
                                                                 const int *__restrict__ ghist, int nt,
                                                                 int32_t *__restrict__ order, int identity,
                                                                 int split_from, int split_log2,
                                                                 int *__restrict__ nitems) {
  __shared__ int sb[ORD_HIST], sx[32], lpb[ORD_BUCKETS];
  __shared__ uint8_t sbk[ORD_LDS_TILES];
  const uint8_t *b = identity ? bk : stage_buckets(sbk, bk, nt);
  order_items(sb, sx, lpb, ghist, b, nt, order, identity, split_from, split_log2, nitems);
}

// Two bitmaps over the same tiles at once (kl_dibr_forward: the rasterizer's and the soft
// mask's bins): one wave per tile counts both; the order kernel writes the rasterizer's items
// and the soft mask's (order_soft_items).
static __global__ void __launch_bounds__(256) tile_bucket2_kernel(const uint32_t *__restrict__ bm0,
                                                                  const uint32_t *__restrict__ bm1, int words, int nt,
                                                                  uint8_t *__restrict__ bk0, uint8_t *__restrict__ bk1,
                                                                  int *__restrict__ gh0, int *__restrict__ gh1,
                                                                  int *__restrict__ zero, int nzero) {
  __shared__ int hist[2][ORD_HIST];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 2 * ORD_HIST; i += blockDim.x) hist[i / ORD_HIST][i % ORD_HIST] = 0;
  if (blockIdx.x == 0 && zero)
    for (int i = threadIdx.x; i < nzero; i += blockDim.x) zero[i] = 0;
  __syncthreads();
  const int t = blockIdx.x * (blockDim.x >> 6) + wid;
  if (t < nt) {
    unsigned n0 = 0, n1 = 0;
    for (int k = lane; k < words; k += 64) {
      n0 += __popc(bm0[bm_index(nt, t, k)]);
      n1 += __popc(bm1[bm_index(nt, t, k)]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      n0 += __shfl_xor(n0, o);
      n1 += __shfl_xor(n1, o);
    }
    if (lane == 0) {
      const int b0 = 31 - __clz(n0 + 1u), b1 = 31 - __clz(n1 + 1u), band = tile_band(t, nt);
      bk0[t] = (uint8_t)b0;
      bk1[t] = (uint8_t)b1;
      atomicAdd(&hist[0][band * ORD_BUCKETS + b0], 1);
      atomicAdd(&hist[1][band * ORD_BUCKETS + b1], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * ORD_HIST; i += blockDim.x) {
    const int h = hist[i / ORD_HIST][i % ORD_HIST];
    if (h) atomicAdd((i < ORD_HIST ? gh0 : gh1) + i % ORD_HIST, h);
  }
}

// Blocks past the first two of the order kernels below zero `zacc` (zn doubles) meanwhile: the
// chip is otherwise idle while two workgroups order (kl_dibr_forward's soft-mask accumulator).
__device__ __forceinline__ void zero_doubles_share(double *__restrict__ z, size_t n, int part, int nparts) {
  const size_t n2 = n / 2, per = (n2 + nparts - 1) / nparts;
  const size_t e0 = (size_t)part * per, e1 = e0 + per < n2 ? e0 + per : n2;
  double2 *z2 = reinterpret_cast<double2 *>(z);
  for (size_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) z2[e] = make_double2(0.0, 0.0);
  if ((n & 1) && part == 0 && threadIdx.x == 0) z[n - 1] = 0.0;
}

static __global__ void __launch_bounds__(1024) tile_order2_kernel(const uint8_t *__restrict__ bk0,
                                                                  const int *__restrict__ gh0,
                                                                  int32_t *__restrict__ order0, int split_from,
                                                                  int split_log2, int *__restrict__ nitems0,
                                                                  const uint8_t *__restrict__ bk1,
                                                                  const int *__restrict__ gh1,
                                                                  int32_t *__restrict__ order1, int nt, int lp_min1,
                                                                  int *__restrict__ nitems1, SoftSplit sp,
                                                                  int skip_empty1, double *__restrict__ zacc,
                                                                  size_t zn) {
  __shared__ int sb[ORD_HIST], sx[32], lpb[ORD_BUCKETS];
  __shared__ uint8_t sbk[ORD_LDS_TILES];
  if (blockIdx.x >= 2) {
    zero_doubles_share(zacc, zn, blockIdx.x - 2, gridDim.x - 2);
    return;
  }
  // two workgroups: block 0 orders the rasterizer's items, block 1 the soft mask's
  const bool soft = blockIdx.x == 1;
  const uint8_t *b = stage_buckets(sbk, soft ? bk1 : bk0, nt);
  if (soft)
    order_soft_items(sb, sx, lpb, b, gh1, nt, order1, lp_min1, nitems1, sp, skip_empty1);
  else
    order_items(sb, sx, lpb, gh0, b, nt, order0, 0, split_from, split_log2, nitems0);
}

// tile_bucket2_kernel + tile_order2_kernel in one launch (nt <= ORD_LDS_TILES): each of the two
// workgroups counts its bitmap's candidate chunks with one thread per tile (the tile's words
// loaded eight at a time) into LDS buckets and histogram, then orders.  Block 0 also zeroes
// zero[0, nzero).  (Counting one tile per wave in turn, a reduction each, took 85 us.)
static __global__ void __launch_bounds__(1024) tile_countorder2_kernel(
    const uint32_t *__restrict__ bm0, const uint32_t *__restrict__ bm1, int words, int32_t *__restrict__ order0,
    int split_from, int split_log2, int *__restrict__ nitems0, int32_t *__restrict__ order1, int nt, int lp_min1,
    int *__restrict__ nitems1, SoftSplit sp, int skip_empty1, int *__restrict__ zero, int nzero,
    double *__restrict__ zacc, size_t zn, uint64_t *dbg) {
  __shared__ int sb[ORD_HIST], sx[32], lpb[ORD_BUCKETS], hist[ORD_HIST];
  __shared__ uint8_t sbk[ORD_LDS_TILES];
  if (blockIdx.x >= 2) {
    zero_doubles_share(zacc, zn, blockIdx.x - 2, gridDim.x - 2);
    return;
  }
  const bool soft = blockIdx.x == 1;
  const uint32_t *bm = soft ? bm1 : bm0;
  if (dbg) dbg += blockIdx.x * 4;  // dev stamps: start, counted, placed prefix, end (wall clock)
  if (dbg && threadIdx.x == 0) dbg[0] = stamp_wall();
  if (!soft && zero)
    for (int i = threadIdx.x; i < nzero; i += blockDim.x) zero[i] = 0;
  if (!soft && order0 == nullptr) return;  // one order only (the fused tile kernel's)
  for (int i = threadIdx.x; i < ORD_HIST; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  // word-major bitmap: a lane per tile, each word load coalesced across the wave; two tiles per
  // lane with up to 2 x 32 words in flight together (one round trip per two tiles for the bench's
  // 25 words and 2,048 tiles: the words were just written by every XCD's binning workgroups, so
  // each round trip is a far one -- stamps: 7.6 us for the count with one tile per round trip).
  // Raw buffer loads: the tile's byte offset in one VGPR, the word's in an SGPR (64 loads in
  // flight need no per-load address registers), and words past the bitmap read as 0.
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)bm, (short)0, words * nt * 4, 0x00020000);
  for (int t0 = threadIdx.x; t0 < nt; t0 += 2 * blockDim.x) {
    const int t1 = t0 + blockDim.x;  // past nt: other words' bits, discarded
    unsigned n0 = 0, n1 = 0;
    for (int k0 = 0; k0 < words; k0 += 32) {
      uint32_t x[32], y[32];
#pragma unroll
      for (int u = 0; u < 32; u++) {
        const int so = (k0 + u) * nt * 4;
        x[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, t0 * 4, so, 0);
        y[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, t1 * 4, so, 0);
      }
#pragma unroll
      for (int u = 0; u < 32; u++) {
        n0 += __popc(x[u]);
        n1 += __popc(y[u]);
      }
    }
    const int q0 = 31 - __clz(n0 + 1u);
    sbk[t0] = (uint8_t)q0;
    atomicAdd(&hist[tile_band(t0, nt) * ORD_BUCKETS + q0], 1);
    if (t1 < nt) {
      const int q1 = 31 - __clz(n1 + 1u);
      sbk[t1] = (uint8_t)q1;
      atomicAdd(&hist[tile_band(t1, nt) * ORD_BUCKETS + q1], 1);
    }
  }
  __syncthreads();
  if (dbg && threadIdx.x == 0) dbg[1] = stamp_wall();
  if (soft)
    order_soft_items(sb, sx, lpb, sbk, hist, nt, order1, lp_min1, nitems1, sp, skip_empty1, dbg);
  else
    order_items(sb, sx, lpb, hist, sbk, nt, order0, 0, split_from, split_log2, nitems0, dbg);
  __syncthreads();
  if (dbg && threadIdx.x == 0) dbg[3] = stamp_wall();
}

// ---- Chip-wide count and order of both bitmaps (kl_dibr_forward; replaces tile_countorder2_kernel,
// whose two ordering workgroups counted 2 x 2,048 tiles alone: 13.9 us at cfg3, 7.6 of it the
// count).  Workgroups [0, nb) count the rasterizer's bitmap, [nb, 2 nb) the soft mask's, one tile
// per thread; each computes its tiles' ranks within (band, bucket) in tile order (per-wave counts
// in LDS) and publishes its (band, bucket) histogram with sc1 stores, then meets its bitmap's other
// count workgroups at a grid barrier (MI355X_MICROARCH.md hand-off table, first row: every storing
// wave waits vmcnt(0), a workgroup barrier, one lane's agent-scope add; the readers load sc1).  Each
// then loads all the histograms, computes its base per key (the earlier workgroups' counts: tile
// order again, the same ranks place_items gives), the parts and prefixes (place_prefix), and writes
// its OWN tiles' items at place_pos -- the same order as before.  (r05 before this: the bitmap's
// last workgroup, found by a ticket, did the prefix and placed all nt tiles alone, reading every
// tile's packed rank back: 3.7 + 3.8 us of the kernel's 12.7 behind the 3.4 us count, stamps.)
// Workgroup 2 nb zeroes `zero` (and `zacc`, when given) meanwhile.
constexpr int CO_THREADS = 512;
constexpr int CO_MAX_BLOCKS = ORD_LDS_TILES / CO_THREADS;  // count workgroups per bitmap
struct CountOrderArgs {
  const uint32_t *bm[2];
  int words, nt, nb;
  int *whist[2];        // per count workgroup: (band, bucket) histogram [nb][ORD_HIST]
  unsigned *ticket;     // [2], zero on entry (the binning kernel's zeroed region): the grid barriers
  int32_t *order[2];
  int *nitems[2];
  int split_from, split_log2;  // the rasterizer's parts
  int lp_min1, skip_empty1;    // the soft mask's
  int noband = 0;              // bit w: bitmap w's items in plain heaviest-first order (no XCD bands)
  SoftSplit sp;
  int *zero;
  int nzero;
  double *zacc;
  size_t zn;
  uint64_t *dbg = nullptr;  // dev stamps (wall clock): count workgroup b at 4 b (start, counted, arrived);
                            // bitmap w's workgroup 0 at 64 + 4 w (barrier passed, prefix, placed)
  // (nt x TILE_H, or nullptr) the soft item holding row r of tile t, -1 for none: the rasterizer
  // flags the items with an uncovered pixel by it (RastTileArgs::soft_live)
  int32_t *row_item = nullptr;
  // (r06) the grid barrier's bounded wait: after this many s_sleep(1) rounds a workgroup stops waiting
  // and counts every tile of its bitmap itself (the same histograms, so the same order); dev param
  // 16 = 1 sets 0 (every workgroup takes that path, for the equality test)
  unsigned spin_limit = 1u << 22;
  // (r06, the _C contract's soft mask) only1: one bitmap, the soft mask's (count workgroups [0, nb)
  // take bitmap 1)
  int only1 = 0;
};

static __global__ void __launch_bounds__(CO_THREADS) tile_countorder_chip_kernel(CountOrderArgs a) {
  __shared__ int s_wk[CO_THREADS / 64][ORD_HIST];  // per-wave key counts; after the barrier: this workgroup's bases
  __shared__ int sb[ORD_HIST], sx[32], lpb[ORD_BUCKETS], hist[ORD_HIST];
  extern __shared__ int s_big[];  // [nb][ORD_HIST]: every count workgroup's histogram
  const int nb = a.nb, nt = a.nt;
  const int ncount = a.only1 ? nb : 2 * nb;
  if ((int)blockIdx.x >= ncount) {
    const int part = blockIdx.x - ncount, nparts = gridDim.x - ncount;
    if (part == 0 && a.zero)
      for (int i = threadIdx.x; i < a.nzero; i += blockDim.x) a.zero[i] = 0;
    if (a.zacc) zero_doubles_share(a.zacc, a.zn, part, nparts);
    return;
  }
  const int which = a.only1 ? 1 : ((int)blockIdx.x >= nb ? 1 : 0);
  const int blk = (int)blockIdx.x - (a.only1 ? 0 : which * nb);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t *const dbg = kDevStamps && a.dbg && blockIdx.x < 16 ? a.dbg + blockIdx.x * 4 : nullptr;
  if (dbg && threadIdx.x == 0) dbg[0] = stamp_wall();
  const int t = blk * CO_THREADS + threadIdx.x;
  for (int i = threadIdx.x; i < (CO_THREADS / 64) * ORD_HIST; i += blockDim.x) (&s_wk[0][0])[i] = 0;
  // the tile's candidate-chunk count: its words (word-major, coalesced across the wave), raw buffer
  // loads from a clamped tile (words past the bitmap read as 0), all in flight together
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.bm[which], (short)0, a.words * nt * 4, 0x00020000);
  const bool flat = (a.noband >> which) & 1;  // one band: plain heaviest-first positions
  // tile tt's bucket q (log2 of its candidate-chunk count + 1) and (band, bucket) key (-1 past nt)
  auto tile_key = [&](int tt, int &qq) -> int {
    const int tc = tt < nt ? tt : nt - 1;
    unsigned n = 0;
    for (int k0 = 0; k0 < a.words; k0 += 32) {
      uint32_t x[32];
#pragma unroll
      for (int u = 0; u < 32; u++) x[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, tc * 4, (k0 + u) * nt * 4, 0);
#pragma unroll
      for (int u = 0; u < 32; u++) n += __popc(x[u]);
    }
    qq = 31 - __clz(n + 1u);
    return tt < nt ? (flat ? 0 : tile_band(tt, nt)) * ORD_BUCKETS + qq : -1;
  };
  int q;
  const int key = tile_key(t, q);
  if (dbg && threadIdx.x == 0) dbg[1] = stamp_wall();
  // rank within the workgroup for its key, in tile order: the wave's own rank (same-key lanes
  // below this one) now, the earlier waves' counts after the barrier
  int wrank = 0;
  {
    uint64_t todo = ballot(key >= 0);
    while (todo) {
      const int kl = __builtin_ctzll(todo);
      const int kk = __builtin_amdgcn_readlane(key, kl);
      const uint64_t same = ballot(key == kk) & todo;
      todo &= ~same;
      if (key == kk)
        wrank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(same >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)same, 0u));
      if (lane == kl) s_wk[wid][kk] = __popcll(same);
    }
  }
  __syncthreads();
  int rank = wrank;  // the tile's rank among this workgroup's tiles of its key
  if (key >= 0)
    for (int w = 0; w < wid; w++) rank += s_wk[w][key];
  for (int k = threadIdx.x; k < ORD_HIST; k += blockDim.x) {
    int h = 0;
#pragma unroll
    for (int w = 0; w < CO_THREADS / 64; w++) h += s_wk[w][k];
    __hip_atomic_store(a.whist[which] + blk * ORD_HIST + k, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- grid barrier of the bitmap's nb count workgroups (all co-resident: at most 2 x 32 + 1
  //      workgroups of 512 threads), on the ticket the binning kernel zeroed
  // (r06) the wait is bounded: a workgroup that has waited spin_limit rounds (the others cannot all be
  // resident -- kl_dibr_forward checks the occupancy before choosing this kernel, so only a GPU shared
  // with other work gets here) counts every tile of the bitmap itself instead
  __shared__ int s_passed;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(a.ticket + which, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dbg) dbg[2] = stamp_wall();
    unsigned spins = 0;
    bool passed = true;
    while (__hip_atomic_load(a.ticket + which, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nb) {
      if (spins++ >= a.spin_limit) {
        passed = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    s_passed = passed;
  }
  __syncthreads();
  uint64_t *const ldbg = kDevStamps && a.dbg && blk == 0 ? a.dbg + 64 + which * 4 : nullptr;
  if (ldbg && threadIdx.x == 0) ldbg[0] = stamp_wall();
  // ---- every count workgroup: all histograms (sc1 loads, eight per thread in flight), its own
  //      base per key (the earlier workgroups' counts: tile order), the totals, parts and prefixes
  //      (place_prefix), then its own tiles' items at place_pos -- the order the r04 kernel gave
  constexpr int BATCH = 8;
  const int nh = nb * ORD_HIST;
  if (s_passed) {
    for (int i0 = threadIdx.x; i0 < nh; i0 += BATCH * blockDim.x) {
      int v[BATCH];
#pragma unroll
      for (int u = 0; u < BATCH; u++) {
        const int i = i0 + u * blockDim.x;
        v[u] = __hip_atomic_load(a.whist[which] + (i < nh ? i : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int u = 0; u < BATCH; u++)
        if (i0 + u * (int)blockDim.x < nh) s_big[i0 + u * blockDim.x] = v[u];
    }
  } else {  // every count workgroup's histogram, counted here from the bitmap
    for (int i = threadIdx.x; i < nh; i += blockDim.x) s_big[i] = 0;
    __syncthreads();
    for (int b = 0; b < nb; b++) {
      int qb;
      const int kb = tile_key(b * CO_THREADS + threadIdx.x, qb);
      if (kb >= 0) atomicAdd(&s_big[b * ORD_HIST + kb], 1);
    }
  }
  __syncthreads();
  int *const wbase = &s_wk[0][0];  // (the per-wave counts are consumed: this workgroup's base per key)
  for (int k = threadIdx.x; k < ORD_HIST; k += blockDim.x) {
    int run = 0, mine = 0;
    for (int b = 0; b < nb; b++) {
      if (b == blk) mine = run;
      run += s_big[b * ORD_HIST + k];
    }
    hist[k] = run;
    wbase[k] = mine;
  }
  __syncthreads();  // hist is read across waves (soft_parts, place_prefix)
  if (ldbg && threadIdx.x == 0) ldbg[3] = stamp_wall();  // (histograms loaded, bases summed)
  if (which == 0) {
    if (threadIdx.x < ORD_BUCKETS) lpb[threadIdx.x] = (int)threadIdx.x >= a.split_from ? a.split_log2 : 0;
  } else {
    soft_parts(sx, lpb, hist, a.lp_min1, a.sp, a.skip_empty1);
  }
  place_prefix(sb, sx, lpb, hist, blk == 0 ? a.nitems[which] : nullptr);
  if (ldbg && threadIdx.x == 0) ldbg[1] = stamp_wall();
  if (key >= 0) {
    const int lp = lpb[q];
    int32_t *const ri = which == 1 ? a.row_item : nullptr;
    if (lp >= 0) {
      const int np = 1 << lp, g = key / ORD_BUCKETS;
      const int r0 = sb[key] + (wbase[key] + rank) * np;
      for (int k = 0; k < np; k++) {
        const int pos = flat ? r0 + k : place_pos(sx, g, r0 + k);
        a.order[which][pos] = t | (k << 24) | (lp << 28);
        if (ri)
          for (int r = k * (TILE_H >> lp); r < (k + 1) * (TILE_H >> lp); r++) ri[(size_t)t * TILE_H + r] = pos;
      }
    } else if (ri) {
      for (int r = 0; r < TILE_H; r++) ri[(size_t)t * TILE_H + r] = -1;
    }
  }
  if (ldbg) {
    __syncthreads();
    if (threadIdx.x == 0) ldbg[2] = stamp_wall();
  }
}

// Whether the 2 nb + 1 workgroups of tile_countorder_chip_kernel (nb per bitmap) can all be resident
// here on the device's occupancy for the kernel's block size and LDS; when they may
// not all fit, the callers take an order kernel without a grid barrier.  The answer depends only on
// the device and nb, so it is computed per call (a host query, no state kept).
static inline bool chip_order_resident(int nb) {
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(tile_countorder_chip_kernel),
                                                   CO_THREADS, (size_t)nb * ORD_HIST * sizeof(int)) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return (int64_t)per_cu * ncu >= 2 * (int64_t)nb + 1;
}

}  // namespace kl
