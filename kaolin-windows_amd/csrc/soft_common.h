// soft_common.h -- per-(pixel, face) arithmetic of the DIB-R soft mask shared by the
// reference-contract kernels (softmask.hip) and the compact fused path (softtile.hip).
#pragma once

#include "binning.h"

namespace kl {

constexpr double SM_EPS = 1e-7;

template <typename T>
__device__ __forceinline__ void soft_dist(T x0, T y0, const T v[6], float multiplier, T &dsq, int &edgeid) {
  T pdis[6];
#pragma unroll
  for (int e = 0; e < 3; e++) {
    const int e2 = (e + 1) % 3;
    const T x1 = v[e * 2], y1 = v[e * 2 + 1];
    const T x2 = v[e2 * 2], y2 = v[e2 * 2 + 1];
    const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
    const T up = A * x0 + Bc * y0 + C;
    const T down = A * A + Bc * Bc;
    T x3 = Bc * Bc * x0 - A * Bc * y0 - A * C;
    T y3 = A * A * y0 - A * Bc * x0 - Bc * C;
    x3 = (T)((double)x3 / ((double)down + SM_EPS));
    y3 = (T)((double)y3 / ((double)down + SM_EPS));
    const T direct = (x3 - x1) * (x3 - x2) + (y3 - y1) * (y3 - y2);
    if (direct > (T)0)
      pdis[e] = (T)(4 * multiplier * multiplier);
    else
      pdis[e] = (T)((double)(up * up) / ((double)down + SM_EPS));
  }
#pragma unroll
  for (int e = 0; e < 3; e++) {
    const T x1 = v[e * 2], y1 = v[e * 2 + 1];
    pdis[e + 3] = (x0 - x1) * (x0 - x1) + (y0 - y1) * (y0 - y1);
  }
  edgeid = 0;
  dsq = pdis[0];
#pragma unroll
  for (int e = 1; e < 6; e++)
    if (dsq > pdis[e]) {
      dsq = pdis[e];
      edgeid = e;
    }
}

// Pixel interval [lo, hi] (lane indices of the row segment starting at pixel ibase,
// clipped to [0, 63]) whose centres c satisfy  x_lo <= c < x_hi  exactly as the
// reference's float/double comparisons decide it: a float estimate, then corrected
// against the exact centre formula (monotone in the index).  A NaN bound never rejects: its
// comparison is false, so it stands for -inf (x_lo) or +inf (x_hi) -- the other bound still
// applies (r06: a single NaN bound had widened the interval to the whole segment, unlike the
// reference's `x0 < xmin || x0 >= xmax`; found by a caller-bbox test of the _C contract path).
// sx = m / W (the reference's float pixel pitch), inv = W / m (estimate only).
template <typename T>
__device__ __forceinline__ void seg_range_s(T x_lo, T x_hi, float sx, float inv, int W, int ibase, int &lo, int &hi) {
  if (!(x_lo == x_lo)) x_lo = (T)-INFINITY;
  if (!(x_hi == x_hi)) x_hi = (T)INFINITY;
  auto est = [&](T c) -> int {  // index = (c / s + W - 1) / 2
    const float t = ((float)c * inv + (float)(W - 1)) * 0.5f - (float)ibase;
    return t < -1.0f ? -1 : (t > 64.0f ? 64 : (int)ceilf(t));
  };
  auto cx = [&](int l) { return (T)(sx * (float)(2 * (ibase + l) + 1 - W)); };  // == pix_x
  lo = min(max(est(x_lo), 0), 64);  // first lane with c >= x_lo
  while (lo > 0 && cx(lo - 1) >= x_lo) lo--;
  while (lo < 64 && !(cx(lo) >= x_lo)) lo++;
  hi = min(max(est(x_hi) - 1, -1), 63);  // last lane with c < x_hi
  while (hi < 63 && cx(hi + 1) < x_hi) hi++;
  while (hi >= 0 && !(cx(hi) < x_hi)) hi--;
}
template <typename T>
__device__ __forceinline__ void seg_range(T x_lo, T x_hi, float m, int W, int ibase, int &lo, int &hi) {
  seg_range_s<T>(x_lo, x_hi, m / (float)W, (float)W / m, W, ibase, lo, hi);
}

// The reference backward's terms for one hit (dibr_soft_mask_cuda.cu:262-340): the
// vertex-coordinate pairs it touches (c0, and c1 for an edge) and their gradients, each
// divided by the multiplier as the reference adds them.  v: the face's 6 multiplied
// coordinates; dLdz = a / (1 - p + EPS) * p with a = -sigmainv * dLdp * (1 - allprob).
template <typename T>
__device__ __forceinline__ void soft_hit_grad(const T v[6], int edgeid, T x0, T y0, T dLdz, float multiplier,
                                              int &c0, int &c1, T &g0x, T &g0y, T &g1x, T &g1y) {
  g1x = (T)0;
  g1y = (T)0;
  c1 = -1;
  if (edgeid >= 3) {
    c0 = edgeid - 3;
    const T x1 = v[c0 * 2], y1 = v[c0 * 2 + 1];
    g0x = dLdz * (T)2 * (x1 - x0) / (T)multiplier;
    g0y = dLdz * (T)2 * (y1 - y0) / (T)multiplier;
  } else {
    c0 = edgeid;
    c1 = (edgeid + 1) % 3;
    const T x1 = v[c0 * 2], y1 = v[c0 * 2 + 1], x2 = v[c1 * 2], y2 = v[c1 * 2 + 1];
    const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
    const T up = A * x0 + Bc * y0 + C;
    const T down = A * A + Bc * Bc;
    const T dsq = (T)((double)(up * up) / ((double)down + SM_EPS));
    const T dzdA = (T)((double)((T)2 * (x0 * up - dsq * A)) / ((double)down + SM_EPS));
    const T dzdB = (T)((double)((T)2 * (y0 * up - dsq * Bc)) / ((double)down + SM_EPS));
    const T dzdC = (T)((double)((T)2 * up) / ((double)down + SM_EPS));
    g0x = dLdz * (dzdB - y2 * dzdC) / (T)multiplier;
    g0y = dLdz * (x2 * dzdC - dzdA) / (T)multiplier;
    g1x = dLdz * (y1 * dzdC - dzdB) / (T)multiplier;
    g1y = dLdz * (dzdA - x1 * dzdC) / (T)multiplier;
  }
}

// Global-memory fallback of the LDS hash adds.  Kept out of line: when both the LDS add and
// this one are inlined into the two arms of a branch, the compiler may sink them into one
// generic-address (flat) atomic, and a flat f64 atomic add is not valid on LDS.
template <typename T>
__device__ __attribute__((noinline)) void global_add_pair(T *g, int c0, int c1, T g0x, T g0y, T g1x, T g1y) {
  atomicAdd(g + c0 * 2, g0x);
  atomicAdd(g + c0 * 2 + 1, g0y);
  if (c1 >= 0) {
    atomicAdd(g + c1 * 2, g1x);
    atomicAdd(g + c1 * 2 + 1, g1y);
  }
}

// Per-face accumulation of (face, coordinate) gradient terms in an LDS hash table
// (linear probing, bounded), flushed with one global atomic per non-zero entry into a
// double accumulator; terms of faces that find no slot go straight to global atomics.
// Every accumulation is in double: the reference's float terms (each rounded as it computes
// them) sum exactly whenever their magnitudes span less than ~2^29, so the rounded result
// does not depend on the order of the atomics (acc_finalize rounds once).
constexpr int SMB_HCAP = 1024;

template <typename T>
struct FaceHash {
  int *key;     // [SMB_HCAP], -1 = empty
  double *val;  // [SMB_HCAP * 6]
  __device__ __forceinline__ void init(int tid, int nthreads) {
    for (int q = tid; q < SMB_HCAP; q += nthreads) key[q] = -1;
    for (int q = tid; q < SMB_HCAP * 6; q += nthreads) val[q] = 0.0;
  }
  __device__ __forceinline__ int slot(int f) {
    unsigned h = ((unsigned)f * 2654435761u) >> 22;  // 10 bits
#pragma unroll 1
    for (int t = 0; t < 16; t++) {
      const int cur = key[h];
      if (cur == f) return (int)h;
      if (cur == -1) {
        const int prev = atomicCAS(&key[h], -1, f);
        if (prev == -1 || prev == f) return (int)h;
      }
      h = (h + 1) & (SMB_HCAP - 1);
    }
    return -1;
  }
  // add the hit's terms (coordinate pairs c0 and, if c1 >= 0, c1) of face f
  __device__ __forceinline__ void add(int f, int c0, int c1, T g0x, T g0y, T g1x, T g1y, double *gface) {
    const int s = slot(f);
    if (s >= 0) {
      atomicAdd(&val[s * 6 + c0 * 2], (double)g0x);
      atomicAdd(&val[s * 6 + c0 * 2 + 1], (double)g0y);
      if (c1 >= 0) {
        atomicAdd(&val[s * 6 + c1 * 2], (double)g1x);
        atomicAdd(&val[s * 6 + c1 * 2 + 1], (double)g1y);
      }
    } else {
      global_add_pair<double>(gface + (size_t)f * 6, c0, c1, g0x, g0y, g1x, g1y);
    }
  }
  __device__ __forceinline__ void flush(int tid, int nthreads, double *gmesh) {
    for (int q = tid; q < SMB_HCAP * 6; q += nthreads) {
      const int k = key[q / 6];
      const double v = val[q];
      if (k >= 0 && v != 0.0) atomicAdd(gmesh + (size_t)k * 6 + q % 6, v);
    }
  }
};

// A wave's fill of [p, p + bytes) with the 32-bit pattern v (bytes of v in memory order): byte
// stores up to the first 16-byte boundary, then 16-byte stores -- 1 KB per wave instruction --
// then the tail bytes.
__device__ __forceinline__ void wave_fill(uint8_t *p, size_t bytes, uint32_t v, int lane) {
  size_t head = (16 - ((uintptr_t)p & 15)) & 15;
  if (head > bytes) head = bytes;
  if ((size_t)lane < head) p[lane] = (uint8_t)(v >> (8 * (((uintptr_t)p + lane) & 3)));
  uint8_t *body = p + head;
  const size_t nvec = (bytes - head) / 16;
  const uint4 q = make_uint4(v, v, v, v);
  for (size_t i = lane; i < nvec; i += 64) reinterpret_cast<uint4 *>(body)[i] = q;
  const size_t done = head + nvec * 16;
  if ((size_t)lane < bytes - done) p[done + lane] = (uint8_t)(v >> (8 * (((uintptr_t)p + done + lane) & 3)));
}

// Forward work items (tileorder.h, order_soft_items): a 4-wave workgroup takes 8 >> lp rows of
// a tile with Q = 4 / (8 >> lp) waves per row.
constexpr int ST_WAVES = 4;
// Backward work items: a forward item's hits taken row-major in pieces of SB_PIECE (one hit per
// thread of a backward workgroup).
constexpr int SB_PIECE = 512;
// LDS of one row: its [K][64] slot lists (face ids, then probabilities in place), the
// filled-slot prefix and the hit total
__host__ __device__ constexpr size_t st_row_lds(int K) {
  return (size_t)K * 64 * sizeof(uint32_t) + 72 * sizeof(int);  // slots | prefix, total
}


// Shards of the soft-mask backward's work-item list (counters DS_CNT_STRIDE ints apart, one per
// 64-byte line): the fused forward appends to shard blockIdx % DS_SHARDS.
constexpr int DS_SHARDS = 8;
constexpr int DS_CNT_STRIDE = 16;
// The fused path's per-face soft sums: 6 doubles padded to 8 (one 64-byte line per face, so a
// face's flush leaves L2 as one request, not two for the half of the faces a 48-byte stride
// puts across a line boundary)
constexpr int DS_ACC_STRIDE = 8;

// The compact soft-mask state (softtile.hip): per pixel the filled-slot count; per hit a
// record (face | type << 28, prob), packed per 64-pixel row segment; per segment its hit
// total; and one scratch int the forward zeroes / the backward re-zeroes after use
// (see kl_dibr_forward).
template <typename T>
struct SoftState {
  uint8_t *hits;
  uint32_t *rec_face;
  T *rec_prob;
  int *seg_tot;
  int *scratch;
};
template <typename T>
int soft_tile_forward(int B, int H, int W, int F, int K, const T *fvi, const int64_t *sel, float sigmainv, double pad,
                      float m, T *mask, const SoftState<T> &s, void *ws, size_t ws_bytes, hipStream_t st);
template <typename T>
int soft_tile_forward_main(int B, int H, int W, int F, int K, const T *fvi, const int64_t *sel, float sigmainv,
                           double pad, float m, T *mask, const SoftState<T> &s, const uint32_t *bitmap,
                           const int32_t *order, const int *nitems, const uint2 *rng, uint8_t *defer,
                           hipStream_t st, bool prefilled, int2 *bwd_items = nullptr, int *bwd_cnt = nullptr,
                           int bwd_cap = 0, const uint8_t *live = nullptr);
int soft_lp_min(int K);
template <typename T>
int soft_tile_backward(int B, int H, int W, int F, int K, const T *grad, const T *mask, const SoftState<T> &s,
                       const T *fvi, float sigmainv, float m, T *gfvi, bool accumulate, void *ws, size_t ws_bytes,
                       hipStream_t st, double *acc_out = nullptr, bool *has_sum = nullptr);
size_t soft_tile_bwd_items_bytes(int B, int H, int W, int K);
// the most backward work items one fused forward can list (per shard)
int soft_bwd_item_cap(int B, int H, int W, int K);
// The fused path's backward on the forward's item list and zeroed accumulator (DibrState):
// the per-face double sums are added into acc (B*F x DS_ACC_STRIDE), not rounded.
template <typename T>
int soft_tile_backward_listed(int B, int H, int W, int F, int K, const T *grad, const T *mask, const SoftState<T> &s,
                              const T *fvi, float sigmainv, float m, const int2 *items, const int *cnt, int cap,
                              double *acc, uint8_t *sflag, hipStream_t st);
// Per-call state of kl_dibr_forward / kl_dibr_backward (kl_dibr_state_bytes):
//   [0, 512)   DS_SHARDS item counters; int 128: the r03 gather's big-face counter (dev path)
//   items      DS_SHARDS x cap backward work items (int2)
struct DibrState {
  int cap;
  size_t off_items, bytes;
  DibrState(int B, int H, int W, int F, int K) {
    (void)F;
    cap = soft_bwd_item_cap(B, H, W, K);
    off_items = 1024;
    bytes = off_items + (size_t)DS_SHARDS * cap * sizeof(int2);
  }
  static constexpr int kZeroInts = 129;  // counters + big-face counter, zeroed by the forward
};
// kl_dibr_backward's soft accumulator (ABI 4; the caller's, zero on entry and left zero): the soft
// mask's per-face double sums (B*F x DS_ACC_STRIDE) and one touched flag byte per face.  The
// soft backward flags the faces it adds to; the gather reads, re-zeroes and unflags only those.
struct DibrSoftAcc {
  size_t off_flags, bytes;
  DibrSoftAcc(int B, int F) {
    off_flags = al256((size_t)B * F * DS_ACC_STRIDE * sizeof(double));
    bytes = off_flags + al256((size_t)B * F);
  }
};
size_t soft_tile_bwd_ws_bytes(int B, int H, int W, int F, int K);
// the _C contract forward on the tile path (softtile.hip, f32, knum <= 255): the reference's slot tensors
size_t soft_tile_slots_ws_bytes(int B, int H, int W, int F);
int soft_tile_forward_slots(int B, int H, int W, int F, int K, const float *fvi, const float *bbox, const int64_t *sel,
                            float sigmainv, float m, float *mask, float *prob, int64_t *cidx, uint8_t *ctype, void *ws,
                            size_t ws_bytes, hipStream_t st);
size_t soft_tile_ws_bytes(int B, int H, int W, int F);

}  // namespace kl
