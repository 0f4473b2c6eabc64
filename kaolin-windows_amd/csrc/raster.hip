// raster.hip -- packed_rasterize_forward / rasterize_backward for gfx950.
//
// Forward (reference: rasterization_cuda.cu:43-236, a per-pixel walk over ALL faces
// of the mesh with the batch looped serially in every thread).  Here the work is
// proportional to what faces actually cover: one thread per face visits the exact
// pixel-centre range of its bbox, runs the reference's per-(pixel, face) arithmetic
// (bbox reject, edge functions, copysign(eps) normalisation, sign test) and ranks
// the hit with a 64-bit atomicMax of (depth, ~face) in a visibility buffer; a
// per-pixel resolve pass then recomputes the winner's weights and interpolates.
// "Max depth, lowest index on ties" is exactly the reference's strict `z0 <= max_z0`
// fold in index order, so face index / weights / features are bit-identical to the
// oracle (NaN depths, which break that order, are replayed sequentially).
//
// Two entry points share it:
//   kl_packed_rasterize_forward  -- the reference's _C contract (packed valid faces,
//                                   coordinates pre-multiplied, explicit bboxes);
//   kl_dibr_rasterize_forward    -- fused front-end path: unpacked (B,F) faces + valid
//                                   mask, multiplier and bboxes applied in-kernel (the
//                                   same float ops the reference front-end runs in
//                                   torch), original face indices written directly.
//
// Backward (rasterization_cuda.cu:238-442):
//   kl_rasterize_backward        -- one thread per pixel, float atomics into the faces
//                                   (the reference's scatter; accepts any face_idx);
//   kl_dibr_rasterize_backward   -- gather: one thread per face sums the pixels of its
//                                   (conservative) screen bbox whose face_idx is that
//                                   face, in row-major order -- no atomics, deterministic.
//                                   Valid whenever face_idx came from the forward (a face
//                                   can only be selected inside its bbox).
#include <algorithm>

#include "dibrtile.h"
#include "rastcommon.h"
#include "rastgrad.h"
#include "soft_common.h"
#include "tileorder.h"
#include "tilewalk.h"

namespace kl {

// ---------------------------------------------------------------- forward
// A face, as the reference's per-pixel loop sees it (rasterization_cuda.cu:95-133):
// bbox and vertices in multiplied coordinates, vertex depths.
template <typename T>
struct RastFace {
  T xmin, ymin, xmax, ymax;
  T v[6];
  T az, bz, cz;
};

template <typename T, typename Src>
__device__ __forceinline__ void load_face(const Src &src, const T *__restrict__ fvz, int64_t f, RastFace<T> &r) {
  src.get(f, r.xmin, r.ymin, r.xmax, r.ymax);
  src.verts(f, r.v);
  r.az = fvz[f * 3 + 0];
  r.bz = fvz[f * 3 + 1];
  r.cz = fvz[f * 3 + 2];
}

template <typename T>
__device__ __forceinline__ bool face_weights(const RastFace<T> &r, T x0, T y0, float eps, T &w0, T &w1, T &w2) {
  if (x0 < r.xmin || x0 >= r.xmax || y0 < r.ymin || y0 >= r.ymax) return false;
  return tri_weights<T>(r.v, x0, y0, eps, w0, w1, w2);
}

template <typename T>
__device__ __forceinline__ T face_depth(const RastFace<T> &r, T w0, T w1, T w2) {
  return w0 * r.az + w1 * r.bz + w2 * r.cz;
}

// Exact pixel interval of one axis whose float centres c satisfy  lo <= c < hi  (the
// reference's bbox test).  Centres are monotone in the index, so the conservative
// interval of axis_range is trimmed by evaluating the exact centre formula at its ends.
// NaN bounds never reject: the whole axis.
template <typename T>
__device__ __forceinline__ void exact_axis(T lo, T hi, float m, int n, bool flip, int &a, int &b) {
  axis_range((double)lo, (double)hi, (double)(m / (float)n), n, flip, a, b);
  if (!(lo == lo) || !(hi == hi)) return;
  auto c = [&](int k) { return flip ? pix_y<T>(m, n, k) : pix_x<T>(m, n, k); };
  auto in = [&](int k) { return !(c(k) < lo || c(k) >= hi); };
  while (a <= b && !in(a)) a++;
  while (b >= a && !in(b)) b--;
}

struct VisBuf {
  unsigned long long *key;  // (P) 0 = empty
  uint32_t *idx;            // (P) double only
  uint8_t *flag;            // (P) NaN depth seen
};

template <int PASS>
__device__ __forceinline__ void vis_update(const VisBuf &vb, int64_t p, float z0, uint32_t local) {
  if (z0 != z0) {
    vb.flag[p] = 1;
    return;
  }
  if (z0 == -INFINITY) return;
  atomicMax(vb.key + p, ((unsigned long long)order32(z0) << 32) | (unsigned long long)(~local));
}
template <int PASS>
__device__ __forceinline__ void vis_update(const VisBuf &vb, int64_t p, double z0, uint32_t local) {
  if (z0 != z0) {
    if (PASS == 0) vb.flag[p] = 1;
    return;
  }
  if (z0 == -INFINITY) return;
  if (PASS == 0)
    atomicMax(vb.key + p, (unsigned long long)order64(z0));
  else if (vb.key[p] == order64(z0))
    atomicMin(vb.idx + p, local);
}

// mesh of packed face f (first_idx) or of dense face f (uniform meshes)
__device__ __forceinline__ void face_mesh(int64_t f, const int64_t *__restrict__ first_idx, int B,
                                          int faces_per_mesh, int &b, int64_t &f0) {
  if (first_idx) {
    int lo = 0, hi = B - 1;  // last b with first_idx[b] <= f
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (first_idx[mid] <= f)
        lo = mid;
      else
        hi = mid - 1;
    }
    b = lo;
    f0 = first_idx[lo];
  } else {
    b = (int)(f / faces_per_mesh);
    f0 = (int64_t)b * faces_per_mesh;
  }
}

constexpr int VIS_SMALL_AREA = 1024;  // faces covering more pixel centres go to the WG kernel
constexpr int LPF = 8;                // lanes per face in the per-face kernels

// Walks a face's exact pixel range [ix0,ix1]x[iy0,iy1] in row-major order, lane s of the
// face's lane group taking elements s, s+LPF, ...  (no divisions in the loop).
template <int STEP = LPF>
struct RangeWalkN {
  int w, area, e, col, row;
  __device__ __forceinline__ RangeWalkN(int ix0, int ix1, int iy0, int iy1, int s) {
    w = ix1 - ix0 + 1;
    area = w * (iy1 - iy0 + 1);
    e = s;
    row = s / w;
    col = s - row * w;
  }
  __device__ __forceinline__ bool more() const { return e < area; }
  __device__ __forceinline__ void next() {
    e += STEP;
    col += STEP;
    while (col >= w) {
      col -= w;
      row++;
    }
  }
};
using RangeWalk = RangeWalkN<LPF>;

// LPF lanes per face; faces whose exact pixel range exceeds VIS_SMALL_AREA are queued
template <typename T, typename Src, int PASS>
__global__ void __launch_bounds__(256) raster_vis_kernel(Src src, const T *__restrict__ fvz,
                                                         const int64_t *__restrict__ first_idx, int B,
                                                         int faces_per_mesh, int64_t nfaces, int H, int W, float m,
                                                         float eps, VisBuf vb, int *__restrict__ big,
                                                         int *__restrict__ nbig) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t f = t / LPF;
  const int s = (int)(t % LPF);
  if (f >= nfaces || !src.valid(f)) return;
  RastFace<T> r;
  load_face(src, fvz, f, r);
  int ix0, ix1, iy0, iy1;
  exact_axis(r.xmin, r.xmax, m, W, false, ix0, ix1);
  if (ix0 > ix1) return;
  exact_axis(r.ymin, r.ymax, m, H, true, iy0, iy1);
  if (iy0 > iy1) return;
  if ((int64_t)(ix1 - ix0 + 1) * (iy1 - iy0 + 1) > VIS_SMALL_AREA) {
    if (PASS == 0 && s == 0) big[atomicAdd(nbig, 1)] = (int)f;
    return;
  }
  int b;
  int64_t f0;
  face_mesh(f, first_idx, B, faces_per_mesh, b, f0);
  const uint32_t local = (uint32_t)(f - f0);
  const int64_t pbase = (int64_t)b * H * W;
  for (RangeWalk rw(ix0, ix1, iy0, iy1, s); rw.more(); rw.next()) {
    const int i = ix0 + rw.col, j = iy0 + rw.row;
    T w0, w1, w2;
    if (face_weights(r, pix_x<T>(m, W, i), pix_y<T>(m, H, j), eps, w0, w1, w2))
      vis_update<PASS>(vb, pbase + (int64_t)j * W + i, face_depth(r, w0, w1, w2), local);
  }
}

// one workgroup per queued large face
template <typename T, typename Src, int PASS>
__global__ void __launch_bounds__(256) raster_vis_big_kernel(Src src, const T *__restrict__ fvz,
                                                             const int64_t *__restrict__ first_idx, int B,
                                                             int faces_per_mesh, int H, int W, float m, float eps,
                                                             VisBuf vb, const int *__restrict__ big,
                                                             const int *__restrict__ nbig) {
  const int n = *nbig;
  for (int k = blockIdx.x; k < n; k += gridDim.x) {
    const int64_t f = big[k];
    RastFace<T> r;
    load_face(src, fvz, f, r);
    int ix0, ix1, iy0, iy1;
    exact_axis(r.xmin, r.xmax, m, W, false, ix0, ix1);
    exact_axis(r.ymin, r.ymax, m, H, true, iy0, iy1);
    int b;
    int64_t f0;
    face_mesh(f, first_idx, B, faces_per_mesh, b, f0);
    const uint32_t local = (uint32_t)(f - f0);
    const int w = ix1 - ix0 + 1;
    const int64_t area = (int64_t)w * (iy1 - iy0 + 1);
    for (int64_t e = threadIdx.x; e < area; e += blockDim.x) {
      const int j = iy0 + (int)(e / w), i = ix0 + (int)(e % w);
      T w0, w1, w2;
      if (face_weights(r, pix_x<T>(m, W, i), pix_y<T>(m, H, j), eps, w0, w1, w2))
        vis_update<PASS>(vb, ((int64_t)b * H + j) * W + i, face_depth(r, w0, w1, w2), local);
    }
  }
}

// One thread per pixel: decode the winner, recompute its weights with the same
// arithmetic (bit-identical to the pass that ranked it) and write the outputs.
// Flagged pixels (NaN depth) replay the reference's sequential fold over all faces.
template <typename T, typename Src>
__global__ void __launch_bounds__(256) raster_resolve_kernel(Src src, const T *__restrict__ fvz,
                                                             const T *__restrict__ feat,
                                                             const int64_t *__restrict__ first_idx,
                                                             int faces_per_mesh, int B, int H, int W, int D,
                                                             float m, float eps, VisBuf vb, T *__restrict__ out_feat,
                                                             int64_t *__restrict__ out_idx, T *__restrict__ out_w) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= (int64_t)B * H * W) return;
  const int b = (int)(p / ((int64_t)H * W));
  const int rem = (int)(p - (int64_t)b * H * W);
  const int j = rem / W, i = rem - j * W;
  const T x0 = pix_x<T>(m, W, i), y0 = pix_y<T>(m, H, j);
  const int64_t f0 = first_idx ? first_idx[b] : (int64_t)b * faces_per_mesh;
  int64_t win = -1;
  T mw0 = 0, mw1 = 0, mw2 = 0;
  if (vb.flag[p]) {
    const int64_t f1 = first_idx ? first_idx[b + 1] : f0 + faces_per_mesh;
    T max_z0 = -INFINITY;
    for (int64_t f = f0; f < f1; f++) {
      if (!src.valid(f)) continue;
      RastFace<T> r;
      load_face(src, fvz, f, r);
      T w0, w1, w2;
      if (!face_weights(r, x0, y0, eps, w0, w1, w2)) continue;
      const T z0 = face_depth(r, w0, w1, w2);
      if (z0 <= max_z0) continue;
      max_z0 = z0;
      win = f;
      mw0 = w0;
      mw1 = w1;
      mw2 = w2;
    }
  } else {
    const unsigned long long key = vb.key[p];
    if (key != 0) {
      win = f0 + (int64_t)(sizeof(T) == 4 ? (uint32_t)~(uint32_t)key : vb.idx[p]);
      RastFace<T> r;
      load_face(src, fvz, win, r);
      face_weights(r, x0, y0, eps, mw0, mw1, mw2);
    }
  }
  out_idx[p] = win >= 0 ? win - f0 : -1;
  out_w[p * 3 + 0] = mw0;
  out_w[p * 3 + 1] = mw1;
  out_w[p * 3 + 2] = mw2;
  if (win >= 0) {
    const T *c = feat + (size_t)win * 3 * D;
    for (int d = 0; d < D; d++) out_feat[p * D + d] = mw0 * c[d] + mw1 * c[D + d] + mw2 * c[2 * D + d];
  } else {
    for (int d = 0; d < D; d++) out_feat[p * D + d] = (T)0;
  }
}

struct RastWs {
  size_t P, nf;
  size_t off_key, off_idx, off_flag, off_big, bytes;
  RastWs(int B, int H, int W, int64_t nfaces) {
    P = (size_t)B * H * W;
    nf = (size_t)(nfaces > 0 ? nfaces : 0);
    off_key = 0;
    off_idx = off_key + P * 8;
    off_flag = off_idx + P * 4;
    off_big = off_flag + ((P + 15) & ~(size_t)15);
    bytes = off_big + (nf + 1) * 4;
  }
};

template <typename T, typename Src>
static int launch_rast_fwd(Src src, int H, int W, int B, int D, int64_t nfaces, int64_t ws_faces, const T *fvz,
                           const T *feat, const int64_t *first_idx, int faces_per_mesh, float m, float eps,
                           T *out_feat, int64_t *out_idx, T *out_w, void *ws, size_t ws_bytes, hipStream_t st) {
  const RastWs L(B, H, W, ws_faces);
  KL_REQUIRE(nfaces <= ws_faces && ws_bytes >= L.bytes, "rasterize forward: workspace too small");
  KL_REQUIRE(nfaces < ((int64_t)1 << 31), "rasterize forward: too many faces");
  if (L.P == 0) return KL_OK;
  char *w = reinterpret_cast<char *>(ws);
  VisBuf vb{reinterpret_cast<unsigned long long *>(w + L.off_key), reinterpret_cast<uint32_t *>(w + L.off_idx),
            reinterpret_cast<uint8_t *>(w + L.off_flag)};
  int *nbig = reinterpret_cast<int *>(w + L.off_big);
  int *big = nbig + 1;
  // key | idx | flag | nbig are contiguous: key and flag/nbig zeroed, idx set to ~0
  KL_CHECK_RC(fill_async(w, 0, L.off_big + 4, st));
  if (sizeof(T) == 8) KL_CHECK_RC(fill_async(w + L.off_idx, 0xff, L.P * 4, st));
  if (nfaces > 0) {
    const unsigned fb = (unsigned)cdiv(nfaces * LPF, 256);
    hipLaunchKernelGGL((raster_vis_kernel<T, Src, 0>), dim3(fb), dim3(256), 0, st, src, fvz, first_idx, B,
                       faces_per_mesh, nfaces, H, W, m, eps, vb, big, nbig);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL((raster_vis_big_kernel<T, Src, 0>), dim3(512), dim3(256), 0, st, src, fvz, first_idx, B,
                       faces_per_mesh, H, W, m, eps, vb, big, nbig);
    KL_CHECK_LAUNCH();
    if (sizeof(T) == 8) {
      hipLaunchKernelGGL((raster_vis_kernel<T, Src, 1>), dim3(fb), dim3(256), 0, st, src, fvz, first_idx, B,
                         faces_per_mesh, nfaces, H, W, m, eps, vb, big, nbig);
      KL_CHECK_LAUNCH();
      hipLaunchKernelGGL((raster_vis_big_kernel<T, Src, 1>), dim3(512), dim3(256), 0, st, src, fvz, first_idx, B,
                         faces_per_mesh, H, W, m, eps, vb, big, nbig);
      KL_CHECK_LAUNCH();
    }
  }
  hipLaunchKernelGGL((raster_resolve_kernel<T, Src>), dim3((unsigned)cdiv((int64_t)L.P, 256)), dim3(256), 0, st, src,
                     fvz, feat, first_idx, faces_per_mesh, B, H, W, D, m, eps, vb, out_feat, out_idx, out_w);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

// ---------------------------------------------------------------- tile forward (fused path)
// One 512-thread workgroup per 64x8 pixel tile, one wave per row, one lane per pixel.
// The tile's candidate chunks (bin bitmap) are expanded 8 chunks (512 faces) per step:
// each wave loads one chunk's faces (vertices x m, depths, validity) -- the next step's
// loads in flight while this step's are tested -- rejects invalid faces and those whose
// bbox misses every pixel centre of the tile (exact row test, exact column interval), and
// appends the rest in index order to an LDS list.  Each row then transposes the list's
// pixel masks so that every pixel lane visits its own candidates in index order and runs
// the reference's per-(pixel, face) loop body (rasterization_cuda.cu:95-171) verbatim:
// bbox-passing faces, edge weights, sign test, depth, strict `z0 <= max_z0` fold.  So
// the fold is the reference's, NaN depths included, with no atomics and no resolve pass.
constexpr int RT_CAP = 512;  // list entries per step: one chunk per wave
constexpr int RT_VS = 12;    // LDS stride of a list entry: 6 coordinates, 3 depths, pad


// VMODE: 0 all faces valid, 1 valid mask, 2 face_normals_z >= 0.  All loads are issued
// up front (clamped index, no branch around them) and the stores come last.
template <typename T, int VMODE>
__global__ void __launch_bounds__(256) raster_bin_kernel(RastSrc<T> src, const T *__restrict__ fvz, int F, BinGeom g,
                                                         PixPitch pp, uint32_t *__restrict__ bitmap,
                                                         T *__restrict__ rec, uint2 *__restrict__ rng,
                                                         uint32_t *__restrict__ sbitmap = nullptr,
                                                         uint2 *__restrict__ srng = nullptr, T spad = 0) {
  __shared__ uint8_t s_bm[4][256];  // bin_mark scratch, one per wave
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.y;
  if (c >= g.chunks || c * 64 >= F) return;
  const int fl = c * 64 + lane;
  const bool live = fl < F;
  const int64_t f = (int64_t)b * F + (live ? fl : F - 1);
  T v[6], z[3];
  src.verts(f, v);
#pragma unroll
  for (int q = 0; q < 3; q++) z[q] = fvz[f * 3 + q];
  bool valid = live;
  if constexpr (VMODE == 1) valid = valid && src.vmask[f] != 0;
  if constexpr (VMODE == 2) valid = valid && src.nz[f] >= (T)0;
  int ix0 = 1, ix1 = 0, iy0 = 1, iy1 = 0;
  if (valid) {
    const T xmin = tmin3(v[0], v[2], v[4]), ymin = tmin3(v[1], v[3], v[5]);
    const T xmax = tmax3(v[0], v[2], v[4]), ymax = tmax3(v[1], v[3], v[5]);
    exact_range(xmin, xmax, pp.sx, pp.xinv, g.width, false, ix0, ix1);
    exact_range(ymin, ymax, pp.sy, pp.yinv, g.height, true, iy0, iy1);
    if (ix0 > ix1 || iy0 > iy1) {
      ix0 = iy0 = 1;
      ix1 = iy1 = 0;
    }
  }
  if (live) {
    T *r = rec + f * RT_REC;
#pragma unroll
    for (int q = 0; q < 6; q++) r[q] = v[q];
#pragma unroll
    for (int q = 0; q < 3; q++) r[6 + q] = z[q];
    rng[f] = make_uint2((uint32_t)ix0 | ((uint32_t)ix1 << 16), (uint32_t)iy0 | ((uint32_t)iy1 << 16));
  }
  const bool has = ix0 <= ix1;
  bin_mark(g, b, c, lane, has ? ix0 / TILE_W : 1, has ? ix1 / TILE_W : 0, has ? iy0 / TILE_H : 1,
           has ? iy1 / TILE_H : 0, bitmap, s_bm[threadIdx.x >> 6]);
  if (sbitmap) {
    // the soft mask's bins of the same faces (kl_dibr_forward): every face, bbox enlarged
    // by boxlen * multiplier as SoftSrc / dibr.py:31-39, and its exact pixel ranges
    int tx0 = 1, tx1 = 0, ty0 = 1, ty1 = 0;
    if (live) {
      const T bx0 = tmin3(v[0], v[2], v[4]) - spad, by0 = tmin3(v[1], v[3], v[5]) - spad;
      const T bx1 = tmax3(v[0], v[2], v[4]) + spad, by1 = tmax3(v[1], v[3], v[5]) + spad;
      int jx0, jx1, jy0, jy1;
      exact_range(bx0, bx1, pp.sx, pp.xinv, g.width, false, jx0, jx1);
      exact_range(by0, by1, pp.sy, pp.yinv, g.height, true, jy0, jy1);
      if (jx0 > jx1 || jy0 > jy1) {
        jx0 = jy0 = 1;
        jx1 = jy1 = 0;
      } else {
        tx0 = jx0 / TILE_W;
        tx1 = jx1 / TILE_W;
        ty0 = jy0 / TILE_H;
        ty1 = jy1 / TILE_H;
      }
      srng[f] = make_uint2((uint32_t)jx0 | ((uint32_t)jx1 << 16), (uint32_t)jy0 | ((uint32_t)jy1 << 16));
    }
    bin_mark(g, b, c, lane, tx0, tx1, ty0, ty1, sbitmap, s_bm[threadIdx.x >> 6]);
  }
}

// raster_bin_kernel's per-face part as a function: the face's record and exact ranges, and its
// tile rectangles (raster; soft when `soft`), empty = tx0 > tx1.
template <typename T, int VMODE>
__device__ __forceinline__ void bin_face(const RastSrc<T> &src, const T *__restrict__ fvz, const BinGeom &g,
                                         const PixPitch &pp, int64_t f, T *__restrict__ rec, uint2 *__restrict__ rng,
                                         bool soft, uint2 *__restrict__ srng, T spad, int4 &rt, int4 &st) {
  T v[6], z[3];
  src.verts(f, v);
#pragma unroll
  for (int q = 0; q < 3; q++) z[q] = fvz[f * 3 + q];
  bool valid = true;
  if constexpr (VMODE == 1) valid = src.vmask[f] != 0;
  if constexpr (VMODE == 2) valid = src.nz[f] >= (T)0;
  int ix0 = 1, ix1 = 0, iy0 = 1, iy1 = 0;
  if (valid) {
    const T xmin = tmin3(v[0], v[2], v[4]), ymin = tmin3(v[1], v[3], v[5]);
    const T xmax = tmax3(v[0], v[2], v[4]), ymax = tmax3(v[1], v[3], v[5]);
    exact_range(xmin, xmax, pp.sx, pp.xinv, g.width, false, ix0, ix1);
    exact_range(ymin, ymax, pp.sy, pp.yinv, g.height, true, iy0, iy1);
    if (ix0 > ix1 || iy0 > iy1) {
      ix0 = iy0 = 1;
      ix1 = iy1 = 0;
    }
  }
  T *r = rec + f * RT_REC;
#pragma unroll
  for (int q = 0; q < 6; q++) r[q] = v[q];
#pragma unroll
  for (int q = 0; q < 3; q++) r[6 + q] = z[q];
  rng[f] = make_uint2((uint32_t)ix0 | ((uint32_t)ix1 << 16), (uint32_t)iy0 | ((uint32_t)iy1 << 16));
  rt = ix0 <= ix1 ? make_int4(ix0 / TILE_W, ix1 / TILE_W, iy0 / TILE_H, iy1 / TILE_H) : make_int4(1, 0, 1, 0);
  st = make_int4(1, 0, 1, 0);
  if (soft) {
    const T bx0 = tmin3(v[0], v[2], v[4]) - spad, by0 = tmin3(v[1], v[3], v[5]) - spad;
    const T bx1 = tmax3(v[0], v[2], v[4]) + spad, by1 = tmax3(v[1], v[3], v[5]) + spad;
    int jx0, jx1, jy0, jy1;
    exact_range(bx0, bx1, pp.sx, pp.xinv, g.width, false, jx0, jx1);
    exact_range(by0, by1, pp.sy, pp.yinv, g.height, true, jy0, jy1);
    if (jx0 > jx1 || jy0 > jy1) {
      jx0 = jy0 = 1;
      jx1 = jy1 = 0;
    } else {
      st = make_int4(jx0 / TILE_W, jx1 / TILE_W, jy0 / TILE_H, jy1 / TILE_H);
    }
    srng[f] = make_uint2((uint32_t)jx0 | ((uint32_t)jx1 << 16), (uint32_t)jy0 | ((uint32_t)jy1 << 16));
  }
}

// Bins without global atomics: one workgroup per (byte of a bitmap word, mesh), i.e. the 512
// faces of 8 chunks, marks its chunks' bits in an LDS byte per tile of the view (LDS
// atomicOr), then stores that byte of every tile's word -- every byte of the bitmaps is
// written, so the bitmaps need no zero fill and take no global atomics.
// LDS: one uint32 per tile and bitmap (bin_word_lds_ok).
constexpr int BIN_WORD_THREADS = 512;  // one face per thread: 8 chunks
inline bool bin_word_lds_ok(const BinGeom &g) { return (size_t)g.tiles_x * g.tiles_y * 2 * 4 <= 64 * 1024; }

// MARKS (r05): the chunk of a face is its wave (512 threads = 8 chunks), so every lane of a wave sets
// the same bit: instead of an LDS atomicOr per (face, tile) -- 87 % of the LDS cycles were bank
// conflicts of lanes hitting the same tile word (r05o counters) -- each lane stores a 1 byte into
// its wave's mark of the tile (tile-major, 8 bytes per tile: plain stores of one value), and the
// tile's byte is gathered from its 8 marks at the end.  LDS 16 bytes per tile (bin_word_marks_ok).
inline bool bin_word_marks_ok(const BinGeom &g) { return (size_t)g.tiles_x * g.tiles_y * 16 <= 64 * 1024; }

template <typename T, int VMODE, bool MARKS>
__global__ void __launch_bounds__(BIN_WORD_THREADS) raster_bin_word_kernel(
    RastSrc<T> src, const T *__restrict__ fvz, int F, BinGeom g, PixPitch pp, uint32_t *__restrict__ bitmap,
    T *__restrict__ rec, uint2 *__restrict__ rng, uint32_t *__restrict__ sbitmap, uint2 *__restrict__ srng, T spad,
    int *__restrict__ zero, int nzero) {
  extern __shared__ uint32_t s_words[];
  const int ntv = g.tiles_x * g.tiles_y;
  const int grp = blockIdx.x, b = blockIdx.y;  // chunks [8 grp, 8 grp + 8)
  // the bucket kernel's histograms, zeroed here instead of by a fill launch
  if (grp == 0 && b == 0)
    for (int t = threadIdx.x; t < nzero; t += blockDim.x) zero[t] = 0;
  uint32_t *sr = s_words, *ss = s_words + (MARKS ? 2 * ntv : ntv);  // MARKS: [tile][8] bytes each
  uint8_t *mr = reinterpret_cast<uint8_t *>(sr), *ms = reinterpret_cast<uint8_t *>(ss);
  const bool soft = sbitmap != nullptr, rast = bitmap != nullptr;  // (the fused tile kernel: soft bins only)
  for (int t = threadIdx.x; t < (MARKS ? 4 : 2) * ntv; t += blockDim.x) s_words[t] = 0;
  __syncthreads();
  const int fl = grp * 512 + (int)threadIdx.x;
  if (fl < F) {
    int4 rt, st;
    bin_face<T, VMODE>(src, fvz, g, pp, (int64_t)b * F + fl, rec, rng, soft, srng, spad, rt, st);
    const int w = (fl >> 6) & 7;
    const uint32_t bit = 1u << w;
    if (rast)
      for (int ty = rt.z; ty <= rt.w; ty++)
        for (int tx = rt.x; tx <= rt.y; tx++) {
          if (MARKS) mr[(ty * g.tiles_x + tx) * 8 + w] = 1;
          else atomicOr(&sr[ty * g.tiles_x + tx], bit);
        }
    for (int ty = st.z; ty <= st.w; ty++)
      for (int tx = st.x; tx <= st.y; tx++) {
        if (MARKS) ms[(ty * g.tiles_x + tx) * 8 + w] = 1;
        else atomicOr(&ss[ty * g.tiles_x + tx], bit);
      }
  }
  __syncthreads();
  const size_t base = (size_t)b * ntv;
  const int word = grp >> 2, byte = grp & 3;  // little-endian: chunk bits 8 byte .. 8 byte + 7
  uint8_t *rb = reinterpret_cast<uint8_t *>(bitmap), *sb = reinterpret_cast<uint8_t *>(sbitmap);
  // 8 mark bytes (0 / 1, byte w = chunk w) -> bit w
  auto gather8 = [](uint64_t x) { return (uint8_t)((x * 0x0102040810204080ull) >> 56); };
  for (int t = threadIdx.x; t < ntv; t += blockDim.x) {
    const size_t o = bm_index(g.ntiles(), base + t, word) * 4 + byte;
    if (MARKS) {
      if (rast) rb[o] = gather8(reinterpret_cast<const uint64_t *>(mr)[t]);
      if (soft) sb[o] = gather8(reinterpret_cast<const uint64_t *>(ms)[t]);
    } else {
      if (rast) rb[o] = (uint8_t)sr[t];
      if (soft) sb[o] = (uint8_t)ss[t];
    }
  }
}

template <typename T>
static int launch_bin_word(const RastSrc<T> &src, const T *fvz, int F, const BinGeom &g, const PixPitch &pp,
                           uint32_t *bitmap, T *rec, uint2 *rng, uint32_t *sbitmap, uint2 *srng, T spad,
                           int *zero, int nzero, hipStream_t st) {
  const dim3 grid((unsigned)(g.words * 4), (unsigned)g.batch);  // every byte of every word
  // dev param 22 = 1: the LDS-atomic marking for A/B (and the only one past 4,096 tiles per view)
  const bool marks = bin_word_marks_ok(g) && g_dev_param[22] != 1;
  const size_t lds = (size_t)g.tiles_x * g.tiles_y * (marks ? 16 : 8);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(BIN_WORD_THREADS), lds, st, src, fvz, F, g, pp, bitmap, rec, rng, sbitmap,
                       srng, spad, zero, nzero);
  };
  if (src.vmask) marks ? go(raster_bin_word_kernel<T, 1, true>) : go(raster_bin_word_kernel<T, 1, false>);
  else if (src.nz) marks ? go(raster_bin_word_kernel<T, 2, true>) : go(raster_bin_word_kernel<T, 2, false>);
  else marks ? go(raster_bin_word_kernel<T, 0, true>) : go(raster_bin_word_kernel<T, 0, false>);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
struct RastTileArgs {
  RastSrc<T> src;
  const T *fvz;
  const T *feat;
  const uint32_t *bitmap;
  const T *rec;
  const uint2 *rng;
  const int32_t *items;  // tileorder.h work items, heaviest first
  const int *nitems;
  BinGeom g;
  int F, D;
  float eps;
  T *out_feat;
  int64_t *out_idx;
  T *out_w;
  uint64_t *dbg;  // dev stamps (kl_dev_set_debug), 8 per wave, or nullptr
  // kl_dibr_forward: the soft mask's outputs for pixels / row segments without hits, written
  // here (mask = covered, hits = 0, seg_tot = defer = 0) so that the soft-mask kernel only
  // touches the ones with hits (nullptr: not written)
  T *soft_mask = nullptr;
  uint8_t *soft_hits = nullptr;
  int *soft_seg = nullptr;
  uint8_t *soft_defer = nullptr;
  // r05: the soft items holding this tile's rows (CountOrderArgs::row_item) and their flags, set
  // here for the items with an uncovered pixel (zeroed by the binning kernel; nullptr: not flagged)
  const int32_t *soft_row_item = nullptr;
  uint8_t *soft_live = nullptr;
};

template <typename T>
__global__ void __launch_bounds__(512) raster_tile_kernel(RastTileArgs<T> a) {
  uint64_t *const dbg = kDevStamps ? a.dbg : nullptr;  // compiled out unless KL_DEV_STAMPS
  constexpr int R = 8;  // waves per workgroup
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const BinGeom &g = a.g;
  // the item: a tile, or one of 2^lg parts of its rows (heavy tiles); 2^lg waves share a row
  if ((int)blockIdx.x >= *a.nitems) return;
  const int32_t item = a.items[blockIdx.x];
  const int tile = item & 0xffffff;
  const int part = (item >> 24) & 15;
  const int lg = (item >> 28) & 7;
  ChunkSeq seq;
  seq.init(a.bitmap + tile, g.words, g.ntiles(), lane);
  const int RG = R >> lg;     // rows of the workgroup
  const int WPR = 1 << lg;    // waves per row
  __shared__ uint32_t L_face[RT_CAP];
  __shared__ uint32_t L_pack[RT_CAP];
  __shared__ __align__(16) T L_v[RT_CAP * RT_VS];
  __shared__ int s_cnt[R];
  __shared__ int s_pre[R * 64];                   // f32 pair walk: entry width prefix << 8 | lo
  __shared__ unsigned long long s_key[R * 64];    // f32 pair walk: per-pixel depth key
  __shared__ unsigned long long s_nan[R];         // f32 pair walk: pixels that saw a NaN depth
  const int r = wid >> lg;          // this wave's row of the workgroup
  const int sub = wid & (WPR - 1);  // and its share of that row's pairs
  if constexpr (sizeof(T) == 4) {
    if ((int)threadIdx.x < RG * 64) s_key[threadIdx.x] = 0;
    if ((int)threadIdx.x < RG) s_nan[threadIdx.x] = 0;
    __syncthreads();
  }
  const int H = g.height, W = g.width;
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int b = tile / (g.tiles_x * g.tiles_y);
  const int j0 = ty * TILE_H + part * RG;  // the workgroup's first row
  const int j = j0 + r;
  const int ibase = tx * TILE_W;
  const int i = ibase + lane;
  const bool px_valid = j < H && i < W;
  const float m = a.src.m;
  const float sx = m / (float)W, sy = m / (float)H;
  const T x0 = (T)(sx * (float)(2 * i + 1 - W));               // == pix_x<T>(m, W, i)
  const T y0 = (T)(sy * (float)(H - 2 * (j < H ? j : H - 1) - 1));  // == pix_y<T>(m, H, j)
  const int64_t f0 = (int64_t)b * a.F;
  const T *rec = a.rec + f0 * RT_REC;
  const uint2 *rng = a.rng + f0;
  // (soft_live) the soft item of this row, loaded now: its flag is set at the end
  const int32_t srow = a.soft_live && sub == 0 ? a.soft_row_item[(size_t)tile * TILE_H + (j0 - ty * TILE_H) + r] : -1;

  T max_z0 = -INFINITY, mw0 = 0, mw1 = 0, mw2 = 0;
  int win = -1;
  uint64_t t0 = 0, w0s = 0, c_fill = 0, c_walk = 0, tq = 0, tr = 0;
  uint64_t c_ph[5] = {0, 0, 0, 0, 0};
  auto phase = [&](int k) {
    if (dbg) {
      const uint64_t t = stamp_clk();
      c_ph[k] += t - tr;
      tr = t;
    }
  };
  int n_entries = 0, n_iters = 0, n_visits = 0;
  if (dbg) {
    t0 = stamp_clk();
    w0s = stamp_wall();
  }

  // A step = one candidate chunk per wave.  Its face data is loaded a step ahead into
  // alternating register sets (no copy between them, so the loads stay in flight while
  // the current step is tested and walked).
  struct Pref {
    T v[9];
    uint2 r;
    int c;
  };
  int pos = 0;
  bool more = false;
  auto issue = [&](Pref &P) {
    more = seq.at(pos, lane) >= 0;
    P.c = more ? seq.at(pos + wid, lane) : -1;
    pos += R;
    // unconditional loads from a clamped index: a guarded load would be waited for at once
    int fl = P.c * 64 + lane;
    fl = fl < 0 ? 0 : (fl < a.F ? fl : a.F - 1);
#pragma unroll
    for (int q = 0; q < 9; q++) P.v[q] = rec[(size_t)fl * RT_REC + q];
    P.r = rng[fl];
  };
  auto step = [&](Pref &cur, Pref &nxt) {
    if (dbg) tq = tr = stamp_clk();
    const int c = cur.c;
    if (dbg) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      phase(4);
    }
    issue(nxt);
    phase(0);
    // the face's exact pixel ranges against this tile's rows and columns
    const int fl = c * 64 + lane;
    const int ix0 = (int)(cur.r.x & 0xffffu), ix1 = (int)(cur.r.x >> 16);
    const int iy0 = (int)(cur.r.y & 0xffffu), iy1 = (int)(cur.r.y >> 16);
    const int ya = max(iy0, j0) - j0, yb = min(iy1, j0 + RG - 1) - j0;
    const uint32_t rows = ya <= yb ? ((2u << yb) - 1u) & ~((1u << ya) - 1u) : 0u;
    const int lo = max(ix0 - ibase, 0), hi = min(ix1 - ibase, 63);
    const bool keep = c >= 0 && fl < a.F && rows != 0 && lo <= hi;
    const T *v = cur.v;
    const uint64_t km = ballot(keep);
    if (lane == 0) s_cnt[wid] = __popcll(km);
    phase(1);
    __syncthreads();
    phase(2);
    int pre = 0, len = 0;
#pragma unroll
    for (int w = 0; w < R; w++) {
      const int cw = s_cnt[w];
      pre += w < wid ? cw : 0;
      len += cw;
    }
    if (keep) {
      const int p = pre + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0u));
      L_face[p] = (uint32_t)fl;
      L_pack[p] = (uint32_t)lo | ((uint32_t)hi << 6) | (rows << 12);
#pragma unroll
      for (int q = 0; q < 9; q++) L_v[p * RT_VS + q] = v[q];
    }
    __syncthreads();
    phase(3);
    n_entries += len;
    if (dbg) {
      const uint64_t t = stamp_clk();
      c_fill += t - tq;
      tq = t;
    }
    if constexpr (sizeof(T) == 4) {
      // this row's (pixel, face) pairs, 64 list entries at a time, evaluated densely: an
      // entry's pixels are the contiguous run [lo, hi], so pair t belongs to the entry whose
      // exclusive width prefix is the last <= t.  Each pair ranks its depth in the pixel's
      // LDS key (max depth, lowest index on ties: the reference's strict fold for non-NaN
      // depths); a NaN depth flags the pixel for the sequential replay below.
      for (int base = 0; base < len; base += 64) {
        const int e = base + lane;
        int lo = 0, wdt = 0;
        if (e < len) {
          const uint32_t pk = L_pack[e];
          if ((pk >> (12 + r)) & 1u) {
            lo = (int)(pk & 63u);
            wdt = (int)((pk >> 6) & 63u) - lo + 1;
          }
        }
        const int inc = wave_incl_scan(wdt);
        const int total = __builtin_amdgcn_readlane(inc, 63);
        if (total == 0) continue;
        s_pre[wid * 64 + lane] = ((inc - wdt) << 8) | lo;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (dbg) {
          n_visits += wdt;
          n_iters += (total + 63) >> 6;
        }
        for (int t = lane + 64 * sub; t < total; t += 64 * WPR) {
          int q = 0;  // owner entry: last q with prefix <= t
#pragma unroll
          for (int stp = 32; stp > 0; stp >>= 1)
            if ((s_pre[wid * 64 + q + stp] >> 8) <= t) q += stp;
          const int pq = s_pre[wid * 64 + q];
          const int pix = (pq & 255) + t - (pq >> 8);
          const T *v = L_v + (base + q) * RT_VS;
          const T xp = (T)(sx * (float)(2 * (ibase + pix) + 1 - W));
          T w0, w1, w2;
          if (!tri_weights<T>(v, xp, y0, a.eps, w0, w1, w2)) continue;
          const float z0 = (float)(w0 * v[6] + w1 * v[7] + w2 * v[8]);
          if (z0 != z0)
            atomicOr(&s_nan[r], 1ull << pix);
          else if (z0 != -INFINITY)
            atomicMax(&s_key[r * 64 + pix],
                      ((unsigned long long)order32(z0) << 32) | (unsigned long long)(~L_face[base + q]));
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      }
    } else {
    // this row's walk: 64 list entries at a time, transposed to per-pixel candidate masks
    for (int base = 0; base < len; base += 64) {
      const int e = base + lane;
      uint64_t rm = 0;
      if (e < len) {
        const uint32_t pk = L_pack[e];
        if ((pk >> (12 + r)) & 1u) {
          const int lo = (int)(pk & 63u), hi = (int)((pk >> 6) & 63u);
          rm = (~0ull >> (63 - hi)) & (~0ull << lo);
        }
      }
      if (!ballot(rm != 0)) continue;
      uint64_t cm = transpose64(rm, lane);
      if (dbg) {
        n_visits += __popcll(cm);
        n_iters += wave_max(__popcll(cm));
      }
      while (cm) {
        const int q = __builtin_ctzll(cm);
        cm &= cm - 1;
        const T *v = L_v + (base + q) * RT_VS;
        T w0, w1, w2;
        if (!tri_weights<T>(v, x0, y0, a.eps, w0, w1, w2)) continue;
        const T z0 = w0 * v[6] + w1 * v[7] + w2 * v[8];
        if (z0 <= max_z0) continue;
        max_z0 = z0;
        win = (int)L_face[base + q];
        mw0 = w0;
        mw1 = w1;
        mw2 = w2;
      }
    }
    }
    if (dbg) c_walk += stamp_clk() - tq;
    __syncthreads();  // the list is rewritten by the next step
  };
  Pref PA, PB;
  issue(PA);
  while (more) {
    step(PA, PB);
    if (!more) break;
    step(PB, PA);
  }
  if (dbg && lane == 0) {
    uint64_t *d = dbg + ((size_t)blockIdx.x * R + wid) * 8;
    d[0] = t0;
    d[1] = stamp_clk();
    d[2] = w0s;
    d[3] = stamp_wall();
    d[4] = c_fill;
    d[5] = c_walk;
    d[6] = ((uint64_t)n_entries << 32) | (uint32_t)n_iters;
    d[7] = ((uint64_t)(pos / R - 1) << 32) | (uint32_t)tile;
  }
  if (dbg) {
    const int tv = n_visits;
    const int sv = wave_max(tv);  // max visits of a lane
    int sum = tv;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (lane == 0) dbg[(size_t)gridDim.x * R * 8 + ((size_t)blockIdx.x * R + wid) * 2] = (uint64_t)sum;
    if (lane == 0) dbg[(size_t)gridDim.x * R * 8 + ((size_t)blockIdx.x * R + wid) * 2 + 1] = (uint64_t)sv;
    if (lane == 0)
      for (int k = 0; k < 5; k++) dbg[(size_t)gridDim.x * R * 10 + ((size_t)blockIdx.x * R + wid) * 5 + k] = c_ph[k];
  }
  if (!px_valid || sub != 0) return;  // the row's keys are complete: every step ends in a barrier
  if constexpr (sizeof(T) == 4) {
    const unsigned long long key = s_key[r * 64 + lane];
    if ((s_nan[r] >> lane) & 1ull) {
      // a NaN depth breaks the total order: replay the reference's fold over every face
      for (int f = 0; f < a.F; f++) {
        const uint2 rr = rng[f];  // exact bbox test (and validity)
        if (i < (int)(rr.x & 0xffffu) || i > (int)(rr.x >> 16) || j < (int)(rr.y & 0xffffu) ||
            j > (int)(rr.y >> 16))
          continue;
        const T *v = rec + (size_t)f * RT_REC;
        T w0, w1, w2;
        if (!tri_weights<T>(v, x0, y0, a.eps, w0, w1, w2)) continue;
        const T z0 = w0 * v[6] + w1 * v[7] + w2 * v[8];
        if (z0 <= max_z0) continue;
        max_z0 = z0;
        win = f;
        mw0 = w0;
        mw1 = w1;
        mw2 = w2;
      }
    } else if (key != 0) {
      win = (int)(~(uint32_t)key);
      tri_weights<T>(rec + (size_t)win * RT_REC, x0, y0, a.eps, mw0, mw1, mw2);  // the arithmetic that ranked it
    }
  }
  const size_t p = ((size_t)b * H + j) * W + i;
  const int D = a.D;
  if (srow >= 0) {  // an uncovered pixel in this row: its soft item has work (px_valid lanes only here)
    const uint64_t unc = ballot(win < 0);
    if (unc && lane == __builtin_ctzll(unc)) a.soft_live[srow] = 1;
  }
  if (a.soft_hits) {
    a.soft_hits[p] = 0;
    a.soft_mask[p] = win >= 0 ? (T)1.0 : (T)0.0;
    if (lane == 0) {
      a.soft_seg[(size_t)(b * H + j) * g.tiles_x + tx] = 0;
      a.soft_defer[(size_t)(b * H + j) * g.tiles_x + tx] = 0;
    }
  }
  a.out_idx[p] = win;
  a.out_w[p * 3 + 0] = mw0;
  a.out_w[p * 3 + 1] = mw1;
  a.out_w[p * 3 + 2] = mw2;
  if (win >= 0) {
    const T *c = a.feat + (size_t)(f0 + win) * 3 * D;
    for (int d = 0; d < D; d++) a.out_feat[p * D + d] = mw0 * c[d] + mw1 * c[D + d] + mw2 * c[2 * D + d];
  } else {
    for (int d = 0; d < D; d++) a.out_feat[p * D + d] = (T)0;
  }
}

// workspace: bin bitmap | ghist (zeroed with the bitmap) | face records | pixel ranges |
// tile buckets | work items | item count  (records sized for sizeof(T) <= 8)
struct RastTileWs {
  size_t off_hist, off_rec, off_rng, off_bk, off_items, off_n, bytes;
  RastTileWs(const BinGeom &g, int B, int F, size_t tsize) {
    const size_t nt = (size_t)g.batch * g.tiles_y * g.tiles_x;
    off_hist = g.bytes();
    off_rec = (off_hist + ORD_HIST * sizeof(int) + 255) & ~(size_t)255;
    off_rng = off_rec + (((size_t)B * F * RT_REC * tsize + 255) & ~(size_t)255);
    off_bk = (off_rng + (size_t)B * F * sizeof(uint2) + 255) & ~(size_t)255;
    off_items = (off_bk + nt + 255) & ~(size_t)255;
    off_n = off_items + nt * TILE_H * sizeof(int32_t);
    bytes = off_n + sizeof(int);
  }
};
inline size_t rast_tile_ws_bytes(int B, int H, int W, int F) {
  return RastTileWs(make_bin_geom(B, H, W, F), B, F, sizeof(double)).bytes;
}

template <typename T>
static int launch_rast_tile(RastSrc<T> src, int H, int W, int B, int D, int F, const T *fvz, const T *feat, float m,
                            float eps, T *out_feat, int64_t *out_idx, T *out_w, void *ws, size_t ws_bytes,
                            hipStream_t st) {
  const BinGeom g = make_bin_geom(B, H, W, F);
  const RastTileWs L(g, B, F, sizeof(T));
  KL_REQUIRE(ws_bytes >= L.bytes, "rasterize forward: workspace too small");
  KL_REQUIRE(H < 65536 && W < 65536, "rasterize forward: height and width must be < 65536");
  const size_t P = (size_t)B * H * W;
  if (P == 0) return KL_OK;
  if (F == 0) {  // no faces: face_idx -1, zero weights and features (the kernels need F > 0)
    KL_CHECK_RC(fill_async(out_idx, 0xff, P * sizeof(int64_t), st));
    KL_CHECK_RC(fill_async(out_w, 0, P * 3 * sizeof(T), st));
    return fill_async(out_feat, 0, P * D * sizeof(T), st);
  }
  char *w = reinterpret_cast<char *>(ws);
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(w);
  int *ghist = reinterpret_cast<int *>(w + L.off_hist);
  T *rec = reinterpret_cast<T *>(w + L.off_rec);
  uint2 *rng = reinterpret_cast<uint2 *>(w + L.off_rng);
  uint8_t *bk = reinterpret_cast<uint8_t *>(w + L.off_bk);
  int32_t *items = reinterpret_cast<int32_t *>(w + L.off_items);
  int *nitems = reinterpret_cast<int *>(w + L.off_n);
  const PixPitch pp{m / (float)W, m / (float)H, (float)W / m, (float)H / m};
  if (bin_word_lds_ok(g) && !(g_dev_flags & (1 << 14))) {  // dev bit 14: the atomic binning
    KL_CHECK_RC(launch_bin_word<T>(src, fvz, F, g, pp, bitmap, rec, rng, nullptr, nullptr, (T)0, ghist, ORD_HIST,
                                   st));
  } else {
  KL_CHECK_RC(fill_async(bitmap, 0, L.off_hist + ORD_HIST * sizeof(int), st));
  const dim3 bgrid((unsigned)cdiv((int64_t)g.chunks * 64, 256), (unsigned)B);
  if (src.vmask)
    hipLaunchKernelGGL((raster_bin_kernel<T, 1>), bgrid, dim3(256), 0, st, src, fvz, F, g, pp, bitmap, rec, rng);
  else if (src.nz)
    hipLaunchKernelGGL((raster_bin_kernel<T, 2>), bgrid, dim3(256), 0, st, src, fvz, F, g, pp, bitmap, rec, rng);
  else
    hipLaunchKernelGGL((raster_bin_kernel<T, 0>), bgrid, dim3(256), 0, st, src, fvz, F, g, pp, bitmap, rec, rng);
  KL_CHECK_LAUNCH();
  }
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  // heaviest tiles first; tiles with >= 2^split_from - 1 candidate chunks are split into
  // 2^split_log2 row parts (f32 only: the f64 walk is one wave per row).  Dev flag bits
  // 16-20 / 21-22 override the two (ablation); bit 12 = grid order, no split.
  int split_from = 5, split_log2 = 2;
  if ((g_dev_flags >> 16) & 31) split_from = (g_dev_flags >> 16) & 31;
  if ((g_dev_flags >> 21) & 3) split_log2 = (g_dev_flags >> 21) & 3;
  if (sizeof(T) != 4) split_log2 = 0;
  const int identity = (g_dev_flags >> 12) & 1;
  if (!identity) {
    hipLaunchKernelGGL(tile_bucket_kernel, dim3((unsigned)cdiv(nt, 4)), dim3(256), 0, st, (const uint32_t *)bitmap,
                       g.words, nt, bk, ghist, nullptr);
    KL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, st, (const uint8_t *)bk, (const int *)ghist, nt, items,
                     identity, split_from, split_log2, nitems);
  KL_CHECK_LAUNCH();
  RastTileArgs<T> args{src, fvz, feat, bitmap, rec, rng, items, nitems, g, F, D, eps, out_feat, out_idx, out_w,
                       reinterpret_cast<uint64_t *>(g_dev_debug)};
  hipLaunchKernelGGL((raster_tile_kernel<T>), dim3((unsigned)(nt << split_log2)), dim3(512), 0, st, args);
  KL_CHECK_LAUNCH();
  return KL_OK;
}


// The single rounding of a gradient summed in double (common.h).
template <typename T>
__global__ void __launch_bounds__(256) acc_finalize_kernel(const double *__restrict__ acc, T *__restrict__ out,
                                                           size_t n, int accumulate, int *__restrict__ reset) {
  if (reset && blockIdx.x == 0 && threadIdx.x == 0) *reset = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = accumulate ? out[i] + (T)acc[i] : (T)acc[i];
}
template <typename T>
int acc_finalize(const double *acc, T *out, size_t n, bool accumulate, hipStream_t st, int *reset) {
  if (n == 0) return reset ? fill_async(reset, 0, sizeof(int), st) : KL_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv((int64_t)n, 256), 8192);
  hipLaunchKernelGGL((acc_finalize_kernel<T>), dim3(blocks), dim3(256), 0, st, acc, out, n, accumulate ? 1 : 0,
                     reset);
  KL_CHECK_LAUNCH();
  return KL_OK;
}
template int acc_finalize<float>(const double *, float *, size_t, bool, hipStream_t, int *);
template int acc_finalize<double>(const double *, double *, size_t, bool, hipStream_t, int *);

// The _C contract's scatter backward (rasterize_backward_cuda takes no multiplier, so the
// faces' pixel ranges are unknown): one thread per pixel, the reference's terms added with
// global atomics into double accumulators, rounded once (acc_finalize) -- the order of the
// atomics does not change the result (the float terms sum exactly in double).
template <typename T>
__global__ void __launch_bounds__(256) rasterize_bwd_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, int B, int H, int W, int F, int D, float eps,
    double *__restrict__ grad_fvi, double *__restrict__ grad_ffeat) {
  const int64_t npix = (int64_t)H * W;
  for (int64_t tp = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; tp < (int64_t)B * npix;
       tp += (int64_t)gridDim.x * blockDim.x) {
    const int64_t fidx = face_idx[tp];
    if (fidx < 0) continue;
    const int b = (int)(tp / npix);
    const int64_t tf = (int64_t)b * F + fidx;
    const T *g = grad_feat + tp * D;
    const T w_a = wts[tp * 3 + 0], w_b = wts[tp * 3 + 1], w_c = wts[tp * 3 + 2];
    for (int d = 0; d < D; d++) {
      const T gd = g[d];
      atomicAdd(grad_ffeat + tf * 3 * D + d, (double)(gd * w_a));
      atomicAdd(grad_ffeat + tf * 3 * D + D + d, (double)(gd * w_b));
      atomicAdd(grad_ffeat + tf * 3 * D + 2 * D + d, (double)(gd * w_c));
    }
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
    BaryGrad<T> bg;
    bg.init(v, w_a, w_b, w_c, eps);
    const T *c = feat + tf * 3 * D;
    double *gv = grad_fvi + tf * 6;
    for (int d = 0; d < D; d++) {
      T o[6];
      bg.terms(g[d], c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
      for (int q = 0; q < 6; q++) atomicAdd(gv + q, (double)o[q]);
    }
  }
}

// ---------------------------------------------------------------- gather backward
// One thread per face visits exactly the pixel range the forward visited for it (the
// same in-kernel bbox and exact_axis), so every pixel the face can have won is seen;
// pixels are taken GATHER_BATCH at a time with their face_idx / weights / grads loads in
// flight together.  Faces whose range exceeds VIS_SMALL_AREA go to a workgroup per face.
// GATHER_BATCH (gather2, r04aw A/B of builds, dibr_backward at cfg3): 1: 74.4, 2: 72.0, 3: 71.1,
// 4: 75.0, 6: 76.5, 8: 77.5 us -- fewer registers per batch slot (93 VGPRs at 2 against 102 at 4)
// buys occupancy that hides more than the deeper batch does.
#ifndef KL_GATHER_BATCH  // A/B builds only
#define KL_GATHER_BATCH 3
#endif
constexpr int GATHER_BATCH = KL_GATHER_BATCH;

template <typename T>
__device__ __forceinline__ bool face_range(const RastSrc<T> &src, int64_t tf, float m, int H, int W, int &ix0,
                                           int &ix1, int &iy0, int &iy1) {
  T x0, y0, x1, y1;
  src.get(tf, x0, y0, x1, y1);
  exact_axis(x0, x1, m, W, false, ix0, ix1);
  exact_axis(y0, y1, m, H, true, iy0, iy1);
  return ix0 <= ix1 && iy0 <= iy1;
}

// The forward's exact pixel ranges of a face (kl_dibr_forward's face_ranges), empty = invalid.
__device__ __forceinline__ bool rng_range(const uint2 *rng, int64_t tf, int &ix0, int &ix1, int &iy0, int &iy1) {
  const uint2 r = rng[tf];
  ix0 = (int)(r.x & 0xffffu);
  ix1 = (int)(r.x >> 16);
  iy0 = (int)(r.y & 0xffffu);
  iy1 = (int)(r.y >> 16);
  return ix0 <= ix1 && iy0 <= iy1;
}

// Per-face sums of the reference's float terms, in double: they are exact whenever the terms'
// magnitudes span less than ~2^29, so the rounded result does not depend on the order of the
// adds (lanes, butterfly) -- it equals the oracle's, which sums the same terms in pixel order.
template <typename T, int MAXD>
struct GatherAcc {
  double gi[6];
  double gf[3 * MAXD];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int q = 0; q < 6; q++) gi[q] = 0.0;
#pragma unroll
    for (int q = 0; q < 3 * MAXD; q++) gf[q] = 0.0;
  }
  // one pixel won by the face: the reference's per-pixel terms (rasterization_cuda.cu:262-399)
  __device__ __forceinline__ void add(const T v[6], const T *c, int D, T w_a, T w_b, T w_c, const T *g, float eps) {
    BaryGrad<T> bg;
    bg.init(v, w_a, w_b, w_c, eps);
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < D) {
        const T gd = g[d];
        gf[d] += (double)(gd * w_a);
        gf[MAXD + d] += (double)(gd * w_b);
        gf[2 * MAXD + d] += (double)(gd * w_c);
        T o[6];
        bg.terms(gd, c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
        for (int q = 0; q < 6; q++) gi[q] += (double)o[q];
      }
    }
  }
};

template <typename T, int MAXD, int LPF_ = LPF>
__device__ __forceinline__ void gather_one(
    int64_t t, const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, const uint8_t *__restrict__ valid,
    const T *__restrict__ nz, int B, int H, int W, int F, int D, float m, float eps, T *__restrict__ grad_fvi,
    T *__restrict__ grad_ffeat, int *__restrict__ big, int *__restrict__ nbig, const uint2 *__restrict__ rng,
    const double *__restrict__ soft) {
  const int64_t tf = t / LPF_;  // LPF_ consecutive lanes per face (whole groups per wave)
  const int s = (int)(t % LPF_);
  const bool in = tf < (int64_t)B * F;
  const int b = in ? (int)(tf / F) : 0;
  const int64_t f = tf - (int64_t)b * F;
  const RastSrc<T> src{fvi, valid, (T)m, nz};
  // the soft mask's sum of coordinate s (written by lane s below), loaded now so that its
  // latency hides behind the walk: an unconditional load from a clamped index
  double sv = 0.0;
  if (soft) sv = soft[(in ? tf : 0) * DS_ACC_STRIDE + (s < 6 ? s : 5)];
  GatherAcc<T, MAXD> acc;
  acc.zero();
  int ix0, ix1, iy0, iy1;
  bool queued = false;
  const bool has = in && (rng ? rng_range(rng, tf, ix0, ix1, iy0, iy1)
                              : (src.valid(tf) && face_range(src, tf, m, H, W, ix0, ix1, iy0, iy1)));
  if (!__any(has)) {
    // no face of the wave covers a pixel (culled / off-screen runs of the mesh): zero gradients
    // (+ the soft sums), no walk and no butterfly
    if (!in) return;
#pragma unroll
    for (int q = 0; q < 6 + 3 * MAXD; q++) {
      if (q % LPF_ != s) continue;
      if (q < 6) {
        grad_fvi[tf * 6 + q] = soft ? (T)0 + (T)sv : (T)0;
      } else {
        const int r = q - 6, ii = r / MAXD, d = r % MAXD;
        if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = (T)0;
      }
    }
    return;
  }
  if (has) {
    if ((int64_t)(ix1 - ix0 + 1) * (iy1 - iy0 + 1) > VIS_SMALL_AREA) {
      queued = true;
      if (s == 0) big[atomicAdd(nbig, 1)] = (int)tf;
    } else {
      T v[6];
#pragma unroll
      for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
      const T *c = feat + tf * 3 * D;
      const int64_t pbase = (int64_t)b * H * W;
      RangeWalkN<LPF_> rw(ix0, ix1, iy0, iy1, s);
      while (rw.more()) {
        // face_idx of GATHER_BATCH pixels in flight together; the (rare) hits then load
        // their weights / grads one by one
        int64_t px[GATHER_BATCH];
        uint32_t hits = 0;
#pragma unroll
        for (int u = 0; u < GATHER_BATCH; u++) {
          px[u] = pbase + (int64_t)(iy0 + rw.row) * W + ix0 + rw.col;
          if (rw.more() && face_idx[px[u]] == f) hits |= 1u << u;
          rw.next();
        }
#pragma unroll 1
        for (; hits; hits &= hits - 1) {
          const int u = __builtin_ctz(hits);
          int64_t p = px[0];
#pragma unroll
          for (int q = 1; q < GATHER_BATCH; q++)
            if (u == q) p = px[q];
          acc.add(v, c, D, wts[p * 3 + 0], wts[p * 3 + 1], wts[p * 3 + 2], grad_feat + p * D, eps);
        }
      }
    }
  }
  // fixed-order butterfly over the face's lane group: every lane ends with the total
#pragma unroll
  for (int o = 1; o < LPF_; o <<= 1) {
#pragma unroll
    for (int q = 0; q < 6; q++) acc.gi[q] += __shfl_xor(acc.gi[q], o);
#pragma unroll
    for (int q = 0; q < 3 * MAXD; q++) acc.gf[q] += __shfl_xor(acc.gf[q], o);
  }
  if (!in || queued) return;  // queued faces are written by the workgroup kernel
  // lane s writes the values q = s, s+LPF_, ...
#pragma unroll
  for (int q = 0; q < 6 + 3 * MAXD; q++) {
    if (q % LPF_ != s) continue;
    if (q < 6) {  // (q == s) + the soft mask's sum, rounded on its own: autograd's add of the two
      grad_fvi[tf * 6 + q] = soft ? (T)acc.gi[q] + (T)sv : (T)acc.gi[q];
    } else {
      const int r = q - 6, ii = r / MAXD, d = r % MAXD;
      if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = (T)acc.gf[r];
    }
  }
}

// One thread per (face, lane) of the LPF-lane groups.  (A persistent grid-stride version, sized
// to the resident waves, measured 82 us against 62 at cfg3: the waves are not dispatch-bound.)
template <typename T, int MAXD, int LPF_ = LPF>
__global__ void __launch_bounds__(256) rasterize_bwd_gather_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, const uint8_t *__restrict__ valid,
    const T *__restrict__ nz, int B, int H, int W, int F, int D, float m, float eps, T *__restrict__ grad_fvi,
    T *__restrict__ grad_ffeat, int *__restrict__ big, int *__restrict__ nbig, const uint2 *__restrict__ rng,
    const double *__restrict__ soft) {
  gather_one<T, MAXD, LPF_>(blockIdx.x * (int64_t)blockDim.x + threadIdx.x, grad_feat, face_idx, wts, fvi, feat,
                            valid, nz, B, H, W, F, D, m, eps, grad_fvi, grad_ffeat, big, nbig, rng, soft);
}

// one 256-thread workgroup per large face; the per-thread partials reduced per wave (butterfly)
// and across the four waves
template <typename T, int MAXD>
__global__ void __launch_bounds__(256) rasterize_bwd_bigface_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, const uint8_t *__restrict__ valid,
    const T *__restrict__ nz, int H, int W, int F, int D, float m, float eps, T *__restrict__ grad_fvi,
    T *__restrict__ grad_ffeat, const int *__restrict__ big, const int *__restrict__ nbig,
    const uint2 *__restrict__ rng, const double *__restrict__ soft) {
  __shared__ double red[4 * (6 + 3 * MAXD)];
  const int n = *nbig;
  const RastSrc<T> src{fvi, valid, (T)m, nz};
  for (int k = blockIdx.x; k < n; k += gridDim.x) {
    const int64_t tf = big[k];
    const int b = (int)(tf / F);
    const int64_t f = tf - (int64_t)b * F;
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
    int ix0, ix1, iy0, iy1;
    if (rng)
      rng_range(rng, tf, ix0, ix1, iy0, iy1);
    else
      face_range(src, tf, m, H, W, ix0, ix1, iy0, iy1);
    const int w = ix1 - ix0 + 1;
    const int64_t area = (int64_t)w * (iy1 - iy0 + 1);
    GatherAcc<T, MAXD> acc;
    acc.zero();
    const T *c = feat + tf * 3 * D;
    for (int64_t e = threadIdx.x; e < area; e += blockDim.x) {
      const int j = iy0 + (int)(e / w), i = ix0 + (int)(e % w);
      const int64_t p = ((int64_t)b * H + j) * W + i;
      if (face_idx[p] != f) continue;
      acc.add(v, c, D, wts[p * 3 + 0], wts[p * 3 + 1], wts[p * 3 + 2], grad_feat + p * D, eps);
    }
    // per wave a butterfly of every value, then the four waves' sums added by thread q
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 6 + 3 * MAXD; q++) {
      double x = q < 6 ? acc.gi[q] : acc.gf[q - 6];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
      if (lane == 0) red[wv * (6 + 3 * MAXD) + q] = x;
    }
    __syncthreads();
    const int q = threadIdx.x;
    if (q < 6 + 3 * MAXD) {
      const double x = red[q] + red[(6 + 3 * MAXD) + q] + red[2 * (6 + 3 * MAXD) + q] + red[3 * (6 + 3 * MAXD) + q];
      if (q < 6) {
        grad_fvi[tf * 6 + q] = soft ? (T)x + (T)soft[tf * DS_ACC_STRIDE + q] : (T)x;
      } else {
        const int r = q - 6, ii = r / MAXD, d = r % MAXD;
        if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = (T)x;
      }
    }
    __syncthreads();  // red is rewritten for the next face
  }
}

// (The chip order kernel's count workgroups meet at a grid barrier: chip_order_resident, tileorder.h,
// checks they can all be resident; when not, kl_dibr_forward takes the two-workgroup order kernel.)

// ---------------------------------------------------------------- gather backward, v2
// The per-face gather reorganised around what bounds it (r03 counters: ~600 VALU per wave of 8
// faces, a third of it the 15-double butterfly; 126 VGPRs of double accumulators; each won pixel's
// weights and grads loaded one after another, a memory round trip each):
//  * 8 lanes per face as before (a wave = 8 faces; a wave whose faces cover no pixel writes their
//    zero gradients and exits after one load);
//  * a batch of 4 pixels per lane loads face_idx, weights and grads together (unconditional
//    loads; a pixel's data is used only if the face won it): one memory round trip per batch
//    instead of one for face_idx and one per won pixel;
//  * every lane adds the reference's per-pixel float terms in double into its OWN LDS partials
//    (value-major, so a wave's adds touch 64 consecutive doubles: no bank or address conflict);
//    then each value's 8 partials are added in lane order and rounded once.  No accumulators in
//    registers, no butterfly; the sum is the same on every run and equals the oracle's pixel-order
//    sum whenever the float terms sum exactly in double (magnitudes within ~2^29, see GatherAcc).
//    Measured dead ends (r04, cfg3, gather alone): one wave per 64 consecutive faces taking its
//    active faces 8 at a time, 120-135 us against 57 -- waves over runs of front faces did 8
//    rounds one after another and set the kernel's end; adding into one LDS slot per face
//    (ds_add_f64 from the face's 8 lanes) serialised the lanes on each address.
//  * faces covering more than VIS_SMALL_AREA pixel centres are summed by the first G2_BIG_BLOCKS
//    workgroups of the same grid (a scan of the ranges, then the whole workgroup per face), so
//    no second launch is needed when there are none.
constexpr int G2_BIG_BLOCKS = 64;
// Row stride of a wave's partials (doubles).  The final sums read value q = s, s + 8 of a face's
// 8 lanes; at a stride of 64 doubles (128 dwords, 0 mod the 64 banks) those reads share a bank
// pair.  r05as A/B (KL_G2_PAD=1: stride 65): LDS bank-conflict share 0.19 -> 0.15 but the kernel
// 49.6 against 48.6 us, cfg3 eager 5,590-5,783 against 5,739-5,763 Mpixels/s -- kept at 64.
#ifndef KL_G2_PAD  // A/B builds only
#define KL_G2_PAD 0
#endif
constexpr int G2_PS = 64 + KL_G2_PAD;

template <typename T, int MAXD, bool ATOM = false>
__device__ __forceinline__ void g2_add(double *__restrict__ part, const T v[6], const T *__restrict__ c, int D, T wa,
                                       T wb, T wc, const T *gv, float eps) {
  // ATOM: ds_add_f64 into the lane's own partials -- 100 VGPRs at D = 3; a read-modify-write lets
  // the compiler keep the partials in registers across the batch (173 VGPRs, 73 against 48 us)
  if constexpr (ATOM) {
    BaryGrad<T> bg;
    bg.init(v, wa, wb, wc, eps);
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < D) {
        const T gd = gv[d];
        atomicAdd(&part[(6 + d) * G2_PS], (double)(gd * wa));
        atomicAdd(&part[(6 + MAXD + d) * G2_PS], (double)(gd * wb));
        atomicAdd(&part[(6 + 2 * MAXD + d) * G2_PS], (double)(gd * wc));
        T o[6];
        bg.terms(gd, c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
        for (int q = 0; q < 6; q++) atomicAdd(&part[q * G2_PS], (double)o[q]);
      }
    }
    return;
  }
  // part: this thread's partials, value q at part[q * G2_PS] (LDS no other thread touches until the sums)
  BaryGrad<T> bg;
  bg.init(v, wa, wb, wc, eps);
#pragma unroll
  for (int d = 0; d < MAXD; d++) {
    if (d < D) {
      const T gd = gv[d];
      part[(6 + d) * G2_PS] += (double)(gd * wa);
      part[(6 + MAXD + d) * G2_PS] += (double)(gd * wb);
      part[(6 + 2 * MAXD + d) * G2_PS] += (double)(gd * wc);
      T o[6];
      bg.terms(gd, c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
      for (int q = 0; q < 6; q++) part[q * G2_PS] += (double)o[q];
    }
  }
}

// value q of a face -> its gradient (q < 6: the vertex-coordinate gradient, + the soft mask's sum
// rounded on its own, sv; else a feature gradient)
// The soft sums live in kl_dibr_backward's zero-kept accumulator: only faces the soft backward
// flagged are read, and their sums are zeroed and their flags cleared as they are read, so the
// accumulator is zero again after every backward (a retained second backward adds into zeros).
// An unflagged face's soft sum is 0: (T)x + 0.0f is (T)x, since (T)x is never -0.0 (x is +0.0 or a
// nonzero sum of float terms, a multiple of 2^-149 of magnitude >= 2^-149).
__device__ __forceinline__ double take_soft(double *__restrict__ soft, int64_t i) {
  const double v = soft[i];
  if (__double_as_longlong(v) != 0) soft[i] = 0.0;
  return v;
}

template <typename T, int MAXD>
__device__ __forceinline__ void g2_store(int64_t tf, int q, double x, int D, double sv, T *__restrict__ grad_fvi,
                                         T *__restrict__ grad_ffeat) {
  if (q < 6) {
    grad_fvi[tf * 6 + q] = (T)x + (T)sv;
  } else {
    const int r = q - 6, ii = r / MAXD, d = r % MAXD;
    if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = (T)x;
  }
}

template <typename T, int MAXD, bool ATOM = false>
__global__ void __launch_bounds__(256) rasterize_bwd_gather2_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, const uint8_t *__restrict__ valid,
    const T *__restrict__ nz, int B, int H, int W, int F, int D, float m, float eps, T *__restrict__ grad_fvi,
    T *__restrict__ grad_ffeat, const uint2 *__restrict__ rng, double *__restrict__ soft,
    uint8_t *__restrict__ sflag, int nbig, int opts) {
  // dev (param 17) opts bit 1: no soft / flag re-zeroing, bit 2: soft read unflagged (timing only)
  const bool rz = !(opts & 2), nofl = opts & 4;
  constexpr int NV = 6 + 3 * MAXD;
  __shared__ double s_part[4][NV][G2_PS];  // per wave: per lane (thread) partial sums, value-major
  __shared__ int s_nbig;
  __shared__ int s_big[256];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nf = (int64_t)B * F;
  const RastSrc<T> src{fvi, valid, (T)m, nz};
  auto range_of = [&](int64_t tf, int &ix0, int &ix1, int &iy0, int &iy1) -> bool {
    return rng ? rng_range(rng, tf, ix0, ix1, iy0, iy1)
               : (src.valid(tf) && face_range(src, tf, m, H, W, ix0, ix1, iy0, iy1));
  };
  double *part = &s_part[wid][0][lane];
  if ((int)blockIdx.x < nbig) {
    // ---- large faces: scan a slice of the faces, then one face at a time with the workgroup;
    //      its 256 partials added in thread order
#pragma unroll
    for (int q = 0; q < NV; q++) part[q * G2_PS] = 0.0;
    const int64_t per = (nf + nbig - 1) / nbig;
    const int64_t f0 = (int64_t)blockIdx.x * per, f1 = f0 + per < nf ? f0 + per : nf;
    for (int64_t base = f0; base < f1; base += 256) {
      if (threadIdx.x == 0) s_nbig = 0;
      __syncthreads();
      {
        const int64_t tf = base + threadIdx.x;
        int ix0, ix1, iy0, iy1;
        if (tf < f1 && range_of(tf, ix0, ix1, iy0, iy1) &&
            (int64_t)(ix1 - ix0 + 1) * (iy1 - iy0 + 1) > VIS_SMALL_AREA)
          s_big[atomicAdd(&s_nbig, 1)] = (int)threadIdx.x;
      }
      __syncthreads();
      const int n = s_nbig;
      for (int k = 0; k < n; k++) {
        const int64_t bf = base + s_big[k];
        const int b = (int)(bf / F);
        const int64_t f = bf - (int64_t)b * F;
        int ix0, ix1, iy0, iy1;
        range_of(bf, ix0, ix1, iy0, iy1);
        T v[6];
#pragma unroll
        for (int q = 0; q < 6; q++) v[q] = fvi[bf * 6 + q];
        const T *c = feat + bf * 3 * D;
        const int w = ix1 - ix0 + 1;
        const int64_t area = (int64_t)w * (iy1 - iy0 + 1);
        for (int64_t e = threadIdx.x; e < area; e += blockDim.x) {
          const int64_t p = ((int64_t)b * H + iy0 + (int)(e / w)) * W + ix0 + (int)(e % w);
          if (face_idx[p] != f) continue;
          T gv[MAXD];
#pragma unroll
          for (int d = 0; d < MAXD; d++) gv[d] = d < D ? grad_feat[p * D + d] : (T)0;
          g2_add<T, MAXD>(part, v, c, D, wts[p * 3 + 0], wts[p * 3 + 1], wts[p * 3 + 2], gv, eps);
        }
        __syncthreads();
        if ((int)threadIdx.x < NV) {
          const int q = threadIdx.x;
          const bool fl = soft && q < 6 && (nofl || sflag[bf]);
          double x = 0.0;
          for (int t = 0; t < 256; t++) x += s_part[t >> 6][q][t & 63];
          g2_store<T, MAXD>(bf, q, x, D, fl ? (rz ? take_soft(soft, bf * DS_ACC_STRIDE + q) : soft[bf * DS_ACC_STRIDE + q]) : 0.0,
                            grad_fvi, grad_ffeat);
          if (rz && fl && q == 0) sflag[bf] = 0;  // after the flag's use: every lane of the wave has read it
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NV; q++) part[q * G2_PS] = 0.0;
      }
      __syncthreads();  // s_nbig / s_big are rewritten
    }
    return;
  }
  // ---- 8 lanes per face, a wave = 8 faces
  const int s = lane & 7;
  const int64_t tf = (((int64_t)(blockIdx.x - nbig) * 256 + threadIdx.x) >> 3);
  const bool in = tf < nf;
  int ix0 = 1, ix1 = 0, iy0 = 1, iy1 = 0;
  const bool has = in && range_of(tf, ix0, ix1, iy0, iy1);
  const bool act = has && (int64_t)(ix1 - ix0 + 1) * (iy1 - iy0 + 1) <= VIS_SMALL_AREA;
  // the face's soft-sum flag (all 8 lanes read the same byte)
  const bool fl = soft && in && (nofl || sflag[tf]);
  if (in && !has) {  // no pixel: zero gradients (+ the soft mask's sums); lane s writes q = s, s + 8, ...
#pragma unroll
    for (int q = s; q < NV; q += 8) {
      if (q < 6) {
        grad_fvi[tf * 6 + q] = fl ? (T)0 + (T)(rz ? take_soft(soft, tf * DS_ACC_STRIDE + q) : soft[tf * DS_ACC_STRIDE + q]) : (T)0;
      } else {
        const int r = q - 6, ii = r / MAXD, d = r % MAXD;
        if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = (T)0;
      }
    }
    if (rz && fl && s == 0) sflag[tf] = 0;  // after the flag's use
  }
  if (!__any(act)) return;  // wave-uniform
#pragma unroll
  for (int q = 0; q < NV; q++) part[q * G2_PS] = 0.0;
  // lane s < 6's soft-mask sum, loaded now so that its latency hides behind the walk
  double soft_v = 0.0;
  if (act && fl && s < 6) soft_v = soft[tf * DS_ACC_STRIDE + s];
  if (act) {
    const int b = (int)(tf / F);
    const int64_t f = tf - (int64_t)b * F;
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
    const T *c = feat + tf * 3 * D;
    const int64_t pbase = (int64_t)b * H * W;
    const int64_t pfirst = pbase + (int64_t)iy0 * W + ix0;
    RangeWalkN<8> rw(ix0, ix1, iy0, iy1, s);
    while (rw.more()) {
      // face_idx, weights and grads of GATHER_BATCH pixels in flight together (the range's first
      // pixel stands in past the range's end)
      int64_t fi[GATHER_BATCH];
      T wv[GATHER_BATCH][3], gv[GATHER_BATCH][MAXD];
      uint32_t inb = 0;
#pragma unroll
      for (int u = 0; u < GATHER_BATCH; u++) {
        int64_t p = pfirst;
        if (rw.more()) {
          p = pbase + (int64_t)(iy0 + rw.row) * W + ix0 + rw.col;
          inb |= 1u << u;
        }
        rw.next();
        fi[u] = face_idx[p];
#pragma unroll
        for (int k = 0; k < 3; k++) wv[u][k] = wts[p * 3 + k];
#pragma unroll
        for (int d = 0; d < MAXD; d++) gv[u][d] = d < D ? grad_feat[p * D + d] : (T)0;
      }
      uint32_t hm = 0;
#pragma unroll
      for (int u = 0; u < GATHER_BATCH; u++)
        if (((inb >> u) & 1u) && fi[u] == f) hm |= 1u << u;
      // the lane's won pixels one per iteration (the wave runs max-over-lanes iterations, not one
      // per batch slot): each iteration selects its pixel's values from the batch registers
      while (__any(hm != 0)) {
        if (hm) {
          const int u = __builtin_ctz(hm);
          hm &= hm - 1;
          T a0 = wv[0][0], a1 = wv[0][1], a2 = wv[0][2], g[MAXD];
#pragma unroll
          for (int d = 0; d < MAXD; d++) g[d] = gv[0][d];
#pragma unroll
          for (int k = 1; k < GATHER_BATCH; k++) {
            if (u == k) {
              a0 = wv[k][0];
              a1 = wv[k][1];
              a2 = wv[k][2];
#pragma unroll
              for (int d = 0; d < MAXD; d++) g[d] = gv[k][d];
            }
          }
          g2_add<T, MAXD, ATOM>(part, v, c, D, a0, a1, a2, g, eps);
        }
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (act) {
    // value q of the face: its 8 lanes' partials in lane order
    const int g0 = lane & ~7;
    for (int q = s; q < NV; q += 8) {
      double x = 0.0;
#pragma unroll
      for (int l = 0; l < 8; l++) x += s_part[wid][q][g0 + l];
      if (q < 6) {  // q == s: the prefetched sum, re-zeroed as take_soft does
        grad_fvi[tf * 6 + q] = (T)x + (T)soft_v;
        if (rz && __double_as_longlong(soft_v) != 0) soft[tf * DS_ACC_STRIDE + q] = 0.0;
      } else {
        g2_store<T, MAXD>(tf, q, x, D, 0.0, grad_fvi, grad_ffeat);
      }
    }
    if (rz && fl && s == 0) sflag[tf] = 0;  // after the flag's use
  }
}

// workspace of the scatter backward: the double accumulators of both gradients
static size_t rast_scatter_ws_bytes(int B, int F, int D) {
  return al256((size_t)B * F * 6 * sizeof(double)) + al256((size_t)B * F * 3 * D * sizeof(double));
}

template <typename T>
static int rasterize_bwd(int B, int H, int W, int F, int D, const void *grad, const int64_t *face_idx,
                         const void *w, const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                         void *ws, size_t ws_bytes, hipStream_t st) {
  const size_t ni = (size_t)B * F * 6, nf = (size_t)B * F * 3 * D;
  const int64_t total = (int64_t)B * H * W;
  if (total == 0 || ni == 0) {
    KL_CHECK_RC(fill_async(gfvi, 0, sizeof(T) * ni, st));
    return fill_async(gfeat, 0, sizeof(T) * nf, st);
  }
  KL_REQUIRE(ws && ws_bytes >= rast_scatter_ws_bytes(B, F, D), "rasterize_backward: workspace too small");
  double *ai = reinterpret_cast<double *>(ws);
  double *af = reinterpret_cast<double *>(reinterpret_cast<char *>(ws) + al256(ni * sizeof(double)));
  KL_CHECK_RC(fill_async(ws, 0, rast_scatter_ws_bytes(B, F, D), st));
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(total, 256), 65536);
  hipLaunchKernelGGL(rasterize_bwd_kernel<T>, dim3(blocks), dim3(256), 0, st, (const T *)grad, face_idx,
                     (const T *)w, (const T *)fvi, (const T *)feat, B, H, W, F, D, eps, ai, af);
  KL_CHECK_LAUNCH();
  KL_CHECK_RC(acc_finalize<T>(ai, (T *)gfvi, ni, false, st));
  return acc_finalize<T>(af, (T *)gfeat, nf, false, st);
}

// gather2 dev ablations (param 17; bits 1, 2: timing only, they break the zero-kept accumulator)
static int gather_opts() { return (g_dev_param[17] & 3) << 1; }

// nbig: a zeroed int (zero_nbig: this call zeroes it first).
template <typename T, int MAXD>
static int rasterize_bwd_gather_maxd(int B, int H, int W, int F, int D, const T *grad, const int64_t *face_idx,
                                     const T *w, const T *fvi, const T *feat, const uint8_t *valid, const T *nz,
                                     float m, float eps, T *gfvi, T *gfeat, int *big, int *nbig, bool zero_nbig,
                                     const uint2 *rng, double *soft, uint8_t *sflag, hipStream_t st) {
  const int64_t nf = (int64_t)B * F;
  if (g_dev_param[7] != 1 || soft) {  // (the r03 gather does not read flagged soft sums)  // dev param 7 = 1: the r03 gather (8 lanes per face, register sums) for A/B
    const int nb = (int)std::min<int64_t>(G2_BIG_BLOCKS, cdiv(nf, 4096));
#if KL_DEV
    if (g_dev_param[8] == 1)  // dev param 8 = 1: read-modify-write partials (A/B: 73 against 48 us at cfg3)
      hipLaunchKernelGGL((rasterize_bwd_gather2_kernel<T, MAXD>), dim3((unsigned)(nb + cdiv(nf * 8, 256))), dim3(256),
                         0, st, grad, face_idx, w, fvi, feat, valid, nz, B, H, W, F, D, m, eps, gfvi, gfeat, rng, soft,
                         sflag, nb, gather_opts());
    else
#endif
      hipLaunchKernelGGL((rasterize_bwd_gather2_kernel<T, MAXD, true>), dim3((unsigned)(nb + cdiv(nf * 8, 256))),
                         dim3(256), 0, st, grad, face_idx, w, fvi, feat, valid, nz, B, H, W, F, D, m, eps, gfvi, gfeat,
                         rng, soft, sflag, nb, gather_opts());
    KL_CHECK_LAUNCH();
    return KL_OK;
  }
#if KL_DEV  // the r03 gather (dev param 7 = 1): a measured dead end, DESIGN.md 3.3
  if (zero_nbig) KL_CHECK_RC(fill_async(nbig, 0, sizeof(int), st));
  // 8 lanes per face (measured: 4 lanes 62.7 us, 8 lanes 58 us, 16 lanes 91 us at cfg3)
  hipLaunchKernelGGL((rasterize_bwd_gather_kernel<T, MAXD>), dim3((unsigned)cdiv(nf * LPF, 256)), dim3(256), 0, st,
                     grad, face_idx, w, fvi, feat, valid, nz, B, H, W, F, D, m, eps, gfvi, gfeat, big, nbig, rng, soft);
  KL_CHECK_LAUNCH();
  // large faces: a workgroup each, grid-stride over the list (dev param 6 overrides the grid)
  const unsigned bgrid = g_dev_param[6] > 0 ? (unsigned)g_dev_param[6] : 256u;
  hipLaunchKernelGGL((rasterize_bwd_bigface_kernel<T, MAXD>), dim3(bgrid), dim3(256), 0, st, grad, face_idx, w, fvi,
                     feat, valid, nz, H, W, F, D, m, eps, gfvi, gfeat, big, nbig, rng, soft);
  KL_CHECK_LAUNCH();
  return KL_OK;
#else
  (void)big;
  (void)nbig;
  (void)zero_nbig;
  return KL_OK;
#endif
}

// The gather backward writes every face's gradient (zeros where nothing was won).
// nbig == nullptr: the big-face counter lives at the head of the workspace and is zeroed here.
template <typename T>
static int rasterize_bwd_gather(int B, int H, int W, int F, int D, const void *grad, const int64_t *face_idx,
                                const void *w, const void *fvi, const void *feat, const uint8_t *valid, const T *nz,
                                float m, float eps, void *gfvi, void *gfeat, void *ws, size_t ws_bytes, int *nbig,
                                hipStream_t st, const uint2 *rng = nullptr, double *soft = nullptr,
                                uint8_t *sflag = nullptr) {
  const int64_t nf = (int64_t)B * F;
  if (nf == 0) return KL_OK;
  if (D > 8) {  // wide features: the scatter kernel
    KL_REQUIRE(soft == nullptr, "rasterize backward: the soft-mask sum needs feat_dim <= 8");
    return rasterize_bwd<T>(B, H, W, F, D, grad, face_idx, w, fvi, feat, eps, gfvi, gfeat, ws, ws_bytes, st);
  }
  KL_REQUIRE(ws_bytes >= (size_t)(nf + 1) * sizeof(int), "rasterize backward: workspace too small");
  KL_REQUIRE(nf < ((int64_t)1 << 31), "rasterize backward: too many faces");
  const bool zero = nbig == nullptr;
  if (zero) nbig = reinterpret_cast<int *>(ws);
  int *big = reinterpret_cast<int *>(ws) + 1;
  const T *g = (const T *)grad;
  const T *wt = (const T *)w;
  const T *fv = (const T *)fvi;
  const T *ft = (const T *)feat;
  // MAXD = D where it is small (the accumulators are doubles: registers set the occupancy)
  if (D <= 2)
    return rasterize_bwd_gather_maxd<T, 2>(B, H, W, F, D, g, face_idx, wt, fv, ft, valid, nz, m, eps, (T *)gfvi,
                                           (T *)gfeat, big, nbig, zero, rng, soft, sflag, st);
  if (D == 3)
    return rasterize_bwd_gather_maxd<T, 3>(B, H, W, F, D, g, face_idx, wt, fv, ft, valid, nz, m, eps, (T *)gfvi,
                                           (T *)gfeat, big, nbig, zero, rng, soft, sflag, st);
  if (D <= 4)
    return rasterize_bwd_gather_maxd<T, 4>(B, H, W, F, D, g, face_idx, wt, fv, ft, valid, nz, m, eps, (T *)gfvi,
                                           (T *)gfeat, big, nbig, zero, rng, soft, sflag, st);
  return rasterize_bwd_gather_maxd<T, 8>(B, H, W, F, D, g, face_idx, wt, fv, ft, valid, nz, m, eps, (T *)gfvi,
                                         (T *)gfeat, big, nbig, zero, rng, soft, sflag, st);
}

// The fused front-end path's forward: the tile rasterizer (dev flag bit 13 selects the
// per-face visibility-buffer path instead, for ablation timing).
template <typename T>
static int dibr_rast_fwd(RastSrc<T> src, int H, int W, int B, int D, int F, const T *fvz, const T *feat, float m,
                         float eps, T *out_feat, int64_t *out_idx, T *out_w, void *ws, size_t ws_bytes,
                         hipStream_t st) {
  if (g_dev_flags & (1 << 13)) {
    const int64_t nf = (int64_t)B * F;
    return launch_rast_fwd<T>(src, H, W, B, D, nf, nf, fvz, feat, nullptr, F, m, eps, out_feat, out_idx, out_w, ws,
                              ws_bytes, st);
  }
  return launch_rast_tile<T>(src, H, W, B, D, F, fvz, feat, m, eps, out_feat, out_idx, out_w, ws, ws_bytes, st);
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_rasterize_workspace_bytes(int batch, int height, int width, int64_t max_faces_per_mesh) {
  return RastWs(batch, height, width, (int64_t)batch * max_faces_per_mesh).bytes;
}

extern "C" int kl_packed_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int64_t num_faces,
                                           int feat_dim, int64_t max_faces_per_mesh, const void *fvz,
                                           const void *fvi, const void *bbox, const void *feat,
                                           const int64_t *first_idx, float multiplier, float eps, void *out_feat,
                                           int64_t *out_idx, void *out_w, void *ws, size_t ws_bytes,
                                           kl_stream stream) {
  const int64_t ws_faces = (int64_t)batch * max_faces_per_mesh;
  if (dtype == KL_F32)
    return launch_rast_fwd<float>(BboxSrc<float>{(const float *)bbox, (const float *)fvi}, height, width, batch,
                                  feat_dim, num_faces, ws_faces, (const float *)fvz, (const float *)feat, first_idx, 0,
                                  multiplier, eps, (float *)out_feat, out_idx, (float *)out_w, ws, ws_bytes,
                                  S(stream));
  if (dtype == KL_F64)
    return launch_rast_fwd<double>(BboxSrc<double>{(const double *)bbox, (const double *)fvi}, height, width, batch,
                                   feat_dim, num_faces, ws_faces, (const double *)fvz, (const double *)feat, first_idx,
                                   0, multiplier, eps, (double *)out_feat, out_idx, (double *)out_w, ws, ws_bytes,
                                   S(stream));
  set_error("packed_rasterize_forward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_dibr_rasterize_workspace_bytes(int batch, int height, int width, int num_faces) {
  const size_t tile = rast_tile_ws_bytes(batch, height, width, num_faces);
  const size_t vis = RastWs(batch, height, width, (int64_t)batch * num_faces).bytes;  // dev ablation path
  const size_t fwd = tile > vis ? tile : vis;
  const size_t bwd = ((size_t)batch * num_faces + 1) * sizeof(int);
  return fwd > bwd ? fwd : bwd;
}

extern "C" int kl_dibr_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int num_faces,
                                         int feat_dim, const void *fvz, const void *fvi, const void *feat,
                                         const uint8_t *valid_faces, const void *fnz, float multiplier, float eps,
                                         void *out_feat, int64_t *out_idx, void *out_w, void *ws, size_t ws_bytes,
                                         kl_stream stream) {
  if (dtype == KL_F32)
    return dibr_rast_fwd<float>(RastSrc<float>{(const float *)fvi, valid_faces, (float)multiplier,
                                               (const float *)fnz}, height, width, batch, feat_dim, num_faces,
                                (const float *)fvz, (const float *)feat, multiplier, eps, (float *)out_feat, out_idx,
                                (float *)out_w, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return dibr_rast_fwd<double>(RastSrc<double>{(const double *)fvi, valid_faces, (double)multiplier,
                                                 (const double *)fnz}, height, width, batch, feat_dim, num_faces,
                                 (const double *)fvz, (const double *)feat, multiplier, eps, (double *)out_feat,
                                 out_idx, (double *)out_w, ws, ws_bytes, S(stream));
  set_error("dibr_rasterize_forward not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_rasterize_backward_workspace_bytes(int batch, int num_faces, int feat_dim) {
  return rast_scatter_ws_bytes(batch, num_faces, feat_dim);
}

extern "C" int kl_rasterize_backward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                     int feat_dim, const void *grad, const int64_t *face_idx, const void *w,
                                     const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                                     void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return rasterize_bwd<float>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat, eps,
                                gfvi, gfeat, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return rasterize_bwd<double>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat, eps,
                                 gfvi, gfeat, ws, ws_bytes, S(stream));
  set_error("rasterize_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_dibr_rasterize_bwd_workspace_bytes(int batch, int height, int width, int num_faces,
                                                        int feat_dim) {
  const size_t gather = ((size_t)batch * num_faces + 1) * sizeof(int);
  return feat_dim > 8 ? std::max(gather, rast_scatter_ws_bytes(batch, num_faces, feat_dim)) : gather;
}

extern "C" int kl_dibr_rasterize_backward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                          int feat_dim, const void *grad, const int64_t *face_idx, const void *w,
                                          const void *fvi, const void *feat, const uint8_t *valid_faces,
                                          const void *fnz, float multiplier, float eps, void *gfvi, void *gfeat,
                                          int *scratch, const uint32_t *face_ranges, void *ws, size_t ws_bytes,
                                          kl_stream stream) {
  const uint2 *fr = reinterpret_cast<const uint2 *>(face_ranges);
  if (dtype == KL_F32)
    return rasterize_bwd_gather<float>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat,
                                       valid_faces, (const float *)fnz, multiplier, eps, gfvi, gfeat, ws, ws_bytes,
                                       scratch, S(stream), fr);
  if (dtype == KL_F64)
    return rasterize_bwd_gather<double>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat,
                                        valid_faces, (const double *)fnz, multiplier, eps, gfvi, gfeat, ws, ws_bytes,
                                        scratch, S(stream), fr);
  set_error("dibr_rasterize_backward not implemented for this dtype");
  return KL_E_INVALID;
}

// ---------------------------------------------------------------- dibr_rasterization
// The whole of dibr_rasterization (dibr.py:119-209) in one call per direction: rasterize
// with valid = face_normals_z >= 0 evaluated in-kernel, then the soft mask of the
// compact path (softtile.hip) on the rasterizer's face index.  The backward runs the
// gather (which writes every face's gradient) and adds the soft-mask terms onto it.
// The state's scratch int is the gather's big-face counter: the forward zeroes it and
// the backward's final add re-zeroes it (retain_graph), so the backward needs no fill of it.
namespace kl {
// Workspace of kl_dibr_forward: the rasterizer's and the soft mask's bins are built by one
// pass over the faces, counted by one bucket kernel and ordered by one order kernel.
//   zeroed: raster bitmap | soft bitmap | raster ghist | soft ghist
//   then:   face records | pixel ranges | raster buckets | soft buckets | raster items |
//           item count | soft order | soft pixel ranges     (records sized for f64)
struct DibrFwdWs {
  size_t off_sbm, off_rgh, off_sgh, off_tk, off_live, zero, off_rec, off_rng, off_rbk, off_sbk, off_items, off_n,
      off_sorder, off_sn, off_srng, off_defer, off_whist, off_rowitem, bytes;
  DibrFwdWs(int B, int H, int W, int F) {
    const BinGeom g = make_bin_geom(B, H, W, F);
    const size_t nt = (size_t)g.batch * g.tiles_y * g.tiles_x;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    off_sbm = g.bytes();
    off_rgh = off_sbm + g.bytes();
    off_sgh = off_rgh + ORD_HIST * sizeof(int);
    off_tk = off_sgh + ORD_HIST * sizeof(int);  // the chip-wide order kernel's two tickets
    off_live = off_tk + 16 * sizeof(int);       // the soft items' live flags (<= 8 items per tile)
    zero = off_live + ((nt * TILE_H + 3) & ~(size_t)3);
    off_rec = up(zero);
    off_rng = up(off_rec + (size_t)B * F * RT_REC * sizeof(double));
    off_rbk = up(off_rng + (size_t)B * F * sizeof(uint2));
    off_sbk = up(off_rbk + nt);
    off_items = up(off_sbk + nt);
    off_n = off_items + nt * TILE_H * sizeof(int32_t);
    off_sorder = up(off_n + sizeof(int));
    off_sn = off_sorder + nt * TILE_H * sizeof(int32_t);
    off_srng = up(off_sn + sizeof(int));
    off_defer = up(off_srng + (size_t)B * F * sizeof(uint2));
    off_whist = up(off_defer + (size_t)B * H * g.tiles_x);  // 2 x nb x ORD_HIST workgroup histograms
    off_rowitem = up(off_whist + 2 * (size_t)cdiv((int64_t)nt, CO_THREADS) * ORD_HIST * sizeof(int));
    bytes = off_rowitem + nt * TILE_H * sizeof(int32_t);  // the soft item of each tile row
  }
};

template <typename T>
static int dibr_fwd(int B, int H, int W, int F, int D, int K, const T *fvz, const T *fvi, const T *feat, const T *fnz,
                    float sigmainv, double pad, float m, float eps, T *out_feat, int64_t *out_idx, T *out_w,
                    T *out_mask, const SoftState<T> &s, void *ws, size_t ws_bytes, hipStream_t st,
                    uint2 *face_ranges) {
  const DibrFwdWs L(B, H, W, F);
  KL_REQUIRE(ws_bytes >= L.bytes, "dibr_rasterization forward: workspace too small");
  KL_REQUIRE(H < 65536 && W < 65536, "dibr_rasterization forward: height and width must be < 65536");
  KL_REQUIRE(K >= 0 && K <= 255, "dibr_rasterization forward: the compact soft mask needs 0 <= knum <= 255");
  KL_REQUIRE(F < (1 << 28), "dibr_rasterization forward: too many faces");
  KL_REQUIRE(s.scratch != nullptr, "dibr_rasterization forward: state (kl_dibr_state_bytes) missing");
  const DibrState S(B, H, W, F, K);
  char *state = reinterpret_cast<char *>(s.scratch);
  int *bcnt = reinterpret_cast<int *>(state);
  int2 *bitems = reinterpret_cast<int2 *>(state + S.off_items);
  double *bacc = nullptr;  // (ABI 4: the backward's soft accumulator is the caller's, kept zero)
  const size_t P = (size_t)B * H * W;
  if (P == 0 || F == 0) {  // no pixels / no faces: no soft-mask hits, nothing listed
    KL_CHECK_RC(fill_async(bcnt, 0, DibrState::kZeroInts * sizeof(int), st));
    if (P == 0) return KL_OK;
    SoftState<T> s0 = s;
    s0.scratch = nullptr;
    KL_CHECK_RC(dibr_rast_fwd<T>(RastSrc<T>{fvi, nullptr, (T)m, fnz}, H, W, B, D, F, fvz, feat, m, eps, out_feat,
                                 out_idx, out_w, ws, ws_bytes, st));
    return soft_tile_forward<T>(B, H, W, F, K, fvi, out_idx, sigmainv, pad, m, out_mask, s0, ws, ws_bytes, st);
  }
  const BinGeom g = make_bin_geom(B, H, W, F);
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  char *w = reinterpret_cast<char *>(ws);
  uint32_t *rbm = reinterpret_cast<uint32_t *>(w);
  uint32_t *sbm = reinterpret_cast<uint32_t *>(w + L.off_sbm);
  int *rgh = reinterpret_cast<int *>(w + L.off_rgh);
  int *sgh = reinterpret_cast<int *>(w + L.off_sgh);
  T *rec = reinterpret_cast<T *>(w + L.off_rec);
  uint2 *rng = face_ranges ? face_ranges : reinterpret_cast<uint2 *>(w + L.off_rng);
  uint8_t *rbk = reinterpret_cast<uint8_t *>(w + L.off_rbk);
  uint8_t *sbk = reinterpret_cast<uint8_t *>(w + L.off_sbk);
  int32_t *items = reinterpret_cast<int32_t *>(w + L.off_items);
  int *nitems = reinterpret_cast<int *>(w + L.off_n);
  int32_t *sorder = reinterpret_cast<int32_t *>(w + L.off_sorder);
  int *snitems = reinterpret_cast<int *>(w + L.off_sn);
  uint2 *srng = reinterpret_cast<uint2 *>(w + L.off_srng);
  const RastSrc<T> src{fvi, nullptr, (T)m, fnz};
  const PixPitch pp{m / (float)W, m / (float)H, (float)W / m, (float)H / m};
  if constexpr (sizeof(T) == 4) {
    // the fused tile kernel (dibrtile.hip): the soft bins only, one order, ONE kernel for the
    // rasterizer and the soft mask (needs bboxes inside the enlarged ones: boxlen >= 0).  Dev param
    // 10 = 2 only: measured slower than the two-kernel path below at cfg3 (105.9 against 32.1 +
    // 51.3 us of tile kernels), kept tested bit-equal to it for the record.
#if KL_DEV  // the fused tile kernel (dev param 10 = 2): a measured dead end, DESIGN.md 3.1
    if (pad >= 0.0 && bin_word_lds_ok(g) && nt <= ORD_LDS_TILES && g_dev_param[10] == 2) {
      KL_CHECK_RC(launch_bin_word<T>(src, fvz, F, g, pp, nullptr, rec, rng, sbm, srng, (T)pad, rgh,
                                     (int)((L.zero - L.off_rgh) / sizeof(int)), st));
      const int lpm = g_dev_param[13] ? g_dev_param[13] : dt_lp_min(K);  // dev param 13: rows 8 >> lp_min
      // block 1 orders; block 0 zeroes the state's counters; the rest zero the backward's accumulator
      const unsigned og = g_dev_param[9] >= 2 ? (unsigned)g_dev_param[9] : 256u;
      hipLaunchKernelGGL(tile_countorder2_kernel, dim3(og), dim3(1024), 0, st, (const uint32_t *)sbm,
                         (const uint32_t *)sbm, g.words, (int32_t *)nullptr, 0, 0, (int *)nullptr, sorder, nt, lpm,
                         snitems, soft_split(), 0, bcnt, DibrState::kZeroInts, bacc, (size_t)0,
                         kDevStamps && g_dev_debug ? reinterpret_cast<uint64_t *>(g_dev_debug) + kOrderStampsAt
                                                   : nullptr);
      KL_CHECK_LAUNCH();
      const DibrTileArgs da{reinterpret_cast<const float *>(rec), rng, srng,
                            SoftSrc<float>{reinterpret_cast<const float *>(fvi), (float)m, (float)pad},
                            reinterpret_cast<const float *>(feat), sbm, sorder, snitems, g, F, D, K, eps, sigmainv,
                            m, reinterpret_cast<float *>(out_feat), out_idx, reinterpret_cast<float *>(out_w),
                            reinterpret_cast<float *>(out_mask), s.hits, s.rec_face,
                            reinterpret_cast<float *>(s.rec_prob), s.seg_tot, bitems, bcnt, S.cap,
                            g_dev_param[12]};
      return dibr_tile_launch(da, lpm, soft_items_bound(nt, lpm, soft_split()), st);
    }
#endif

  }
  if (bin_word_lds_ok(g) && !(g_dev_flags & (1 << 14))) {  // dev bit 14: the atomic binning
    KL_CHECK_RC(launch_bin_word<T>(src, fvz, F, g, pp, rbm, rec, rng, sbm, srng, (T)pad, rgh,
                                   (int)((L.zero - L.off_rgh) / sizeof(int)), st));  // + histograms zeroed
  } else {
  KL_CHECK_RC(fill_async(w, 0, L.zero, st));
  const dim3 bgrid((unsigned)cdiv((int64_t)g.chunks * 64, 256), (unsigned)B);
  if (fnz)
    hipLaunchKernelGGL((raster_bin_kernel<T, 2>), bgrid, dim3(256), 0, st, src, fvz, F, g, pp, rbm, rec, rng, sbm,
                       srng, (T)pad);
  else
    hipLaunchKernelGGL((raster_bin_kernel<T, 0>), bgrid, dim3(256), 0, st, src, fvz, F, g, pp, rbm, rec, rng, sbm,
                       srng, (T)pad);
  KL_CHECK_LAUNCH();
  }
  // heavy tiles (>= 2^split_from - 1 candidate chunks) split into 2^split_log2 row parts (dev
  // params 4 / 5 override, for sweeps)
  const int split_from = g_dev_param[4] ? g_dev_param[4] : 5;
  const int split_log2 = sizeof(T) == 4 ? (g_dev_param[5] ? g_dev_param[5] : 2) : 0;
  // r05: the soft items' live flags (set by the rasterizer, read by the soft kernel first) where the
  // chip order kernel lists each tile row's item; dev param 26 = 1: off (A/B)
  bool live = false;
  if (nt <= ORD_LDS_TILES && !(g_dev_flags & (1 << 20)) && g_dev_param[15] != 1 &&
      chip_order_resident((int)cdiv(nt, CO_THREADS))) {
    // counts over the chip, orders by each bitmap's last count workgroup (tileorder.h); the other
    // workgroups zero the backward's soft-mask accumulator meanwhile (dev param 15 = 1: the r04
    // two-workgroup kernel below, for A/B)
    const int nb = (int)cdiv(nt, CO_THREADS);
    CountOrderArgs ca{};
    ca.bm[0] = rbm;
    ca.bm[1] = sbm;
    ca.words = g.words;
    ca.nt = nt;
    ca.nb = nb;
    ca.whist[0] = reinterpret_cast<int *>(w + L.off_whist);
    ca.whist[1] = ca.whist[0] + (size_t)nb * ORD_HIST;
    ca.ticket = reinterpret_cast<unsigned *>(w + L.off_tk);
    ca.order[0] = items;
    ca.order[1] = sorder;
    ca.nitems[0] = nitems;
    ca.nitems[1] = snitems;
    ca.split_from = split_from;
    ca.split_log2 = split_log2;
    ca.lp_min1 = soft_lp_min(K);
    ca.skip_empty1 = 1;
    // the soft mask's items in plain heaviest-first order (r05: 1-3 us faster than XCD bands, whose
    // band-local ranks started heavy silhouette items late); dev param 18 = 1 + v sets the bits to v
    // (bit 0 the rasterizer's, bit 1 the soft mask's) for A/B
    ca.noband = g_dev_param[18] ? (g_dev_param[18] - 1) & 3 : 2;
    ca.sp = soft_split();
    ca.zero = bcnt;
    ca.nzero = DibrState::kZeroInts;
    ca.zacc = nullptr;
    ca.zn = 0;
    ca.dbg = kDevStamps && g_dev_debug ? reinterpret_cast<uint64_t *>(g_dev_debug) + kOrderStampsAt : nullptr;
    live = g_dev_param[26] != 1;
    ca.row_item = live ? reinterpret_cast<int32_t *>(w + L.off_rowitem) : nullptr;
    if (g_dev_param[16] == 1) ca.spin_limit = 0;  // dev: every workgroup counts the whole bitmap (test)
    const unsigned zg = 1u;  // one workgroup zeroes the state's counters
    hipLaunchKernelGGL(tile_countorder_chip_kernel, dim3((unsigned)(2 * nb) + zg), dim3(CO_THREADS),
                       (size_t)nb * ORD_HIST * sizeof(int), st, ca);
    KL_CHECK_LAUNCH();
  } else if (nt <= ORD_LDS_TILES && !(g_dev_flags & (1 << 20))) {  // counts and orders in one launch
    // + 254 workgroups that zero the backward's soft-mask accumulator while two order
    const unsigned og = g_dev_param[9] >= 2 ? (unsigned)g_dev_param[9] : 256u;  // dev: grid (2 = no zero fill)
    hipLaunchKernelGGL(tile_countorder2_kernel, dim3(og), dim3(1024), 0, st, (const uint32_t *)rbm,
                       (const uint32_t *)sbm, g.words, items, split_from, split_log2, nitems, sorder, nt,
                       soft_lp_min(K), snitems, soft_split(), 1, bcnt, DibrState::kZeroInts, bacc,
                       (size_t)0,
                       kDevStamps && g_dev_debug ? reinterpret_cast<uint64_t *>(g_dev_debug) + kOrderStampsAt : nullptr);
    KL_CHECK_LAUNCH();
  } else {  // counts (a wave per tile) then orders (dev bit 20: this path, for A/B timing)
    hipLaunchKernelGGL(tile_bucket2_kernel, dim3((unsigned)cdiv(nt, 4)), dim3(256), 0, st, (const uint32_t *)rbm,
                       (const uint32_t *)sbm, g.words, nt, rbk, sbk, rgh, sgh, bcnt, DibrState::kZeroInts);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(tile_order2_kernel, dim3(256), dim3(1024), 0, st, (const uint8_t *)rbk, (const int *)rgh,
                       items, split_from, split_log2, nitems, (const uint8_t *)sbk, (const int *)sgh, sorder, nt,
                       soft_lp_min(K), snitems, soft_split(), 1, bacc, (size_t)0);
    KL_CHECK_LAUNCH();
  }
  uint8_t *defer = reinterpret_cast<uint8_t *>(w + L.off_defer);
  RastTileArgs<T> args{src, fvz, feat, rbm, rec, rng, items, nitems, g, F, D, eps, out_feat, out_idx, out_w,
                       reinterpret_cast<uint64_t *>(g_dev_debug)};
  args.soft_mask = out_mask;
  args.soft_hits = s.hits;
  args.soft_seg = s.seg_tot;
  args.soft_defer = defer;
  uint8_t *live_flags = live ? reinterpret_cast<uint8_t *>(w + L.off_live) : nullptr;
  args.soft_row_item = live ? reinterpret_cast<const int32_t *>(w + L.off_rowitem) : nullptr;
  args.soft_live = live_flags;
  hipLaunchKernelGGL((raster_tile_kernel<T>), dim3((unsigned)(nt << split_log2)), dim3(512), 0, st, args);
  KL_CHECK_LAUNCH();
  return soft_tile_forward_main<T>(B, H, W, F, K, fvi, out_idx, sigmainv, pad, m, out_mask, s, sbm, sorder, snitems,
                                   srng, defer, st, true, bitems, bcnt, S.cap, live_flags);
}

template <typename T>
static int dibr_bwd(int B, int H, int W, int F, int D, int K, const T *grad_feat, const T *grad_mask,
                    const int64_t *face_idx, const T *w, const T *fvi, const T *feat, const T *fnz, const T *mask,
                    const SoftState<T> &s, float sigmainv, float m, float eps, T *gfvi, T *gfeat, void *soft_acc,
                    void *ws, size_t ws_bytes, hipStream_t st, const uint2 *face_ranges) {
  KL_REQUIRE(D <= 8, "dibr_rasterization backward: feature dimension > 8 is not supported by the fused path");
  KL_REQUIRE(s.scratch != nullptr, "dibr_rasterization backward: state (kl_dibr_state_bytes) missing");
  // The soft-mask terms first, summed in double into the state's accumulator (zeroed by the
  // forward) over the work items the forward listed -- no plan kernel, no fill -- then the gather
  // on the same stream, which adds each face's soft sum, rounded on its own, to the face's own
  // rounded gradient as it writes it (autograd's add of the two gradients).  (r03: a plan kernel
  // listed the items and zeroed the accumulator, 8.6 us per backward at cfg3; until r03x the two
  // halves ran on two streams joined by a final add, ~16 us of fork / join gaps in the graph.)
  const DibrState S(B, H, W, F, K);
  char *state = reinterpret_cast<char *>(s.scratch);
  const bool has_soft = grad_mask != nullptr && K > 0 && (int64_t)B * H * W > 0 && (int64_t)B * F > 0;
  KL_REQUIRE(soft_acc != nullptr || !has_soft, "dibr_rasterization backward: soft accumulator (kl_dibr_soft_acc_bytes) missing");
  const DibrSoftAcc A(B, F);
  double *acc = reinterpret_cast<double *>(soft_acc);
  uint8_t *sflag = has_soft ? reinterpret_cast<uint8_t *>(soft_acc) + A.off_flags : nullptr;
  int rc = KL_OK;
  if (has_soft)
    rc = soft_tile_backward_listed<T>(B, H, W, F, K, grad_mask, mask, s, fvi, sigmainv, m,
                                      reinterpret_cast<const int2 *>(state + S.off_items),
                                      reinterpret_cast<const int *>(state), S.cap, acc, sflag, st);
  if (rc == KL_OK)
    rc = rasterize_bwd_gather<T>(B, H, W, F, D, grad_feat, face_idx, w, fvi, feat, nullptr, fnz, m, eps, gfvi, gfeat,
                                 ws, ws_bytes, nullptr, st, face_ranges, has_soft ? acc : nullptr, sflag);
  // the accumulator must be zero for the next call: on ANY failure (the soft kernel may have added
  // into it before a later step failed, and the gather that re-zeroes it may not have run) clear it
  if (rc != KL_OK && has_soft) (void)fill_async(soft_acc, 0, A.bytes, st);
  return rc;
}
}  // namespace kl

extern "C" size_t kl_dibr_workspace_bytes(int batch, int height, int width, int num_faces) {
  const size_t a = kl_dibr_rasterize_workspace_bytes(batch, height, width, num_faces);  // F == 0 / dev path
  const size_t b = soft_tile_ws_bytes(batch, height, width, num_faces);
  const size_t c = DibrFwdWs(batch, height, width, num_faces).bytes;
  return std::max(a, std::max(b, c));
}

extern "C" size_t kl_dibr_bwd_workspace_bytes(int batch, int height, int width, int num_faces, int knum) {
  (void)knum;
  return kl_dibr_rasterize_bwd_workspace_bytes(batch, height, width, num_faces, 8);
}

extern "C" size_t kl_dibr_state_bytes(int batch, int height, int width, int num_faces, int knum) {
  return DibrState(batch, height, width, num_faces, knum).bytes;
}

extern "C" size_t kl_dibr_soft_acc_bytes(int batch, int num_faces) { return DibrSoftAcc(batch, num_faces).bytes; }

extern "C" int kl_dibr_forward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim,
                               int knum, const void *fvz, const void *fvi, const void *feat, const void *fnz,
                               float sigmainv, double bbox_pad, float multiplier, float eps, void *out_feat,
                               int64_t *out_idx, void *out_w, void *out_mask, uint8_t *hits, uint32_t *rec_face,
                               void *rec_prob, int *seg_tot, void *state, uint32_t *face_ranges, void *ws,
                               size_t ws_bytes, kl_stream stream) {
  uint2 *fr = reinterpret_cast<uint2 *>(face_ranges);
  if (dtype == KL_F32)
    return dibr_fwd<float>(batch, height, width, num_faces, feat_dim, knum, (const float *)fvz, (const float *)fvi,
                           (const float *)feat, (const float *)fnz, sigmainv, bbox_pad, multiplier, eps,
                           (float *)out_feat, out_idx, (float *)out_w, (float *)out_mask,
                           SoftState<float>{hits, rec_face, (float *)rec_prob, seg_tot, (int *)state}, ws, ws_bytes,
                           S(stream), fr);
  if (dtype == KL_F64)
    return dibr_fwd<double>(batch, height, width, num_faces, feat_dim, knum, (const double *)fvz, (const double *)fvi,
                            (const double *)feat, (const double *)fnz, sigmainv, bbox_pad, multiplier, eps,
                            (double *)out_feat, out_idx, (double *)out_w, (double *)out_mask,
                            SoftState<double>{hits, rec_face, (double *)rec_prob, seg_tot, (int *)state}, ws, ws_bytes,
                            S(stream), fr);
  set_error("dibr_rasterization not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_backward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim,
                                int knum, const void *grad_feat, const void *grad_mask, const int64_t *face_idx,
                                const void *w, const void *fvi, const void *feat, const void *fnz, const void *mask,
                                const uint8_t *hits, const uint32_t *rec_face, const void *rec_prob,
                                const int *seg_tot, float sigmainv, float multiplier, float eps, void *gfvi,
                                void *gfeat, void *state, const uint32_t *face_ranges, void *soft_acc, void *ws,
                                size_t ws_bytes, kl_stream stream) {
  const uint2 *fr = reinterpret_cast<const uint2 *>(face_ranges);
  if (dtype == KL_F32)
    return dibr_bwd<float>(
        batch, height, width, num_faces, feat_dim, knum, (const float *)grad_feat, (const float *)grad_mask, face_idx,
        (const float *)w, (const float *)fvi, (const float *)feat, (const float *)fnz, (const float *)mask,
        SoftState<float>{(uint8_t *)hits, (uint32_t *)rec_face, (float *)rec_prob, (int *)seg_tot, (int *)state},
        sigmainv, multiplier, eps, (float *)gfvi, (float *)gfeat, soft_acc, ws, ws_bytes, S(stream), fr);
  if (dtype == KL_F64)
    return dibr_bwd<double>(
        batch, height, width, num_faces, feat_dim, knum, (const double *)grad_feat, (const double *)grad_mask,
        face_idx, (const double *)w, (const double *)fvi, (const double *)feat, (const double *)fnz,
        (const double *)mask,
        SoftState<double>{(uint8_t *)hits, (uint32_t *)rec_face, (double *)rec_prob, (int *)seg_tot, (int *)state},
        sigmainv, multiplier, eps, (double *)gfvi, (double *)gfeat, soft_acc, ws, ws_bytes, S(stream), fr);
  set_error("dibr_rasterization backward not implemented for this dtype");
  return KL_E_INVALID;
}
