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
#include "soft_common.h"

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

// The reference's per-(pixel, face) test, statement for statement: bbox reject, edge
// functions, copysign(eps) normalisation, barycentric sign test.  true => (w0,w1,w2)
// are the face's weights at the pixel centre (x0, y0).
template <typename T>
__device__ __forceinline__ bool face_weights(const RastFace<T> &r, T x0, T y0, float eps, T &w0, T &w1, T &w2) {
  if (x0 < r.xmin || x0 >= r.xmax || y0 < r.ymin || y0 >= r.ymax) return false;
  const T aex = r.v[0] - x0, aey = r.v[1] - y0;
  const T bex = r.v[2] - x0, bey = r.v[3] - y0;
  const T cex = r.v[4] - x0, cey = r.v[5] - y0;
  w0 = bex * cey - bey * cex;
  w1 = cex * aey - cey * aex;
  w2 = aex * bey - aey * bex;
  T norm = w0 + w1 + w2;
  norm = (T)((double)norm + copysign((double)eps, (double)norm));
  w0 /= norm;
  w1 /= norm;
  w2 /= norm;
  return !(w0 < (T)0 || w1 < (T)0 || w2 < (T)0);
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

// Depth-ordered visibility through one 64-bit atomicMax per covered (face, pixel):
//   float : key = order(z0) << 32 | ~local_face   -> max depth, lowest index on ties,
//           which is exactly the reference's `if (z0 <= max_z0) continue` fold over
//           faces in index order;
//   double: pass 0 maxes order(z0) (64 bit), pass 1 mins the index among the faces
//           that reach it.
// order() maps floats to unsigned keys monotonically with -0 == +0.  z0 = -inf never
// wins in the reference (-inf <= -inf), so it is dropped.  A NaN z0 breaks the total
// order (the reference then keeps the LAST passing face); such pixels are flagged and
// re-walked sequentially by the resolve kernel.
__device__ __forceinline__ uint32_t order32(float z) {
  uint32_t u = __float_as_uint(z == 0.0f ? 0.0f : z);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint64_t order64(double z) {
  uint64_t u = (uint64_t)__double_as_longlong(z == 0.0 ? 0.0 : z);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
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
struct RangeWalk {
  int w, area, e, col, row;
  __device__ __forceinline__ RangeWalk(int ix0, int ix1, int iy0, int iy1, int s) {
    w = ix1 - ix0 + 1;
    area = w * (iy1 - iy0 + 1);
    e = s;
    row = s / w;
    col = s - row * w;
  }
  __device__ __forceinline__ bool more() const { return e < area; }
  __device__ __forceinline__ void next() {
    e += LPF;
    col += LPF;
    while (col >= w) {
      col -= w;
      row++;
    }
  }
};

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

// d(interpolated feature)/d(face vertices) of one pixel (rasterization_cuda.cu:287-399).
// Calls acc(slot, value) for the 6 vertex-coordinate slots, per feature d.
template <typename T>
struct BaryGrad {
  T dw1dax, dw1day, dw1dbx, dw1dby, dw1dcx, dw1dcy;
  T dw2dax, dw2day, dw2dbx, dw2dby, dw2dcx, dw2dcy;
  T k3sq;
  __device__ __forceinline__ void init(const T v[6], T w_a, T w_b, T w_c, float eps) {
    const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
    const T x0 = w_a * ax + w_b * bx + w_c * cx;
    const T y0 = w_a * ay + w_b * by + w_c * cy;
    const T m = bx - ax, p = by - ay, n = cx - ax, q = cy - ay, s = x0 - ax, t = y0 - ay;
    const T k1 = s * q - n * t;
    const T k2 = m * t - s * p;
    T k3 = m * q - n * p;
    k3 = (T)((double)k3 + copysign((double)eps, (double)k3));
    const T zero = (T)0;
    const T dk1dm = zero, dk1dn = -t, dk1dp = zero, dk1dq = s, dk1ds = q, dk1dt = -n;
    const T dk2dm = t, dk2dn = zero, dk2dp = -s, dk2dq = zero, dk2ds = -p, dk2dt = m;
    const T dk3dm = q, dk3dn = -p, dk3dp = -n, dk3dq = m, dk3ds = zero, dk3dt = zero;
    const T dw1dm = dk1dm * k3 - dk3dm * k1, dw1dn = dk1dn * k3 - dk3dn * k1;
    const T dw1dp = dk1dp * k3 - dk3dp * k1, dw1dq = dk1dq * k3 - dk3dq * k1;
    const T dw1ds = dk1ds * k3 - dk3ds * k1, dw1dt = dk1dt * k3 - dk3dt * k1;
    const T dw2dm = dk2dm * k3 - dk3dm * k2, dw2dn = dk2dn * k3 - dk3dn * k2;
    const T dw2dp = dk2dp * k3 - dk3dp * k2, dw2dq = dk2dq * k3 - dk3dq * k2;
    const T dw2ds = dk2ds * k3 - dk3ds * k2, dw2dt = dk2dt * k3 - dk3dt * k2;
    dw1dax = -(dw1dm + dw1dn + dw1ds);
    dw1day = -(dw1dp + dw1dq + dw1dt);
    dw1dbx = dw1dm; dw1dby = dw1dp; dw1dcx = dw1dn; dw1dcy = dw1dq;
    dw2dax = -(dw2dm + dw2dn + dw2ds);
    dw2day = -(dw2dp + dw2dq + dw2dt);
    dw2dbx = dw2dm; dw2dby = dw2dp; dw2dcx = dw2dn; dw2dcy = dw2dq;
    k3sq = k3 * k3;
  }
  // the six dL/d(vertex coordinate) terms of feature channel with grad gd and values c0..c2
  __device__ __forceinline__ void terms(T gd, T c0, T c1, T c2, T out[6]) const {
    const T dIdax = (c1 - c0) * dw1dax + (c2 - c0) * dw2dax;
    const T dIday = (c1 - c0) * dw1day + (c2 - c0) * dw2day;
    const T dIdbx = (c1 - c0) * dw1dbx + (c2 - c0) * dw2dbx;
    const T dIdby = (c1 - c0) * dw1dby + (c2 - c0) * dw2dby;
    const T dIdcx = (c1 - c0) * dw1dcx + (c2 - c0) * dw2dcx;
    const T dIdcy = (c1 - c0) * dw1dcy + (c2 - c0) * dw2dcy;
    const T dldI = gd / k3sq;
    out[0] = dldI * dIdax;
    out[1] = dldI * dIday;
    out[2] = dldI * dIdbx;
    out[3] = dldI * dIdby;
    out[4] = dldI * dIdcx;
    out[5] = dldI * dIdcy;
  }
};

template <typename T>
__global__ void __launch_bounds__(256) rasterize_bwd_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, int B, int H, int W, int F, int D, float eps,
    T *__restrict__ grad_fvi, T *__restrict__ grad_ffeat) {
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
      atomicAdd(grad_ffeat + tf * 3 * D + d, gd * w_a);
      atomicAdd(grad_ffeat + tf * 3 * D + D + d, gd * w_b);
      atomicAdd(grad_ffeat + tf * 3 * D + 2 * D + d, gd * w_c);
    }
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
    BaryGrad<T> bg;
    bg.init(v, w_a, w_b, w_c, eps);
    const T *c = feat + tf * 3 * D;
    T *gv = grad_fvi + tf * 6;
    for (int d = 0; d < D; d++) {
      T o[6];
      bg.terms(g[d], c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
      for (int q = 0; q < 6; q++) atomicAdd(gv + q, o[q]);
    }
  }
}

// ---------------------------------------------------------------- gather backward
// One thread per face visits exactly the pixel range the forward visited for it (the
// same in-kernel bbox and exact_axis), so every pixel the face can have won is seen;
// pixels are taken 8 at a time with their face_idx / weights / grads loads in flight
// together.  Faces whose range exceeds VIS_SMALL_AREA go to a workgroup per face.
constexpr int GATHER_BATCH = 4;

template <typename T>
__device__ __forceinline__ bool face_range(const RastSrc<T> &src, int64_t tf, float m, int H, int W, int &ix0,
                                           int &ix1, int &iy0, int &iy1) {
  T x0, y0, x1, y1;
  src.get(tf, x0, y0, x1, y1);
  exact_axis(x0, x1, m, W, false, ix0, ix1);
  exact_axis(y0, y1, m, H, true, iy0, iy1);
  return ix0 <= ix1 && iy0 <= iy1;
}

template <typename T, int MAXD>
struct GatherAcc {
  T gi[6];
  T gf[3 * MAXD];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int q = 0; q < 6; q++) gi[q] = (T)0;
#pragma unroll
    for (int q = 0; q < 3 * MAXD; q++) gf[q] = (T)0;
  }
  // one pixel won by the face: the reference's per-pixel terms (rasterization_cuda.cu:262-399)
  __device__ __forceinline__ void add(const T v[6], const T *c, int D, T w_a, T w_b, T w_c, const T *g, float eps) {
    BaryGrad<T> bg;
    bg.init(v, w_a, w_b, w_c, eps);
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < D) {
        const T gd = g[d];
        gf[d] += gd * w_a;
        gf[MAXD + d] += gd * w_b;
        gf[2 * MAXD + d] += gd * w_c;
        T o[6];
        bg.terms(gd, c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
        for (int q = 0; q < 6; q++) gi[q] += o[q];
      }
    }
  }
};

template <typename T, int MAXD>
__global__ void __launch_bounds__(256) rasterize_bwd_gather_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, const uint8_t *__restrict__ valid,
    const T *__restrict__ nz, int B, int H, int W, int F, int D, float m, float eps, T *__restrict__ grad_fvi,
    T *__restrict__ grad_ffeat, int *__restrict__ big, int *__restrict__ nbig) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t tf = t / LPF;  // LPF consecutive lanes per face (whole groups per wave)
  const int s = (int)(t % LPF);
  const bool in = tf < (int64_t)B * F;
  const int b = in ? (int)(tf / F) : 0;
  const int64_t f = tf - (int64_t)b * F;
  const RastSrc<T> src{fvi, valid, (T)m, nz};
  GatherAcc<T, MAXD> acc;
  acc.zero();
  int ix0, ix1, iy0, iy1;
  bool queued = false;
  if (in && src.valid(tf) && face_range(src, tf, m, H, W, ix0, ix1, iy0, iy1)) {
    if ((int64_t)(ix1 - ix0 + 1) * (iy1 - iy0 + 1) > VIS_SMALL_AREA) {
      queued = true;
      if (s == 0) big[atomicAdd(nbig, 1)] = (int)tf;
    } else {
      T v[6];
#pragma unroll
      for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
      const T *c = feat + tf * 3 * D;
      const int64_t pbase = (int64_t)b * H * W;
      RangeWalk rw(ix0, ix1, iy0, iy1, s);
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
  for (int o = 1; o < LPF; o <<= 1) {
#pragma unroll
    for (int q = 0; q < 6; q++) acc.gi[q] += __shfl_xor(acc.gi[q], o);
#pragma unroll
    for (int q = 0; q < 3 * MAXD; q++) acc.gf[q] += __shfl_xor(acc.gf[q], o);
  }
  if (!in || queued) return;  // queued faces are written by the workgroup kernel
  // lane s writes the values q = s, s+LPF, ...
#pragma unroll
  for (int q = 0; q < 6 + 3 * MAXD; q++) {
    if (q % LPF != s) continue;
    if (q < 6) {
      grad_fvi[tf * 6 + q] = acc.gi[q];
    } else {
      const int r = q - 6, ii = r / MAXD, d = r % MAXD;
      if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = acc.gf[r];
    }
  }
}

// one 256-thread workgroup per large face; block reduction of the per-thread partials
template <typename T, int MAXD>
__global__ void __launch_bounds__(256) rasterize_bwd_bigface_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, const uint8_t *__restrict__ valid,
    const T *__restrict__ nz, int H, int W, int F, int D, float m, float eps, T *__restrict__ grad_fvi,
    T *__restrict__ grad_ffeat, const int *__restrict__ big, const int *__restrict__ nbig) {
  __shared__ T red[256];
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
    for (int q = 0; q < 6 + 3 * MAXD; q++) {
      red[threadIdx.x] = q < 6 ? acc.gi[q] : acc.gf[q - 6];
      __syncthreads();
      for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        if (q < 6) {
          grad_fvi[tf * 6 + q] = red[0];
        } else {
          const int r = q - 6, ii = r / MAXD, d = r % MAXD;
          if (d < D) grad_ffeat[tf * 3 * D + ii * D + d] = red[0];
        }
      }
      __syncthreads();
    }
  }
}

template <typename T>
static int rasterize_bwd(int B, int H, int W, int F, int D, const void *grad, const int64_t *face_idx,
                         const void *w, const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                         hipStream_t st) {
  KL_CHECK_RC(fill_async(gfvi, 0, sizeof(T) * (size_t)B * F * 6, st));
  KL_CHECK_RC(fill_async(gfeat, 0, sizeof(T) * (size_t)B * F * 3 * D, st));
  const int64_t total = (int64_t)B * H * W;
  if (total == 0) return KL_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(total, 256), 65536);
  hipLaunchKernelGGL(rasterize_bwd_kernel<T>, dim3(blocks), dim3(256), 0, st, (const T *)grad, face_idx,
                     (const T *)w, (const T *)fvi, (const T *)feat, B, H, W, F, D, eps, (T *)gfvi, (T *)gfeat);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

// nbig: a zeroed int (zero_nbig: this call zeroes it first).
template <typename T, int MAXD>
static int rasterize_bwd_gather_maxd(int B, int H, int W, int F, int D, const T *grad, const int64_t *face_idx,
                                     const T *w, const T *fvi, const T *feat, const uint8_t *valid, const T *nz,
                                     float m, float eps, T *gfvi, T *gfeat, int *big, int *nbig, bool zero_nbig,
                                     hipStream_t st) {
  if (zero_nbig) KL_CHECK_RC(fill_async(nbig, 0, sizeof(int), st));
  const int64_t nf = (int64_t)B * F;
  hipLaunchKernelGGL((rasterize_bwd_gather_kernel<T, MAXD>), dim3((unsigned)cdiv(nf * LPF, 256)), dim3(256), 0, st, grad,
                     face_idx, w, fvi, feat, valid, nz, B, H, W, F, D, m, eps, gfvi, gfeat, big, nbig);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL((rasterize_bwd_bigface_kernel<T, MAXD>), dim3(256), dim3(256), 0, st, grad, face_idx, w, fvi,
                     feat, valid, nz, H, W, F, D, m, eps, gfvi, gfeat, big, nbig);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

// The gather backward writes every face's gradient (zeros where nothing was won).
// nbig == nullptr: the big-face counter lives at the head of the workspace and is zeroed here.
template <typename T>
static int rasterize_bwd_gather(int B, int H, int W, int F, int D, const void *grad, const int64_t *face_idx,
                                const void *w, const void *fvi, const void *feat, const uint8_t *valid, const T *nz,
                                float m, float eps, void *gfvi, void *gfeat, void *ws, size_t ws_bytes, int *nbig,
                                hipStream_t st) {
  const int64_t nf = (int64_t)B * F;
  if (nf == 0) return KL_OK;
  KL_REQUIRE(ws_bytes >= (size_t)(nf + 1) * sizeof(int), "rasterize backward: workspace too small");
  KL_REQUIRE(nf < ((int64_t)1 << 31), "rasterize backward: too many faces");
  const bool zero = nbig == nullptr;
  if (zero) nbig = reinterpret_cast<int *>(ws);
  int *big = reinterpret_cast<int *>(ws) + 1;
  const T *g = (const T *)grad;
  const T *wt = (const T *)w;
  const T *fv = (const T *)fvi;
  const T *ft = (const T *)feat;
  if (D <= 4)
    return rasterize_bwd_gather_maxd<T, 4>(B, H, W, F, D, g, face_idx, wt, fv, ft, valid, nz, m, eps, (T *)gfvi,
                                           (T *)gfeat, big, nbig, zero, st);
  if (D <= 8)
    return rasterize_bwd_gather_maxd<T, 8>(B, H, W, F, D, g, face_idx, wt, fv, ft, valid, nz, m, eps, (T *)gfvi,
                                           (T *)gfeat, big, nbig, zero, st);
  // wide features: the scatter kernel
  return rasterize_bwd<T>(B, H, W, F, D, grad, face_idx, w, fvi, feat, eps, gfvi, gfeat, st);
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
  const size_t fwd = RastWs(batch, height, width, (int64_t)batch * num_faces).bytes;
  const size_t bwd = ((size_t)batch * num_faces + 1) * sizeof(int);
  return fwd > bwd ? fwd : bwd;
}

extern "C" int kl_dibr_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int num_faces,
                                         int feat_dim, const void *fvz, const void *fvi, const void *feat,
                                         const uint8_t *valid_faces, const void *fnz, float multiplier, float eps,
                                         void *out_feat, int64_t *out_idx, void *out_w, void *ws, size_t ws_bytes,
                                         kl_stream stream) {
  const int64_t nf = (int64_t)batch * num_faces;
  if (dtype == KL_F32)
    return launch_rast_fwd<float>(RastSrc<float>{(const float *)fvi, valid_faces, (float)multiplier,
                                                 (const float *)fnz}, height, width,
                                  batch, feat_dim, nf, nf, (const float *)fvz, (const float *)feat, nullptr,
                                  num_faces, multiplier, eps, (float *)out_feat, out_idx, (float *)out_w, ws, ws_bytes,
                                  S(stream));
  if (dtype == KL_F64)
    return launch_rast_fwd<double>(RastSrc<double>{(const double *)fvi, valid_faces, (double)multiplier,
                                                   (const double *)fnz}, height,
                                   width, batch, feat_dim, nf, nf, (const double *)fvz, (const double *)feat, nullptr,
                                   num_faces, multiplier, eps, (double *)out_feat, out_idx, (double *)out_w, ws,
                                   ws_bytes, S(stream));
  set_error("dibr_rasterize_forward not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_rasterize_backward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                     int feat_dim, const void *grad, const int64_t *face_idx, const void *w,
                                     const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                                     kl_stream stream) {
  if (dtype == KL_F32)
    return rasterize_bwd<float>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat, eps,
                                gfvi, gfeat, S(stream));
  if (dtype == KL_F64)
    return rasterize_bwd<double>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat, eps,
                                 gfvi, gfeat, S(stream));
  set_error("rasterize_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_rasterize_backward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                          int feat_dim, const void *grad, const int64_t *face_idx, const void *w,
                                          const void *fvi, const void *feat, const uint8_t *valid_faces,
                                          const void *fnz, float multiplier, float eps, void *gfvi, void *gfeat,
                                          int *scratch, void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return rasterize_bwd_gather<float>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat,
                                       valid_faces, (const float *)fnz, multiplier, eps, gfvi, gfeat, ws, ws_bytes,
                                       scratch, S(stream));
  if (dtype == KL_F64)
    return rasterize_bwd_gather<double>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat,
                                        valid_faces, (const double *)fnz, multiplier, eps, gfvi, gfeat, ws, ws_bytes,
                                        scratch, S(stream));
  set_error("dibr_rasterize_backward not implemented for this dtype");
  return KL_E_INVALID;
}

// ---------------------------------------------------------------- dibr_rasterization
// The whole of dibr_rasterization (dibr.py:119-209) in one call per direction: rasterize
// with valid = face_normals_z >= 0 evaluated in-kernel, then the soft mask of the
// compact path (softtile.hip) on the rasterizer's face index.  The backward runs the
// gather (which writes every face's gradient) and adds the soft-mask terms onto it.
// The state's scratch int is the gather's big-face counter: the forward zeroes it and
// the soft-mask backward re-zeroes it, so the backward needs no fill of its own.
namespace kl {
template <typename T>
static int dibr_fwd(int B, int H, int W, int F, int D, int K, const T *fvz, const T *fvi, const T *feat, const T *fnz,
                    float sigmainv, double pad, float m, float eps, T *out_feat, int64_t *out_idx, T *out_w,
                    T *out_mask, const SoftState<T> &s, void *ws, size_t ws_bytes, hipStream_t st) {
  const int64_t nf = (int64_t)B * F;
  KL_CHECK_RC(launch_rast_fwd<T>(RastSrc<T>{fvi, nullptr, (T)m, fnz}, H, W, B, D, nf, nf, fvz, feat, nullptr, F, m,
                                 eps, out_feat, out_idx, out_w, ws, ws_bytes, st));
  return soft_tile_forward<T>(B, H, W, F, K, fvi, out_idx, sigmainv, pad, m, out_mask, s, ws, ws_bytes, st);
}

template <typename T>
static int dibr_bwd(int B, int H, int W, int F, int D, int K, const T *grad_feat, const T *grad_mask,
                    const int64_t *face_idx, const T *w, const T *fvi, const T *feat, const T *fnz, const T *mask,
                    const SoftState<T> &s, float sigmainv, float m, float eps, T *gfvi, T *gfeat, void *ws,
                    size_t ws_bytes, hipStream_t st) {
  KL_REQUIRE(D <= 8, "dibr_rasterization backward: feature dimension > 8 is not supported by the fused path");
  KL_CHECK_RC(rasterize_bwd_gather<T>(B, H, W, F, D, grad_feat, face_idx, w, fvi, feat, nullptr, fnz, m, eps, gfvi,
                                      gfeat, ws, ws_bytes, s.scratch, st));
  return soft_tile_backward<T>(B, H, W, F, K, grad_mask, mask, s, fvi, sigmainv, m, gfvi, true, ws, ws_bytes, st);
}
}  // namespace kl

extern "C" size_t kl_dibr_workspace_bytes(int batch, int height, int width, int num_faces) {
  const size_t a = kl_dibr_rasterize_workspace_bytes(batch, height, width, num_faces);
  const size_t b = soft_tile_ws_bytes(batch, height, width, num_faces);
  return a > b ? a : b;
}

extern "C" size_t kl_dibr_bwd_workspace_bytes(int batch, int height, int width, int num_faces, int knum) {
  const size_t a = kl_dibr_rasterize_workspace_bytes(batch, height, width, num_faces);
  const size_t b = soft_tile_bwd_ws_bytes(batch, height, width, knum);
  return a > b ? a : b;
}

extern "C" int kl_dibr_forward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim,
                               int knum, const void *fvz, const void *fvi, const void *feat, const void *fnz,
                               float sigmainv, double bbox_pad, float multiplier, float eps, void *out_feat,
                               int64_t *out_idx, void *out_w, void *out_mask, uint8_t *hits, uint32_t *rec_face,
                               void *rec_prob, int *seg_tot, int *scratch, void *ws, size_t ws_bytes,
                               kl_stream stream) {
  if (dtype == KL_F32)
    return dibr_fwd<float>(batch, height, width, num_faces, feat_dim, knum, (const float *)fvz, (const float *)fvi,
                           (const float *)feat, (const float *)fnz, sigmainv, bbox_pad, multiplier, eps,
                           (float *)out_feat, out_idx, (float *)out_w, (float *)out_mask,
                           SoftState<float>{hits, rec_face, (float *)rec_prob, seg_tot, scratch}, ws, ws_bytes,
                           S(stream));
  if (dtype == KL_F64)
    return dibr_fwd<double>(batch, height, width, num_faces, feat_dim, knum, (const double *)fvz, (const double *)fvi,
                            (const double *)feat, (const double *)fnz, sigmainv, bbox_pad, multiplier, eps,
                            (double *)out_feat, out_idx, (double *)out_w, (double *)out_mask,
                            SoftState<double>{hits, rec_face, (double *)rec_prob, seg_tot, scratch}, ws, ws_bytes,
                            S(stream));
  set_error("dibr_rasterization not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_backward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim,
                                int knum, const void *grad_feat, const void *grad_mask, const int64_t *face_idx,
                                const void *w, const void *fvi, const void *feat, const void *fnz, const void *mask,
                                const uint8_t *hits, const uint32_t *rec_face, const void *rec_prob,
                                const int *seg_tot, float sigmainv, float multiplier, float eps, void *gfvi,
                                void *gfeat, int *scratch, void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return dibr_bwd<float>(
        batch, height, width, num_faces, feat_dim, knum, (const float *)grad_feat, (const float *)grad_mask, face_idx,
        (const float *)w, (const float *)fvi, (const float *)feat, (const float *)fnz, (const float *)mask,
        SoftState<float>{(uint8_t *)hits, (uint32_t *)rec_face, (float *)rec_prob, (int *)seg_tot, scratch},
        sigmainv, multiplier, eps, (float *)gfvi, (float *)gfeat, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return dibr_bwd<double>(
        batch, height, width, num_faces, feat_dim, knum, (const double *)grad_feat, (const double *)grad_mask,
        face_idx, (const double *)w, (const double *)fvi, (const double *)feat, (const double *)fnz,
        (const double *)mask,
        SoftState<double>{(uint8_t *)hits, (uint32_t *)rec_face, (double *)rec_prob, (int *)seg_tot, scratch},
        sigmainv, multiplier, eps, (double *)gfvi, (double *)gfeat, ws, ws_bytes, S(stream));
  set_error("dibr_rasterization backward not implemented for this dtype");
  return KL_E_INVALID;
}
