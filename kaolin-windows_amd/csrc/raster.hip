// raster.hip -- packed_rasterize_forward / rasterize_backward for gfx950.
//
// Forward (reference: rasterization_cuda.cu:43-236, a per-pixel walk over ALL faces
// of the mesh with the batch looped serially in every thread): here faces are first
// binned to 64x8 pixel tiles (binning.h), then one wave per 64-pixel row segment walks
// only the candidate 64-face chunks of its tile, in ascending face order.  Per chunk
// the wave loads the 64 faces once (one per lane, coalesced), ballots which of them can
// touch its row, and broadcasts each surviving face through the scalar unit
// (v_readlane) to all 64 pixel lanes.  The per-pixel arithmetic is the reference's,
// statement for statement (bbox reject, edge functions, copysign(eps) normalisation,
// strict depth test), so face index / weights / features are bit-identical to the
// oracle for the same inputs.
//
// Two entry points share that walk:
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
#include "binning.h"

namespace kl {

template <typename T, typename Src>
__global__ void __launch_bounds__(256) rasterize_fwd_kernel(
    Src src, const T *__restrict__ fvz, const T *__restrict__ feat, const int64_t *__restrict__ first_idx,
    int faces_per_mesh, const uint32_t *__restrict__ bitmap, BinGeom g, int D, float multiplier, float eps,
    T *__restrict__ out_feat, int64_t *__restrict__ out_idx, T *__restrict__ out_w) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  const int tx = blockIdx.x;
  const int H = g.height, W = g.width;
  if (j >= H) return;
  const int i = tx * TILE_W + lane;
  const bool px_valid = i < W;
  int64_t f0, f1;
  if (first_idx) {
    f0 = first_idx[b];
    f1 = first_idx[b + 1];
  } else {
    f0 = (int64_t)b * faces_per_mesh;
    f1 = f0 + faces_per_mesh;
  }

  const T x0 = pix_x<T>(multiplier, W, px_valid ? i : W - 1);
  const T y0 = pix_y<T>(multiplier, H, j);
  // pixel-centre extent of this row segment (for the per-chunk ballot)
  const int ilast = min(tx * TILE_W + 63, W - 1);
  const T xlo = pix_x<T>(multiplier, W, tx * TILE_W);
  const T xhi = pix_x<T>(multiplier, W, ilast);
  const T sxlo = xlo < xhi ? xlo : xhi, sxhi = xlo < xhi ? xhi : xlo;

  T max_z0 = -INFINITY, mw0 = 0, mw1 = 0, mw2 = 0;
  int64_t max_f = -1;

  const uint32_t *words = bitmap + ((size_t)(b * g.tiles_y + j / TILE_H) * g.tiles_x + tx) * g.words;
  for (int wi = 0; wi < g.words; wi++) {
    uint32_t word = words[wi];
    while (word) {
      const int c = wi * 32 + __builtin_ctz(word);
      word &= word - 1;
      const int64_t base = f0 + (int64_t)c * 64;
      const int64_t f = base + lane;
      const bool fv = f < f1 && src.valid(f);
      T bx0 = 0, by0 = 0, bx1 = 0, by1 = 0;
      if (fv) src.get(f, bx0, by0, bx1, by1);
      // may this face cover some pixel centre of the row segment?  (NaN-safe: NaN never rejects)
      const bool touch = fv && !(y0 < by0 || y0 >= by1 || sxhi < bx0 || sxlo >= bx1);
      uint64_t mask = ballot(touch);
      if (!mask) continue;
      T v[6] = {0, 0, 0, 0, 0, 0};
      T az = 0, bz = 0, cz = 0;
      if (touch) {
        src.verts(f, v);
        const T *z = fvz + f * 3;
        az = z[0];
        bz = z[1];
        cz = z[2];
      }
      while (mask) {
        const int s = __builtin_ctzll(mask);
        mask &= mask - 1;
        const T xmin = bcast(bx0, s), ymin = bcast(by0, s), xmax = bcast(bx1, s), ymax = bcast(by1, s);
        const T Ax = bcast(v[0], s), Ay = bcast(v[1], s), Bx = bcast(v[2], s), By = bcast(v[3], s);
        const T Cx = bcast(v[4], s), Cy = bcast(v[5], s);
        const T Az = bcast(az, s), Bz = bcast(bz, s), Cz = bcast(cz, s);
        if (x0 < xmin || x0 >= xmax || y0 < ymin || y0 >= ymax) continue;
        const T aex = Ax - x0, aey = Ay - y0;
        const T bex = Bx - x0, bey = By - y0;
        const T cex = Cx - x0, cey = Cy - y0;
        T w0 = bex * cey - bey * cex;
        T w1 = cex * aey - cey * aex;
        T w2 = aex * bey - aey * bex;
        T norm = w0 + w1 + w2;
        norm = (T)((double)norm + copysign((double)eps, (double)norm));
        w0 /= norm;
        w1 /= norm;
        w2 /= norm;
        if (w0 < (T)0 || w1 < (T)0 || w2 < (T)0) continue;
        const T z0 = w0 * Az + w1 * Bz + w2 * Cz;
        if (z0 <= max_z0) continue;
        max_z0 = z0;
        max_f = base + s;
        mw0 = w0;
        mw1 = w1;
        mw2 = w2;
      }
    }
  }
  if (!px_valid) return;
  const size_t pix = ((size_t)b * H + j) * W + i;
  out_idx[pix] = max_f >= 0 ? max_f - f0 : -1;
  out_w[pix * 3 + 0] = mw0;
  out_w[pix * 3 + 1] = mw1;
  out_w[pix * 3 + 2] = mw2;
  if (max_f >= 0) {
    const T *r = feat + (size_t)max_f * 3 * D;
    for (int d = 0; d < D; d++) out_feat[pix * D + d] = mw0 * r[d] + mw1 * r[D + d] + mw2 * r[2 * D + d];
  } else {
    for (int d = 0; d < D; d++) out_feat[pix * D + d] = (T)0;
  }
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
constexpr int GATHER_MAX_AREA = 1024;  // faces with larger screen bboxes go to the WG path

template <typename T>
__device__ __forceinline__ bool conservative_range(const T v[6], int H, int W, int &ix0, int &ix1, int &iy0,
                                                   int &iy1) {
  const T xmin = tmin3(v[0], v[2], v[4]), xmax = tmax3(v[0], v[2], v[4]);
  const T ymin = tmin3(v[1], v[3], v[5]), ymax = tmax3(v[1], v[3], v[5]);
  // unscaled pixel centres: x(i) = (2i+1-W)/W ; the forward compared in x multiplier
  // space, which differs by rounding only -> +-1 pixel margin inside axis_range.
  axis_range((double)xmin, (double)xmax, 1.0 / (double)W, W, false, ix0, ix1);
  axis_range((double)ymin, (double)ymax, 1.0 / (double)H, H, true, iy0, iy1);
  return ix0 <= ix1 && iy0 <= iy1;
}

template <typename T, int MAXD>
__global__ void __launch_bounds__(256) rasterize_bwd_gather_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, int B, int H, int W, int F, int D, float eps,
    T *__restrict__ grad_fvi, T *__restrict__ grad_ffeat, int *__restrict__ big, int *__restrict__ nbig) {
  const int64_t tf = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (tf >= (int64_t)B * F) return;
  const int b = (int)(tf / F);
  const int64_t f = tf - (int64_t)b * F;
  T v[6];
#pragma unroll
  for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
  int ix0, ix1, iy0, iy1;
  T gi[6] = {0, 0, 0, 0, 0, 0};
  T gf[3 * MAXD];
#pragma unroll
  for (int q = 0; q < 3 * MAXD; q++) gf[q] = (T)0;
  if (conservative_range(v, H, W, ix0, ix1, iy0, iy1)) {
    const int area = (ix1 - ix0 + 1) * (iy1 - iy0 + 1);
    if (area > GATHER_MAX_AREA) {
      big[atomicAdd(nbig, 1)] = (int)tf;
      return;  // the WG kernel writes this face
    }
    const T *c = feat + tf * 3 * D;
    for (int j = iy0; j <= iy1; j++) {
      for (int i = ix0; i <= ix1; i++) {
        const int64_t p = ((int64_t)b * H + j) * W + i;
        if (face_idx[p] != f) continue;
        const T w_a = wts[p * 3 + 0], w_b = wts[p * 3 + 1], w_c = wts[p * 3 + 2];
        const T *g = grad_feat + p * D;
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
    }
  }
#pragma unroll
  for (int q = 0; q < 6; q++) grad_fvi[tf * 6 + q] = gi[q];
#pragma unroll
  for (int d = 0; d < MAXD; d++) {
    if (d < D) {
      grad_ffeat[tf * 3 * D + d] = gf[d];
      grad_ffeat[tf * 3 * D + D + d] = gf[MAXD + d];
      grad_ffeat[tf * 3 * D + 2 * D + d] = gf[2 * MAXD + d];
    }
  }
}

// one 256-thread workgroup per large face; block reduction of the per-thread partials
template <typename T, int MAXD>
__global__ void __launch_bounds__(256) rasterize_bwd_bigface_kernel(
    const T *__restrict__ grad_feat, const int64_t *__restrict__ face_idx, const T *__restrict__ wts,
    const T *__restrict__ fvi, const T *__restrict__ feat, int H, int W, int F, int D, float eps,
    T *__restrict__ grad_fvi, T *__restrict__ grad_ffeat, const int *__restrict__ big, const int *__restrict__ nbig) {
  __shared__ T red[256];
  const int n = *nbig;
  for (int k = blockIdx.x; k < n; k += gridDim.x) {
    const int64_t tf = big[k];
    const int b = (int)(tf / F);
    const int64_t f = tf - (int64_t)b * F;
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[tf * 6 + q];
    int ix0, ix1, iy0, iy1;
    conservative_range(v, H, W, ix0, ix1, iy0, iy1);
    const int w = ix1 - ix0 + 1;
    const int64_t area = (int64_t)w * (iy1 - iy0 + 1);
    T acc[6 + 3 * MAXD];
#pragma unroll
    for (int q = 0; q < 6 + 3 * MAXD; q++) acc[q] = (T)0;
    const T *c = feat + tf * 3 * D;
    for (int64_t e = threadIdx.x; e < area; e += blockDim.x) {
      const int j = iy0 + (int)(e / w), i = ix0 + (int)(e % w);
      const int64_t p = ((int64_t)b * H + j) * W + i;
      if (face_idx[p] != f) continue;
      const T w_a = wts[p * 3 + 0], w_b = wts[p * 3 + 1], w_c = wts[p * 3 + 2];
      const T *g = grad_feat + p * D;
      BaryGrad<T> bg;
      bg.init(v, w_a, w_b, w_c, eps);
#pragma unroll
      for (int d = 0; d < MAXD; d++) {
        if (d < D) {
          const T gd = g[d];
          acc[6 + d] += gd * w_a;
          acc[6 + MAXD + d] += gd * w_b;
          acc[6 + 2 * MAXD + d] += gd * w_c;
          T o[6];
          bg.terms(gd, c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
          for (int q = 0; q < 6; q++) acc[q] += o[q];
        }
      }
    }
    for (int q = 0; q < 6 + 3 * MAXD; q++) {
      red[threadIdx.x] = acc[q];
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

template <typename T, typename Src>
static int launch_rast_fwd(Src src, int H, int W, int B, int D, int64_t maxf, const T *fvz, const T *feat,
                           const int64_t *first_idx, int faces_per_mesh, float m, float eps, T *out_feat,
                           int64_t *out_idx, T *out_w, void *ws, size_t ws_bytes, hipStream_t st) {
  BinGeom g = make_bin_geom(B, H, W, maxf);
  KL_REQUIRE(ws_bytes >= g.bytes(), "rasterize forward: workspace too small");
  if (B == 0 || H == 0 || W == 0) return KL_OK;
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(ws);
  int rc = launch_binning<T, Src>(src, first_idx, faces_per_mesh, g, m, bitmap, st);
  if (rc) return rc;
  dim3 grid(g.tiles_x, (unsigned)cdiv(H, 4), B);
  hipLaunchKernelGGL((rasterize_fwd_kernel<T, Src>), grid, dim3(256), 0, st, src, fvz, feat, first_idx,
                     faces_per_mesh, bitmap, g, D, m, eps, out_feat, out_idx, out_w);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
static int rasterize_bwd(int B, int H, int W, int F, int D, const void *grad, const int64_t *face_idx,
                         const void *w, const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                         hipStream_t st) {
  KL_CHECK_HIP(hipMemsetAsync(gfvi, 0, sizeof(T) * (size_t)B * F * 6, st));
  KL_CHECK_HIP(hipMemsetAsync(gfeat, 0, sizeof(T) * (size_t)B * F * 3 * D, st));
  const int64_t total = (int64_t)B * H * W;
  if (total == 0) return KL_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(total, 256), 65536);
  hipLaunchKernelGGL(rasterize_bwd_kernel<T>, dim3(blocks), dim3(256), 0, st, (const T *)grad, face_idx,
                     (const T *)w, (const T *)fvi, (const T *)feat, B, H, W, F, D, eps, (T *)gfvi, (T *)gfeat);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T, int MAXD>
static int rasterize_bwd_gather_maxd(int B, int H, int W, int F, int D, const T *grad, const int64_t *face_idx,
                                     const T *w, const T *fvi, const T *feat, float eps, T *gfvi, T *gfeat,
                                     int *big, int *nbig, hipStream_t st) {
  KL_CHECK_HIP(hipMemsetAsync(nbig, 0, sizeof(int), st));
  const int64_t nf = (int64_t)B * F;
  hipLaunchKernelGGL((rasterize_bwd_gather_kernel<T, MAXD>), dim3((unsigned)cdiv(nf, 256)), dim3(256), 0, st, grad,
                     face_idx, w, fvi, feat, B, H, W, F, D, eps, gfvi, gfeat, big, nbig);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL((rasterize_bwd_bigface_kernel<T, MAXD>), dim3(256), dim3(256), 0, st, grad, face_idx, w, fvi,
                     feat, H, W, F, D, eps, gfvi, gfeat, big, nbig);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
static int rasterize_bwd_gather(int B, int H, int W, int F, int D, const void *grad, const int64_t *face_idx,
                                const void *w, const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                                void *ws, size_t ws_bytes, hipStream_t st) {
  const int64_t nf = (int64_t)B * F;
  if (nf == 0) return KL_OK;
  KL_REQUIRE(ws_bytes >= (size_t)(nf + 1) * sizeof(int), "rasterize backward: workspace too small");
  int *nbig = reinterpret_cast<int *>(ws);
  int *big = nbig + 1;
  const T *g = (const T *)grad;
  const T *wt = (const T *)w;
  const T *fv = (const T *)fvi;
  const T *ft = (const T *)feat;
  if (D <= 4)
    return rasterize_bwd_gather_maxd<T, 4>(B, H, W, F, D, g, face_idx, wt, fv, ft, eps, (T *)gfvi, (T *)gfeat, big,
                                           nbig, st);
  if (D <= 8)
    return rasterize_bwd_gather_maxd<T, 8>(B, H, W, F, D, g, face_idx, wt, fv, ft, eps, (T *)gfvi, (T *)gfeat, big,
                                           nbig, st);
  // wide features: the scatter kernel
  return rasterize_bwd<T>(B, H, W, F, D, grad, face_idx, w, fvi, feat, eps, gfvi, gfeat, st);
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_rasterize_workspace_bytes(int batch, int height, int width, int64_t max_faces_per_mesh) {
  return make_bin_geom(batch, height, width, max_faces_per_mesh).bytes();
}

extern "C" int kl_packed_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int64_t num_faces,
                                           int feat_dim, int64_t max_faces_per_mesh, const void *fvz,
                                           const void *fvi, const void *bbox, const void *feat,
                                           const int64_t *first_idx, float multiplier, float eps, void *out_feat,
                                           int64_t *out_idx, void *out_w, void *ws, size_t ws_bytes,
                                           kl_stream stream) {
  (void)num_faces;
  if (dtype == KL_F32)
    return launch_rast_fwd<float>(BboxSrc<float>{(const float *)bbox, (const float *)fvi}, height, width, batch,
                                  feat_dim, max_faces_per_mesh, (const float *)fvz, (const float *)feat, first_idx, 0,
                                  multiplier, eps, (float *)out_feat, out_idx, (float *)out_w, ws, ws_bytes,
                                  S(stream));
  if (dtype == KL_F64)
    return launch_rast_fwd<double>(BboxSrc<double>{(const double *)bbox, (const double *)fvi}, height, width, batch,
                                   feat_dim, max_faces_per_mesh, (const double *)fvz, (const double *)feat, first_idx,
                                   0, multiplier, eps, (double *)out_feat, out_idx, (double *)out_w, ws, ws_bytes,
                                   S(stream));
  set_error("packed_rasterize_forward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_dibr_rasterize_workspace_bytes(int batch, int height, int width, int num_faces) {
  const size_t fwd = make_bin_geom(batch, height, width, num_faces).bytes();
  const size_t bwd = ((size_t)batch * num_faces + 1) * sizeof(int);
  return fwd > bwd ? fwd : bwd;
}

extern "C" int kl_dibr_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int num_faces,
                                         int feat_dim, const void *fvz, const void *fvi, const void *feat,
                                         const uint8_t *valid_faces, float multiplier, float eps, void *out_feat,
                                         int64_t *out_idx, void *out_w, void *ws, size_t ws_bytes,
                                         kl_stream stream) {
  if (dtype == KL_F32)
    return launch_rast_fwd<float>(RastSrc<float>{(const float *)fvi, valid_faces, (float)multiplier}, height, width,
                                  batch, feat_dim, num_faces, (const float *)fvz, (const float *)feat, nullptr,
                                  num_faces, multiplier, eps, (float *)out_feat, out_idx, (float *)out_w, ws, ws_bytes,
                                  S(stream));
  if (dtype == KL_F64)
    return launch_rast_fwd<double>(RastSrc<double>{(const double *)fvi, valid_faces, (double)multiplier}, height,
                                   width, batch, feat_dim, num_faces, (const double *)fvz, (const double *)feat,
                                   nullptr, num_faces, multiplier, eps, (double *)out_feat, out_idx, (double *)out_w,
                                   ws, ws_bytes, S(stream));
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
                                          const void *fvi, const void *feat, float eps, void *gfvi, void *gfeat,
                                          void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return rasterize_bwd_gather<float>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat, eps,
                                       gfvi, gfeat, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return rasterize_bwd_gather<double>(batch, height, width, num_faces, feat_dim, grad, face_idx, w, fvi, feat, eps,
                                        gfvi, gfeat, ws, ws_bytes, S(stream));
  set_error("dibr_rasterize_backward not implemented for this dtype");
  return KL_E_INVALID;
}
