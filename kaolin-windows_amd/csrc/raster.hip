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
// Backward (rasterization_cuda.cu:238-442): one thread per pixel, analytic d(bary)/d(v)
// with k3 += copysign(eps); accumulation by float atomics into the face arrays.
#include "binning.h"

namespace kl {

template <typename T>
struct RastState {
  T max_z0, w0, w1, w2;
  int max_f;
};

template <typename T>
__global__ void __launch_bounds__(256) rasterize_fwd_kernel(
    const T *__restrict__ fvz, const T *__restrict__ fvi, const T *__restrict__ bboxes,
    const T *__restrict__ feat, const int64_t *__restrict__ first_idx, const uint32_t *__restrict__ bitmap,
    BinGeom g, int D, float multiplier, float eps, T *__restrict__ out_feat, int64_t *__restrict__ out_idx,
    T *__restrict__ out_w) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  const int tx = blockIdx.x;
  const int H = g.height, W = g.width;
  if (j >= H) return;
  const int i = tx * TILE_W + lane;
  const bool px_valid = i < W;
  const int64_t f0 = first_idx[b], f1 = first_idx[b + 1];

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
      const bool fv = f < f1;
      T bx0 = 0, by0 = 0, bx1 = 0, by1 = 0;
      if (fv) {
        const T *bb = bboxes + f * 4;
        bx0 = bb[0];
        by0 = bb[1];
        bx1 = bb[2];
        by1 = bb[3];
      }
      // may this face cover some pixel centre of the row segment?  (NaN-safe: NaN never rejects)
      const bool touch = fv && !(y0 < by0 || y0 >= by1 || sxhi < bx0 || sxlo >= bx1);
      uint64_t mask = ballot(touch);
      if (!mask) continue;
      T ax = 0, ay = 0, bxv = 0, byv = 0, cx = 0, cy = 0, az = 0, bz = 0, cz = 0;
      if (touch) {
        const T *v = fvi + f * 6;
        ax = v[0]; ay = v[1]; bxv = v[2]; byv = v[3]; cx = v[4]; cy = v[5];
        const T *z = fvz + f * 3;
        az = z[0]; bz = z[1]; cz = z[2];
      }
      while (mask) {
        const int s = __builtin_ctzll(mask);
        mask &= mask - 1;
        const T xmin = bcast(bx0, s), ymin = bcast(by0, s), xmax = bcast(bx1, s), ymax = bcast(by1, s);
        const T Ax = bcast(ax, s), Ay = bcast(ay, s), Bx = bcast(bxv, s), By = bcast(byv, s);
        const T Cx = bcast(cx, s), Cy = bcast(cy, s);
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
    const T *v = fvi + tf * 6;
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
    const T dw1dax = -(dw1dm + dw1dn + dw1ds), dw1day = -(dw1dp + dw1dq + dw1dt);
    const T dw1dbx = dw1dm, dw1dby = dw1dp, dw1dcx = dw1dn, dw1dcy = dw1dq;
    const T dw2dax = -(dw2dm + dw2dn + dw2ds), dw2day = -(dw2dp + dw2dq + dw2dt);
    const T dw2dbx = dw2dm, dw2dby = dw2dp, dw2dcx = dw2dn, dw2dcy = dw2dq;
    const T *c = feat + tf * 3 * D;
    T *gv = grad_fvi + tf * 6;
    for (int d = 0; d < D; d++) {
      const T c0 = c[d], c1 = c[D + d], c2 = c[2 * D + d];
      const T dIdax = (c1 - c0) * dw1dax + (c2 - c0) * dw2dax;
      const T dIday = (c1 - c0) * dw1day + (c2 - c0) * dw2day;
      const T dIdbx = (c1 - c0) * dw1dbx + (c2 - c0) * dw2dbx;
      const T dIdby = (c1 - c0) * dw1dby + (c2 - c0) * dw2dby;
      const T dIdcx = (c1 - c0) * dw1dcx + (c2 - c0) * dw2dcx;
      const T dIdcy = (c1 - c0) * dw1dcy + (c2 - c0) * dw2dcy;
      const T dldI = g[d] / (k3 * k3);
      atomicAdd(gv + 0, dldI * dIdax);
      atomicAdd(gv + 1, dldI * dIday);
      atomicAdd(gv + 2, dldI * dIdbx);
      atomicAdd(gv + 3, dldI * dIdby);
      atomicAdd(gv + 4, dldI * dIdcx);
      atomicAdd(gv + 5, dldI * dIdcy);
    }
  }
}

template <typename T>
static int rasterize_fwd(int H, int W, int B, int64_t Nv, int D, int64_t maxf, const void *fvz, const void *fvi,
                         const void *bbox, const void *feat, const int64_t *first_idx, float m, float eps,
                         void *out_feat, int64_t *out_idx, void *out_w, void *ws, size_t ws_bytes,
                         hipStream_t st) {
  (void)Nv;
  BinGeom g = make_bin_geom(B, H, W, maxf);
  KL_REQUIRE(ws_bytes >= g.bytes(), "packed_rasterize_forward: workspace too small");
  if (B == 0 || H == 0 || W == 0) return KL_OK;
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(ws);
  int rc = launch_binning<T>((const T *)bbox, first_idx, 0, g, m, bitmap, st);
  if (rc) return rc;
  dim3 grid(g.tiles_x, (unsigned)cdiv(H, 4), B);
  hipLaunchKernelGGL(rasterize_fwd_kernel<T>, grid, dim3(256), 0, st, (const T *)fvz, (const T *)fvi,
                     (const T *)bbox, (const T *)feat, first_idx, bitmap, g, D, m, eps, (T *)out_feat, out_idx,
                     (T *)out_w);
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
  if (dtype == KL_F32)
    return rasterize_fwd<float>(height, width, batch, num_faces, feat_dim, max_faces_per_mesh, fvz, fvi, bbox,
                                feat, first_idx, multiplier, eps, out_feat, out_idx, out_w, ws, ws_bytes,
                                S(stream));
  if (dtype == KL_F64)
    return rasterize_fwd<double>(height, width, batch, num_faces, feat_dim, max_faces_per_mesh, fvz, fvi, bbox,
                                 feat, first_idx, multiplier, eps, out_feat, out_idx, out_w, ws, ws_bytes,
                                 S(stream));
  set_error("packed_rasterize_forward_cuda not implemented for this dtype");
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
