// softmask.hip -- DIB-R soft silhouette (dibr_soft_mask forward / backward) for gfx950.
//
// Reference forward (dibr_soft_mask_cuda.cu:27-184): for every pixel NOT covered by a
// rasterized face, walk ALL faces of its mesh in index order, keep the first `knum`
// whose enlarged bbox contains the pixel centre, and store for each its probability
// exp(-sigmainv * d^2 / m^2), index and distance type; mask = 1 - prod(1 - p).
//
// Here: faces are binned to 64x8 tiles (binning.h, order-preserving 64-face chunks);
// one wave owns a 64-pixel row segment, walks only candidate chunks in ascending order
// and stops as soon as every lane is covered or has `knum` hits.  Hits are staged in
// LDS ([slot][lane] layout, conflict-free), then the wave writes its whole contiguous
// output range (64 pixels x knum slots of prob / idx / type, padding included) with
// lane-contiguous stores -- the K-slot tensors are ~95% of the op's HBM traffic, so
// they are written exactly once and coalesced.  Per-hit arithmetic is the reference's,
// including its float/double promotions (EPS = 1e-7 is a double literal there).
//
// Backward (dibr_soft_mask_cuda.cu:230-353): one thread per pixel, atomics into the
// face-vertex gradient.
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

// LDS per wave: code[K][64] (face << 3 | type) + prob[K][64] + kid[64]
template <typename T, typename Src>
__global__ void __launch_bounds__(128) soft_mask_fwd_kernel(
    Src src, const int64_t *__restrict__ sel,
    const uint32_t *__restrict__ bitmap, BinGeom g, int F, int K, float sigmainv, float multiplier,
    T *__restrict__ out_mask, T *__restrict__ out_prob, int64_t *__restrict__ out_idx,
    uint8_t *__restrict__ out_type) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  const size_t per_wave = (size_t)K * 64 * (sizeof(uint32_t) + sizeof(T)) + 64 * sizeof(int);
  unsigned char *mine = smem + per_wave * wid;
  T *s_prob = reinterpret_cast<T *>(mine);
  uint32_t *s_code = reinterpret_cast<uint32_t *>(mine + (size_t)K * 64 * sizeof(T));
  int *s_kid = reinterpret_cast<int *>(mine + (size_t)K * 64 * (sizeof(T) + sizeof(uint32_t)));

  const int j = blockIdx.y * waves + wid;
  const int b = blockIdx.z;
  const int tx = blockIdx.x;
  const int H = g.height, W = g.width;
  if (j >= H) return;
  const int i = tx * TILE_W + lane;
  const bool px_valid = i < W;
  const size_t pix = ((size_t)b * H + j) * W + (px_valid ? i : W - 1);
  const bool covered = px_valid ? (sel[pix] >= 0) : true;

  const T x0 = pix_x<T>(multiplier, W, px_valid ? i : W - 1);
  const T y0 = pix_y<T>(multiplier, H, j);
  const int ilast = min(tx * TILE_W + 63, W - 1);
  const T xa = pix_x<T>(multiplier, W, tx * TILE_W), xb = pix_x<T>(multiplier, W, ilast);
  const T sxlo = xa < xb ? xa : xb, sxhi = xa < xb ? xb : xa;

  int kid = 0;
  bool active = !covered && K > 0;
  const uint32_t *words = bitmap + ((size_t)(b * g.tiles_y + j / TILE_H) * g.tiles_x + tx) * g.words;
  const int64_t f0 = (int64_t)b * F;
  for (int wi = 0; wi < g.words && ballot(active); wi++) {
    uint32_t word = words[wi];
    while (word && ballot(active)) {
      const int c = wi * 32 + __builtin_ctz(word);
      word &= word - 1;
      const int fl = c * 64 + lane;  // face index within the mesh
      const bool fv = fl < F;
      T bx0 = 0, by0 = 0, bx1 = 0, by1 = 0;
      if (fv) src.get(f0 + fl, bx0, by0, bx1, by1);
      const bool touch = fv && !(y0 < by0 || y0 >= by1 || sxhi < bx0 || sxlo >= bx1);
      uint64_t mask = ballot(touch);
      if (!mask) continue;
      T v[6] = {0, 0, 0, 0, 0, 0};
      if (touch) src.verts(f0 + fl, v);
      while (mask) {
        const int s = __builtin_ctzll(mask);
        mask &= mask - 1;
        const T xmin = bcast(bx0, s), ymin = bcast(by0, s), xmax = bcast(bx1, s), ymax = bcast(by1, s);
        T vb[6];
#pragma unroll
        for (int q = 0; q < 6; q++) vb[q] = bcast(v[q], s);
        if (active && !(x0 < xmin || x0 >= xmax || y0 < ymin || y0 >= ymax)) {
          T dsq;
          int edgeid;
          soft_dist<T>(x0, y0, vb, multiplier, dsq, edgeid);
          const T z = (T)sigmainv * dsq / (T)multiplier / (T)multiplier;
          const T pr = kl_exp<T>(-z);
          s_prob[kid * 64 + lane] = pr;
          s_code[kid * 64 + lane] = ((uint32_t)(c * 64 + s) << 3) | (uint32_t)(edgeid + 1);
          kid++;
          if (kid >= K) active = false;
        }
        if (!ballot(active)) break;
      }
    }
  }
  // soft mask value: 1 - prod(1 - p) in double, slot order (dibr_soft_mask_cuda.cu:174-182)
  if (px_valid) {
    T res;
    if (covered) {
      res = (T)1.0;
    } else {
      T allprob = (T)1.0;
      for (int k = 0; k < kid; k++) allprob = (T)((double)allprob * (1.0 - (double)s_prob[k * 64 + lane]));
      res = (T)(1.0 - (double)allprob);
    }
    out_mask[pix] = res;
  }
  s_kid[lane] = px_valid ? kid : 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // write this wave's contiguous slot range [pix0*K, (pix0+n)*K)
  const int n = min(64, W - tx * TILE_W);
  const size_t e0 = (((size_t)b * H + j) * W + (size_t)tx * TILE_W) * K;
  const int ne = n * K;
  for (int e = lane; e < ne; e += 64) {
    const int p = e / K, k = e - p * K;
    const bool hit = k < s_kid[p];
    const uint32_t code = hit ? s_code[k * 64 + p] : 0u;
    out_idx[e0 + e] = hit ? (int64_t)(code >> 3) : (int64_t)-1;
    out_prob[e0 + e] = hit ? s_prob[k * 64 + p] : (T)0;
    out_type[e0 + e] = (uint8_t)(code & 7u);
  }
}

template <typename T, bool SCALE>
__global__ void __launch_bounds__(256) soft_mask_bwd_kernel(
    const T *__restrict__ grad, const T *__restrict__ mask, const int64_t *__restrict__ sel,
    const T *__restrict__ prob, const int64_t *__restrict__ cidx, const uint8_t *__restrict__ ctype,
    const T *__restrict__ fvi, int B, int H, int W, int F, int K, float sigmainv, float multiplier,
    T *__restrict__ gfvi) {
  // SCALE: fvi holds unscaled coordinates, multiplied here exactly as the front-end's
  // `face_vertices_image * multiplier` (dibr.py:31) would have
  const T ms = (T)multiplier;
  auto V = [&](size_t k) -> T { return SCALE ? fvi[k] * ms : fvi[k]; };
  const int64_t npix = (int64_t)H * W;
  for (int64_t tp = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; tp < (int64_t)B * npix;
       tp += (int64_t)gridDim.x * blockDim.x) {
    if (sel[tp] >= 0) continue;
    const int b = (int)(tp / npix);
    const int rem = (int)(tp - (int64_t)b * npix);
    const int j = rem / W, i = rem - j * W;
    const T x0 = pix_x<T>(multiplier, W, i);
    const T y0 = pix_y<T>(multiplier, H, j);
    const T dLdp = grad[tp];
    const T allprob = mask[tp];
    const size_t pk = (size_t)tp * K;
    for (int k = 0; k < K; k++) {
      const int64_t f = cidx[pk + k];
      if (f < 0) break;
      const size_t s6 = ((size_t)b * F + f) * 6;
      const T pr = prob[pk + k];
      const T dLdz = (T)(-1.0 * (double)sigmainv * (double)dLdp * (1.0 - (double)allprob) /
                         (1.0 - (double)pr + SM_EPS) * (double)pr);
      const int edgeid = (int)ctype[pk + k] - 1;
      if (edgeid >= 3) {
        const size_t ps = s6 + (edgeid - 3) * 2;
        const T x1 = V(ps), y1 = V(ps + 1);
        const T dLdx1 = dLdz * (T)2 * (x1 - x0);
        const T dLdy1 = dLdz * (T)2 * (y1 - y0);
        atomicAdd(gfvi + ps + 0, dLdx1 / (T)multiplier);
        atomicAdd(gfvi + ps + 1, dLdy1 / (T)multiplier);
      } else {
        const size_t ps = s6 + edgeid * 2, ps2 = s6 + ((edgeid + 1) % 3) * 2;
        const T x1 = V(ps), y1 = V(ps + 1), x2 = V(ps2), y2 = V(ps2 + 1);
        const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
        const T up = A * x0 + Bc * y0 + C;
        const T down = A * A + Bc * Bc;
        const T dsq = (T)((double)(up * up) / ((double)down + SM_EPS));
        const T dzdA = (T)((double)((T)2 * (x0 * up - dsq * A)) / ((double)down + SM_EPS));
        const T dzdB = (T)((double)((T)2 * (y0 * up - dsq * Bc)) / ((double)down + SM_EPS));
        const T dzdC = (T)((double)((T)2 * up) / ((double)down + SM_EPS));
        const T dLdx1 = dLdz * (dzdB - y2 * dzdC);
        const T dLdy1 = dLdz * (x2 * dzdC - dzdA);
        const T dLdx2 = dLdz * (y1 * dzdC - dzdB);
        const T dLdy2 = dLdz * (dzdA - x1 * dzdC);
        atomicAdd(gfvi + ps + 0, dLdx1 / (T)multiplier);
        atomicAdd(gfvi + ps + 1, dLdy1 / (T)multiplier);
        atomicAdd(gfvi + ps2 + 0, dLdx2 / (T)multiplier);
        atomicAdd(gfvi + ps2 + 1, dLdy2 / (T)multiplier);
      }
    }
  }
}

template <typename T>
static size_t sm_lds_per_wave(int K) {
  return (size_t)K * 64 * (sizeof(uint32_t) + sizeof(T)) + 64 * sizeof(int);
}

template <typename T, typename Src>
static int soft_mask_fwd(Src src, int B, int H, int W, int F, int K, const int64_t *sel, float sigmainv, float m,
                         void *mask, void *prob, int64_t *cidx, uint8_t *ctype, void *ws, size_t ws_bytes,
                         hipStream_t st) {
  BinGeom g = make_bin_geom(B, H, W, F);
  KL_REQUIRE(ws_bytes >= g.bytes(), "dibr_soft_mask_forward: workspace too small");
  KL_REQUIRE(K >= 0, "dibr_soft_mask_forward: knum must be >= 0");
  KL_REQUIRE(F < (1 << 28), "dibr_soft_mask_forward: too many faces");
  if (B == 0 || H == 0 || W == 0) return KL_OK;
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(ws);
  int rc = launch_binning<T, Src>(src, nullptr, F, g, m, bitmap, st);
  if (rc) return rc;
  const size_t pw = sm_lds_per_wave<T>(K);
  int waves = 2;
  if (pw * 2 > 160 * 1024) waves = 1;
  KL_REQUIRE(pw * waves <= 160 * 1024, "dibr_soft_mask_forward: knum too large for the LDS staging buffer");
  dim3 grid(g.tiles_x, (unsigned)cdiv(H, waves), B);
  hipLaunchKernelGGL((soft_mask_fwd_kernel<T, Src>), grid, dim3(64 * waves), pw * waves, st, src, sel, bitmap, g, F, K,
                     sigmainv, m, (T *)mask, (T *)prob, cidx, ctype);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T, bool SCALE>
static int soft_mask_bwd(int B, int H, int W, int F, int K, const void *grad, const void *mask,
                         const int64_t *sel, const void *prob, const int64_t *cidx, const uint8_t *ctype,
                         const void *fvi, float sigmainv, float m, void *gfvi, hipStream_t st) {
  KL_CHECK_HIP(hipMemsetAsync(gfvi, 0, sizeof(T) * (size_t)B * F * 6, st));
  const int64_t total = (int64_t)B * H * W;
  if (total == 0) return KL_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(total, 256), 65536);
  hipLaunchKernelGGL((soft_mask_bwd_kernel<T, SCALE>), dim3(blocks), dim3(256), 0, st, (const T *)grad,
                     (const T *)mask, sel, (const T *)prob, cidx, ctype, (const T *)fvi, B, H, W, F, K, sigmainv, m,
                     (T *)gfvi);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_soft_mask_workspace_bytes(int batch, int height, int width, int num_faces) {
  return make_bin_geom(batch, height, width, num_faces).bytes();
}

extern "C" int kl_dibr_soft_mask_forward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                         int knum, const void *fvi, const void *bbox, const int64_t *sel,
                                         float sigmainv, float multiplier, void *mask, void *prob,
                                         int64_t *cidx, uint8_t *ctype, void *ws, size_t ws_bytes,
                                         kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_fwd<float>(BboxSrc<float>{(const float *)bbox, (const float *)fvi}, batch, height, width,
                                num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype, ws, ws_bytes,
                                S(stream));
  if (dtype == KL_F64)
    return soft_mask_fwd<double>(BboxSrc<double>{(const double *)bbox, (const double *)fvi}, batch, height, width,
                                 num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype, ws, ws_bytes,
                                 S(stream));
  set_error("dibr_soft_mask_forward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_soft_mask_forward_fused(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                               int knum, const void *fvi, const int64_t *sel, float sigmainv,
                                               double pad, float multiplier, void *mask, void *prob,
                                               int64_t *cidx, uint8_t *ctype, void *ws, size_t ws_bytes,
                                               kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_fwd<float>(SoftSrc<float>{(const float *)fvi, (float)multiplier, (float)pad}, batch, height,
                                width, num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype, ws,
                                ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_mask_fwd<double>(SoftSrc<double>{(const double *)fvi, (double)multiplier, pad}, batch, height, width,
                                 num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype, ws, ws_bytes,
                                 S(stream));
  set_error("dibr_soft_mask_forward not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_soft_mask_backward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                          int knum, const void *grad, const void *mask, const int64_t *sel,
                                          const void *prob, const int64_t *cidx, const uint8_t *ctype,
                                          const void *fvi, float sigmainv, float multiplier, void *gfvi,
                                          kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_bwd<float, false>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype, fvi,
                                       sigmainv, multiplier, gfvi, S(stream));
  if (dtype == KL_F64)
    return soft_mask_bwd<double, false>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype,
                                        fvi, sigmainv, multiplier, gfvi, S(stream));
  set_error("dibr_soft_mask_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_soft_mask_backward_fused(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                                int knum, const void *grad, const void *mask, const int64_t *sel,
                                                const void *prob, const int64_t *cidx, const uint8_t *ctype,
                                                const void *fvi, float sigmainv, float multiplier, void *gfvi,
                                                kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_bwd<float, true>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype, fvi,
                                      sigmainv, multiplier, gfvi, S(stream));
  if (dtype == KL_F64)
    return soft_mask_bwd<double, true>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype,
                                       fvi, sigmainv, multiplier, gfvi, S(stream));
  set_error("dibr_soft_mask_backward not implemented for this dtype");
  return KL_E_INVALID;
}
