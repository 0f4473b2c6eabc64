// texture.hip -- texture_mapping (kaolin/render/mesh/utils.py:23-75), the caller-side lookup the
// reference's DIB-R tutorial runs on the rasterizer's uv map (dibr_tutorial.ipynb cell 12).
//
// The reference clamps the coordinates to [0, 1], maps them to [-1, 1] with y reversed and calls
// torch.nn.functional.grid_sample(..., align_corners=False, padding_mode='border').  Here the
// whole chain is one launch forward and one backward, with grid_sample's own arithmetic
// (aten/src/ATen/native/cuda/GridSampler.cu: unnormalize, border clip, the four bilinear corner
// weights and their accumulation order, and the multiply-adds torch's ROCm build contracts into
// fma -- written as explicit fma here, since this library compiles with -ffp-contract=off), so
// the forward equals the torch chain's and the coordinate gradient equals autograd's through it.
//
// The texture gradient is where the torch chain spends its time: grid_sample's backward adds
// every (pixel, channel, corner) term with a float atomic, zero incoming gradients included --
// in the tutorial every uncovered pixel (uv = 0 after the mask) samples the same corner texel,
// so ~half a million pixels serialise on three addresses (10.8 ms per call at 4 x 512^2).  Here
// terms with a zero incoming gradient are skipped (they add nothing) and the rest are summed in
// double and rounded once: for f32, deterministic and equal to the exact sum of torch's float
// terms wherever those span less than ~2^29 (torch's own float atomics round in arbitrary order);
// f64 terms added with double atomics round in arrival order.
#include "common.h"

namespace kl {

// grid_sampler_compute_source_index for align_corners=False, padding 'border' (GridSampler.cuh):
// unnormalize ((c + 1) * size - 1) / 2, clip_coordinates (min(size - 1, max(x, 0)), a NaN
// clipped to 0 as fmax does), safe_downgrade_to_int_range (non-finite -> -100: out of bounds)
template <typename T>
__device__ __forceinline__ T tex_source(T c, int size) {
  T x = fma(c + (T)1, (T)size, (T)-1) / (T)2;  // torch's build contracts a * b - 1
  x = fmin((T)(size - 1), fmax(x, (T)0));
  return isfinite(x) ? x : (T)-100;
}
// ..._set_grad: clip_coordinates_set_grad (borders count as clipped: gradient 0 there; a NaN passes
// with gradient 1), then the same downgrade; `mult` is the coordinate's gradient factor size / 2
// times the clip gradient
template <typename T>
__device__ __forceinline__ T tex_source_grad(T c, int size, T &mult) {
  T x = fma(c + (T)1, (T)size, (T)-1) / (T)2;
  const T lim = (T)(size - 1);
  T gclip = (T)1;
  if (x <= (T)0) {
    gclip = (T)0;
    x = (T)0;
  } else if (x >= lim) {
    gclip = (T)0;
    x = lim;
  }
  mult = (T)size / (T)2 * gclip;
  return isfinite(x) ? x : (T)-100;
}

// the reference's pre-processing of one coordinate pair: clamp to [0, 1], * 2 - 1, y negated;
// `gx`, `gy`: torch.clamp's gradient mask (inclusive bounds) times the chain's exact factors
template <typename T>
__device__ __forceinline__ void tex_grid(T u, T v, T &gx, T &gy, T &cx, T &cy) {
  const T uc = u < (T)0 ? (T)0 : (u > (T)1 ? (T)1 : u);
  const T vc = v < (T)0 ? (T)0 : (v > (T)1 ? (T)1 : v);
  cx = uc * (T)2 - (T)1;
  cy = -(vc * (T)2 - (T)1);
  gx = (u >= (T)0 && u <= (T)1) ? (T)2 : (T)0;
  gy = (v >= (T)0 && v <= (T)1) ? (T)-2 : (T)0;
  if (u != u) gx = (T)0;  // clamp propagates NaN; its gradient mask is false there
  if (v != v) gy = (T)0;
}

__device__ __forceinline__ bool tex_in(int x, int y, int W, int H) { return x >= 0 && x < W && y >= 0 && y < H; }

// One thread per (mesh, point): out (B, N, C), contiguous.
template <typename T, int MODE>
__global__ void __launch_bounds__(256) texture_fwd_kernel(int B, int64_t N, int C, int TH, int TW,
                                                          const T *__restrict__ coords, const T *__restrict__ tex,
                                                          T *__restrict__ out) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * N) return;
  const int b = (int)(t / N);
  T gx, gy, cx, cy;
  tex_grid<T>(coords[t * 2], coords[t * 2 + 1], gx, gy, cx, cy);
  const T ix = tex_source<T>(cx, TW), iy = tex_source<T>(cy, TH);
  const T *tb = tex + (size_t)b * C * TH * TW;
  const size_t plane = (size_t)TH * TW;
  if (MODE == 0) {  // nearest: nearbyint (half to even)
    const int xn = (int)rint(ix), yn = (int)rint(iy);
    const bool in = tex_in(xn, yn, TW, TH);
    for (int c = 0; c < C; c++) out[t * C + c] = in ? tb[c * plane + (size_t)yn * TW + xn] : (T)0;
    return;
  }
  const T fx = floor(ix), fy = floor(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const T ix_se = fx + (T)1, iy_se = fy + (T)1;
  const T nw = (ix_se - ix) * (iy_se - iy);
  const T ne = (ix - fx) * (iy_se - iy);
  const T sw = (ix_se - ix) * (iy - fy);
  const T se = (ix - fx) * (iy - fy);
  const bool b_nw = tex_in(x0, y0, TW, TH), b_ne = tex_in(x0 + 1, y0, TW, TH);
  const bool b_sw = tex_in(x0, y0 + 1, TW, TH), b_se = tex_in(x0 + 1, y0 + 1, TW, TH);
  for (int c = 0; c < C; c++) {
    const T *p = tb + c * plane;
    T o = (T)0;
    // out += value * weight as the contracted fma of torch's build
    if (b_nw) o = fma(p[(size_t)y0 * TW + x0], nw, o);
    if (b_ne) o = fma(p[(size_t)y0 * TW + x0 + 1], ne, o);
    if (b_sw) o = fma(p[(size_t)(y0 + 1) * TW + x0], sw, o);
    if (b_se) o = fma(p[(size_t)(y0 + 1) * TW + x0 + 1], se, o);
    out[t * C + c] = o;
  }
}

// One thread per (mesh, point): the coordinate gradient (grid_sampler_2d_backward_kernel's
// gix / giy, times the clip / unnormalize and pre-processing factors), and the texture terms
// with a non-zero incoming gradient added in double into `acc` (B, C, TH, TW).
template <typename T, int MODE>
__global__ void __launch_bounds__(256) texture_bwd_kernel(int B, int64_t N, int C, int TH, int TW,
                                                          const T *__restrict__ gout, const T *__restrict__ coords,
                                                          const T *__restrict__ tex, T *__restrict__ gcoords,
                                                          double *__restrict__ acc) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * N) return;
  const int b = (int)(t / N);
  T gx, gy, cx, cy, mx, my;
  tex_grid<T>(coords[t * 2], coords[t * 2 + 1], gx, gy, cx, cy);
  const T ix = tex_source_grad<T>(cx, TW, mx), iy = tex_source_grad<T>(cy, TH, my);
  const size_t plane = (size_t)TH * TW;
  const T *tb = tex + (size_t)b * C * plane;
  double *ab = acc ? acc + (size_t)b * C * plane : nullptr;
  if (MODE == 0) {
    const int xn = (int)rint(ix), yn = (int)rint(iy);
    if (ab && tex_in(xn, yn, TW, TH))
      for (int c = 0; c < C; c++) {
        const T g = gout[t * C + c];
        if (g != (T)0) atomicAdd(ab + c * plane + (size_t)yn * TW + xn, (double)g);
      }
    if (gcoords) {
      gcoords[t * 2] = (T)0;
      gcoords[t * 2 + 1] = (T)0;
    }
    return;
  }
  const T fx = floor(ix), fy = floor(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const T ix_nw = fx, iy_nw = fy, ix_ne = fx + (T)1, iy_ne = fy, ix_sw = fx, iy_sw = fy + (T)1;
  const T ix_se = fx + (T)1, iy_se = fy + (T)1;
  const T nw = (ix_se - ix) * (iy_se - iy);
  const T ne = (ix - ix_sw) * (iy_sw - iy);
  const T sw = (ix_ne - ix) * (iy - iy_ne);
  const T se = (ix - ix_nw) * (iy - iy_nw);
  const bool b_nw = tex_in(x0, y0, TW, TH), b_ne = tex_in(x0 + 1, y0, TW, TH);
  const bool b_sw = tex_in(x0, y0 + 1, TW, TH), b_se = tex_in(x0 + 1, y0 + 1, TW, TH);
  const size_t o_nw = (size_t)y0 * TW + x0;
  T gix = (T)0, giy = (T)0;
  for (int c = 0; c < C; c++) {
    const T g = gout[t * C + c];
    const T *p = tb + c * plane;
    double *a = ab ? ab + c * plane : nullptr;
    if (b_nw) {
      const T val = p[o_nw];
      gix = fma(-(val * (iy_se - iy)), g, gix);
      giy = fma(-(val * (ix_se - ix)), g, giy);
      if (a && g != (T)0) atomicAdd(a + o_nw, (double)(nw * g));
    }
    if (b_ne) {
      const T val = p[o_nw + 1];
      gix = fma(val * (iy_sw - iy), g, gix);
      giy = fma(-(val * (ix - ix_sw)), g, giy);
      if (a && g != (T)0) atomicAdd(a + o_nw + 1, (double)(ne * g));
    }
    if (b_sw) {
      const T val = p[o_nw + TW];
      gix = fma(-(val * (iy - iy_ne)), g, gix);
      giy = fma(val * (ix_ne - ix), g, giy);
      if (a && g != (T)0) atomicAdd(a + o_nw + TW, (double)(sw * g));
    }
    if (b_se) {
      const T val = p[o_nw + TW + 1];
      gix = fma(val * (iy - iy_nw), g, gix);
      giy = fma(val * (ix - ix_nw), g, giy);
      if (a && g != (T)0) atomicAdd(a + o_nw + TW + 1, (double)(se * g));
    }
  }
  if (gcoords) {
    gcoords[t * 2] = mx * gix * gx;
    gcoords[t * 2 + 1] = my * giy * gy;
  }
}

template <typename T>
static int texture_fwd(int mode, int B, int64_t N, int C, int TH, int TW, const void *coords, const void *tex,
                       void *out, hipStream_t st) {
  const int64_t n = (int64_t)B * N;
  if (n == 0 || C == 0) return KL_OK;
  const dim3 grid((unsigned)cdiv(n, 256));
  if (mode == 0)
    hipLaunchKernelGGL((texture_fwd_kernel<T, 0>), grid, dim3(256), 0, st, B, N, C, TH, TW, (const T *)coords,
                       (const T *)tex, (T *)out);
  else
    hipLaunchKernelGGL((texture_fwd_kernel<T, 1>), grid, dim3(256), 0, st, B, N, C, TH, TW, (const T *)coords,
                       (const T *)tex, (T *)out);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
static int texture_bwd(int mode, int B, int64_t N, int C, int TH, int TW, const void *gout, const void *coords,
                       const void *tex, void *gcoords, void *gtex, void *ws, size_t ws_bytes, hipStream_t st) {
  const size_t nt = (size_t)B * C * TH * TW;
  double *acc = nullptr;
  if (gtex) {
    KL_REQUIRE(ws && ws_bytes >= nt * sizeof(double), "texture_mapping backward: workspace too small");
    acc = (double *)ws;
    KL_CHECK_RC(fill_async(acc, 0, nt * sizeof(double), st));
  }
  const int64_t n = (int64_t)B * N;
  if (n > 0 && C > 0) {
    const dim3 grid((unsigned)cdiv(n, 256));
    if (mode == 0)
      hipLaunchKernelGGL((texture_bwd_kernel<T, 0>), grid, dim3(256), 0, st, B, N, C, TH, TW, (const T *)gout,
                         (const T *)coords, (const T *)tex, (T *)gcoords, acc);
    else
      hipLaunchKernelGGL((texture_bwd_kernel<T, 1>), grid, dim3(256), 0, st, B, N, C, TH, TW, (const T *)gout,
                         (const T *)coords, (const T *)tex, (T *)gcoords, acc);
    KL_CHECK_LAUNCH();
  } else if (gcoords && n > 0) {
    KL_CHECK_RC(fill_async(gcoords, 0, (size_t)n * 2 * sizeof(T), st));
  }
  return gtex ? acc_finalize<T>(acc, (T *)gtex, nt, false, st) : KL_OK;
}

}  // namespace kl

using namespace kl;

extern "C" int kl_texture_mapping_forward(kl_dtype dtype, int mode, int batch, int64_t num_points, int channels,
                                          int tex_height, int tex_width, const void *coords, const void *texture,
                                          void *out, kl_stream stream) {
  KL_REQUIRE(mode == 0 || mode == 1, "texture_mapping: mode must be 'nearest' (0) or 'bilinear' (1)");
  KL_REQUIRE(batch >= 0 && num_points >= 0 && channels >= 0 && tex_height > 0 && tex_width > 0,
             "texture_mapping: bad sizes");
  if (dtype == KL_F32)
    return texture_fwd<float>(mode, batch, num_points, channels, tex_height, tex_width, coords, texture, out,
                              S(stream));
  if (dtype == KL_F64)
    return texture_fwd<double>(mode, batch, num_points, channels, tex_height, tex_width, coords, texture, out,
                               S(stream));
  set_error("texture_mapping not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_texture_mapping_bwd_workspace_bytes(int batch, int channels, int tex_height, int tex_width) {
  return (size_t)batch * channels * tex_height * tex_width * sizeof(double);
}

extern "C" int kl_texture_mapping_backward(kl_dtype dtype, int mode, int batch, int64_t num_points, int channels,
                                           int tex_height, int tex_width, const void *grad_out, const void *coords,
                                           const void *texture, void *grad_coords, void *grad_texture, void *ws,
                                           size_t ws_bytes, kl_stream stream) {
  KL_REQUIRE(mode == 0 || mode == 1, "texture_mapping: mode must be 'nearest' (0) or 'bilinear' (1)");
  KL_REQUIRE(batch >= 0 && num_points >= 0 && channels >= 0 && tex_height > 0 && tex_width > 0,
             "texture_mapping: bad sizes");
  if (dtype == KL_F32)
    return texture_bwd<float>(mode, batch, num_points, channels, tex_height, tex_width, grad_out, coords, texture,
                              grad_coords, grad_texture, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return texture_bwd<double>(mode, batch, num_points, channels, tex_height, tex_width, grad_out, coords, texture,
                               grad_coords, grad_texture, ws, ws_bytes, S(stream));
  set_error("texture_mapping backward not implemented for this dtype");
  return KL_E_INVALID;
}
