// maskiou.hip -- mask_iou (kaolin/metrics/render.py:18-40), the silhouette loss the DIB-R tutorial
// puts on dibr_soft_mask's output, fused: one pass over both masks for the two per-view sums and
// one pass for both gradients.
//
// The reference is six torch ops forward (mul, add, two dim=1 sums, div, mean) and about a dozen
// backward; its two sums are reductions to B values, which torch runs with few workgroups per
// output (~24 us each at 4 x 512^2).  Here each view's strip is split over many workgroups, the
// products / differences are formed in the input dtype exactly as torch forms them
// (sil_mul = l * r, sil_add - sil_mul = (l + r) - l * r), summed in double and added in a fixed
// order (deterministic), and rounded once to the dtype; the loss follows the reference's float
// ops.  The gradients are autograd's through the reference's ops, evaluated per element in the
// same order (mean / rsub, div, sum, sub, mul, add):
//   g_in = (-g) / B,  den = down + 1e-10,  g_up = g_in / den,  g_den = -g_in * ((up / den) / den)
//   grad_lhs = (g_up - g_den) * rhs + g_den,  grad_rhs = (g_up - g_den) * lhs + g_den
// (bit-equal to torch's given the same up / down; up / down themselves are the exactly rounded
// sums, where torch's float reductions round per partial).
#include "common.h"

namespace kl {

constexpr int MIOU_THREADS = 256;

template <typename T>
__global__ void __launch_bounds__(MIOU_THREADS) miou_partial_kernel(const T *__restrict__ l, const T *__restrict__ r,
                                                                   int64_t N, double *__restrict__ part) {
  __shared__ double s_u[MIOU_THREADS / 64], s_d[MIOU_THREADS / 64];
  const int b = blockIdx.y;
  const T *lb = l + (int64_t)b * N, *rb = r + (int64_t)b * N;
  double up = 0.0, dn = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)MIOU_THREADS + threadIdx.x; i < N; i += (int64_t)gridDim.x * MIOU_THREADS) {
    const T x = lb[i], y = rb[i];
    const T m = x * y;
    up += (double)m;
    dn += (double)((x + y) - m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    up += __shfl_xor(up, o);
    dn += __shfl_xor(dn, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s_u[threadIdx.x >> 6] = up;
    s_d[threadIdx.x >> 6] = dn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double u = 0.0, d = 0.0;
#pragma unroll
    for (int w = 0; w < MIOU_THREADS / 64; w++) {
      u += s_u[w];
      d += s_d[w];
    }
    part[((size_t)b * gridDim.x + blockIdx.x) * 2] = u;
    part[((size_t)b * gridDim.x + blockIdx.x) * 2 + 1] = d;
  }
}

// one workgroup: a wave per view adds its partials (lane l the partials l, l + 64, ... in order,
// then a fixed butterfly: deterministic; one thread adding all of them serially took 13.7 us at
// 4 x 512^2); thread 0 then forms the loss
template <typename T>
__global__ void __launch_bounds__(MIOU_THREADS) miou_final_kernel(const double *__restrict__ part, int B, int nbx,
                                                                 T *__restrict__ up, T *__restrict__ down,
                                                                 T *__restrict__ loss) {
  const int lane = threadIdx.x & 63;
  for (int b = threadIdx.x >> 6; b < B; b += MIOU_THREADS / 64) {  // uniform per wave
    double u = 0.0, d = 0.0;
    for (int k = lane; k < nbx; k += 64) {
      u += part[((size_t)b * nbx + k) * 2];
      d += part[((size_t)b * nbx + k) * 2 + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      u += __shfl_xor(u, o);
      d += __shfl_xor(d, o);
    }
    if (lane == 0) {
      up[b] = (T)u;
      down[b] = (T)d;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    T s = (T)0;  // torch.mean: the views' ratios summed in order, times 1 / B
    for (int b = 0; b < B; b++) s += up[b] / (down[b] + (T)1e-10);
    loss[0] = (T)1.0 - s * ((T)1 / (T)B);
  }
}

template <typename T>
__global__ void __launch_bounds__(MIOU_THREADS) miou_bwd_kernel(const T *__restrict__ g, const T *__restrict__ l,
                                                               const T *__restrict__ r, const T *__restrict__ up,
                                                               const T *__restrict__ down, int B, int64_t N,
                                                               T *__restrict__ gl, T *__restrict__ gr) {
  const int b = blockIdx.y;
  const T gin = (-g[0]) / (T)B;
  const T den = down[b] + (T)1e-10;
  const T gup = gin / den;
  const T gden = -gin * ((up[b] / den) / den);
  const T a = gup - gden;
  const int64_t o = (int64_t)b * N;
  for (int64_t i = blockIdx.x * (int64_t)MIOU_THREADS + threadIdx.x; i < N; i += (int64_t)gridDim.x * MIOU_THREADS) {
    if (gl) gl[o + i] = a * r[o + i] + gden;
    if (gr) gr[o + i] = a * l[o + i] + gden;
  }
}

static int miou_blocks(int64_t N) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(256, cdiv(N, (int64_t)MIOU_THREADS * 8)));
}

template <typename T>
static int miou_fwd(int B, int64_t N, const T *l, const T *r, T *up, T *down, T *loss, void *ws, size_t ws_bytes,
                    hipStream_t st) {
  const int nbx = miou_blocks(N);
  KL_REQUIRE(B > 0 && N > 0, "mask_iou: empty masks");
  KL_REQUIRE(ws_bytes >= (size_t)B * nbx * 2 * sizeof(double), "mask_iou: workspace too small");
  hipLaunchKernelGGL((miou_partial_kernel<T>), dim3((unsigned)nbx, (unsigned)B), dim3(MIOU_THREADS), 0, st, l, r, N,
                     (double *)ws);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL((miou_final_kernel<T>), dim3(1), dim3(MIOU_THREADS), 0, st, (const double *)ws, B, nbx, up, down,
                     loss);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
static int miou_bwd(int B, int64_t N, const T *g, const T *l, const T *r, const T *up, const T *down, T *gl, T *gr,
                    hipStream_t st) {
  if (B <= 0 || N <= 0 || (!gl && !gr)) return KL_OK;
  hipLaunchKernelGGL((miou_bwd_kernel<T>), dim3((unsigned)miou_blocks(N), (unsigned)B), dim3(MIOU_THREADS), 0, st, g,
                     l, r, up, down, B, N, gl, gr);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_mask_iou_workspace_bytes(int batch, int64_t pixels_per_mask) {
  return (size_t)std::max(batch, 1) * miou_blocks(pixels_per_mask) * 2 * sizeof(double);
}

extern "C" int kl_mask_iou_forward(kl_dtype dtype, int batch, int64_t pixels_per_mask, const void *lhs,
                                   const void *rhs, void *iou_up, void *iou_down, void *loss, void *workspace,
                                   size_t workspace_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return miou_fwd<float>(batch, pixels_per_mask, (const float *)lhs, (const float *)rhs, (float *)iou_up,
                           (float *)iou_down, (float *)loss, workspace, workspace_bytes, S(stream));
  if (dtype == KL_F64)
    return miou_fwd<double>(batch, pixels_per_mask, (const double *)lhs, (const double *)rhs, (double *)iou_up,
                            (double *)iou_down, (double *)loss, workspace, workspace_bytes, S(stream));
  set_error("mask_iou: f32 / f64 only");
  return KL_E_INVALID;
}

extern "C" int kl_mask_iou_backward(kl_dtype dtype, int batch, int64_t pixels_per_mask, const void *grad_loss,
                                    const void *lhs, const void *rhs, const void *iou_up, const void *iou_down,
                                    void *grad_lhs, void *grad_rhs, kl_stream stream) {
  if (dtype == KL_F32)
    return miou_bwd<float>(batch, pixels_per_mask, (const float *)grad_loss, (const float *)lhs, (const float *)rhs,
                           (const float *)iou_up, (const float *)iou_down, (float *)grad_lhs, (float *)grad_rhs,
                           S(stream));
  if (dtype == KL_F64)
    return miou_bwd<double>(batch, pixels_per_mask, (const double *)grad_loss, (const double *)lhs,
                            (const double *)rhs, (const double *)iou_up, (const double *)iou_down,
                            (double *)grad_lhs, (double *)grad_rhs, S(stream));
  set_error("mask_iou backward: f32 / f64 only");
  return KL_E_INVALID;
}
