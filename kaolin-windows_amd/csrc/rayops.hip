// rayops.hip -- packed ray operations on the raytrace output:
// diff, inclusive_sum, sum_reduce, cumsum and cumprod over packs of consecutive rows.
//
// Reference: kaolin/render/spc/raytrace.py:86-296 (front-ends) over
// raytrace_cuda.cu:309-483 / 609-759 (kernels) and raytrace.cpp:285-402 (bindings).
//
// Layout: feats is (num_feats, feat_dim) row-major; a pack is a run of rows
// [pack_indices[p], pack_indices[p+1]) (the last one runs to num_feats).  Rows before the
// first pack belong to no pack and keep the reference's initial value (0, or 1 for cumprod;
// the reference allocates at::zeros / at::ones and leaves them untouched).
//
// One lane per (pack, feature column): lane t -> column t % feat_dim of pack t / feat_dim - 1
// (the extra pack -1 is the prefix before the first pack), so neighbouring lanes walk
// neighbouring columns of the same rows and each step of the walk is one coalesced row
// read.  Every lane walks its pack in the reference's order with the reference's operand
// order (in op prev), so the scans are bit-identical to the reference's sequential loops;
// half arithmetic is float arithmetic rounded to half after every step (at::Half's).
// sum_reduce replaces the reference's atomicAdd (unordered) with the same sequential walk
// from each pack's first row: deterministic, and within rounding of any atomic order.
#include <hip/hip_fp16.h>

#include <hipcub/hipcub.hpp>

#include "common.h"

namespace kl {

template <typename S>
struct Acc {
  using T = S;
};
template <>
struct Acc<__half> {
  using T = float;
};

template <typename S>
__device__ __forceinline__ typename Acc<S>::T up(S v) {
  return (typename Acc<S>::T)v;
}
template <typename S>
__device__ __forceinline__ S down(typename Acc<S>::T v) {
  return (S)v;
}

struct OpAdd {
  template <typename A>
  __device__ static A apply(A a, A b) { return a + b; }
  static constexpr int init = 0;
};
struct OpMul {
  template <typename A>
  __device__ static A apply(A a, A b) { return a * b; }
  static constexpr int init = 1;
};

// pack p's row range; p == -1 is the prefix [0, first pack)
template <typename I>
__device__ __forceinline__ void pack_range(int64_t p, const I *__restrict__ idx, int64_t num_packs, int64_t num_feats,
                                           int64_t &begin, int64_t &end) {
  if (p < 0) {
    begin = 0;
    end = num_packs > 0 ? (int64_t)idx[0] : num_feats;
  } else {
    begin = (int64_t)idx[p];
    end = p == num_packs - 1 ? num_feats : (int64_t)idx[p + 1];
  }
  begin = max(begin, (int64_t)0);
  end = min(end, num_feats);
}

// raytrace_cuda.cu:391-483 (cumsum / cumprod, forward and reverse kernels)
template <typename S, typename OP>
__global__ void __launch_bounds__(256) pack_scan_kernel(int64_t num_feats, int64_t dim, const S *__restrict__ in,
                                                        const int32_t *__restrict__ idx, int64_t num_packs,
                                                        int exclusive, int reverse, S *__restrict__ out) {
  using A = typename Acc<S>::T;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (num_packs + 1) * dim) return;
  const int64_t p = t / dim - 1, j = t - (t / dim) * dim;
  int64_t begin, end;
  pack_range(p, idx, num_packs, num_feats, begin, end);
  const S init = down<S>((A)OP::init);
  if (p < 0) {
    for (int64_t i = begin; i < end; i++) out[i * dim + j] = init;
    return;
  }
  if (begin >= end) return;
  if (!reverse) {
    A acc = exclusive ? (A)OP::init : up(in[begin * dim + j]);
    out[begin * dim + j] = exclusive ? init : in[begin * dim + j];
    for (int64_t i = begin + 1; i < end; i++) {
      acc = up(down<S>(OP::apply(up(in[(i - exclusive) * dim + j]), acc)));
      out[i * dim + j] = down<S>(acc);
    }
  } else {
    A acc = exclusive ? (A)OP::init : up(in[(end - 1) * dim + j]);
    out[(end - 1) * dim + j] = exclusive ? init : in[(end - 1) * dim + j];
    for (int64_t i = end - 2; i >= begin; i--) {
      acc = up(down<S>(OP::apply(up(in[(i + exclusive) * dim + j]), acc)));
      out[i * dim + j] = down<S>(acc);
    }
  }
}

// raytrace_cuda.cu:309-325 (diff): out[i] = in[i+1] - in[i] inside a pack, 0 on its last row
template <typename S>
__global__ void __launch_bounds__(256) pack_diff_kernel(int64_t num_feats, int64_t dim, const S *__restrict__ in,
                                                        const int64_t *__restrict__ idx, int64_t num_packs,
                                                        S *__restrict__ out) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (num_packs + 1) * dim) return;
  const int64_t p = t / dim - 1, j = t - (t / dim) * dim;
  int64_t begin, end;
  pack_range(p, idx, num_packs, num_feats, begin, end);
  const S zero = down<S>(0);
  if (p < 0) {
    for (int64_t i = begin; i < end; i++) out[i * dim + j] = zero;
    return;
  }
  if (begin >= end) return;
  S cur = in[begin * dim + j];
  for (int64_t i = begin; i < end - 1; i++) {
    const S nxt = in[(i + 1) * dim + j];
    out[i * dim + j] = down<S>(up(nxt) - up(cur));
    cur = nxt;
  }
  out[(end - 1) * dim + j] = zero;
}

// raytrace_cuda.cu:327-346 (sum_reduce): row inclusive_sum[i]-1 of out accumulates row i.
// The lane of a pack's first row walks the pack; rows whose id is < 1 or >= num_out are
// dropped (the reference wrote them out of bounds).
template <typename S>
__global__ void __launch_bounds__(256) sum_reduce_kernel(int64_t num_feats, int64_t dim, const S *__restrict__ in,
                                                         const int32_t *__restrict__ isum, int64_t num_out,
                                                         S *__restrict__ out) {
  using A = typename Acc<S>::T;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= num_feats * dim) return;
  const int64_t i = t / dim, j = t - i * dim;
  const int32_t id = isum[i];
  if (i > 0 && isum[i - 1] == id) return;
  if (id < 1 || id > num_out) return;
  A acc = (A)0;
  for (int64_t k = i; k < num_feats && isum[k] == id; k++) acc = up(down<S>(acc + up(in[k * dim + j])));
  out[(int64_t)(id - 1) * dim + j] = down<S>(acc);
}

template <typename S, typename OP>
static int pack_scan(int64_t nf, int64_t dim, const void *in, const int32_t *idx, int64_t np, int ex, int rev,
                     void *out, hipStream_t st) {
  const int64_t n = (np + 1) * dim;
  hipLaunchKernelGGL((pack_scan_kernel<S, OP>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, nf, dim,
                     (const S *)in, idx, np, ex, rev, (S *)out);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename S>
static int pack_diff(int64_t nf, int64_t dim, const void *in, const int64_t *idx, int64_t np, void *out,
                     hipStream_t st) {
  const int64_t n = (np + 1) * dim;
  hipLaunchKernelGGL(pack_diff_kernel<S>, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, nf, dim, (const S *)in, idx,
                     np, (S *)out);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename S>
static int sum_reduce(int64_t nf, int64_t dim, const void *in, const int32_t *isum, int64_t nout, void *out,
                      hipStream_t st) {
  KL_CHECK_RC(fill_async(out, 0, (size_t)(nout * dim) * sizeof(S), st));
  const int64_t n = nf * dim;
  if (n == 0) return KL_OK;
  hipLaunchKernelGGL(sum_reduce_kernel<S>, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, nf, dim, (const S *)in,
                     isum, nout, (S *)out);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

#define KL_FLOAT_DISPATCH(dtype, FN, ...)                         \
  switch (dtype) {                                                \
    case KL_F32: return FN<float>(__VA_ARGS__);                   \
    case KL_F64: return FN<double>(__VA_ARGS__);                  \
    case KL_F16: return FN<__half>(__VA_ARGS__);                  \
    default: set_error("expected a Half, Float or Double tensor"); \
      return KL_E_INVALID;                                        \
  }

}  // namespace kl

using namespace kl;

static int check_pack_args(int64_t nf, int64_t dim, int64_t np) {
  KL_REQUIRE(nf >= 0 && dim >= 0 && np >= 0, "packed ray op: negative size");
  KL_REQUIRE(np < ((int64_t)1 << 40) && dim < ((int64_t)1 << 20), "packed ray op: size out of range");
  return KL_OK;
}

extern "C" int kl_pack_diff(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                            const int64_t *pack_indices, int64_t num_packs, void *out, kl_stream stream) {
  KL_CHECK_RC(check_pack_args(num_feats, feat_dim, num_packs));
  if (num_feats == 0 || feat_dim == 0) return KL_OK;
  KL_FLOAT_DISPATCH(dtype, pack_diff, num_feats, feat_dim, feats, pack_indices, num_packs, out, S(stream));
}

extern "C" int kl_pack_cumsum(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                              const int32_t *pack_indices, int64_t num_packs, int exclusive, int reverse, void *out,
                              kl_stream stream) {
  KL_CHECK_RC(check_pack_args(num_feats, feat_dim, num_packs));
  if (num_feats == 0 || feat_dim == 0) return KL_OK;
  const int ex = exclusive ? 1 : 0, rev = reverse ? 1 : 0;
  switch (dtype) {
    case KL_F32: return pack_scan<float, OpAdd>(num_feats, feat_dim, feats, pack_indices, num_packs, ex, rev, out, S(stream));
    case KL_F64: return pack_scan<double, OpAdd>(num_feats, feat_dim, feats, pack_indices, num_packs, ex, rev, out, S(stream));
    case KL_F16: return pack_scan<__half, OpAdd>(num_feats, feat_dim, feats, pack_indices, num_packs, ex, rev, out, S(stream));
    default: set_error("cumsum: expected a Half, Float or Double tensor"); return KL_E_INVALID;
  }
}

extern "C" int kl_pack_cumprod(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                               const int32_t *pack_indices, int64_t num_packs, int exclusive, int reverse, void *out,
                               kl_stream stream) {
  KL_CHECK_RC(check_pack_args(num_feats, feat_dim, num_packs));
  if (num_feats == 0 || feat_dim == 0) return KL_OK;
  const int ex = exclusive ? 1 : 0, rev = reverse ? 1 : 0;
  switch (dtype) {
    case KL_F32: return pack_scan<float, OpMul>(num_feats, feat_dim, feats, pack_indices, num_packs, ex, rev, out, S(stream));
    case KL_F64: return pack_scan<double, OpMul>(num_feats, feat_dim, feats, pack_indices, num_packs, ex, rev, out, S(stream));
    case KL_F16: return pack_scan<__half, OpMul>(num_feats, feat_dim, feats, pack_indices, num_packs, ex, rev, out, S(stream));
    default: set_error("cumprod: expected a Half, Float or Double tensor"); return KL_E_INVALID;
  }
}

extern "C" int kl_sum_reduce(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                             const int32_t *inclusive_sum, int64_t num_out, void *out, kl_stream stream) {
  KL_CHECK_RC(check_pack_args(num_feats, feat_dim, num_out));
  if (num_out == 0 || feat_dim == 0) return KL_OK;
  KL_FLOAT_DISPATCH(dtype, sum_reduce, num_feats, feat_dim, feats, inclusive_sum, num_out, out, S(stream));
}

extern "C" size_t kl_inclusive_sum_workspace_bytes(int64_t num) {
  size_t tb = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, tb, (const int32_t *)nullptr, (int32_t *)nullptr, (int)num);
  return tb > 0 ? tb : 1;
}

// raytrace_cuda.cu:650-663 (inclusive_sum_cuda_impl: cub::DeviceScan::InclusiveSum over int32)
extern "C" int kl_inclusive_sum_i32(int64_t num, const int32_t *info, int32_t *out, void *ws, size_t ws_bytes,
                                    kl_stream stream) {
  KL_REQUIRE(num >= 0 && num < ((int64_t)1 << 31), "inclusive_sum: size out of range");
  if (num == 0) return KL_OK;
  size_t tb = ws_bytes;
  KL_CHECK_HIP(hipcub::DeviceScan::InclusiveSum(ws, tb, info, out, (int)num, S(stream)));
  return KL_OK;
}
