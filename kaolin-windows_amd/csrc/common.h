// common.h -- shared helpers for the gfx950 kernels of libkaolin_hip.so.
// Compiled with -ffp-contract=off: every multiply-add is rounded twice, exactly as
// written, so results match the CPU oracle bit for bit (explicit fmaf() only where
// the reference wrote fmaf()).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <string>

#include "../../include/kaolin_hip.h"

namespace kl {

void set_error(const std::string &msg);
// Development controls exist only in the dev build (make dev: -DKL_DEV=1, kaolin/_lib/dev/): A/B
// switches between the product path and measured alternatives, forced fallbacks for the tests
// that cover them (tests marked devlib), stamps.  In the product library they are compile-time
// zeros: no process-global mutable state, and every branch they select -- the dead ends DESIGN.md
// records (the fused tile kernel, the fused / depth-first raytrace marches, the scalar-record p2m
// kernel, the r03 gather) -- is compiled out.
#ifndef KL_DEV
#define KL_DEV 0
#endif
#if KL_DEV
extern int g_dev_flags;    // kl_dev_set_flags (ablation timing only; 0 = the product path)
extern void *g_dev_debug;  // kl_dev_set_debug (per-wave stamps; nullptr = none)
extern int g_dev_param[32];  // kl_dev_set_param (tuning sweeps, forced fallbacks; 0 = the built-in value)
extern int g_dev_stat[4];    // kl_dev_get_stat (what the last call took)
#define KL_DEV_STAT(i, v) (::kl::g_dev_stat[(i)] = (v))
#else
constexpr int g_dev_flags = 0;
constexpr void *g_dev_debug = nullptr;
constexpr int g_dev_param[32] = {};
#define KL_DEV_STAT(i, v) ((void)0)
#endif

// shader-clock and 100 MHz wall-clock stamps for the dev timing buffer
// Dev stamps (kl_dev_set_debug) are compiled in only with -DKL_DEV_STAMPS=1 (make STAMPS=1):
// the bookkeeping costs registers even when the buffer is null.
#ifndef KL_DEV_STAMPS
#define KL_DEV_STAMPS 0
#endif
constexpr bool kDevStamps = KL_DEV_STAMPS != 0;
// The dev stamp buffer is shared by every stamping kernel (raster_tile_kernel and
// soft_tile_fwd_kernel write per-wave stamps from index 0, up to ~2M entries at cfg3): the order
// kernel's 8 stamps go this far in (the buffer must hold kOrderStampsAt + 8 entries).
constexpr size_t kOrderStampsAt = (size_t)1 << 24;
__device__ __forceinline__ uint64_t stamp_clk() { return __builtin_readcyclecounter(); }
__device__ __forceinline__ uint64_t stamp_wall() { return __builtin_amdgcn_s_memrealtime(); }
// memset as a kernel launch on `st` (graph-capture friendly); returns a kl_status
int fill_async(void *p, int value, size_t bytes, hipStream_t st);
// Reads `bytes` of device memory to the host once the stream reaches this point: a copy into a
// thread-local pinned buffer (allocated once, grown when needed, never freed) and a stream
// synchronise.  hipHostMalloc / hipHostFree per call, or a copy into pageable memory, cost
// tens to hundreds of microseconds each (mesh_to_spc's three reads, r04).
int host_read(void *dst, const void *src, size_t bytes, hipStream_t st);
// out[i] = (T)acc[i], or out[i] + (T)acc[i] with accumulate: the single rounding of a gradient
// summed in double (raster.hip)
// `reset` (optional): an int zeroed by the same launch.
template <typename T>
int acc_finalize(const double *acc, T *out, size_t n, bool accumulate, hipStream_t st, int *reset = nullptr);
inline size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

#define KL_CHECK_HIP(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::kl::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));               \
      return KL_E_HIP;                                                                  \
    }                                                                                   \
  } while (0)

#define KL_CHECK_LAUNCH() KL_CHECK_HIP(hipGetLastError())

#define KL_CHECK_RC(expr)                                                               \
  do {                                                                                  \
    const int _rc = (expr);                                                             \
    if (_rc) return _rc;                                                                \
  } while (0)

#define KL_REQUIRE(cond, msg)                                                           \
  do {                                                                                  \
    if (!(cond)) {                                                                      \
      ::kl::set_error(msg);                                                             \
      return KL_E_INVALID;                                                              \
    }                                                                                   \
  } while (0)

inline hipStream_t S(kl_stream s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr int WAVE = 64;

// Pixel centres (rasterization_cuda.cu:85-86, dibr_soft_mask_cuda.cu:74-75):
// `multiplier / width * (2 * wididx + 1 - width)` is evaluated in float.
template <typename T>
__device__ __forceinline__ T pix_x(float m, int W, int i) {
  return (T)((m / (float)W) * (float)(2 * i + 1 - W));
}
template <typename T>
__device__ __forceinline__ T pix_y(float m, int H, int j) {
  return (T)((m / (float)H) * (float)(H - 2 * j - 1));
}

// wave64 helpers
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int lane_id() { return __lane_id(); }

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o);
    v = u < v ? u : v;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o);
    v = u > v ? u : v;
  }
  return v;
}
// wave_max by DPP for 32-bit values (a running maximum within rows of 16 lanes, then the row 15 / 31
// broadcasts; lane 63's result read back as a scalar) -- no LDS round trips.  All 64 lanes must be
// active.  NaN: like `u > v ? u : v`, a NaN is kept only where it entered first, so callers pass
// no NaN (p2m's thresholds are finite or +inf).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_max_step(float v) {
  const float u = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROW_MASK, 0xf,
                                                             false));
  return u > v ? u : v;
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = dpp_max_step<0x111, 0xf>(v);  // row_shr:1
  v = dpp_max_step<0x112, 0xf>(v);  // row_shr:2
  v = dpp_max_step<0x114, 0xf>(v);  // row_shr:4
  v = dpp_max_step<0x118, 0xf>(v);  // row_shr:8
  v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15
  v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
template <typename T>
__device__ __forceinline__ T wave_max_all(T v) {
  if constexpr (sizeof(T) == 4) return wave_max_dpp(v);
  else return wave_max(v);
}

// Broadcast lane `src` (wave-uniform) of v to all lanes through the scalar unit.
__device__ __forceinline__ float bcast(float v, int src) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ int bcast(int v, int src) { return __builtin_amdgcn_readlane(v, src); }
__device__ __forceinline__ double bcast(double v, int src) {
  int64_t b = __double_as_longlong(v);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), src);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

// Inclusive prefix sum over the 64 lanes of a wave by DPP -- no LDS round trips (a __shfl_up
// scan is six dependent ds_bpermute): row_shr 1, 2, 4, 8 within each row of 16 lanes (lanes
// without a source keep the 0 of `old`), then lane 15's sum broadcast into rows 1 and 3 and lane
// 31's into rows 2 and 3.  All 64 lanes must be active (an inactive source lane reads as no source).
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// The same within each 32-lane half of the wave (the row 15 broadcast only: rows 1 and 3 take the
// sums of rows 0 and 2).  All 64 lanes must be active.
__device__ __forceinline__ int wave_incl_scan32(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  return v;
}

// Exclusive prefix sum over a workgroup (<= 1024 threads): wave scans (DPP), then
// the wave totals in `s_wave` (>= 16 ints of LDS).  Returns the thread's exclusive prefix;
// *total gets the workgroup sum.  Every thread must call it (two barriers).
__device__ __forceinline__ int block_exclusive_scan(int v, int *s_wave, int *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) s_wave[wid] = inc;
  __syncthreads();
  int before = 0, all = 0;
  for (int w = 0; w < nw; w++) {
    const int t = s_wave[w];
    before += w < wid ? t : 0;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + inc - v;
}

// Last-workgroup hand-off (MI355X_MICROARCH.md's measured `sc1` row): every workgroup's published
// values are complete (vmcnt(0)) before its barrier and its agent-scope add on a ticket; the
// workgroup that takes the last ticket returns true and may then read the published values with
// agent-scope loads.  Two levels of tickets, 128 B apart: tk[32 * (1 + g)] for each group g of
// GL_GROUP workgroups, then the groups' last workgroups on the top ticket tk[0] -- 2,048 adds on
// one address cost ~25 us (r05w), a group's 32 ~0.4 us.  Each last taker re-zeroes its ticket, so
// the tickets are zero again after every grid (zero them once: gl_ticket_words).  Workgroup-uniform.
constexpr int GL_GROUP = 32;
__host__ __device__ constexpr size_t gl_ticket_words(int grid) { return 32 * (size_t)(1 + (grid + GL_GROUP - 1) / GL_GROUP); }
__device__ __forceinline__ bool grid_last(unsigned *tk, int *s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned G = gridDim.x, grp = blockIdx.x / GL_GROUP;
    const unsigned ng = (G + GL_GROUP - 1) / GL_GROUP;
    const unsigned gsize = min((unsigned)GL_GROUP, G - grp * GL_GROUP);
    unsigned *t1 = tk + 32 * (1 + grp);
    bool last = false;
    if (__hip_atomic_fetch_add(t1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(t1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
      if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *s_flag = last ? 1 : 0;
  }
  __syncthreads();
  return *s_flag != 0;
}

// Adds v of every lane into *dst (64-bit): a wave sum, then one vector atomic per wave.
// Every lane of the wave must call it (lanes with nothing to add pass 0).
__device__ __forceinline__ void wave_add_u64(unsigned long long *dst, unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, v);
}

// Adds v of every thread into *dst: wave sums, then one atomic per workgroup (one returning
// word takes ~90 atomics per us, so a wave each from a large grid queues behind it).  Every
// thread of the workgroup must call it (one barrier); s_w: one word of LDS per wave.
__device__ __forceinline__ void block_add_u64(unsigned long long *dst, unsigned long long v,
                                              unsigned long long *s_w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < (int)((blockDim.x + 63) >> 6); w++) t += s_w[w];
    if (t) atomicAdd(dst, t);
  }
}

template <typename T>
__device__ __forceinline__ T kl_exp(T x);
template <>
__device__ __forceinline__ float kl_exp<float>(float x) { return expf(x); }
template <>
__device__ __forceinline__ double kl_exp<double>(double x) { return exp(x); }

template <typename T>
__device__ __forceinline__ T kl_sqrt(T x);
template <>
__device__ __forceinline__ float kl_sqrt<float>(float x) { return sqrtf(x); }
template <>
__device__ __forceinline__ double kl_sqrt<double>(double x) { return sqrt(x); }

}  // namespace kl
