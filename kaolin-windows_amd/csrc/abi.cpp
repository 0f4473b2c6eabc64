// abi.cpp -- error channel and version of the libkaolin_hip.so C ABI.
#include <algorithm>
#include <cstring>

#include <string>

#include "common.h"

namespace kl {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
#if KL_DEV
int g_dev_flags = 0;
void *g_dev_debug = nullptr;
int g_dev_param[32] = {};
int g_dev_stat[4] = {};
#endif
}  // namespace kl

#if KL_DEV  // the dev build only (make dev): none of these is in the product library

// Development hook (not part of include/kaolin_hip.h): bit flags that switch parts of
// some kernels off for ablation timing (scripts/dev/ablate.py).  Results are wrong
// while any flag is set; 0 (the default) is the product path.
extern "C" void kl_dev_set_flags(int flags) { kl::g_dev_flags = flags; }
// Development hook: a device buffer some kernels write per-wave timing stamps into
// (scripts/dev/stamps.py); nullptr (the default) in the product path.
extern "C" void kl_dev_set_debug(void *buf) { kl::g_dev_debug = buf; }
// Development hook: tuning parameters for sweeps (scripts/dev/stamps.py); 0 = built-in value.
// 0..3: the soft-mask forward's split thresholds / caps (tileorder.h, SoftSplit).
extern "C" void kl_dev_set_param(int idx, int value) {
  if (idx >= 0 && idx < 32) kl::g_dev_param[idx] = value;
}
// Development hook: what the last call took (tests assert a fallback branch ran).
// 0: mesh_to_spc -- 0 the node-rank path, 1 its per-level fallback (the pair buffers overflowed).
// 1: raytrace (host-sized entry) -- 4 the hit-list march (the default), 5 the hit-list march
//    outgrew its list buffers and the per-level march was rerun, 0 the per-level march alone
//    (dev param 15 = 2), 1 the fused march (15 = 3), 2 the fused march truncated and the per-level
//    march rerun, 3 the depth-first march (15 = 4).
extern "C" int kl_dev_get_stat(int idx) { return idx >= 0 && idx < 4 ? kl::g_dev_stat[idx] : 0; }
// 1 in the dev build (tests/conftest.py: the devlib tests need it)
extern "C" int kl_dev_build() { return 1; }
#endif

namespace kl {
// Byte fill as an ordinary kernel: 16-byte stores over the aligned body, bytes at the
// ends.  Used instead of hipMemsetAsync so that every fill is a kernel node when the
// caller captures our work in a HIP graph.
__global__ void __launch_bounds__(256) fill_kernel(uint8_t *__restrict__ p, size_t bytes, uint32_t v4) {
  const size_t head = (16 - ((uintptr_t)p & 15)) & 15;
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t nt = (size_t)gridDim.x * blockDim.x;
  if (head >= bytes) {
    for (size_t i = t; i < bytes; i += nt) p[i] = (uint8_t)v4;
    return;
  }
  if (t < head) p[t] = (uint8_t)v4;
  uint8_t *body = p + head;
  const size_t nvec = (bytes - head) / 16;
  const uint4 v = make_uint4(v4, v4, v4, v4);
  for (size_t i = t; i < nvec; i += nt) reinterpret_cast<uint4 *>(body)[i] = v;
  const size_t done = head + nvec * 16;
  if (t < bytes - done) p[done + t] = (uint8_t)v4;
}

int host_read(void *dst, const void *src, size_t bytes, hipStream_t st) {
  static thread_local void *pinned = nullptr;
  static thread_local size_t pinned_bytes = 0;
  if (bytes > pinned_bytes) {
    const size_t want = bytes < 4096 ? 4096 : bytes;
    void *p = nullptr;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      set_error("host_read: pinned allocation failed");
      return KL_E_HIP;
    }
    if (pinned) (void)hipHostFree(pinned);  // grown: rare (the first calls only)
    pinned = p;
    pinned_bytes = want;
  }
  if (hipMemcpyAsync(pinned, src, bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    set_error("host_read: device to host copy failed");
    return KL_E_HIP;
  }
  std::memcpy(dst, pinned, bytes);
  return KL_OK;
}

int fill_async(void *p, int value, size_t bytes, hipStream_t st) {
  if (bytes == 0) return KL_OK;
  const uint32_t b = (uint32_t)(value & 0xff);
  const uint32_t v4 = b | (b << 8) | (b << 16) | (b << 24);
  // one 16-byte store per thread in one pass (r06, scripts/dev/fill_bench.hip on 537 MB: 79.8 us, 6.7 TB/s,
  // against 127 us for a 4096-workgroup grid-stride loop); the loop only past 2^20 workgroups (16 GB)
  const size_t blocks = std::min<size_t>((bytes / 16 + 255) / 256 + 1, (size_t)1 << 20);
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (uint8_t *)p, bytes, v4);
  KL_CHECK_LAUNCH();
  return KL_OK;
}
}  // namespace kl


extern "C" const char *kl_last_error(void) { return kl::g_last_error.c_str(); }

extern "C" int kl_stream_is_capturing(kl_stream stream) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(reinterpret_cast<hipStream_t>(stream), &cs) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return cs == hipStreamCaptureStatusActive ? 1 : 0;
}
// 2: workspace arguments before the stream in kl_rasterize_backward, kl_dibr_soft_mask_backward(_fused),
//    kl_unbatched_triangle_distance_backward; num_faces in kl_soft_mask_compact_bwd_workspace_bytes
extern "C" int kl_abi_version(void) { return KL_ABI_VERSION; }

// ---- Training-loop helper (not a reference op): L = <a, ga> + <b, gb>.
// A loss of this shape is what bench.py's step computes; two torch.dot calls plus their add cost
// four launches.  ONE launch: each workgroup folds float4 strips of both pairs in double and
// publishes its partial; the workgroup whose ticket comes last adds the partials in block order
// (deterministic) and resets the ticket.  The hand-off is MI355X_MICROARCH.md's first measured
// `sc1` row: one lane per workgroup stores its 8-B partial `sc1` (a relaxed agent-scope atomic
// store), waits vmcnt(0), then adds to its group's agent-scope ticket (common.h grid_last: two
// levels, r05); the last adder's workgroup loads
// the partials `sc1` behind a workgroup barrier -- no release / acquire fences (a device-scope
// release per block measured 29 us here in r03, hence the old second launch).  One workgroup per
// CU, as that row was measured.
namespace kl {
constexpr int DOT2_BLOCKS = 256;

// Both pairs' float4 strips as one index space (a's, then b's), DOT2_U strips per thread in flight
// together: at cfg3 every thread folds exactly 4 (r06: the former per-pair loop ran its 3 + 1
// iterations one memory round trip after another, 9.6 us).  Scalar tails last.
constexpr int DOT2_U = 4;
__device__ __forceinline__ double dot_pairs(const float *__restrict__ a, const float *__restrict__ ga, size_t na,
                                            const float *__restrict__ b, const float *__restrict__ gb, size_t nb,
                                            size_t t, size_t nt) {
  double s = 0.0;
  const size_t n4a = ((uintptr_t)a % 16 == 0 && (uintptr_t)ga % 16 == 0) ? na / 4 : 0;
  const size_t n4b = ((uintptr_t)b % 16 == 0 && (uintptr_t)gb % 16 == 0) ? nb / 4 : 0;
  const size_t n4 = n4a + n4b;
  const float4 *a4 = reinterpret_cast<const float4 *>(a), *ga4 = reinterpret_cast<const float4 *>(ga);
  const float4 *b4 = reinterpret_cast<const float4 *>(b), *gb4 = reinterpret_cast<const float4 *>(gb);
  for (size_t i0 = t; i0 < n4; i0 += DOT2_U * nt) {
    float4 x[DOT2_U], y[DOT2_U];
#pragma unroll
    for (int u = 0; u < DOT2_U; u++) {
      size_t i = i0 + u * nt;
      i = i < n4 ? i : i0;  // (a valid strip stands in past the end)
      x[u] = i < n4a ? a4[i] : b4[i - n4a];
      y[u] = i < n4a ? ga4[i] : gb4[i - n4a];
    }
#pragma unroll
    for (int u = 0; u < DOT2_U; u++)
      if (i0 + u * nt < n4)
        s += (double)(x[u].x * y[u].x) + (double)(x[u].y * y[u].y) + (double)(x[u].z * y[u].z) +
             (double)(x[u].w * y[u].w);
  }
  for (size_t i = n4a * 4 + t; i < na; i += nt) s += (double)(a[i] * ga[i]);
  for (size_t i = n4b * 4 + t; i < nb; i += nt) s += (double)(b[i] * gb[i]);
  return s;
}

constexpr int DOT2_THREADS = 1024;  // 16 waves: the loads in flight of one workgroup per CU

__device__ __forceinline__ double block_sum(double s, double *red) {
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int w = 0; w < DOT2_THREADS / 64; w++) r += red[w];
  __syncthreads();  // red is reused by the last workgroup's second sum
  return r;
}

__global__ void __launch_bounds__(DOT2_THREADS) dot2_kernel(const float *__restrict__ a, const float *__restrict__ ga, size_t na,
                                                   const float *__restrict__ b, const float *__restrict__ gb,
                                                   size_t nb, double *__restrict__ partial,
                                                   unsigned int *__restrict__ ticket, float *__restrict__ out) {
  __shared__ double red[DOT2_THREADS / 64];
  __shared__ int s_last;
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  const double s = block_sum(dot_pairs(a, ga, na, b, gb, nb, t, nt), red);
  if (threadIdx.x == 0) __hip_atomic_store(partial + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!grid_last(ticket, &s_last)) return;
  double v = 0.0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x)
    v += __hip_atomic_load(partial + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v = block_sum(v, red);
  if (threadIdx.x == 0) out[0] = (float)v;
}
}  // namespace kl

// workspace: the partials, then the tickets (zero before the first call; every call leaves them zero)
extern "C" size_t kl_loss_dot2_workspace_bytes(void) {
  return kl::DOT2_BLOCKS * sizeof(double) + kl::gl_ticket_words(kl::DOT2_BLOCKS) * 4;
}

extern "C" int kl_loss_dot2(const float *a, const float *ga, int64_t na, const float *b, const float *gb, int64_t nb,
                            void *ws, float *out, kl_stream stream) {
  if (na < 0 || nb < 0 || !out || !ws) {
    kl::set_error("kl_loss_dot2: bad arguments");
    return KL_E_INVALID;
  }
  double *partial = (double *)ws;
  unsigned int *ticket = (unsigned int *)(partial + kl::DOT2_BLOCKS);
  const int64_t vec = (na + nb) / 4;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kl::DOT2_BLOCKS, (vec + 2047) / 2048));
  hipLaunchKernelGGL(kl::dot2_kernel, dim3(blocks), dim3(kl::DOT2_THREADS), 0, (hipStream_t)stream, a, ga, (size_t)na, b, gb,
                     (size_t)nb, partial, ticket, out);
  KL_CHECK_LAUNCH();
  return KL_OK;
}
