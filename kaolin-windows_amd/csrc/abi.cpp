// abi.cpp -- error channel and version of the libkaolin_hip.so C ABI.
#include <algorithm>
#include <string>

#include "common.h"

namespace kl {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
int g_dev_flags = 0;
void *g_dev_debug = nullptr;
}  // namespace kl

// Development hook (not part of include/kaolin_hip.h): bit flags that switch parts of
// some kernels off for ablation timing (scripts/dev/ablate.py).  Results are wrong
// while any flag is set; 0 (the default) is the product path.
extern "C" void kl_dev_set_flags(int flags) { kl::g_dev_flags = flags; }
// Development hook: a device buffer some kernels write per-wave timing stamps into
// (scripts/dev/stamps.py); nullptr (the default) in the product path.
extern "C" void kl_dev_set_debug(void *buf) { kl::g_dev_debug = buf; }

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

int fill_async(void *p, int value, size_t bytes, hipStream_t st) {
  if (bytes == 0) return KL_OK;
  const uint32_t b = (uint32_t)(value & 0xff);
  const uint32_t v4 = b | (b << 8) | (b << 16) | (b << 24);
  const size_t blocks = std::min<size_t>((bytes / 16 + 255) / 256 + 1, 4096);
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (uint8_t *)p, bytes, v4);
  KL_CHECK_LAUNCH();
  return KL_OK;
}
}  // namespace kl

extern "C" const char *kl_last_error(void) { return kl::g_last_error.c_str(); }
extern "C" int kl_abi_version(void) { return 1; }
