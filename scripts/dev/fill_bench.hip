// Zero-fill variants of a 537 MB buffer (cfg4's voxelgrid), HIP events (development aid).
// build: hipcc -O3 --offload-arch=gfx950 -o scripts/dev/_bin/fill_bench scripts/dev/fill_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) fill_gs(uint4 *p, size_t n) {  // the library's form: grid-stride, 1 x 16 B
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  const uint4 v = make_uint4(0, 0, 0, 0);
  for (size_t i = t; i < n; i += nt) p[i] = v;
}
template <int U>
__global__ void __launch_bounds__(256) fill_blk(uint4 *p, size_t n) {  // U x 16 B per thread, one pass
  const size_t b = (blockIdx.x * (size_t)U) * blockDim.x + threadIdx.x;
  const uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = b + (size_t)u * blockDim.x;
    if (i < n) p[i] = v;
  }
}
template <int U>
__global__ void __launch_bounds__(256) fill_nt(uint4 *p, size_t n) {  // nontemporal stores
  const size_t b = (blockIdx.x * (size_t)U) * blockDim.x + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = b + (size_t)u * blockDim.x;
    if (i < n) {
      __builtin_nontemporal_store(0u, &p[i].x); __builtin_nontemporal_store(0u, &p[i].y);
      __builtin_nontemporal_store(0u, &p[i].z); __builtin_nontemporal_store(0u, &p[i].w);
    }
  }
}

int main() {
  const size_t bytes = (size_t)512 * 512 * 512 * 4, n = bytes / 16;
  uint4 *p;
  hipMalloc(&p, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char *name, auto fn) {
    for (int w = 0; w < 3; w++) fn();
    hipEventRecord(a);
    for (int r = 0; r < 20; r++) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e12);
  };
  run("grid-stride 4096x256", [&] { fill_gs<<<4096, 256>>>(p, n); });
  run("grid-stride 16384x256", [&] { fill_gs<<<16384, 256>>>(p, n); });
  run("one pass U=1", [&] { fill_blk<1><<<(unsigned)((n + 255) / 256), 256>>>(p, n); });
  run("one pass U=4", [&] { fill_blk<4><<<(unsigned)((n + 1023) / 1024), 256>>>(p, n); });
  run("one pass U=8", [&] { fill_blk<8><<<(unsigned)((n + 2047) / 2048), 256>>>(p, n); });
  run("nontemporal U=4", [&] { fill_nt<4><<<(unsigned)((n + 1023) / 1024), 256>>>(p, n); });
  run("hipMemsetAsync", [&] { hipMemsetAsync(p, 0, bytes, 0); });
  run("hipMemsetD32Async", [&] { hipMemsetD32Async((hipDeviceptr_t)p, 0, bytes / 4, 0); });
  hipFree(p);
  return 0;
}
