// voxel.hip -- trianglemeshes_to_voxelgrids surface voxelisation for gfx950.
//
// Reference (kaolin/ops/conversions/trianglemesh.py:29-110 -> ops/mesh/trianglemesh.py:339-457
// -> ops/conversions/pointcloud.py:22-75): iteratively split every triangle whose longest
// squared edge exceeds ((R-1)/R^2)^2 into four (midpoints v4=(v1+v3)/2, v5=(v1+v2)/2,
// v6=(v2+v3)/2), torch.unique the growing vertex list each round, then round-half-even
// every vertex * (R-1), keep [0, R-1]^3 and scatter ones into a dense grid.
//
// The occupied set is the union over faces of an independent recursion, so here:
//   * original vertices are marked directly;
//   * triangles expand breadth-first, one launch per subdivision level; only children that
//     need a further split are appended (device counter; order is irrelevant for a set), so
//     the last round writes nothing;
//   * every midpoint is rounded and stored straight into the dense output grid with
//     a plain (idempotent) store -- no unique(), no sparse tensor, no sort.
// Midpoints, edge lengths and rounding use the reference's arithmetic in the input
// precision, so the occupied voxel set is bit-identical.
#include "common.h"

#include <hip/hip_fp16.h>

namespace kl {

template <typename T>
struct Tri {
  T v[9];
};

template <typename G>
__device__ __forceinline__ G one_val() { return G(1); }
template <>
__device__ __forceinline__ __half one_val<__half>() { return __float2half(1.0f); }

template <typename T, typename G>
__device__ __forceinline__ void mark_point(T x, T y, T z, int R, G *grid) {
  const T mult = (T)(R - 1);
  const T fx = rint(x * mult), fy = rint(y * mult), fz = rint(z * mult);
  const T hi = (T)(R - 1);
  if (!(fx >= (T)0 && fy >= (T)0 && fz >= (T)0 && fx <= hi && fy <= hi && fz <= hi)) return;
  const int64_t ix = (int64_t)fx, iy = (int64_t)fy, iz = (int64_t)fz;
  grid[(ix * R + iy) * R + iz] = one_val<G>();
}

template <typename T, typename G>
__global__ void mark_vertices_kernel(int64_t V, const T *__restrict__ pts, int R, G *__restrict__ grid) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < V) mark_point<T, G>(pts[i * 3], pts[i * 3 + 1], pts[i * 3 + 2], R, grid);
}

template <typename T>
__global__ void gather_tris_kernel(int64_t F, const T *__restrict__ pts, const int64_t *__restrict__ faces,
                                   Tri<T> *__restrict__ tris) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= F) return;
  Tri<T> t;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int64_t v = faces[f * 3 + k];
    t.v[k * 3 + 0] = pts[v * 3 + 0];
    t.v[k * 3 + 1] = pts[v * 3 + 1];
    t.v[k * 3 + 2] = pts[v * 3 + 2];
  }
  tris[f] = t;
}

template <typename T>
__device__ __forceinline__ T edge2(const T *a, const T *b) {
  const T dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
  return dx * dx + dy * dy + dz * dz;
}

template <typename T>
__device__ __forceinline__ bool needs_split(const T *v, T thr) {
  const T e1 = edge2(v + 0, v + 3), e2 = edge2(v + 3, v + 6), e3 = edge2(v + 6, v + 0);
  T mx = e1;
  if (e2 > mx) mx = e2;  // torch.max over the three (NaN-free inputs)
  if (e3 > mx) mx = e3;
  return mx > thr;
}

// One subdivision round over triangles that need a split (level 0: every face, tested
// here).  The three midpoints are marked; of the four children only those that need a
// split themselves (the reference's next-round test on their own coordinates) are written:
// the others add no vertex the grid does not already hold.  The workgroup's kept children
// are counted first and reserved with ONE returning atomic (one per wave and child took 156 /
// 365 us at cfg4's first two rounds: a returning atomic on one word saturates near 88 per us).
template <typename T>
__device__ __forceinline__ void make_child(const Tri<T> &t, const T *v4, const T *v5, const T *v6, int c, Tri<T> &o) {
#pragma unroll
  for (int k = 0; k < 3; k++) {  // (v1,v4,v5),(v2,v5,v6),(v4,v5,v6),(v3,v4,v6)
    if (c == 0) { o.v[k] = t.v[k]; o.v[3 + k] = v4[k]; o.v[6 + k] = v5[k]; }
    if (c == 1) { o.v[k] = t.v[3 + k]; o.v[3 + k] = v5[k]; o.v[6 + k] = v6[k]; }
    if (c == 2) { o.v[k] = v4[k]; o.v[3 + k] = v5[k]; o.v[6 + k] = v6[k]; }
    if (c == 3) { o.v[k] = t.v[6 + k]; o.v[3 + k] = v4[k]; o.v[6 + k] = v6[k]; }
  }
}

template <typename T, typename G>
__global__ void __launch_bounds__(256) subdivide_kernel(int64_t n, const Tri<T> *__restrict__ in, bool test_input,
                                                        T thr, int R, G *__restrict__ grid, Tri<T> *__restrict__ out,
                                                        unsigned long long *__restrict__ counter) {
  __shared__ int s_wave[16];
  __shared__ unsigned long long s_base;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  bool live = false;
  Tri<T> t;
  if (i < n) {
    t = in[i];
    live = !test_input || needs_split(t.v, thr);
  }
  T v4[3], v5[3], v6[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    v4[k] = (t.v[k] + t.v[6 + k]) / (T)2;
    v5[k] = (t.v[k] + t.v[3 + k]) / (T)2;
    v6[k] = (t.v[3 + k] + t.v[6 + k]) / (T)2;
  }
  uint32_t keep = 0;
  if (live) {
    mark_point<T, G>(v4[0], v4[1], v4[2], R, grid);
    mark_point<T, G>(v5[0], v5[1], v5[2], R, grid);
    mark_point<T, G>(v6[0], v6[1], v6[2], R, grid);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      Tri<T> o;
      make_child(t, v4, v5, v6, c, o);
      if (needs_split(o.v, thr)) keep |= 1u << c;
    }
  }
  int total = 0;
  const int pre = block_exclusive_scan(__popc(keep), s_wave, &total);
  if (total == 0) return;  // uniform: every thread saw the same total
  if (threadIdx.x == 0) s_base = atomicAdd(counter, (unsigned long long)total);
  __syncthreads();
  unsigned long long o = s_base + (unsigned long long)pre;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    if (!(keep >> c & 1)) continue;
    make_child(t, v4, v5, v6, c, out[o]);
    o++;
  }
}

template <typename T, typename G>
static int voxel_mark(int64_t V, const T *pts, int64_t F, const int64_t *faces, int R, G *grid, kl_alloc_fn alloc,
                      void *ctx, hipStream_t st) {
  if (V > 0) {
    hipLaunchKernelGGL((mark_vertices_kernel<T, G>), dim3((unsigned)cdiv(V, 256)), dim3(256), 0, st, V, pts, R, grid);
    KL_CHECK_LAUNCH();
  }
  if (F == 0) return KL_OK;
  const double thr_d = (double)(R - 1) / ((double)R * (double)R);
  const T thr = (T)(thr_d * thr_d);  // python float, compared in the tensor dtype
  Tri<T> *cur = (Tri<T> *)alloc(ctx, (size_t)F * sizeof(Tri<T>));
  unsigned long long *counter = (unsigned long long *)alloc(ctx, 64);
  if (!cur || !counter) {
    set_error("trianglemeshes_to_voxelgrids: allocation failed");
    return KL_E_ALLOC;
  }
  unsigned long long *hcount = nullptr;
  KL_CHECK_HIP(hipHostMalloc((void **)&hcount, sizeof(unsigned long long), hipHostMallocDefault));
  hipLaunchKernelGGL(gather_tris_kernel<T>, dim3((unsigned)cdiv(F, 256)), dim3(256), 0, st, F, pts, faces, cur);
  KL_CHECK_LAUNCH();
  int64_t n = F;
  int rc = KL_OK;
  for (int level = 0; n > 0 && level < 64; level++) {
    Tri<T> *nxt = (Tri<T> *)alloc(ctx, (size_t)n * 4 * sizeof(Tri<T>));
    if (!nxt) {
      set_error("trianglemeshes_to_voxelgrids: allocation failed");
      rc = KL_E_ALLOC;
      break;
    }
    rc = fill_async(counter, 0, sizeof(unsigned long long), st);
    if (rc) break;
    hipLaunchKernelGGL((subdivide_kernel<T, G>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, n, cur, level == 0,
                       thr, R, grid, nxt, counter);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(hcount, counter, sizeof(unsigned long long), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      set_error("voxelgrid subdivision launch failed");
      rc = KL_E_HIP;
      break;
    }
    n = (int64_t)*hcount;
    cur = nxt;
  }
  (void)hipHostFree(hcount);
  return rc;
}

template <typename T>
static int voxel_dispatch_grid(int64_t V, const void *pts, int64_t F, const int64_t *faces, int R, kl_dtype gdt,
                               void *grid, kl_alloc_fn alloc, void *ctx, hipStream_t st) {
  switch (gdt) {
    case KL_F32: return voxel_mark<T, float>(V, (const T *)pts, F, faces, R, (float *)grid, alloc, ctx, st);
    case KL_F64: return voxel_mark<T, double>(V, (const T *)pts, F, faces, R, (double *)grid, alloc, ctx, st);
    case KL_F16: return voxel_mark<T, __half>(V, (const T *)pts, F, faces, R, (__half *)grid, alloc, ctx, st);
    case KL_U8: return voxel_mark<T, uint8_t>(V, (const T *)pts, F, faces, R, (uint8_t *)grid, alloc, ctx, st);
    default: break;
  }
  set_error("voxelgrid: unsupported grid dtype");
  return KL_E_INVALID;
}

}  // namespace kl

using namespace kl;

extern "C" int kl_voxelgrid_mark(int64_t V, const float *pts, int64_t F, const int64_t *faces, int R,
                                 kl_dtype grid_dtype, void *grid, kl_alloc_fn alloc, void *ctx, kl_stream stream) {
  KL_REQUIRE(R > 1, "trianglemeshes_to_voxelgrids: resolution must be > 1");
  KL_REQUIRE(alloc != nullptr, "trianglemeshes_to_voxelgrids: allocator required");
  return voxel_dispatch_grid<float>(V, pts, F, faces, R, grid_dtype, grid, alloc, ctx, S(stream));
}

extern "C" int kl_voxelgrid_mark_f64(int64_t V, const double *pts, int64_t F, const int64_t *faces, int R,
                                     kl_dtype grid_dtype, void *grid, kl_alloc_fn alloc, void *ctx,
                                     kl_stream stream) {
  KL_REQUIRE(R > 1, "trianglemeshes_to_voxelgrids: resolution must be > 1");
  KL_REQUIRE(alloc != nullptr, "trianglemeshes_to_voxelgrids: allocator required");
  return voxel_dispatch_grid<double>(V, pts, F, faces, R, grid_dtype, grid, alloc, ctx, S(stream));
}
