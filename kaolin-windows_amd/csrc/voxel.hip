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

#include <algorithm>

namespace kl {

template <typename T>
struct Tri {
  T v[9];
};

// (r06) the front-end's normalisation (v - origin) / scale (trianglemesh.py:78-80: a tensor subtraction
// then a division, each rounded in the vertex dtype) applied as the vertices are read, so the call
// needs no normalised copy; o == nullptr: the points are normalised already
template <typename T>
struct Norm {
  const T *o = nullptr, *s = nullptr;
  __device__ __forceinline__ T operator()(T v, int c) const { return o ? (v - o[c]) / s[0] : v; }
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

// (r06) z0 / z1 (optional): words block 0 zeroes on the way (the async path's status word and level
// counters: two launches fewer per call)
template <typename T, typename G>
__global__ void mark_vertices_kernel(int64_t V, const T *__restrict__ pts, int R, G *__restrict__ grid,
                                     Norm<T> nm = Norm<T>{}, uint32_t *z0 = nullptr, int n0 = 0,
                                     uint32_t *z1 = nullptr, int n1 = 0) {
  if (blockIdx.x == 0) {
    for (int k = threadIdx.x; k < n0; k += blockDim.x) z0[k] = 0;
    for (int k = threadIdx.x; k < n1; k += blockDim.x) z1[k] = 0;
  }
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < V) mark_point<T, G>(nm(pts[i * 3], 0), nm(pts[i * 3 + 1], 1), nm(pts[i * 3 + 2], 2), R, grid);
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
  unsigned long long hcount_v = 0, *hcount = &hcount_v;
  hipLaunchKernelGGL(gather_tris_kernel<T>, dim3((unsigned)cdiv(F, 256)), dim3(256), 0, st, F, pts, faces, cur);
  KL_CHECK_LAUNCH();
  int64_t n = F;
  int rc = KL_OK;
  // two buffers, ping-pong: a level's children overwrite the level before its parents (each
  // level only reads the previous one); a buffer is re-allocated only when a level needs more
  // room than it has, so the allocations are the growth steps, not one per level
  Tri<T> *buf[2] = {cur, nullptr};
  size_t cap[2] = {(size_t)F, 0};
  int ci = 0;
  for (int level = 0; n > 0 && level < 64; level++) {
    const int ni = 1 - ci;
    if (cap[ni] < (size_t)n * 4) {
      buf[ni] = (Tri<T> *)alloc(ctx, (size_t)n * 4 * sizeof(Tri<T>));
      cap[ni] = (size_t)n * 4;
    }
    Tri<T> *nxt = buf[ni];
    if (!nxt) {
      set_error("trianglemeshes_to_voxelgrids: allocation failed");
      rc = KL_E_ALLOC;
      break;
    }
    rc = fill_async(counter, 0, sizeof(unsigned long long), st);
    if (rc) break;
    hipLaunchKernelGGL((subdivide_kernel<T, G>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, n, buf[ci],
                       level == 0, thr, R, grid, nxt, counter);
    if (hipGetLastError() != hipSuccess) {
      set_error("voxelgrid subdivision launch failed");
      rc = KL_E_HIP;
      break;
    }
    rc = host_read(hcount, counter, sizeof(unsigned long long), st);
    if (rc) break;
    n = (int64_t)*hcount;
    ci = ni;
  }
  return rc;
}

// ---- the capturable subdivision: nothing is read back to the host.
// The levels run from fixed-capacity ping-pong buffers with every count kept on the device: a
// level's kernel reads its input count from the counter the level before advanced, and its grid
// strides over it.  The number of launched levels is fixed on the host from R alone: vertices
// normalised into [0,1]^3 (the default origin / scale) have squared edges <= 3, and midpoint
// splitting quarters them per level, so ceil(log4(3 / thr)) + 2 levels drain such a mesh.  Two
// cases leave work beyond what the buffers hold -- a level with more than `capacity` children to
// keep, or triangles still needing a split at the last launched level (a caller origin / scale
// that leaves the unit cube) -- and there the thread finishes the triangle's subtree depth-first
// itself.  The union of marked voxels does not depend on the order the subtrees are visited in,
// so the grid is the host-sized path's bit for bit.  A depth-first walk longer than
// VOX_DFS_BUDGET nodes stops and sets status bit 0 (the host-sized path fails its allocation
// at such sizes); status bit 1 records that some level overflowed `capacity` (speed only).
constexpr int VOX_DFS_BUDGET = 1 << 20;
constexpr int VOX_MAX_LEVELS = 64;  // as the host-sized loop: levels 0..63 are subdivided
constexpr size_t VOX_COUNTER_BYTES = 1024;  // level counters (65 x 8 B), then the tail kernel's ticket
constexpr size_t VOX_TICKET_AT = 768;

template <typename T>
__device__ __forceinline__ void midpoints(const Tri<T> &t, T *v4, T *v5, T *v6) {
#pragma unroll
  for (int k = 0; k < 3; k++) {
    v4[k] = (t.v[k] + t.v[6 + k]) / (T)2;
    v5[k] = (t.v[k] + t.v[3 + k]) / (T)2;
    v6[k] = (t.v[3 + k] + t.v[6 + k]) / (T)2;
  }
}

template <typename T>
__device__ __forceinline__ void child_of(const Tri<T> &t, int c, Tri<T> &o) {
  T v4[3], v5[3], v6[3];
  midpoints(t, v4, v5, v6);
  make_child(t, v4, v5, v6, c, o);
}

// marks t's three midpoints; returns the mask of its children that need a split (none at the
// last subdivided level: their midpoints are never made)
template <typename T, typename G>
__device__ __forceinline__ uint32_t expand(const Tri<T> &t, int level, T thr, int R, G *grid) {
  T v4[3], v5[3], v6[3];
  midpoints(t, v4, v5, v6);
  mark_point<T, G>(v4[0], v4[1], v4[2], R, grid);
  mark_point<T, G>(v5[0], v5[1], v5[2], R, grid);
  mark_point<T, G>(v6[0], v6[1], v6[2], R, grid);
  if (level >= VOX_MAX_LEVELS - 1) return 0;
  uint32_t keep = 0;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    Tri<T> o;
    make_child(t, v4, v5, v6, c, o);
    if (needs_split(o.v, thr)) keep |= 1u << c;
  }
  return keep;
}

// root (at `level`, needing a split) and its whole subtree, depth-first; the stack holds one
// triangle and its unvisited children per level below root
template <typename T, typename G>
__device__ __noinline__ void subdivide_dfs(Tri<T> root, int level, T thr, int R, G *grid, unsigned *status) {
  Tri<T> stk[VOX_MAX_LEVELS];
  uint8_t msk[VOX_MAX_LEVELS];
  stk[0] = root;
  msk[0] = (uint8_t)expand<T, G>(root, level, thr, R, grid);
  int sp = 0, budget = VOX_DFS_BUDGET;
  while (sp >= 0) {
    const uint32_t m = msk[sp];
    if (!m) {
      sp--;
      continue;
    }
    if (--budget < 0) {
      atomicOr(status, 1u);
      return;
    }
    // one thread over budget stops the others (the grid is incomplete either way)
    if ((budget & 1023) == 0 && (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u)) return;
    msk[sp] = (uint8_t)(m & (m - 1));
    Tri<T> ch;
    child_of(stk[sp], __ffs(m) - 1, ch);
    // expand() returns 0 at level 63, so sp + 1 <= 63 - level
    msk[sp + 1] = (uint8_t)expand<T, G>(ch, level + sp + 1, thr, R, grid);
    stk[sp + 1] = ch;
    sp++;
  }
}

// One level.  faces != null: level 0, the triangles gathered from (pts, faces) and tested here;
// else the first min(*n_in, cap) triangles of `in`.  last: every kept child is finished
// depth-first instead of appended.  The loop trip count is uniform over the workgroup.
#ifndef VOX_MIN_WAVES  // subdivide_async / tail kernels' minimum waves per SIMD (A/B builds)
#define VOX_MIN_WAVES 5  // r06: 96 VGPRs, 5 waves (98 / 97 and 4 unbounded), no spills: 1-2 % faster
#endif
// one level's grid-strided loop (subdivide_async_kernel and, per level, subdivide_tail_kernel); n is
// uniform over the grid
template <typename T, typename G>
__device__ __forceinline__ void subdivide_level(const T *__restrict__ pts, const int64_t *__restrict__ faces,
                                                Norm<T> nm, const Tri<T> *__restrict__ in, int64_t n, int level,
                                                bool last, int64_t cap, T thr, int R, G *__restrict__ grid,
                                                Tri<T> *__restrict__ out, unsigned long long *__restrict__ n_out,
                                                unsigned *__restrict__ status, int *s_wave,
                                                unsigned long long *s_base) {
  for (int64_t b0 = blockIdx.x * 256ll; b0 < n; b0 += (int64_t)gridDim.x * 256) {
    const int64_t i = b0 + threadIdx.x;
    Tri<T> t;
    uint32_t keep = 0;
    if (i < n) {
      bool live = true;
      if (faces) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const int64_t v = faces[i * 3 + k];
          t.v[k * 3 + 0] = nm(pts[v * 3 + 0], 0);
          t.v[k * 3 + 1] = nm(pts[v * 3 + 1], 1);
          t.v[k * 3 + 2] = nm(pts[v * 3 + 2], 2);
        }
        live = needs_split(t.v, thr);
      } else {
        t = in[i];
      }
      if (live) keep = expand<T, G>(t, level, thr, R, grid);
    }
    if (last) {  // grid-uniform
      for (uint32_t m = keep; m; m &= m - 1) {
        Tri<T> ch;
        child_of(t, __ffs(m) - 1, ch);
        subdivide_dfs<T, G>(ch, level + 1, thr, R, grid, status);
      }
      continue;
    }
    int total = 0;
    const int pre = block_exclusive_scan(__popc(keep), s_wave, &total);
    if (total == 0) continue;  // uniform
    if (threadIdx.x == 0) *s_base = atomicAdd(n_out, (unsigned long long)total);
    __syncthreads();
    unsigned long long o = *s_base + (unsigned long long)pre;
    __syncthreads();  // s_base is rewritten by the next trip
    for (uint32_t m = keep; m; m &= m - 1, o++) {
      Tri<T> ch;
      child_of(t, __ffs(m) - 1, ch);
      if (o < (unsigned long long)cap) {
        out[o] = ch;
      } else {
        atomicOr(status, 2u);
        subdivide_dfs<T, G>(ch, level + 1, thr, R, grid, status);
      }
    }
  }
}

template <typename T, typename G>
__global__ void __launch_bounds__(256, VOX_MIN_WAVES) subdivide_async_kernel(
    const T *__restrict__ pts, const int64_t *__restrict__ faces, int64_t F, const Tri<T> *__restrict__ in,
    const unsigned long long *__restrict__ n_in, int level, int last, int64_t cap, T thr, int R, G *__restrict__ grid,
    Tri<T> *__restrict__ out, unsigned long long *__restrict__ n_out, unsigned *__restrict__ status,
    Norm<T> nm = Norm<T>{}) {
  __shared__ int s_wave[4];
  __shared__ unsigned long long s_base;
  const int64_t n = faces ? F : (int64_t)min(*n_in, (unsigned long long)cap);
  subdivide_level<T, G>(pts, faces, nm, in, n, level, last != 0, cap, thr, R, grid, out, n_out, status, s_wave, &s_base);
}

// (r06) Levels k0 .. levels - 1 in ONE launch of co-resident workgroups: each level as
// subdivide_async_kernel's, then a grid barrier (release fence, an agent-scope ticket, acquire
// fence: the children written on one XCD are read on any other) before the next level reads its
// count.  A level with no input ends the kernel: at cfg4 (R = 512) the subdivision is done after
// level 2, and the nine empty levels it launched one by one cost ~5 us each.  The wait is bounded: a
// workgroup that waits spin_limit rounds sets status bit 2 (grid incomplete; the eager call raises)
// and stops.  buf: the two ping-pong buffers (level k reads buf[(k + 1) & 1], writes buf[k & 1]).
template <typename T, typename G>
__global__ void __launch_bounds__(256, VOX_MIN_WAVES) subdivide_tail_kernel(Tri<T> *__restrict__ buf0, Tri<T> *__restrict__ buf1,
                                                             unsigned long long *__restrict__ counter, int k0,
                                                             int levels, int64_t cap, T thr, int R,
                                                             G *__restrict__ grid, unsigned *__restrict__ status,
                                                             unsigned *__restrict__ ticket, unsigned spin_limit) {
  __shared__ int s_wave[4];
  __shared__ unsigned long long s_base;
  __shared__ int s_go;
  for (int k = k0; k < levels; k++) {
    const int64_t n = (int64_t)min(__hip_atomic_load(counter + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                   (unsigned long long)cap);
    if (n == 0) return;  // grid-uniform: read after the barrier, every add to it done
    const bool last = k == levels - 1;
    subdivide_level<T, G>(nullptr, nullptr, Norm<T>{}, (k & 1) ? buf0 : buf1, n, k, last, cap, thr, R, grid,
                          (k & 1) ? buf1 : buf0, counter + k + 1, status, s_wave, &s_base);
    if (last) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this level's children and count
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned target = gridDim.x * (unsigned)(k - k0 + 1);
      __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      int go = 1;
      while (__hip_atomic_load(ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (spins++ >= spin_limit) {
          atomicOr(status, 4u);
          go = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_go = go;
    }
    __syncthreads();
    if (!s_go) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

template <typename T>
static size_t voxel_async_ws_bytes(int64_t cap) {
  return VOX_COUNTER_BYTES + 2 * (size_t)std::max<int64_t>(cap, 0) * sizeof(Tri<T>);
}

// levels launched: enough to drain a mesh inside the unit cube (see above), at most 64
static int voxel_async_levels(int R) {
  const double e = (double)(R - 1) / ((double)R * (double)R);
  const int k = (int)std::ceil(std::log(3.0 / (e * e)) / std::log(4.0)) + 2;
  return std::max(1, std::min(VOX_MAX_LEVELS, k));
}

// co-resident workgroups of subdivide_tail_kernel<T, G> (0: not all resident / query failed)
template <typename T, typename G>
static int voxel_tail_grid(int64_t cap) {
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(subdivide_tail_kernel<T, G>),
                                                   256, 0) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (int)std::max<int64_t>(0, std::min<int64_t>({(int64_t)per_cu * ncu, cdiv(cap, 256), 2048}));
}

// levels launched one by one before subdivide_tail_kernel takes the rest (dev param 21: 1 = every level
// its own launch, as r05; 2 + v = v levels first)
constexpr int VOX_HEAD_LEVELS = 3;

template <typename T, typename G>
static int voxel_mark_async(int64_t V, const T *pts, int64_t F, const int64_t *faces, int R, G *grid, int64_t cap,
                            unsigned *status, void *ws, size_t ws_bytes, hipStream_t st, Norm<T> nm = Norm<T>{}) {
  KL_REQUIRE(cap >= 0, "trianglemeshes_to_voxelgrids: capacity must be >= 0");
  KL_REQUIRE(ws_bytes >= voxel_async_ws_bytes<T>(cap), "trianglemeshes_to_voxelgrids: workspace too small");
  KL_REQUIRE(status != nullptr, "trianglemeshes_to_voxelgrids: status required");
  unsigned long long *counter = reinterpret_cast<unsigned long long *>(ws);
  // the status word and (F > 0) the level counters with the tail kernel's ticket: zeroed by the
  // vertex kernel's block 0, or by fills when there are no vertices
  uint32_t *zc = F > 0 ? reinterpret_cast<uint32_t *>(counter) : nullptr;
  const int nzc = F > 0 ? (int)(VOX_COUNTER_BYTES / 4) : 0;
  if (V > 0) {
    hipLaunchKernelGGL((mark_vertices_kernel<T, G>), dim3((unsigned)cdiv(V, 256)), dim3(256), 0, st, V, pts, R, grid,
                       nm, (uint32_t *)status, 1, zc, nzc);
    KL_CHECK_LAUNCH();
  } else {
    KL_CHECK_RC(fill_async(status, 0, sizeof(unsigned), st));
    if (zc) KL_CHECK_RC(fill_async(zc, 0, VOX_COUNTER_BYTES, st));
  }
  if (F == 0) return KL_OK;
  const double thr_d = (double)(R - 1) / ((double)R * (double)R);
  const T thr = (T)(thr_d * thr_d);
  Tri<T> *buf[2] = {reinterpret_cast<Tri<T> *>((char *)ws + VOX_COUNTER_BYTES), nullptr};
  buf[1] = buf[0] + cap;
  const int levels = voxel_async_levels(R);
  const unsigned g_rest = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(cap, 256), 2048));
  const int dp = g_dev_param[21];
  int k0 = dp == 1 ? levels : dp >= 2 ? std::max(1, dp - 2) : VOX_HEAD_LEVELS;
  const int tg = k0 < levels ? voxel_tail_grid<T, G>(cap) : 0;
  if (tg <= 0) k0 = levels;
  for (int k = 0; k < std::min(k0, levels); k++) {
    // level k reads buf[(k - 1) & 1] (count counter[k]) and appends to buf[k & 1] (counter[k + 1])
    const unsigned g = k == 0 ? (unsigned)std::min<int64_t>(cdiv(F, 256), 4096) : g_rest;
    hipLaunchKernelGGL((subdivide_async_kernel<T, G>), dim3(g), dim3(256), 0, st, pts, k == 0 ? faces : nullptr, F,
                       (const Tri<T> *)buf[(k + 1) & 1], (const unsigned long long *)counter + k, k,
                       (int)(k == levels - 1), cap, thr, R, grid, buf[k & 1], counter + k + 1, status, nm);
    KL_CHECK_LAUNCH();
  }
  if (k0 < levels) {
    unsigned *ticket = reinterpret_cast<unsigned *>(reinterpret_cast<char *>(ws) + VOX_TICKET_AT);
    hipLaunchKernelGGL((subdivide_tail_kernel<T, G>), dim3((unsigned)tg), dim3(256), 0, st, buf[0], buf[1], counter,
                       k0, levels, cap, thr, R, grid, status, ticket, 1u << 22);
    KL_CHECK_LAUNCH();
  }
  return KL_OK;
}

template <typename T>
static int voxel_async_dispatch(int64_t V, const void *pts, int64_t F, const int64_t *faces, int R, kl_dtype gdt,
                                void *grid, int64_t cap, unsigned *status, void *ws, size_t ws_bytes,
                                hipStream_t st) {
  const T *p = (const T *)pts;
  switch (gdt) {
    case KL_F32: return voxel_mark_async<T, float>(V, p, F, faces, R, (float *)grid, cap, status, ws, ws_bytes, st);
    case KL_F64: return voxel_mark_async<T, double>(V, p, F, faces, R, (double *)grid, cap, status, ws, ws_bytes, st);
    case KL_F16: return voxel_mark_async<T, __half>(V, p, F, faces, R, (__half *)grid, cap, status, ws, ws_bytes, st);
    case KL_U8: return voxel_mark_async<T, uint8_t>(V, p, F, faces, R, (uint8_t *)grid, cap, status, ws, ws_bytes, st);
    default: break;
  }
  set_error("voxelgrid: unsupported grid dtype");
  return KL_E_INVALID;
}

// (r06) kl_voxelgrid_async: the grid zero-filled here (16-byte stores: 78 us for cfg4's 537 MB
// against torch.zeros' 104) and the vertices normalised as they are read (Norm)
template <typename T>
static int voxel_full_dispatch(int64_t V, const void *verts, const void *origin, const void *scale, int64_t F,
                               const int64_t *faces, int R, kl_dtype gdt, void *grid, int64_t cap, unsigned *status,
                               void *ws, size_t ws_bytes, hipStream_t st) {
  KL_REQUIRE(origin != nullptr && scale != nullptr, "trianglemeshes_to_voxelgrids: origin and scale required");
  const T *p = (const T *)verts;
  const Norm<T> nm{(const T *)origin, (const T *)scale};
  const size_t nvox = (size_t)R * R * R;
  switch (gdt) {
    case KL_F32:
      KL_CHECK_RC(fill_async(grid, 0, nvox * 4, st));
      return voxel_mark_async<T, float>(V, p, F, faces, R, (float *)grid, cap, status, ws, ws_bytes, st, nm);
    case KL_F64:
      KL_CHECK_RC(fill_async(grid, 0, nvox * 8, st));
      return voxel_mark_async<T, double>(V, p, F, faces, R, (double *)grid, cap, status, ws, ws_bytes, st, nm);
    case KL_F16:
      KL_CHECK_RC(fill_async(grid, 0, nvox * 2, st));
      return voxel_mark_async<T, __half>(V, p, F, faces, R, (__half *)grid, cap, status, ws, ws_bytes, st, nm);
    case KL_U8:
      KL_CHECK_RC(fill_async(grid, 0, nvox, st));
      return voxel_mark_async<T, uint8_t>(V, p, F, faces, R, (uint8_t *)grid, cap, status, ws, ws_bytes, st, nm);
    default: break;
  }
  set_error("voxelgrid: unsupported grid dtype");
  return KL_E_INVALID;
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

// ---- default origin / scale (trianglemesh.py:74-77): per mesh, origin = min over the
// vertices of each coordinate, scale = max over the coordinates of (max - origin).  Min / max
// are order-independent, so a block reduction plus atomicMin / atomicMax on order-preserving
// integer keys gives torch.min / torch.max's values exactly; a NaN coordinate makes the mesh's
// results NaN, as torch's reductions propagate it.  (torch's two dim=1 reductions over the
// 100k x 3 vertices took ~100 us at cfg4: three outputs per mesh parallelise poorly.)
template <typename T>
struct OKey;
template <>
struct OKey<float> {
  using U = unsigned int;
  __device__ static U key(float f) {
    const U b = __float_as_uint(f);
    return (b >> 31) ? ~b : (b | 0x80000000u);
  }
  __device__ static float val(U k) { return __uint_as_float((k >> 31) ? (k & 0x7fffffffu) : ~k); }
};
template <>
struct OKey<double> {
  using U = unsigned long long;
  __device__ static U key(double f) {
    const U b = (U)__double_as_longlong(f);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  }
  __device__ static double val(U k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
  }
};

// acc per mesh: [min x, y, z, max x, y, z, nan x, y, z]
template <typename T>
__global__ void __launch_bounds__(256) bounds_init_kernel(int B, typename OKey<T>::U *__restrict__ acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * 9) acc[i] = (i % 9) < 3 ? ~(typename OKey<T>::U)0 : (typename OKey<T>::U)0;
}

template <typename T>
__global__ void __launch_bounds__(256) bounds_reduce_kernel(int64_t V, const T *__restrict__ pts,
                                                            typename OKey<T>::U *__restrict__ acc) {
  using U = typename OKey<T>::U;
  __shared__ U s_r[4][9];
  const int b = blockIdx.y;
  U mn[3] = {~(U)0, ~(U)0, ~(U)0}, mx[3] = {0, 0, 0};
  U nan[3] = {0, 0, 0};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const T v = pts[((int64_t)b * V + i) * 3 + c];
      if (v != v) nan[c] = 1;
      const U k = OKey<T>::key(v);
      mn[c] = k < mn[c] ? k : mn[c];
      mx[c] = k > mx[c] ? k : mx[c];
    }
  }
  U r[9] = {mn[0], mn[1], mn[2], mx[0], mx[1], mx[2], nan[0], nan[1], nan[2]};
#pragma unroll
  for (int q = 0; q < 9; q++)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const U u = __shfl_xor(r[q], o);
      r[q] = q < 3 ? (u < r[q] ? u : r[q]) : (u > r[q] ? u : r[q]);
    }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < 9; q++) s_r[wid][q] = r[q];
  __syncthreads();
  if (threadIdx.x < 9) {
    const int q = threadIdx.x;
    U a = s_r[0][q];
    for (int w = 1; w < 4; w++) a = q < 3 ? (s_r[w][q] < a ? s_r[w][q] : a) : (s_r[w][q] > a ? s_r[w][q] : a);
    if (q < 3)
      atomicMin(acc + b * 9 + q, a);
    else
      atomicMax(acc + b * 9 + q, a);
  }
}

template <typename T>
__global__ void bounds_final_kernel(int B, const typename OKey<T>::U *__restrict__ acc, T *__restrict__ origin,
                                    T *__restrict__ scale) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const typename OKey<T>::U *a = acc + b * 9;
  T s = (T)0;
  for (int c = 0; c < 3; c++) {
    const bool nan = a[6 + c] != 0;  // torch's min / max propagate a NaN of the coordinate
    const T lo = nan ? (T)NAN : OKey<T>::val(a[c]), hi = nan ? (T)NAN : OKey<T>::val(a[3 + c]);
    origin[b * 3 + c] = lo;
    const T d = hi - lo;  // torch.max(dim=1): NaN propagates
    if (c == 0 || d > s || d != d) s = (s != s) ? s : d;
  }
  scale[b] = s;
}

template <typename T>
static int voxel_bounds(int B, int64_t V, const T *pts, T *origin, T *scale, void *ws, size_t ws_bytes,
                        hipStream_t st) {
  using U = typename OKey<T>::U;
  KL_REQUIRE(ws_bytes >= (size_t)B * 9 * sizeof(U), "voxelgrid bounds: workspace too small");
  KL_REQUIRE(V > 0, "voxelgrid bounds: no vertices");
  if (B == 0) return KL_OK;
  U *acc = reinterpret_cast<U *>(ws);
  hipLaunchKernelGGL(bounds_init_kernel<T>, dim3((unsigned)cdiv(B * 9, 256)), dim3(256), 0, st, B, acc);
  KL_CHECK_LAUNCH();
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(V, 256), 256);
  hipLaunchKernelGGL(bounds_reduce_kernel<T>, dim3(gx, B), dim3(256), 0, st, V, pts, acc);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL(bounds_final_kernel<T>, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, st, B, (const U *)acc, origin,
                     scale);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_voxelgrid_bounds_workspace_bytes(int batch) { return (size_t)(batch > 0 ? batch : 1) * 9 * 8; }

extern "C" int kl_voxelgrid_bounds(kl_dtype dtype, int batch, int64_t num_vertices, const void *vertices,
                                   void *origin, void *scale, void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return voxel_bounds<float>(batch, num_vertices, (const float *)vertices, (float *)origin, (float *)scale, ws,
                               ws_bytes, S(stream));
  if (dtype == KL_F64)
    return voxel_bounds<double>(batch, num_vertices, (const double *)vertices, (double *)origin, (double *)scale, ws,
                                ws_bytes, S(stream));
  set_error("trianglemeshes_to_voxelgrids bounds: f32 / f64 only");
  return KL_E_INVALID;
}

extern "C" int kl_voxelgrid_mark(int64_t V, const float *pts, int64_t F, const int64_t *faces, int R,
                                 kl_dtype grid_dtype, void *grid, kl_alloc_fn alloc, void *ctx, kl_stream stream) {
  KL_REQUIRE(R > 1, "trianglemeshes_to_voxelgrids: resolution must be > 1");
  KL_REQUIRE(alloc != nullptr, "trianglemeshes_to_voxelgrids: allocator required");
  return voxel_dispatch_grid<float>(V, pts, F, faces, R, grid_dtype, grid, alloc, ctx, S(stream));
}

extern "C" size_t kl_voxelgrid_mark_async_workspace_bytes(kl_dtype point_dtype, int64_t capacity) {
  return point_dtype == KL_F64 ? voxel_async_ws_bytes<double>(capacity) : voxel_async_ws_bytes<float>(capacity);
}

extern "C" int kl_voxelgrid_mark_async(kl_dtype point_dtype, int64_t V, const void *pts, int64_t F,
                                       const int64_t *faces, int R, kl_dtype grid_dtype, void *grid, int64_t capacity,
                                       uint32_t *status, void *ws, size_t ws_bytes, kl_stream stream) {
  KL_REQUIRE(R > 1, "trianglemeshes_to_voxelgrids: resolution must be > 1");
  if (point_dtype == KL_F32)
    return voxel_async_dispatch<float>(V, pts, F, faces, R, grid_dtype, grid, capacity, status, ws, ws_bytes,
                                       S(stream));
  if (point_dtype == KL_F64)
    return voxel_async_dispatch<double>(V, pts, F, faces, R, grid_dtype, grid, capacity, status, ws, ws_bytes,
                                        S(stream));
  set_error("trianglemeshes_to_voxelgrids: f32 / f64 points only");
  return KL_E_INVALID;
}

extern "C" int kl_voxelgrid_async(kl_dtype dtype, int64_t V, const void *vertices, const void *origin,
                                  const void *scale, int64_t F, const int64_t *faces, int R, kl_dtype grid_dtype,
                                  void *grid, int64_t capacity, uint32_t *status, void *ws, size_t ws_bytes,
                                  kl_stream stream) {
  KL_REQUIRE(R > 1, "trianglemeshes_to_voxelgrids: resolution must be > 1");
  if (dtype == KL_F32)
    return voxel_full_dispatch<float>(V, vertices, origin, scale, F, faces, R, grid_dtype, grid, capacity, status, ws,
                                      ws_bytes, S(stream));
  if (dtype == KL_F64)
    return voxel_full_dispatch<double>(V, vertices, origin, scale, F, faces, R, grid_dtype, grid, capacity, status, ws,
                                       ws_bytes, S(stream));
  set_error("trianglemeshes_to_voxelgrids: f32 / f64 vertices only");
  return KL_E_INVALID;
}

extern "C" int kl_voxelgrid_mark_f64(int64_t V, const double *pts, int64_t F, const int64_t *faces, int R,
                                     kl_dtype grid_dtype, void *grid, kl_alloc_fn alloc, void *ctx,
                                     kl_stream stream) {
  KL_REQUIRE(R > 1, "trianglemeshes_to_voxelgrids: resolution must be > 1");
  KL_REQUIRE(alloc != nullptr, "trianglemeshes_to_voxelgrids: allocator required");
  return voxel_dispatch_grid<double>(V, pts, F, faces, R, grid_dtype, grid, alloc, ctx, S(stream));
}
