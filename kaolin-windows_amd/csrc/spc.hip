// spc.hip -- structured point cloud paths for gfx950: mesh -> SPC conversion,
// morton -> octree, octree scan / point generation and the level-synchronous ray march.
//
// References:
//   mesh_to_spc       kaolin/csrc/ops/conversions/mesh_to_spc/mesh_to_spc_cuda.cu:59-463
//   morton_to_octree  kaolin/csrc/ops/spc/spc_cuda.cu:45-163
//   scan_octrees      kaolin/csrc/ops/spc/scan_octrees.cu:43-114
//   generate_points   kaolin/csrc/ops/spc/generate_points.cu:28-81 (+ spc_utils.cuh:140-160)
//   raytrace          kaolin/csrc/render/spc/raytrace_cuda.cu:63-304,485-607
//                     kaolin/csrc/render/spc/spc_render_utils.cuh:21-143
//
// Differences in structure (not in results):
//   * every kernel runs on the caller's stream (the reference used the legacy default
//     stream with synchronous cudaMemcpy);
//   * mesh_to_spc keeps each level's nodes as a sorted list numbered by a scan of its octree row
//     (no sort; mesh_to_spc_nodes): one host read per call, none in the fixed-capacity form; the
//     per-level path (one 4-byte count read per level) remains the overflow fallback; the whole
//     pyramid of scan_octrees is computed on device and read back once;
//   * the child order of the ray march (VOXEL_ORDER) is derived, not tabulated:
//     children sorted by (popcount(code ^ j), j).
#include "common.h"

#include <hipcub/hipcub.hpp>

#include <vector>

namespace kl {

constexpr int SPC_MAX_LEVELS = 15;

__host__ __device__ __forceinline__ uint64_t to_morton(int x, int y, int z) {
  uint64_t m = 0;
  const uint64_t X = (uint16_t)x, Y = (uint16_t)y, Z = (uint16_t)z;
#pragma unroll
  for (unsigned i = 0; i < SPC_MAX_LEVELS; i++) {
    const unsigned i2 = i + i;
    m |= (Z & (1ull << i)) << i2;
    m |= (Y & (1ull << i)) << (i2 + 1);
    m |= (X & (1ull << i)) << (i2 + 2);
  }
  return m;
}

__host__ __device__ __forceinline__ void to_point(uint64_t m, int16_t &px, int16_t &py, int16_t &pz) {
  uint16_t x = 0, y = 0, z = 0;
#pragma unroll
  for (int i = 0; i < SPC_MAX_LEVELS; i++) {
    x |= (uint16_t)((m & (1ull << (3 * i + 2))) >> (2 * i + 2));
    y |= (uint16_t)((m & (1ull << (3 * i + 1))) >> (2 * i + 1));
    z |= (uint16_t)((m & (1ull << (3 * i + 0))) >> (2 * i + 0));
  }
  px = (int16_t)x;
  py = (int16_t)y;
  pz = (int16_t)z;
}

// ------------------------------------------------------------------ scan helper
// Exclusive scan of n uint32 into out (n+1 entries, out[n] = total); returns total on host.
struct Scratch {
  kl_alloc_fn alloc;
  void *ctx;
  void *get(size_t bytes) { return alloc(ctx, bytes > 0 ? bytes : 16); }
};

// Temporaries of one phase from ONE allocation: each allocation through the caller's allocator
// is a host callback (torch's caching allocator via ctypes, ~5-10 us), and after a host read the
// GPU idles while the host allocates.  Requests past the chunk go to the parent allocator;
// outputs handed back to the caller must come from the parent itself.
struct Bump {
  Scratch *parent;
  char *p;
  size_t left;
};
static void *bump_alloc(void *ctx, size_t bytes) {
  Bump *b = static_cast<Bump *>(ctx);
  const size_t need = (std::max<size_t>(bytes, 16) + 255) & ~(size_t)255;
  if (b->p && need <= b->left) {
    void *r = b->p;
    b->p += need;
    b->left -= need;
    return r;
  }
  return b->parent->get(bytes);
}
static size_t al256b(size_t v) { return (std::max<size_t>(v, 16) + 255) & ~(size_t)255; }
static size_t scan_tmp_bytes(int64_t n) {
  size_t tb = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n + 1);
  return tb;
}

static int exclusive_scan(const uint32_t *in, uint32_t *out, int64_t n, Scratch &sc, hipStream_t st,
                          uint32_t *total_host) {
  size_t tb = 0;
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int)n + 1, st));
  void *tmp = sc.get(tb);
  if (!tmp) return KL_E_ALLOC;
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, (int)n + 1, st));
  if (total_host) return host_read(total_host, out + n, sizeof(uint32_t), st);
  return KL_OK;
}

// ------------------------------------------------------------------ mesh_to_spc
struct D3 {
  double x, y, z;
};
__device__ __forceinline__ D3 d3(double x, double y, double z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 dsub(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ double ddot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ D3 dcross(D3 a, D3 b) {
  return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ D3 dnorm(D3 v) {
  const double inv = 1.0 / sqrt(ddot(v, v));
  return d3(inv * v.x, inv * v.y, inv * v.z);
}

// TriangleVoxelSAT (mesh_to_spc_cuda.cu:96-111): fp64 projections, float-cast compare
__device__ __forceinline__ bool sat_axis(D3 v0, D3 v1, D3 v2, float h, D3 axis) {
  const double d0 = ddot(v0, axis), d1 = ddot(v1, axis), d2 = ddot(v2, axis);
  const double maxd = fmax(d0, fmax(d1, d2));
  const double mind = fmin(d0, fmin(d1, d2));
  const double r = (double)h * (fabs(axis.x) + fabs(axis.y) + fabs(axis.z));
  const float fd = (float)fmax(-maxd, mind);
  const float fr = (float)r;
  return fd <= fr;
}

__device__ bool tri_voxel_test(const float *fa, const float *fb, const float *fc, float cx, float cy, float cz,
                               float h) {
  const D3 va = d3((double)(fa[0] - cx), (double)(fa[1] - cy), (double)(fa[2] - cz));
  const D3 vb = d3((double)(fb[0] - cx), (double)(fb[1] - cy), (double)(fb[2] - cz));
  const D3 vc = d3((double)(fc[0] - cx), (double)(fc[1] - cy), (double)(fc[2] - cz));
  const D3 ab = dnorm(dsub(vb, va)), bc = dnorm(dsub(vc, vb)), ca = dnorm(dsub(va, vc));
  if (!sat_axis(va, vb, vc, h, d3(0.0, -ab.z, ab.y))) return false;
  if (!sat_axis(va, vb, vc, h, d3(0.0, -bc.z, bc.y))) return false;
  if (!sat_axis(va, vb, vc, h, d3(0.0, -ca.z, ca.y))) return false;
  if (!sat_axis(va, vb, vc, h, d3(ab.z, 0.0, -ab.x))) return false;
  if (!sat_axis(va, vb, vc, h, d3(bc.z, 0.0, -bc.x))) return false;
  if (!sat_axis(va, vb, vc, h, d3(ca.z, 0.0, -ca.x))) return false;
  if (!sat_axis(va, vb, vc, h, d3(-ab.y, ab.x, 0.0))) return false;
  if (!sat_axis(va, vb, vc, h, d3(-bc.y, bc.x, 0.0))) return false;
  if (!sat_axis(va, vb, vc, h, d3(-ca.y, ca.x, 0.0))) return false;
  if (!sat_axis(va, vb, vc, h, d3(1, 0, 0))) return false;
  if (!sat_axis(va, vb, vc, h, d3(0, 1, 0))) return false;
  if (!sat_axis(va, vb, vc, h, d3(0, 0, 1))) return false;
  if (!sat_axis(va, vb, vc, h, dcross(ab, bc))) return false;
  return true;
}

// A float pre-test of tri_voxel_test: false only where tri_voxel_test is false (the SAT is a
// conjunction of independent axis tests, so any axis that separates decides it).
//  * The box axes (1,0,0), (0,1,0), (0,0,1): sat_axis projects v_k exactly (d_k = v_k.x * 1 +
//    v_k.y * 0 + v_k.z * 0 = v_k.x for finite coordinates, already a float) and compares
//    (float)max(-max d, min d) with (float)(h * 1) = h -- the same float comparison as here, so
//    these three decide exactly as the full test does.
//  * The triangle's normal, conservatively: with E1 = vb - va, E2 = vc - vb and N = E1 x E2 in
//    float, S = max(-max_k v_k.N, min_k v_k.N) - h |N|_1 differs from the exact (unit-normal)
//    separation, scaled by |e1 x e2|, by far less than 2^-14 (Vm + h) 12 |E1|inf |E2|inf (Vm the
//    largest |coordinate| of the v_k; float products and sums of 3 terms, the edge roundings, the
//    full test's own double rounding and its two float casts are each a few 2^-24 of that), so
//    S > that slack proves the full test's normal axis separates.  Non-finite inputs or a
//    degenerate triangle (slack 0) are left to the full test.
// Most of a level's proposals (8 children of each occupied parent per face) are separated by a
// box axis or the plane; the full fp64 test then runs only on this test's survivors, compacted
// into coherent waves (r04's first step; now the per-level fallback's and the root's pre-test).
__device__ __forceinline__ bool tri_voxel_maybe(const float *fa, const float *fb, const float *fc, float cx, float cy,
                                                float cz, float h) {
  const float ax = fa[0] - cx, ay = fa[1] - cy, az = fa[2] - cz;
  const float bx = fb[0] - cx, by = fb[1] - cy, bz = fb[2] - cz;
  const float qx = fc[0] - cx, qy = fc[1] - cy, qz = fc[2] - cz;
  const float vm = fmaxf(fmaxf(fmaxf(fabsf(ax), fabsf(ay)), fmaxf(fabsf(az), fabsf(bx))),
                         fmaxf(fmaxf(fabsf(by), fabsf(bz)), fmaxf(fmaxf(fabsf(qx), fabsf(qy)), fabsf(qz))));
  if (!(vm < 1e30f)) return true;  // NaN / inf / huge: the full test decides
  if (fminf(ax, fminf(bx, qx)) > h || fmaxf(ax, fmaxf(bx, qx)) < -h) return false;
  if (fminf(ay, fminf(by, qy)) > h || fmaxf(ay, fmaxf(by, qy)) < -h) return false;
  if (fminf(az, fminf(bz, qz)) > h || fmaxf(az, fmaxf(bz, qz)) < -h) return false;
  const float e1x = bx - ax, e1y = by - ay, e1z = bz - az;
  const float e2x = qx - bx, e2y = qy - by, e2z = qz - bz;
  const float nx = e1y * e2z - e1z * e2y, ny = e1z * e2x - e1x * e2z, nz = e1x * e2y - e1y * e2x;
  const float d0 = ax * nx + ay * ny + az * nz, d1 = bx * nx + by * ny + bz * nz, d2 = qx * nx + qy * ny + qz * nz;
  const float sep = fmaxf(-fmaxf(d0, fmaxf(d1, d2)), fminf(d0, fminf(d1, d2))) - h * (fabsf(nx) + fabsf(ny) + fabsf(nz));
  const float e1m = fmaxf(fabsf(e1x), fmaxf(fabsf(e1y), fabsf(e1z))), e2m = fmaxf(fabsf(e2x), fmaxf(fabsf(e2y), fabsf(e2z)));
  const float slack = (12.0f / 16384.0f) * (vm + h) * e1m * e2m;
  return !(sep > slack);
}

__device__ __forceinline__ void voxel_center(uint64_t m, uint32_t level, float &cx, float &cy, float &cz,
                                             float &h) {
  const float two_level = (float)(1u << level);
  const float vs = 2.0f / two_level;
  h = (float)(0.5 * vs);
  int16_t px, py, pz;
  to_point(m, px, py, pz);
  cx = fmaf((float)px, vs, h - 1.0f);
  cy = fmaf((float)py, vs, h - 1.0f);
  cz = fmaf((float)pz, vs, h - 1.0f);
}

__global__ void m2s_decide_kernel(int64_t num, const float *__restrict__ fv, const uint64_t *__restrict__ morton,
                                  const int64_t *__restrict__ tri, uint32_t *__restrict__ occ, uint32_t level,
                                  uint32_t not_done) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t > num) return;
  if (t == num) {
    occ[t] = 0;
    return;
  }
  float cx, cy, cz, h;
  voxel_center(morton[t], level, cx, cy, cz, h);
  const float *v = fv + tri[t] * 9;
  occ[t] = tri_voxel_maybe(v, v + 3, v + 6, cx, cy, cz, h) && tri_voxel_test(v, v + 3, v + 6, cx, cy, cz, h)
               ? (not_done ? 8u : 1u)
               : 0u;
}

__global__ void m2s_subdivide_kernel(int64_t num, const uint64_t *__restrict__ min_, const int64_t *__restrict__ tin,
                                     uint64_t *__restrict__ mout, int64_t *__restrict__ tout,
                                     const uint32_t *__restrict__ occ, const uint32_t *__restrict__ psum,
                                     int subdivide) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= num || !occ[t]) return;
  const int64_t tr = tin[t];
  uint32_t o = psum[t];
  if (!subdivide) {
    mout[o] = min_[t];
    tout[o] = tr;
    return;
  }
  int16_t px, py, pz;
  to_point(min_[t], px, py, pz);
  for (uint32_t i = 0; i < 8; i++) {
    mout[o] = to_morton(2 * px + (i >> 2), 2 * py + ((i >> 1) & 1), 2 * pz + (i & 1));
    tout[o] = tr;
    o++;
  }
}

__global__ void mark_unique_kernel(int64_t num, const uint64_t *__restrict__ m, uint32_t *__restrict__ flag) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t > num) return;
  flag[t] = (t == num) ? 0u : ((t == 0 || m[t - 1] != m[t]) ? 1u : 0u);
}

// float closest point (spc_math.h:229-258), used for the leaf barycentrics
struct F3 {
  float x, y, z;
};
__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 fsub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ F3 fadd(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ F3 fmul(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float fdot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ F3 fcross(F3 a, F3 b) {
  return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float fpe(F3 v, F3 e, F3 p) {
  const F3 pv = fsub(p, v);
  const float len = fdot(e, e);
  return fdot(pv, e) / len;
}
__device__ __forceinline__ bool fna(F3 v, F3 e, F3 n, F3 p) { return fdot(fcross(n, e), fsub(p, v)) <= 0; }

__device__ F3 tri_closest(F3 v1, F3 v2, F3 v3, F3 p) {
  const F3 e12 = fsub(v2, v1), e23 = fsub(v3, v2), e31 = fsub(v1, v3);
  const F3 n = fcross(fsub(v1, v2), e31);
  const float uab = fpe(v1, e12, p), uca = fpe(v3, e31, p);
  if (uca > 1 && uab < 0) return v1;
  const float ubc = fpe(v2, e23, p);
  if (uab > 1 && ubc < 0) return v2;
  if (ubc > 1 && uca < 0) return v3;
  if (uab <= 1.f && uab >= 0.f && fna(v1, e12, n, p)) return fadd(v1, fmul(e12, uab));
  if (ubc <= 1.f && ubc >= 0.f && fna(v2, e23, n, p)) return fadd(v2, fmul(e23, ubc));
  if (uca <= 1.f && uca >= 0.f && fna(v3, e31, n, p)) return fadd(v3, fmul(e31, uca));
  const float inv = 1.0f / sqrtf(fdot(n, n));
  const F3 un = fmul(n, inv);
  const float dist = (p.x - v1.x) * un.x + (p.y - v1.y) * un.y + (p.z - v1.z) * un.z;
  return fsub(p, fmul(un, dist));
}

// compaction of the sorted (morton, face) pairs to unique leaves + barycentrics
__global__ void m2s_leaves_kernel(int64_t num, const uint64_t *__restrict__ ms, const int64_t *__restrict__ ts,
                                  const uint32_t *__restrict__ flag, const uint32_t *__restrict__ psum,
                                  const float *__restrict__ fv, uint32_t level, uint64_t *__restrict__ mout,
                                  int64_t *__restrict__ fout, float *__restrict__ bary) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= num || !flag[t]) return;
  const uint32_t o = psum[t];
  const uint64_t m = ms[t];
  const int64_t f = ts[t];
  mout[o] = m;
  fout[o] = f;
  float cx, cy, cz, h;
  voxel_center(m, level, cx, cy, cz, h);
  const float *v = fv + f * 9;
  const F3 v1 = f3(v[0], v[1], v[2]), v2 = f3(v[3], v[4], v[5]), v3 = f3(v[6], v[7], v[8]);
  const F3 cp = tri_closest(v1, v2, v3, f3(cx, cy, cz));
  const F3 cr = fcross(fsub(v1, v2), fsub(v1, v3));
  const float delta = fdot(cr, cr);
  const F3 d1 = fsub(cp, v1), d2 = fsub(cp, v2), d3v = fsub(cp, v3);
  F3 q = fcross(d2, d3v);
  const float da = sqrtf(fdot(q, q));
  q = fcross(d1, d3v);
  const float db = sqrtf(fdot(q, q));
  q = fcross(d1, d2);
  const float dc = sqrtf(fdot(q, q));
  const float rs = 1.0f / sqrtf(delta);
  float bx = da * rs, by = db * rs, bz = dc * rs;
  if (bx < 0.0f) bx = 0.f;
  if (by < 0.0f) by = 0.f;
  if (bz < 0.0f) bz = 0.f;
  const float s = (float)(1. / (double)(bx + by + bz));
  bary[o * 2 + 0] = bx * s;
  bary[o * 2 + 1] = by * s;
}

// ------------------------------------------------------------------ morton -> octree
__global__ void parent_flag_kernel(int64_t num, const uint64_t *__restrict__ m, uint32_t *__restrict__ flag) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t > num) return;
  flag[t] = (t == num) ? 0u : ((t == 0 || (m[t - 1] >> 3) != (m[t] >> 3)) ? 1u : 0u);
}

__global__ void compact_nodes_kernel(int64_t num, const uint64_t *__restrict__ m, const uint32_t *__restrict__ flag,
                                     const uint32_t *__restrict__ psum, uint64_t *__restrict__ parent,
                                     uint8_t *__restrict__ bytes) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= num || !flag[t]) return;
  const uint32_t o = psum[t];
  parent[o] = m[t] >> 3;
  uint32_t code = 0;
  do {
    code |= 1u << (uint32_t)(m[t] & 7);
    t++;
  } while (t < num && !flag[t]);
  bytes[o] = (uint8_t)code;
}

static int morton_to_octree_impl(int64_t n, const uint64_t *morton, uint32_t level, Scratch &sc, uint8_t **octree,
                                 int64_t *num_nodes, hipStream_t st) {
  std::vector<uint8_t *> lv(level, nullptr);
  std::vector<int64_t> ln(level, 0);
  const uint64_t *cur = morton;
  int64_t prev = n;
  for (uint32_t i = level; i > 0; i--) {
    uint32_t *flag = (uint32_t *)sc.get((prev + 1) * sizeof(uint32_t));
    uint32_t *psum = (uint32_t *)sc.get((prev + 2) * sizeof(uint32_t));
    if (!flag || !psum) return KL_E_ALLOC;
    const unsigned g = (unsigned)cdiv(prev + 1, 256);
    hipLaunchKernelGGL(parent_flag_kernel, dim3(g), dim3(256), 0, st, prev, cur, flag);
    KL_CHECK_LAUNCH();
    uint32_t cnt = 0;
    int rc = exclusive_scan(flag, psum, prev, sc, st, &cnt);
    if (rc) return rc;
    uint64_t *par = (uint64_t *)sc.get((size_t)cnt * sizeof(uint64_t));
    uint8_t *bytes = (uint8_t *)sc.get(cnt);
    if (!par || !bytes) return KL_E_ALLOC;
    if (prev > 0) {
      hipLaunchKernelGGL(compact_nodes_kernel, dim3((unsigned)cdiv(prev, 256)), dim3(256), 0, st, prev, cur, flag,
                         psum, par, bytes);
      KL_CHECK_LAUNCH();
    }
    lv[i - 1] = bytes;
    ln[i - 1] = cnt;
    cur = par;
    prev = cnt;
  }
  int64_t total = 0;
  for (uint32_t l = 0; l < level; l++) total += ln[l];
  uint8_t *out = (uint8_t *)sc.get((size_t)total);
  if (!out) return KL_E_ALLOC;
  int64_t o = 0;
  for (uint32_t l = 0; l < level; l++) {
    if (ln[l]) KL_CHECK_HIP(hipMemcpyAsync(out + o, lv[l], ln[l], hipMemcpyDeviceToDevice, st));
    o += ln[l];
  }
  *octree = out;
  *num_nodes = total;
  return KL_OK;
}

__global__ void iota_kernel(int64_t n, int64_t *__restrict__ t, uint64_t *__restrict__ m) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) {
    t[i] = i;
    m[i] = 0;
  }
}

// proposals (face, voxel) tested per level by the last mesh_to_spc call on this thread
// (N_l of SURVEY.md §8d's cfg4 byte count; read by kl_mesh_to_spc_level_counts)
static thread_local int64_t t_m2s_counts[SPC_MAX_LEVELS + 1];
static thread_local int t_m2s_levels = 0;

static int mesh_to_spc_impl(int64_t F, const float *fv, uint32_t L, Scratch &sc, uint8_t **octree,
                            int64_t *num_nodes, int64_t **face_idx, float **bary, int64_t *num_leaves,
                            hipStream_t st) {
  t_m2s_levels = 0;
  *num_nodes = 0;
  *num_leaves = 0;
  *octree = nullptr;
  *face_idx = nullptr;
  *bary = nullptr;
  int64_t cnt = F;
  uint64_t *m0 = (uint64_t *)sc.get(cnt * sizeof(uint64_t));
  int64_t *t0 = (int64_t *)sc.get(cnt * sizeof(int64_t));
  if (!m0 || !t0) return KL_E_ALLOC;
  if (cnt > 0) {
    hipLaunchKernelGGL(iota_kernel, dim3((unsigned)cdiv(cnt, 256)), dim3(256), 0, st, cnt, t0, m0);
    KL_CHECK_LAUNCH();
  }
  for (uint32_t l = 0; l <= L; l++) {
    t_m2s_counts[l] = cnt;
    t_m2s_levels = (int)l + 1;
    uint32_t *occ = (uint32_t *)sc.get((cnt + 1) * sizeof(uint32_t));
    uint32_t *psum = (uint32_t *)sc.get((cnt + 2) * sizeof(uint32_t));
    if (!occ || !psum) return KL_E_ALLOC;
    hipLaunchKernelGGL(m2s_decide_kernel, dim3((unsigned)cdiv(cnt + 1, 256)), dim3(256), 0, st, cnt, fv, m0, t0,
                       occ, l, L - l);
    KL_CHECK_LAUNCH();
    uint32_t next = 0;
    int rc = exclusive_scan(occ, psum, cnt, sc, st, &next);
    if (rc) return rc;
    if (next == 0) return KL_OK;  // empty: (0,) u8, (0,) i64, (0,3) f32 built by the caller
    uint64_t *m1 = (uint64_t *)sc.get((size_t)next * sizeof(uint64_t));
    int64_t *t1 = (int64_t *)sc.get((size_t)next * sizeof(int64_t));
    if (!m1 || !t1) return KL_E_ALLOC;
    hipLaunchKernelGGL(m2s_subdivide_kernel, dim3((unsigned)cdiv(cnt, 256)), dim3(256), 0, st, cnt, m0, t0, m1, t1,
                       occ, psum, l < L ? 1 : 0);
    KL_CHECK_LAUNCH();
    m0 = m1;
    t0 = t1;
    cnt = next;
  }
  // stable radix sort of (morton, face) on the 3L significant bits: keeps generation
  // order (= ascending face id) among equal mortons, as CUB's SortPairs did.
  uint64_t *ms = (uint64_t *)sc.get(cnt * sizeof(uint64_t));
  int64_t *ts = (int64_t *)sc.get(cnt * sizeof(int64_t));
  if (!ms || !ts) return KL_E_ALLOC;
  size_t tb = 0;
  const int end_bit = (int)(3 * L) > 0 ? (int)(3 * L) : 1;
  KL_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, m0, ms, t0, ts, (int)cnt, 0, end_bit, st));
  void *tmp = sc.get(tb);
  if (!tmp) return KL_E_ALLOC;
  KL_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, m0, ms, t0, ts, (int)cnt, 0, end_bit, st));
  uint32_t *flag = (uint32_t *)sc.get((cnt + 1) * sizeof(uint32_t));
  uint32_t *psum = (uint32_t *)sc.get((cnt + 2) * sizeof(uint32_t));
  if (!flag || !psum) return KL_E_ALLOC;
  hipLaunchKernelGGL(mark_unique_kernel, dim3((unsigned)cdiv(cnt + 1, 256)), dim3(256), 0, st, cnt, ms, flag);
  KL_CHECK_LAUNCH();
  uint32_t uniq = 0;
  int rc = exclusive_scan(flag, psum, cnt, sc, st, &uniq);
  if (rc) return rc;
  uint64_t *mu = (uint64_t *)sc.get((size_t)uniq * sizeof(uint64_t));
  int64_t *fu = (int64_t *)sc.get((size_t)uniq * sizeof(int64_t));
  float *bu = (float *)sc.get((size_t)uniq * 2 * sizeof(float));
  if (!mu || !fu || !bu) return KL_E_ALLOC;
  hipLaunchKernelGGL(m2s_leaves_kernel, dim3((unsigned)cdiv(cnt, 256)), dim3(256), 0, st, cnt, ms, ts, flag, psum, fv,
                     L, mu, fu, bu);
  KL_CHECK_LAUNCH();
  rc = morton_to_octree_impl(uniq, mu, L, sc, octree, num_nodes, st);
  if (rc) return rc;
  *face_idx = fu;
  *bary = bu;
  *num_leaves = uniq;
  return KL_OK;
}

// ------------------------------------------------------------------ mesh_to_spc, device-sized
// A returning atomic on one word saturates at ~88 per us (MI355X_MICROARCH.md), so the level
// counters and the output are sharded M2S_SHARDS ways by workgroup (blockIdx % M2S_SHARDS,
// which also keeps a shard on one XCD): shard g of a level is the region [g * seg,
// (g + 1) * seg) of the buffer with its own counter.  A level's input is the previous
// level's shards, indexed as one sequence (their counts' prefix).
constexpr int M2S_SHARDS = 32;

// The shards' counts as one sequence: prefix sums in LDS (filled by the workgroup), item i's
// buffer position by a binary search over them.
struct ShardIn {
  unsigned long long *pre;  // LDS, M2S_SHARDS + 1
  __device__ __forceinline__ void load(unsigned long long *lds, const unsigned long long *c, unsigned long long seg) {
    pre = lds;
    if (threadIdx.x == 0) {
      unsigned long long a = 0;
      pre[0] = 0;
      for (int g = 0; g < M2S_SHARDS; g++) {
        a += c[g] < seg ? c[g] : seg;
        pre[g + 1] = a;
      }
    }
    __syncthreads();
  }
  __device__ __forceinline__ unsigned long long total() const { return pre[M2S_SHARDS]; }
  // buffer position of logical item i (< total)
  __device__ __forceinline__ unsigned long long pos(unsigned long long i, unsigned long long seg) const {
    int lo = 0, hi = M2S_SHARDS - 1;  // last g with pre[g] <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= i)
        lo = mid;
      else
        hi = mid - 1;
    }
    return (unsigned long long)lo * seg + (i - pre[lo]);
  }
};

// The level kernels' grid: a span of up to M2S_MAX_CHUNKS chunks of 256 pairs per workgroup,
// one reservation per workgroup and level.
constexpr int M2S_GRID = 2048;
constexpr int M2S_MAX_CHUNKS = 64;
constexpr int M2S_KEEP = 4;  // chunks whose (node, face) m2s_node_kernel keeps in registers (r06)

// ---- the 8 children of a parent (voxel, face) pair at once (m2s_children_pt).
// The reference's decision for a child c (tri_voxel_test: 13 SAT axes, each passing iff
// (float)max(-max_k d_k, min_k d_k) <= (float)(h |a|_1), d_k = v_k . a, v_k = fl(f_k - c)) is
// derived per axis from the PARENT's projections: with C the parent's centre and w_k = fl(f_k - C),
// the child centre is c = C + delta, delta in {-h, +h}^3 (C and every child centre are exact
// floats), so d_k = w_k . a - delta . a up to rounding, and the axis's separation is
//   S = max(s - max_k P_k, min_k P_k - s) - h |a|_1,  P_k = w_k . a,  s = delta . a,
// one add per sign pattern of delta.  Each axis is evaluated with float edges E = fl(f_b - f_a)
// (unnormalised: a positive scale does not change the sign of S) and a margin M bounding the
// difference to the reference's own S in that scale -- its rounded v_k (the edges it builds
// differ from E by at most tau = 2^-22 U per component, U = max |w_k| + 2h + max |E|), its
// normalisation, its double products and float casts, and this float evaluation (a few 2^-24 U
// |a|_1 each):
//   * box axes: decided EXACTLY, on the reference's own float differences f_k - (C +- h);
//   * edge-cross axes (x/y/z cross each edge): |dS| <= 2 tau (V + 2h) + 2^-20 (V + 2h) |a|_1 <
//     M = 2^-17 U^2;
//   * the normal, E1 x E2 (r04: a margin linear in the edge scale Em = max |E|): every term of dS
//     carries a factor of the axis (|n|_inf <= 2 Em^2) or of its error against the reference's
//     rounded edges (|dn|_inf <= 4 tau Em + 2 tau^2 + 2^-21 Em^2 <= 2^-20 U Em + 2 tau^2): the
//     rounded v_k / w_k (<= 2.3 * 2^-20 U^2 Em), v.dn (<= 3 * 2^-20 U^2 Em), the float dot, s, R
//     and S (<= 3.7 * 2^-20 U^2 Em) and the reference's float casts of fd / fr (<= 0.8 * 2^-20
//     U^2 Em), in all |dS| <= 10 * 2^-20 U^2 Em + 6 U tau^2 < M = 2^-15 U^2 (Em + 2^-10 U)
//     (tau^2 <= 2^-46 U^2).  The r03 bound 2^-15 U^3 took Em <= U: with a triangle much smaller
//     than the voxel (the first levels: cfg4's edges are ~1/100 of a level-2 voxel) a passing
//     child's normal-axis separation, ~ -h |n|_1, fell inside it, and every such child ran the
//     full test.
// S > M proves the reference rejects the child on that axis, S < -M that it passes it; a child
// every axis passes is accepted, one some axis rejects is rejected, and the rest (|S| <= M on
// some axis, none rejecting) run the reference's test itself.  A reference edge of length 0
// (its NaN axis rejects) needs |E| <= tau, where |S| < M: never decided here.  Non-finite or
// huge inputs (U >= 1e12) leave all 8 children to the full test.
// -> bit c set iff child c (to_morton(2p + (c >> 2), 2q + ((c >> 1) & 1), 2r + (c & 1))) passes.
__device__ __forceinline__ void m2s_axis4(float pmax, float pmin, float R, float hp, float hq, float M,
                                          uint32_t &rej4, uint32_t &amb4) {
  // sign patterns j = (bp << 1) | bq of the two nonzero components: s = +-hp +-hq
  rej4 = 0;
  amb4 = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const float sv = ((j >> 1) ? hp : -hp) + ((j & 1) ? hq : -hq);
    const float S = fmaxf(sv - pmax, pmin - sv) - R;
    rej4 |= (S > M ? 1u : 0u) << j;
    amb4 |= (!(S < -M) && !(S > M) ? 1u : 0u) << j;
  }
}

__device__ uint32_t m2s_children_pt(const float *v, int px, int py, int pz, uint32_t level) {
  const float two_level = (float)(1u << level);
  const float vs = 2.0f / two_level;  // child size
  const float h = (float)(0.5 * vs);  // child half-size (voxel_center at `level`)
  // parent centre: child (2p, 2q, 2r)'s centre + h, exact
  const float Cx = fmaf((float)(2 * px), vs, h - 1.0f) + h;
  const float Cy = fmaf((float)(2 * py), vs, h - 1.0f) + h;
  const float Cz = fmaf((float)(2 * pz), vs, h - 1.0f) + h;
  const float w[3][3] = {{v[0] - Cx, v[1] - Cy, v[2] - Cz}, {v[3] - Cx, v[4] - Cy, v[5] - Cz},
                         {v[6] - Cx, v[7] - Cy, v[8] - Cz}};
  const float E[3][3] = {{v[3] - v[0], v[4] - v[1], v[5] - v[2]},   // ab
                         {v[6] - v[3], v[7] - v[4], v[8] - v[5]},   // bc
                         {v[0] - v[6], v[1] - v[7], v[2] - v[8]}};  // ca
  float V = 0.f, Em = 0.f;
#pragma unroll
  for (int k = 0; k < 3; k++)
#pragma unroll
    for (int q = 0; q < 3; q++) {
      V = fmaxf(V, fabsf(w[k][q]));
      Em = fmaxf(Em, fabsf(E[k][q]));
    }
  const float U = V + 2.0f * h + Em;
  uint32_t rej = 0, amb = 0;
  if (!(U < 1e12f)) {
    amb = 0xffu;
  } else {
    // box axes, exactly as the reference: per axis and half, the children's own differences
    const float cen[3] = {Cx, Cy, Cz};
    const uint32_t half_mask[3][2] = {{0x0fu, 0xf0u}, {0x33u, 0xccu}, {0x55u, 0xaau}};
#pragma unroll
    for (int q = 0; q < 3; q++)
#pragma unroll
      for (int b = 0; b < 2; b++) {
        const float c = b ? cen[q] + h : cen[q] - h;
        const float u0 = v[q] - c, u1 = v[3 + q] - c, u2 = v[6 + q] - c;
        const float fd = fmaxf(-fmaxf(u0, fmaxf(u1, u2)), fminf(u0, fminf(u1, u2)));
        if (!(fd <= h)) rej |= half_mask[q][b];
      }
    // edge-cross axes: x x e = (0, -e.z, e.y), y x e = (e.z, 0, -e.x), z x e = (-e.y, e.x, 0)
    const float Me = (1.0f / 131072.0f) * U * U;
#pragma unroll
    for (int e = 0; e < 3; e++) {
      const float ex = E[e][0], ey = E[e][1], ez = E[e][2];
      uint32_t r4, a4;
      {  // (0, -ez, ey): patterns over (y, z): child bits (c >> 1) & 1, c & 1
        float P[3];
#pragma unroll
        for (int k = 0; k < 3; k++) P[k] = w[k][1] * -ez + w[k][2] * ey;
        m2s_axis4(fmaxf(P[0], fmaxf(P[1], P[2])), fminf(P[0], fminf(P[1], P[2])), h * (fabsf(ez) + fabsf(ey)),
                  h * -ez, h * ey, Me, r4, a4);
        rej |= r4 | (r4 << 4);
        amb |= a4 | (a4 << 4);
      }
      {  // (ez, 0, -ex): patterns over (x, z)
        float P[3];
#pragma unroll
        for (int k = 0; k < 3; k++) P[k] = w[k][0] * ez + w[k][2] * -ex;
        m2s_axis4(fmaxf(P[0], fmaxf(P[1], P[2])), fminf(P[0], fminf(P[1], P[2])), h * (fabsf(ez) + fabsf(ex)),
                  h * ez, h * -ex, Me, r4, a4);
        auto spread = [](uint32_t m4) {  // j = (bx << 1) | bz -> children bx * 4 + bz + {0, 2}
          return ((m4 & 1u) ? 0x05u : 0u) | ((m4 & 2u) ? 0x0au : 0u) | ((m4 & 4u) ? 0x50u : 0u) |
                 ((m4 & 8u) ? 0xa0u : 0u);
        };
        rej |= spread(r4);
        amb |= spread(a4);
      }
      {  // (-ey, ex, 0): patterns over (x, y)
        float P[3];
#pragma unroll
        for (int k = 0; k < 3; k++) P[k] = w[k][0] * -ey + w[k][1] * ex;
        m2s_axis4(fmaxf(P[0], fmaxf(P[1], P[2])), fminf(P[0], fminf(P[1], P[2])), h * (fabsf(ey) + fabsf(ex)),
                  h * -ey, h * ex, Me, r4, a4);
        auto spread = [](uint32_t m4) {  // j = (bx << 1) | by -> children bx * 4 + by * 2 + {0, 1}
          return ((m4 & 1u) ? 0x03u : 0u) | ((m4 & 2u) ? 0x0cu : 0u) | ((m4 & 4u) ? 0x30u : 0u) |
                 ((m4 & 8u) ? 0xc0u : 0u);
        };
        rej |= spread(r4);
        amb |= spread(a4);
      }
    }
    // the normal E1 x E2 (the reference's cross(ab, bc))
    {
      const float nx = E[0][1] * E[1][2] - E[0][2] * E[1][1];
      const float ny = E[0][2] * E[1][0] - E[0][0] * E[1][2];
      const float nz = E[0][0] * E[1][1] - E[0][1] * E[1][0];
      float P[3];
#pragma unroll
      for (int k = 0; k < 3; k++) P[k] = w[k][0] * nx + w[k][1] * ny + w[k][2] * nz;
      const float pmax = fmaxf(P[0], fmaxf(P[1], P[2])), pmin = fminf(P[0], fminf(P[1], P[2]));
      const float R = h * (fabsf(nx) + fabsf(ny) + fabsf(nz));
      const float Mn = (1.0f / 32768.0f) * U * U * (Em + (1.0f / 1024.0f) * U);
      const float hx = h * nx, hy = h * ny, hz = h * nz;
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const float sv = ((c >> 2) ? hx : -hx) + (((c >> 1) & 1) ? hy : -hy) + ((c & 1) ? hz : -hz);
        const float S = fmaxf(sv - pmax, pmin - sv) - R;
        rej |= (S > Mn ? 1u : 0u) << c;
        amb |= (!(S < -Mn) && !(S > Mn) ? 1u : 0u) << c;
      }
    }
  }
  uint32_t pass = ~(rej | amb) & 0xffu;
  uint32_t need = amb & ~rej & 0xffu;
  while (need) {  // the reference's test itself, on its own child centre
    const int c = __builtin_ctz(need);
    need &= need - 1;
    // the child's centre as voxel_center computes it
    const float cx = fmaf((float)(2 * px + (c >> 2)), vs, h - 1.0f);
    const float cy = fmaf((float)(2 * py + ((c >> 1) & 1)), vs, h - 1.0f);
    const float cz = fmaf((float)(2 * pz + (c & 1)), vs, h - 1.0f);
    if (tri_voxel_test(v, v + 3, v + 6, cx, cy, cz, h)) pass |= 1u << c;
  }
  return pass;
}

// ---- mesh_to_spc by node ranks (r04, m2s_node_kernel / m2s_rank_kernel): no sort, one host read.
// Level l's nodes are a list in morton order (U_l nodes).  Node j's octree byte oct_l[j] -- the OR
// of the child masks its (node, face) pairs decide -- IS the octree row, and the exclusive popcount
// scan S_l of the row numbers the next level: child c of node j is node
//   S_l[j] + popc(oct_l[j] & ((1 << c) - 1))
// of level l + 1, again in morton order (the parents are, and children follow in c); M_l keeps the
// nodes' points (x | y << 16 | z << 32: no morton decode per pair).  A level's
// pairs are appended in any order as (key = parent * 8 + c, face) and the next level resolves the
// key through the parent level's S and octree row.  At the last level each (parent, child) slot
// keeps its least face (atomicMin), the face the reference's stable sort puts first (generation
// order is ascending face id, m2s_key_kernel's comment).  Per call: the root test, then per level
// one decision launch and one scan launch (single pass, ordered tiles with look-back), the counts
// read once at the end, and one launch writing the leaves' faces and barycentrics.
struct M2sCtl {
  unsigned long long counts[(SPC_MAX_LEVELS + 2) * M2S_SHARDS];  // pairs per level and shard
  uint32_t U[SPC_MAX_LEVELS + 2];       // nodes per level
  uint32_t O[SPC_MAX_LEVELS + 2];       // the level's first byte in the octree arena
  uint32_t ticket[SPC_MAX_LEVELS + 2];  // tile tickets of the level's scan
  // 0, or the launch sequence number (m2s_seq_*) of the first launch that overflowed a buffer.  A
  // launch stops at its start only on an overflow of an EARLIER launch (seq < its own): that test
  // is the same for all its workgroups, however late they start.  (Stopping on any overflow let a
  // late scan workgroup return without publishing its tile while the tiles after it waited for it.)
  int overflow;
  uint32_t zero;
  uint32_t root_S[2];  // the level above the root: one node whose child 0 is the root
  uint32_t root_oct;   // its octree byte (1)
};

constexpr int M2S_TILE = 1024;  // nodes per scan tile (256 threads x 4)

// launch sequence of the node-rank path: root 1, then per level l the node kernel (2 l) and the scan
// of level l - 1's row (2 l + 1)
constexpr int M2S_SEQ_ROOT = 1;
__host__ __device__ constexpr int m2s_seq_node(uint32_t level) { return 2 * (int)level; }
__host__ __device__ constexpr int m2s_seq_rank(uint32_t l) { return 2 * (int)l + 3; }
__device__ __forceinline__ bool m2s_dead(const M2sCtl *ctl, int seq) {
  const int ov = *(const volatile int *)&ctl->overflow;
  return ov != 0 && ov < seq;
}

__device__ void leaf_out_pt(int px, int py, int pz, int64_t f, const float *__restrict__ fv, uint32_t level,
                            uint32_t o, int64_t *__restrict__ fout, float *__restrict__ bary);

// a node's point packed in 64 bits (x | y << 16 | z << 32): a child is 2 p + m2s_child_off(c)
__device__ __forceinline__ uint64_t m2s_child_off(uint32_t c) {
  return (uint64_t)(c >> 2) | ((uint64_t)((c >> 1) & 1) << 16) | ((uint64_t)(c & 1) << 32);
}

// level 0: the root voxel against every face; the passing faces are the pairs (key 0, face)
__global__ void __launch_bounds__(256) m2s_root_kernel(int64_t F, const float *__restrict__ fv, uint32_t *__restrict__ kout,
                                                       uint32_t *__restrict__ fout, unsigned long long seg,
                                                       M2sCtl *__restrict__ ctl, uint64_t *__restrict__ M0,
                                                       uint64_t *__restrict__ slots, uint32_t *__restrict__ fmin8,
                                                       uint32_t L) {
  __shared__ int s_wave[4];
  __shared__ unsigned long long s_base;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctl->root_S[0] = 0;
    ctl->root_S[1] = 1;
    ctl->root_oct = 1;
    ctl->U[0] = 1;
    ctl->O[0] = 0;
    M0[0] = 0;
    if (L >= 2) slots[0] = 0;
  }
  if (blockIdx.x == 0 && L == 1 && threadIdx.x < 8) fmin8[threadIdx.x] = 0xffffffffu;
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  bool pass = false;
  if (f < F) {
    float cx, cy, cz, h;
    voxel_center(0, 0, cx, cy, cz, h);
    const float *v = fv + f * 9;
    pass = tri_voxel_maybe(v, v + 3, v + 6, cx, cy, cz, h) && tri_voxel_test(v, v + 3, v + 6, cx, cy, cz, h);
  }
  int total = 0;
  const int pre = block_exclusive_scan(pass ? 1 : 0, s_wave, &total);
  const int g = blockIdx.x % M2S_SHARDS;
  if (threadIdx.x == 0) s_base = total ? atomicAdd(ctl->counts + g, (unsigned long long)total) : 0ull;
  __syncthreads();
  if (total == 0) return;
  if (s_base + (unsigned long long)total > seg) {
    if (threadIdx.x == 0) ctl->overflow = M2S_SEQ_ROOT;
    return;
  }
  if (pass) {
    const unsigned long long o = (unsigned long long)g * seg + s_base + (unsigned long long)pre;
    kout[o] = 0;
    fout[o] = (uint32_t)f;
  }
}

// the node a pair's key names: (its index at the pair's level, its morton)
__device__ __forceinline__ uint32_t m2s_node(uint32_t key, const uint32_t *__restrict__ Spp,
                                             const uint8_t *__restrict__ octpp) {
  const uint32_t jp = key >> 3, c = key & 7;
  return Spp[jp] + (uint32_t)__popc((uint32_t)octpp[jp] & ((1u << c) - 1u));
}

// One level l >= 1: each thread takes a pair of level l - 1, decides its node's 8 children
// (m2s_children), flags them in the node's 8 child slots, and appends (node * 8 + c, face) for the
// passing children (sharded, one reservation per workgroup) -- or, at the
// last level, keeps the least face per (node, child) slot.  The scan kernel then forms each node's
// octree byte from its slots.
template <bool LAST>
__global__ void __launch_bounds__(256) m2s_node_kernel(const float *__restrict__ fv, const uint32_t *__restrict__ kin,
                                                       const uint32_t *__restrict__ fin, uint32_t *__restrict__ kout,
                                                       uint32_t *__restrict__ fout, unsigned long long seg,
                                                       M2sCtl *__restrict__ ctl, uint32_t level,
                                                       const uint32_t *__restrict__ Spp,
                                                       const uint8_t *__restrict__ octpp_base,
                                                       const uint32_t *__restrict__ opp,
                                                       const uint64_t *__restrict__ Mp, uint8_t *__restrict__ slots,
                                                       uint32_t *__restrict__ fmin8) {
  __shared__ int s_wave[4];
  __shared__ unsigned long long s_base;
  __shared__ unsigned long long s_pre[M2S_SHARDS + 1];
  __shared__ uint8_t s_kids[M2S_MAX_CHUNKS][256];
  // After an overflow the shards hold unwritten holes below their clamped counts (the overflowing
  // workgroups reserved past seg and wrote nothing): the levels after it must not read them (their
  // face ids would index fv out of bounds).  The host then runs the per-level path.
  if (m2s_dead(ctl, m2s_seq_node(level))) return;
  ShardIn in;
  in.load(s_pre, ctl->counts + (level - 1) * M2S_SHARDS, seg);
  const unsigned long long n = in.total();
  const int g = blockIdx.x % M2S_SHARDS;
  // whole chunks of 256 pairs per workgroup (the first levels' ~200 k pairs fill 782 workgroups'
  // lanes instead of spreading ~98 over each of 2,048)
  const unsigned long long span = ((n + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
  const unsigned long long lo = (unsigned long long)blockIdx.x * span;
  const unsigned long long hi = lo + span < n ? lo + span : n;
  if (lo >= hi) return;
  const int nch = (int)((hi - lo + blockDim.x - 1) / blockDim.x);
  if (nch > M2S_MAX_CHUNKS) {
    if (threadIdx.x == 0) ctl->overflow = m2s_seq_node(level);
    return;
  }
  const uint8_t *octpp = octpp_base + *opp;
  int mine = 0;
  // (r06) the first M2S_KEEP chunks' node and face per thread kept in registers for the append pass
  // below, which re-resolved them (a chain of dependent loads per chunk); cfg4's levels have 1-3
  // chunks per workgroup
  uint32_t keep_j[M2S_KEEP], keep_f[M2S_KEEP];
#pragma unroll 1
  for (int k = 0; k < nch; k++) {
    const unsigned long long i = lo + (unsigned long long)k * blockDim.x + threadIdx.x;
    uint32_t kids = 0, j = 0, f = 0;
    if (i < hi) {
      const unsigned long long p = in.pos(i, seg);
      f = fin[p];
      j = m2s_node(kin[p], Spp, octpp);
      const uint64_t q = Mp[j];
      kids = m2s_children_pt(fv + (int64_t)f * 9, (int)(q & 0xffff), (int)((q >> 16) & 0xffff), (int)(q >> 32), level);
    }
#pragma unroll
    for (int u = 0; u < M2S_KEEP; u++)
      if (k == u) {
        keep_j[u] = j;
        keep_f[u] = f;
      }
    if (LAST) {  // the least face per (node, child) slot; a slot left at ~0 is no child
      for (uint32_t c = kids; c; c &= c - 1) atomicMin(fmin8 + j * 8 + __builtin_ctz(c), f);
    } else {
      // the node's child flags: plain byte stores of 1 (idempotent, merged in the XCDs' L2s),
      // not atomics -- global atomics execute at the memory side, ~12 ns apiece per address, and
      // the first levels send every pair to a few nodes (293 us at level 3 with atomicOr)
      uint8_t *fl = slots + (size_t)j * 8;
#pragma unroll
      for (int c = 0; c < 8; c++)
        if ((kids >> c) & 1) fl[c] = 1;
      s_kids[k][threadIdx.x] = (uint8_t)kids;
      mine += __popc(kids);
    }
  }
  if (LAST) return;
  // the children's pairs, appended in any order (the next level's nodes are numbered by the scan,
  // not by position): one reservation per workgroup (per wave and chunk: 21 -> 31 us per level)
  int total = 0;
  (void)block_exclusive_scan(mine, s_wave, &total);
  unsigned long long *cnt_out = ctl->counts + level * M2S_SHARDS;
  if (threadIdx.x == 0) s_base = total ? atomicAdd(cnt_out + g, (unsigned long long)total) : 0ull;
  __syncthreads();
  unsigned long long o0 = s_base;
  if (total == 0) return;
  if (o0 + (unsigned long long)total > seg) {
    if (threadIdx.x == 0) ctl->overflow = m2s_seq_node(level);
    return;
  }
  o0 += (unsigned long long)g * seg;
#pragma unroll 1
  for (int k = 0; k < nch; k++) {
    const uint32_t kids = s_kids[k][threadIdx.x];
    int ctot = 0;
    const int pre = block_exclusive_scan(__popc(kids), s_wave, &ctot);
    if (kids) {
      uint32_t f = 0, j8 = 0;
      if (k < M2S_KEEP) {
#pragma unroll
        for (int u = 0; u < M2S_KEEP; u++)
          if (k == u) {
            f = keep_f[u];
            j8 = keep_j[u] * 8;
          }
      } else {
        const unsigned long long i = lo + (unsigned long long)k * blockDim.x + threadIdx.x;
        const unsigned long long p = in.pos(i, seg);
        f = fin[p];
        j8 = m2s_node(kin[p], Spp, octpp) * 8;
      }
      unsigned long long o = o0 + (unsigned long long)pre;
      for (uint32_t c = kids; c; c &= c - 1) {
        kout[o] = j8 + (uint32_t)__builtin_ctz(c);
        fout[o] = f;
        o++;
      }
    }
    o0 += (unsigned long long)ctot;
  }
}

// Level l's octree row (l < L) from its nodes' child slots (flags, or at l = L - 1 the least-face
// slots: a child iff not ~0) and its scan: S_l (exclusive popcounts, S_l[U_l] = U_{l+1}), the next
// level's count and arena offset, and for each child its point (M_{l+1}) and zeroed slots (flags
// for l + 2 < L, least faces ~0 for l + 2 == L).  Single
// pass: workgroup b takes tile b (tiles past the grid by ticket), publishes the tile's sum tagged
// with the level (aggregate, then inclusive once the prefix is known) and looks back over the
// earlier tiles' tags, 64 per round; a workgroup only waits on tiles of workgroups dispatched or
// ticketed before it, so the wait always ends.
__global__ void __launch_bounds__(256) m2s_rank_kernel(M2sCtl *__restrict__ ctl, uint32_t l, uint32_t L,
                                                       uint8_t *__restrict__ arena, const uint64_t *__restrict__ Ml,
                                                       uint32_t *__restrict__ Sl, uint64_t *__restrict__ Mn,
                                                       const uint64_t *__restrict__ slots,
                                                       uint64_t *__restrict__ slots_next,
                                                       unsigned long long *__restrict__ status,
                                                       uint32_t *__restrict__ fmin8, uint32_t ncap, uint32_t oct_cap,
                                                       uint32_t fmin_cap) {
  __shared__ int s_wave[4];
  __shared__ uint32_t s_tile, s_prefix;
  if (m2s_dead(ctl, m2s_seq_rank(l))) return;  // the same answer for every workgroup (M2sCtl)
  const uint32_t n = ctl->U[l], O = ctl->O[l], On = O + n;
  const uint32_t ntiles = (n + M2S_TILE - 1) / M2S_TILE;
  const bool has_next = l + 1 < L, init_fmin = l + 2 == L, init_flags = l + 2 < L, last = l + 1 == L;
  const unsigned long long tag_agg = (unsigned long long)(2 * l + 2) << 32,
                           tag_inc = (unsigned long long)(2 * l + 3) << 32;
  uint8_t *oct = arena + O;
  // tile blockIdx.x first (workgroups are dispatched in index order, so a tile's predecessors are
  // held by workgroups already running), then tiles past the grid by ticket
  if (blockIdx.x >= ntiles) return;
  uint32_t t = blockIdx.x;
  for (;;) {
    const uint32_t j0 = t * M2S_TILE + threadIdx.x * 4;
    uint32_t b[4];
    int local = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t j = j0 + q;
      uint32_t byte = 0;
      if (j < n) {
        if (last) {
          const uint4 *f4 = (const uint4 *)(fmin8 + (size_t)j * 8);
          const uint4 a = f4[0], c = f4[1];
          byte = (a.x != ~0u ? 1u : 0u) | (a.y != ~0u ? 2u : 0u) | (a.z != ~0u ? 4u : 0u) | (a.w != ~0u ? 8u : 0u) |
                 (c.x != ~0u ? 16u : 0u) | (c.y != ~0u ? 32u : 0u) | (c.z != ~0u ? 64u : 0u) |
                 (c.w != ~0u ? 128u : 0u);
        } else {
          const uint64_t v = slots[j];
#pragma unroll
          for (int c = 0; c < 8; c++) byte |= ((v >> (8 * c)) & 0xffu) ? 1u << c : 0u;
        }
        oct[j] = (uint8_t)byte;
      }
      b[q] = byte;
      local += __popc(byte);
    }
    int agg = 0;
    const int ex = block_exclusive_scan(local, s_wave, &agg);
    if (threadIdx.x < 64) {  // wave 0: publish, then look back 64 tiles per round
      uint32_t prefix = 0;
      if (t == 0) {
        if (threadIdx.x == 0)
          __hip_atomic_store(status, tag_inc | (uint32_t)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        if (threadIdx.x == 0)
          __hip_atomic_store(status + t, tag_agg | (uint32_t)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int64_t end = t;  // lane i reads tile end - 1 - i (before tile 0: an inclusive 0)
        for (;;) {
          const int64_t k = end - 1 - (int64_t)threadIdx.x;
          const unsigned long long v =
              k >= 0 ? __hip_atomic_load(status + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag_inc;
          const unsigned long long tg = v & 0xffffffff00000000ull;
          const uint64_t inc = ballot(tg == tag_inc), any = ballot(tg == tag_inc || tg == tag_agg);
          if (inc) {  // the nearest inclusive tile, once every tile after it has published
            const int f = __builtin_ctzll(inc);
            const uint64_t need = f == 63 ? ~0ull : ((2ull << f) - 1);
            if ((any & need) == need) {
              uint32_t x = (int)threadIdx.x <= f ? (uint32_t)v : 0u;
#pragma unroll
              for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
              prefix += x;
              break;
            }
          } else if (any == ~0ull) {  // 64 aggregates: add them, look further back
            uint32_t x = (uint32_t)v;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
            prefix += x;
            end -= 64;
            continue;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (threadIdx.x == 0)
          __hip_atomic_store(status + t, tag_inc | (prefix + (uint32_t)agg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (threadIdx.x == 0) s_prefix = prefix;
    }
    __syncthreads();
    uint32_t s = s_prefix + (uint32_t)ex;
    bool over = false;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t j = j0 + q;
      if (j >= n) break;
      Sl[j] = s;
      if (has_next && b[q]) {
        const uint64_t m2 = Ml[j] * 2;
        for (uint32_t c = b[q]; c; c &= c - 1, s++) {
          if (s >= ncap || On + s >= oct_cap || (init_fmin && s * 8ull + 8 > fmin_cap)) {
            over = true;
            continue;
          }
          Mn[s] = m2 + m2s_child_off((uint32_t)__builtin_ctz(c));
          if (init_flags) slots_next[s] = 0;
          if (init_fmin) {
#pragma unroll
            for (int e = 0; e < 8; e++) fmin8[s * 8 + e] = 0xffffffffu;
          }
        }
      } else {
        s += (uint32_t)__popc(b[q]);
      }
    }
    if (over) ctl->overflow = m2s_seq_rank(l);
    if (t + 1 == ntiles && threadIdx.x == 0) {
      const uint32_t total = s_prefix + (uint32_t)agg;
      Sl[n] = total;
      ctl->U[l + 1] = total;
      ctl->O[l + 1] = On;
      if (total > ncap || (has_next && On + total > oct_cap)) ctl->overflow = m2s_seq_rank(l);
    }
    if (ntiles <= gridDim.x) break;
    __syncthreads();  // s_prefix and s_tile are rewritten for the next tile
    if (threadIdx.x == 0) s_tile = gridDim.x + atomicAdd(&ctl->ticket[l], 1u);
    __syncthreads();
    t = s_tile;
    if (t >= ntiles) break;
  }
}

// the leaves (after the one host read): per (parent, child) slot of the last level's parents, a
// leaf's number, least face, morton and barycentrics
__global__ void m2s_node_leaves_kernel(int64_t nslots, const M2sCtl *__restrict__ ctl, uint32_t L,
                                       const uint8_t *__restrict__ arena, const uint32_t *__restrict__ Sp,
                                       const uint64_t *__restrict__ Mp, const uint32_t *__restrict__ fmin8,
                                       const float *__restrict__ fv, int64_t *__restrict__ fout,
                                       float *__restrict__ bary) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  const uint32_t jp = (uint32_t)(s >> 3), c = (uint32_t)(s & 7);
  const uint32_t b = arena[ctl->O[L - 1] + jp];
  if (!((b >> c) & 1)) return;
  const uint32_t o = Sp[jp] + (uint32_t)__popc(b & ((1u << c) - 1u));
  const uint64_t q = Mp[jp] * 2 + m2s_child_off(c);
  leaf_out_pt((int)(q & 0xffff), (int)((q >> 16) & 0xffff), (int)(q >> 32), (int64_t)fmin8[s], fv, L, o, fout, bary);
}

// leaf o: its face and the face's barycentrics at the voxel centre (spc_math.h:229-258)
__device__ __forceinline__ void leaf_bary(float cx, float cy, float cz, int64_t f, const float *__restrict__ fv,
                                          uint32_t o, int64_t *__restrict__ fout, float *__restrict__ bary) {
  fout[o] = f;
  const float *v = fv + f * 9;
  const F3 v1 = f3(v[0], v[1], v[2]), v2 = f3(v[3], v[4], v[5]), v3 = f3(v[6], v[7], v[8]);
  const F3 cp = tri_closest(v1, v2, v3, f3(cx, cy, cz));
  const F3 cr = fcross(fsub(v1, v2), fsub(v1, v3));
  const float delta = fdot(cr, cr);
  const F3 d1 = fsub(cp, v1), d2 = fsub(cp, v2), d3v = fsub(cp, v3);
  F3 q = fcross(d2, d3v);
  const float da = sqrtf(fdot(q, q));
  q = fcross(d1, d3v);
  const float db = sqrtf(fdot(q, q));
  q = fcross(d1, d2);
  const float dc = sqrtf(fdot(q, q));
  const float rs = 1.0f / sqrtf(delta);
  float bx = da * rs, by = db * rs, bz = dc * rs;
  if (bx < 0.0f) bx = 0.f;
  if (by < 0.0f) by = 0.f;
  if (bz < 0.0f) bz = 0.f;
  const float sc = (float)(1. / (double)(bx + by + bz));
  bary[o * 2 + 0] = bx * sc;
  bary[o * 2 + 1] = by * sc;
}

// the same from the leaf's point (voxel_center's arithmetic)
__device__ void leaf_out_pt(int px, int py, int pz, int64_t f, const float *__restrict__ fv, uint32_t level,
                            uint32_t o, int64_t *__restrict__ fout, float *__restrict__ bary) {
  const float vs = 2.0f / (float)(1u << level);
  const float h = (float)(0.5 * vs);
  leaf_bary(fmaf((float)px, vs, h - 1.0f), fmaf((float)py, vs, h - 1.0f), fmaf((float)pz, vs, h - 1.0f), f, fv, o,
            fout, bary);
}

// The node-rank path's workspace: pair buffers of 96 pairs per face per level (cfg4: 1.18 M of
// 19.2 M at L = 9), in shards; nodes per level and octree bytes: a quarter of that; the last
// level's least-face slots (8 per parent) reuse the pair buffer that level would have written
// (2 cap words >= 8 ncap).
struct M2sNodes {
  unsigned long long cap = 0, seg = 0;
  uint32_t ncap = 0, oct_cap = 0, fmin_cap = 0;
  int64_t tiles = 0;
  size_t qb = 0, mbytes = 0, sbytes = 0, ctl_bytes = 0, total = 0;
  uint32_t *Qk[2], *Qf[2], *S[2];
  uint64_t *M[2], *SL[2];
  uint8_t *arena = nullptr;
  M2sCtl *ctl = nullptr;
  unsigned long long *status = nullptr;
  bool plan(int64_t F) {
    cap = (unsigned long long)std::max<int64_t>(F * 96, (int64_t)1 << 20);
    // dev param 14: the pair capacity itself (tests force the overflow branch with a small one)
    if (g_dev_param[14] > 0) cap = (unsigned long long)std::max(g_dev_param[14], 64 * M2S_SHARDS);
    if (F >= ((int64_t)1 << 31) || cap >= (1ull << 31)) return false;
    seg = cap / M2S_SHARDS;
    ncap = (uint32_t)(cap / 4);
    oct_cap = ncap;
    fmin_cap = (uint32_t)(2 * cap);
    tiles = cdiv(ncap, M2S_TILE);
    qb = al256b((size_t)cap * 4);
    mbytes = al256b((size_t)ncap * 8);
    sbytes = al256b(((size_t)ncap + 1) * 4);
    ctl_bytes = al256b(sizeof(M2sCtl) + (size_t)tiles * 8);
    total = 4 * qb + 4 * mbytes + 2 * sbytes + al256b(oct_cap + 4) + ctl_bytes;
    return true;
  }
  void place(char *p) {
    for (int k = 0; k < 2; k++) {
      Qk[k] = (uint32_t *)p;  // key then face: the pair of arrays is also 2 cap contiguous words
      Qf[k] = (uint32_t *)(p + qb);
      p += 2 * qb;
    }
    for (int k = 0; k < 2; k++, p += mbytes) M[k] = (uint64_t *)p;
    for (int k = 0; k < 2; k++, p += mbytes) SL[k] = (uint64_t *)p;  // child slots of levels l, l + 1
    for (int k = 0; k < 2; k++, p += sbytes) S[k] = (uint32_t *)p;
    arena = (uint8_t *)p;
    p += al256b(oct_cap + 4);
    ctl = (M2sCtl *)p;
    status = (unsigned long long *)(p + sizeof(M2sCtl));
  }
  uint32_t *fmin8(uint32_t L) const { return Qk[L & 1]; }
};

// the root test and levels 1..L (nothing read back): the octree rows in the arena, the counts in ctl
static int m2s_nodes_levels(int64_t F, const float *fv, uint32_t L, M2sNodes &w, hipStream_t st) {
  M2sCtl *ctl = w.ctl;
  uint32_t *fmin8 = w.fmin8(L);
  KL_CHECK_RC(fill_async(ctl, 0, w.ctl_bytes, st));
  if (F == 0) return KL_OK;
  hipLaunchKernelGGL(m2s_root_kernel, dim3((unsigned)cdiv(F, 256)), dim3(256), 0, st, F, fv, w.Qk[0], w.Qf[0], w.seg,
                     ctl, w.M[0], w.SL[0], fmin8, L);
  KL_CHECK_LAUNCH();
  const unsigned grid = (unsigned)std::max<int64_t>(M2S_GRID, cdiv((int64_t)w.cap, 256 * M2S_MAX_CHUNKS));
  const unsigned rgrid = (unsigned)std::min<int64_t>(256, std::max<int64_t>(w.tiles, 1));  // one per CU
  for (uint32_t l = 1; l <= L; l++) {
    // level l - 2's S and octree row resolve the keys of level l - 1's pairs (level -1: ctl's root)
    const uint32_t *Spp = l >= 2 ? w.S[l & 1] : ctl->root_S;
    const uint8_t *octpp = l >= 2 ? w.arena : (const uint8_t *)&ctl->root_oct;
    const uint32_t *opp = l >= 2 ? &ctl->O[l - 2] : &ctl->zero;
    const int a = (l - 1) & 1;
    if (l < L)
      hipLaunchKernelGGL(m2s_node_kernel<false>, dim3(grid), dim3(256), 0, st, fv, w.Qk[a], w.Qf[a], w.Qk[a ^ 1],
                         w.Qf[a ^ 1], w.seg, ctl, l, Spp, octpp, opp, w.M[a], (uint8_t *)w.SL[a], fmin8);
    else
      hipLaunchKernelGGL(m2s_node_kernel<true>, dim3(grid), dim3(256), 0, st, fv, w.Qk[a], w.Qf[a], w.Qk[a ^ 1],
                         w.Qf[a ^ 1], w.seg, ctl, l, Spp, octpp, opp, w.M[a], (uint8_t *)w.SL[a], fmin8);
    KL_CHECK_LAUNCH();
    // level l - 1's row scanned: S_{l-1}, U_l, O_l, M_l
    hipLaunchKernelGGL(m2s_rank_kernel, dim3(rgrid), dim3(256), 0, st, ctl, l - 1, L, w.arena, w.M[a], w.S[a],
                       w.M[a ^ 1], w.SL[a], w.SL[a ^ 1], w.status, fmin8, w.ncap, w.oct_cap, w.fmin_cap);
    KL_CHECK_LAUNCH();
  }
  return KL_OK;
}

// mesh_to_spc by node ranks (m2s_node_kernel): returns KL_OK, an error, or 1 = not taken
// (capacity): the caller runs the per-level path.  One host read (the counts, after the levels).
static int mesh_to_spc_nodes(int64_t F, const float *fv, uint32_t L, Scratch &sc, uint8_t **octree,
                             int64_t *num_nodes, int64_t **face_idx, float **bary, int64_t *num_leaves,
                             hipStream_t st) {
  *octree = nullptr;
  *face_idx = nullptr;
  *bary = nullptr;
  *num_nodes = 0;
  *num_leaves = 0;
  M2sNodes w;
  if (F <= 0 || L == 0 || !w.plan(F)) return 1;
  char *base = (char *)sc.get(w.total);
  if (!base) return KL_E_ALLOC;
  w.place(base);
  KL_CHECK_RC(m2s_nodes_levels(F, fv, L, w, st));
  std::vector<char> hbuf(sizeof(M2sCtl));
  M2sCtl &h = *(M2sCtl *)hbuf.data();
  KL_CHECK_RC(host_read(&h, w.ctl, sizeof(M2sCtl), st));
  if (h.overflow) return 1;
  t_m2s_counts[0] = F;
  for (uint32_t l = 1; l <= L; l++) {
    unsigned long long t = 0;
    for (int g = 0; g < M2S_SHARDS; g++) t += h.counts[(l - 1) * M2S_SHARDS + g];
    t_m2s_counts[l] = 8 * (int64_t)t;
  }
  t_m2s_levels = (int)L + 1;
  const int64_t leaves = h.U[L];
  if (leaves == 0) return KL_OK;  // empty: (0,) u8, (0,) i64, (0,3) f32 built by the caller
  const int64_t nodes = h.O[L];
  // (r06) the three outputs from ONE allocation (each is a host callback into the caller's allocator,
  // made while the GPU idles after the count read): face ids | barycentrics | octree, 256-B aligned
  const size_t ofu = 0, obu = al256b((size_t)leaves * sizeof(int64_t)),
               oout = obu + al256b((size_t)leaves * 2 * sizeof(float));
  char *blk = (char *)sc.get(oout + (size_t)nodes);
  if (!blk) return KL_E_ALLOC;
  int64_t *fu = (int64_t *)(blk + ofu);
  float *bu = (float *)(blk + obu);
  uint8_t *out = (uint8_t *)(blk + oout);
  KL_CHECK_HIP(hipMemcpyAsync(out, w.arena, (size_t)nodes, hipMemcpyDeviceToDevice, st));
  const int64_t nslots = 8 * (int64_t)h.U[L - 1];
  const int b = (int)((L - 1) & 1);
  hipLaunchKernelGGL(m2s_node_leaves_kernel, dim3((unsigned)cdiv(nslots, 256)), dim3(256), 0, st, nslots, w.ctl, L,
                     w.arena, w.S[b], w.M[b], w.fmin8(L), fv, fu, bu);
  KL_CHECK_LAUNCH();
  *octree = out;
  *num_nodes = nodes;
  *face_idx = fu;
  *bary = bu;
  *num_leaves = leaves;
  return KL_OK;
}

// The fixed-capacity form's last step, sized on the device: result = (nodes, leaves, status), status
// 0 = written, 1 = an output capacity too small (nothing written; nodes / leaves say what is
// needed), 2 = the workspace's pair buffers overflowed (counts unknown: run the eager call).
__global__ void m2s_fixed_final_kernel(const M2sCtl *__restrict__ ctl, uint32_t L, const uint8_t *__restrict__ arena,
                                       const uint32_t *__restrict__ Sp, const uint64_t *__restrict__ Mp,
                                       const uint32_t *__restrict__ fmin8, const float *__restrict__ fv,
                                       int64_t node_cap, int64_t leaf_cap, uint8_t *__restrict__ octree,
                                       int64_t *__restrict__ fout, float *__restrict__ bary,
                                       int64_t *__restrict__ result) {
  const int64_t leaves = ctl->U[L], nodes = leaves ? (int64_t)ctl->O[L] : 0;
  const int over = ctl->overflow;
  const int status = over ? 2 : (nodes > node_cap || leaves > leaf_cap ? 1 : 0);
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
  if (t0 == 0) {
    result[0] = over ? 0 : nodes;
    result[1] = over ? 0 : leaves;
    result[2] = status;
  }
  if (status || leaves == 0) return;
  for (int64_t t = t0; t < nodes; t += step) octree[t] = arena[t];
  const int64_t nslots = 8 * (int64_t)ctl->U[L - 1];
  const uint32_t OL1 = ctl->O[L - 1];
  for (int64_t s = t0; s < nslots; s += step) {
    const uint32_t jp = (uint32_t)(s >> 3), c = (uint32_t)(s & 7);
    const uint32_t b = arena[OL1 + jp];
    if (!((b >> c) & 1)) continue;
    const uint32_t o = Sp[jp] + (uint32_t)__popc(b & ((1u << c) - 1u));
    const uint64_t q = Mp[jp] * 2 + m2s_child_off(c);
    leaf_out_pt((int)(q & 0xffff), (int)((q >> 16) & 0xffff), (int)(q >> 32), (int64_t)fmin8[s], fv, L, o, fout, bary);
  }
}

// ------------------------------------------------------------------ scan_octrees
__global__ void popc_kernel(int64_t n, const uint8_t *__restrict__ o, uint32_t *__restrict__ c) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < n) c[t] = (uint32_t)__popc(o[t]);
  if (t == n) c[t] = 0;
}

// pyramid walk of scan_octrees.cu:66-103 on device (one thread)
__global__ void pyramid_kernel(const int32_t *__restrict__ ex, uint32_t osize, int32_t *__restrict__ pyr,
                               int32_t *__restrict__ level_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int STR = SPC_MAX_LEVELS + 2;
  for (int i = 0; i < 2 * STR; i++) pyr[i] = 0;
  int32_t *Pmid = pyr, *PmidSum = pyr + STR;
  uint32_t prevSum = 0, sum = 1;
  Pmid[0] = 1;
  PmidSum[0] = 0;
  PmidSum[1] = 1;
  int level = 0;
  while (sum <= osize && level < SPC_MAX_LEVELS) {
    const uint32_t currSum = (uint32_t)ex[prevSum + 1];
    const uint32_t Lsize = currSum - prevSum;
    prevSum = currSum;
    Pmid[++level] = (int32_t)Lsize;
    sum += Lsize;
    PmidSum[level + 1] = (int32_t)sum;
  }
  *level_out = level;
}

// nodes_to_morton (spc_utils.cuh:140-160)
__global__ void nodes_to_morton_kernel(const uint8_t *__restrict__ octree, const int32_t *__restrict__ incl,
                                       const uint64_t *__restrict__ min_, uint64_t *__restrict__ mall, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint8_t bits = octree[t];
  const uint64_t code = min_[t];
  int addr = incl[t];
  for (int i = 7; i >= 0; i--)
    if (bits & (1u << i)) mall[addr--] = 8 * code + (uint64_t)i;
}

__global__ void morton_to_points_kernel(const uint64_t *__restrict__ m, int16_t *__restrict__ p, int64_t n) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= n) return;
  int16_t x, y, z;
  to_point(m[t], x, y, z);
  p[t * 3 + 0] = x;
  p[t * 3 + 1] = y;
  p[t * 3 + 2] = z;
}

// points_to_morton (point_utils_cuda.cu, spc_math.h:93-107): one lane per point; the 6 B
// point is read as three int16 loads (rows of 6 B are not 4-B aligned) and the code is
// written as one 8-B store, so a wave moves 384 B in and 512 B out.
__global__ void points_to_morton_kernel(const int16_t *__restrict__ p, int64_t *__restrict__ m, int64_t n) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= n) return;
  m[t] = (int64_t)to_morton(p[t * 3 + 0], p[t * 3 + 1], p[t * 3 + 2]);
}

// ------------------------------------------------------------------ raytrace
__device__ __forceinline__ float ray_aabb(const float o_q[3], const float d[3], const float inv[3],
                                          const float sgn[3], const float org[3], float r) {
  const float o0 = o_q[0] - org[0], o1 = o_q[1] - org[1], o2 = o_q[2] - org[2];
  const float cmax = fmaxf(fmaxf(fabsf(o0), fabsf(o1)), fabsf(o2));
  float winding = cmax < r ? -1.0f : 1.0f;
  winding *= r;
  if (winding < 0) return winding;
  const float d0 = fmaf(winding, sgn[0], -o0) * inv[0];
  const float d1 = fmaf(winding, sgn[1], -o1) * inv[1];
  const float d2 = fmaf(winding, sgn[2], -o2) * inv[2];
  const float ltxy = fmaf(d[1], d0, o1), ltxz = fmaf(d[2], d0, o2);
  const float ltyx = fmaf(d[0], d1, o0), ltyz = fmaf(d[2], d1, o2);
  const float ltzx = fmaf(d[0], d2, o0), ltzy = fmaf(d[1], d2, o1);
  const bool t0 = (d0 >= 0.0f) && (fabsf(ltxy) <= r) && (fabsf(ltxz) <= r);
  const bool t1 = (d1 >= 0.0f) && (fabsf(ltyx) <= r) && (fabsf(ltyz) <= r);
  const bool t2 = (d2 >= 0.0f) && (fabsf(ltzx) <= r) && (fabsf(ltzy) <= r);
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
  if (t0) s0 = sgn[0];
  else if (t1) s1 = sgn[1];
  else if (t2) s2 = sgn[2];
  float dd = 0.0f;
  if (s0 != 0.0f) dd = d0;
  else if (s1 != 0.0f) dd = d1;
  else if (s2 != 0.0f) dd = d2;
  if (dd != 0.0f) return dd;
  return 0.0f;
}

// children of a node in front-to-back order from the origin's octant code: increasing Hamming
// distance to the code, then index (rt_children) -- one nibble per child index, 8 per code
__constant__ uint32_t c_rt_perm[8] = {0x76534210u, 0x67425301u, 0x57416302u, 0x46507213u,
                                      0x37216504u, 0x26307415u, 0x15307426u, 0x04216537u};

struct RayIn {
  const uint8_t *octree;
  const int16_t *points;
  const int32_t *exsum;
  const float *ro, *rd;
};

// decide (raytrace_cuda.cu:63-222): info = children count / keep flag; depth at the target level
// (fixed-capacity entry: the count is read from dnum on the device and info is zeroed up to span)
__device__ __forceinline__ void rt_decide_one(const RayIn &in, int64_t t, const int2 *__restrict__ nug,
                                              uint32_t *__restrict__ info, float *__restrict__ depth, uint32_t level,
                                              int last, int with_depth, int with_exit) {
  const int ridx = nug[t].x, pidx = nug[t].y;
  const int16_t *p = in.points + (int64_t)pidx * 3;
  const float o[3] = {in.ro[ridx * 3], in.ro[ridx * 3 + 1], in.ro[ridx * 3 + 2]};
  const float d[3] = {in.rd[ridx * 3], in.rd[ridx * 3 + 1], in.rd[ridx * 3 + 2]};
  const float r = (float)(1.0 / (double)(float)(1u << level));
  const float vc[3] = {fmaf(r, fmaf(2.0f, (float)p[0], 1.0f), -1.0f), fmaf(r, fmaf(2.0f, (float)p[1], 1.0f), -1.0f),
                       fmaf(r, fmaf(2.0f, (float)p[2], 1.0f), -1.0f)};
  const float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f, signbit(d[2]) ? 1.0f : -1.0f};
  const float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
  if (last && with_depth) {
    if (with_exit) {
      const float xs[3] = {signbit(-d[0]) ? 1.0f : -1.0f, signbit(-d[1]) ? 1.0f : -1.0f,
                           signbit(-d[2]) ? 1.0f : -1.0f};
      const float en = ray_aabb(o, d, inv, sgn, vc, r);
      const float ex = ray_aabb(o, d, inv, xs, vc, r);
      depth[t * 2] = en;
      depth[t * 2 + 1] = ex;
      info[t] = (en > 0.0f && ex > 0.0f) ? 1u : 0u;
    } else {
      const float dv = ray_aabb(o, d, inv, sgn, vc, r);
      depth[t] = dv;
      info[t] = dv > 0.0f ? 1u : 0u;
    }
  } else {
    const float dv = ray_aabb(o, d, inv, sgn, vc, r);
    if (!last)
      info[t] = dv != 0.0f ? (uint32_t)__popc(in.octree[pidx]) : 0u;
    else
      info[t] = dv > 0.0f ? 1u : 0u;
  }
}

__global__ void rt_decide_kernel(RayIn in, int64_t num, const int2 *__restrict__ nug, uint32_t *__restrict__ info,
                                 float *__restrict__ depth, uint32_t level, int last, int with_depth, int with_exit) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t == num) info[t] = 0;
  if (t >= num) return;
  rt_decide_one(in, t, nug, info, depth, level, last, with_depth, with_exit);
}

__device__ __forceinline__ void rt_subdivide_one(const RayIn &in, int64_t t, const int2 *__restrict__ nin,
                                                 int2 *__restrict__ nout, const uint32_t *__restrict__ info,
                                                 const uint32_t *__restrict__ psum, uint32_t level, int64_t cap) {
  if (!info[t]) return;
  const int ridx = nin[t].x, pidx = nin[t].y;
  const int16_t *p = in.points + (int64_t)pidx * 3;
  uint32_t base = psum[t];
  const uint8_t ob = in.octree[pidx];
  const uint32_t s = (uint32_t)in.exsum[pidx];
  const float scale = (float)(1.0 / (double)(float)(1u << level));
  const float *org = in.ro + (int64_t)ridx * 3;
  const float x = (float)((double)(0.5f * org[0] + 0.5f) - (double)scale * ((double)(float)p[0] + 0.5));
  const float y = (float)((double)(0.5f * org[1] + 0.5f) - (double)scale * ((double)(float)p[1] + 0.5));
  const float z = (float)((double)(0.5f * org[2] + 0.5f) - (double)scale * ((double)(float)p[2] + 0.5));
  uint32_t code = 0;
  if (x > 0) code = 4;
  if (y > 0) code += 2;
  if (z > 0) code += 1;
  // front-to-back: children by increasing Hamming distance to `code`, then index
  for (int h = 0; h <= 3; h++)
    for (uint32_t j = 0; j < 8; j++) {
      if (__popc(code ^ j) != h || !(ob & (1u << j))) continue;
      const uint32_t c = (uint32_t)__popc(ob & ((2u << j) - 1));
      if (base < cap) nout[base] = make_int2(ridx, (int)(s + c));
      base++;
    }
}

__global__ void rt_subdivide_kernel(RayIn in, int64_t num, const int2 *__restrict__ nin, int2 *__restrict__ nout,
                                    const uint32_t *__restrict__ info, const uint32_t *__restrict__ psum,
                                    uint32_t level, int64_t cap) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < num) rt_subdivide_one(in, t, nin, nout, info, psum, level, cap);
}

__global__ void rt_compact_kernel(int64_t num, const int2 *__restrict__ nin, const float *__restrict__ din,
                                  int2 *__restrict__ nout, float *__restrict__ dout, int dd,
                                  const uint32_t *__restrict__ info, const uint32_t *__restrict__ psum, int64_t cap) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= num || !info[t]) return;
  const uint32_t o = psum[t];
  if (o >= cap) return;
  nout[o] = nin[t];
  if (dout)
    for (int k = 0; k < dd; k++) dout[(int64_t)o * dd + k] = din[t * dd + k];
}

__global__ void rt_init_kernel(int64_t n, int2 *__restrict__ nug, uint32_t *__restrict__ dnum,
                               int64_t *__restrict__ result) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < n) nug[t] = make_int2((int)t, 0);
  if (t == 0 && dnum) {
    *dnum = (uint32_t)n;
    result[0] = 0;
    result[1] = 0;
  }
}

// fixed-capacity entry, after a level's scan: the next level's count on the device, clipped to
// the capacity (the nuggets kept are then a prefix of the full list: the lists stay in ray,
// front-to-back order and a nugget's children follow its predecessors'); result = (rows,
// truncated)
__global__ void rt_count_kernel(const uint32_t *__restrict__ psum, uint32_t cap, uint32_t *__restrict__ dnum,
                                int64_t *__restrict__ result, int last) {
  if (threadIdx.x != 0) return;
  const uint32_t n = psum[*dnum];  // the scan's total, at the level's count
  *dnum = n < cap ? n : cap;
  if (n > cap) result[1] = 1;
  if (last) result[0] = n < cap ? n : cap;
}

// Fixed-capacity level kernels: a fixed grid strides over the level's count read on the device
// (a grid sized to the capacity paid ~10 us per launch for its empty workgroups at 13 M rows).
constexpr int RTF_GRID = 2048;

__global__ void __launch_bounds__(256) rtf_decide_kernel(RayIn in, const uint32_t *__restrict__ dnum,
                                                         const int2 *__restrict__ nug, uint32_t *__restrict__ info,
                                                         float *__restrict__ depth, uint32_t level, int last,
                                                         int with_depth, int with_exit) {
  const int64_t num = *dnum;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < num; t += (int64_t)gridDim.x * 256)
    rt_decide_one(in, t, nug, info, depth, level, last, with_depth, with_exit);
}

__global__ void __launch_bounds__(256) rtf_subdivide_kernel(RayIn in, const uint32_t *__restrict__ dnum,
                                                            const int2 *__restrict__ nin, int2 *__restrict__ nout,
                                                            const uint32_t *__restrict__ info,
                                                            const uint32_t *__restrict__ psum, uint32_t level,
                                                            int64_t cap) {
  const int64_t num = *dnum;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < num; t += (int64_t)gridDim.x * 256)
    rt_subdivide_one(in, t, nin, nout, info, psum, level, cap);
}

__global__ void __launch_bounds__(256) rtf_compact_kernel(const uint32_t *__restrict__ dnum,
                                                          const int2 *__restrict__ nin, const float *__restrict__ din,
                                                          int2 *__restrict__ nout, float *__restrict__ dout, int dd,
                                                          const uint32_t *__restrict__ info,
                                                          const uint32_t *__restrict__ psum, int64_t cap) {
  const int64_t num = *dnum;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < num; t += (int64_t)gridDim.x * 256) {
    if (!info[t]) continue;
    const uint32_t o = psum[t];
    if (o >= cap) continue;
    nout[o] = nin[t];
    if (dout)
      for (int k = 0; k < dd; k++) dout[(int64_t)o * dd + k] = din[t * dd + k];
  }
}

// Exclusive scan of in[0, *dn) into out[0, *dn], out[*dn] = the total, with the count read on the
// device: tile sums, one workgroup scanning them, then each tile's scan plus its offset.  Tiles
// past the count exit at once.
constexpr int DSCAN_PER = 16, DSCAN_TILE = 256 * DSCAN_PER;

__global__ void __launch_bounds__(256) dscan_tile_sum_kernel(const uint32_t *__restrict__ in,
                                                             const uint32_t *__restrict__ dn,
                                                             uint32_t *__restrict__ tsum) {
  __shared__ int s_wave[4];
  const int64_t n = *dn, base = blockIdx.x * (int64_t)DSCAN_TILE;
  if (base >= n) return;  // uniform
  int v = 0;
#pragma unroll
  for (int k = 0; k < DSCAN_PER; k++) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i < n) v += (int)in[i];
  }
  int tot = 0;
  (void)block_exclusive_scan(v, s_wave, &tot);
  if (threadIdx.x == 0) tsum[blockIdx.x] = (uint32_t)tot;
}

__global__ void __launch_bounds__(1024) dscan_tile_offset_kernel(uint32_t *__restrict__ tsum,
                                                                 const uint32_t *__restrict__ dn,
                                                                 uint32_t *__restrict__ out) {
  __shared__ int s_wave[16];
  const int64_t n = *dn;
  const int nt = (int)((n + DSCAN_TILE - 1) / DSCAN_TILE);
  uint32_t carry = 0;
  for (int b0 = 0; b0 < nt; b0 += 1024) {
    const int i = b0 + threadIdx.x;
    const int v = i < nt ? (int)tsum[i] : 0;
    int tot = 0;
    const int ex = block_exclusive_scan(v, s_wave, &tot);
    if (i < nt) tsum[i] = carry + (uint32_t)ex;
    carry += (uint32_t)tot;
  }
  if (threadIdx.x == 0) out[n] = carry;
}

__global__ void __launch_bounds__(256) dscan_apply_kernel(const uint32_t *__restrict__ in,
                                                          const uint32_t *__restrict__ dn,
                                                          const uint32_t *__restrict__ toff,
                                                          uint32_t *__restrict__ out) {
  __shared__ int s_wave[4];
  const int64_t n = *dn, base = blockIdx.x * (int64_t)DSCAN_TILE;
  if (base >= n) return;  // uniform
  const int64_t i0 = base + threadIdx.x * DSCAN_PER;
  uint32_t v[DSCAN_PER];
  int sum = 0;
#pragma unroll
  for (int k = 0; k < DSCAN_PER; k++) {
    v[k] = i0 + k < n ? in[i0 + k] : 0u;
    sum += (int)v[k];
  }
  int tot = 0;
  uint32_t run = toff[blockIdx.x] + (uint32_t)block_exclusive_scan(sum, s_wave, &tot);
#pragma unroll
  for (int k = 0; k < DSCAN_PER; k++) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
  }
}

// ---- Fused level march (r05): ONE launch per level.  Each workgroup takes tiles of RTL_TILE
// nuggets by ticket, decides them (the reference's ray_aabb, raytrace_cuda.cu:63-222), scans the
// children counts with a decoupled look-back over the tiles (a tile only waits on tiles with
// smaller tickets, held by workgroups already running), and writes the children front to back
// (raytrace_cuda.cu:224-269) -- or, at the target level, the kept nuggets and depths -- at their
// final positions.  The last tile leaves the level's count on the device for the next launch.
// Replaces decide + scan (3 launches) + subdivide + count per level and the host count read of
// every level: the eager call reads 8 bytes once, at the end.
// 16 nuggets per thread (their loads in flight together); one workgroup per CU takes the tiles in
// ticket order, so most tiles find an inclusive predecessor close by (with a workgroup per tile
// and 4 nuggets per thread, ~1,600 tiles at cfg4's deepest level all looked back at once, up to
// 25 rounds of 64 tiles each: the fused march took 2.35 ms against the per-level march's 1.17)
constexpr int RTL_PER = 16, RTL_TILE = 256 * RTL_PER;
struct RtlCtl {
  uint32_t dnum[SPC_MAX_LEVELS + 2];    // nuggets of each level, clipped to the capacity
  uint32_t total[SPC_MAX_LEVELS + 2];   // the same, unclipped
  uint32_t ticket[SPC_MAX_LEVELS + 2];  // tile tickets of each level
  uint32_t truncated;                   // some level had more nuggets than the capacity
};

#if KL_DEV  // the fused level march (dev param 15 = 3): a measured dead end, DESIGN.md 3.5
constexpr int RTL_GRID = 256;
__device__ __forceinline__ void rt_children(const RayIn &in, int ridx, int pidx, uint32_t level, uint32_t base,
                                            int2 *__restrict__ nout, uint32_t cap) {
  const int16_t *p = in.points + (int64_t)pidx * 3;
  const uint8_t ob = in.octree[pidx];
  const uint32_t s = (uint32_t)in.exsum[pidx];
  const float scale = (float)(1.0 / (double)(float)(1u << level));
  const float *org = in.ro + (int64_t)ridx * 3;
  const float x = (float)((double)(0.5f * org[0] + 0.5f) - (double)scale * ((double)(float)p[0] + 0.5));
  const float y = (float)((double)(0.5f * org[1] + 0.5f) - (double)scale * ((double)(float)p[1] + 0.5));
  const float z = (float)((double)(0.5f * org[2] + 0.5f) - (double)scale * ((double)(float)p[2] + 0.5));
  uint32_t code = 0;
  if (x > 0) code = 4;
  if (y > 0) code += 2;
  if (z > 0) code += 1;
  // front-to-back: children by increasing Hamming distance to `code`, then index
  for (int h = 0; h <= 3; h++)
    for (uint32_t j = 0; j < 8; j++) {
      if (__popc(code ^ j) != h || !(ob & (1u << j))) continue;
      const uint32_t c = (uint32_t)__popc(ob & ((2u << j) - 1));
      if (base < cap) nout[base] = make_int2(ridx, (int)(s + c));
      base++;
    }
}

__global__ void __launch_bounds__(256) rt_level_kernel(RayIn in, RtlCtl *__restrict__ ctl,
                                                       const int2 *__restrict__ nin, int2 *__restrict__ nout,
                                                       float *__restrict__ dout, unsigned long long *__restrict__ status,
                                                       int64_t num_rays, uint32_t level, int last, int with_depth,
                                                       int with_exit, uint32_t cap) {
  __shared__ int s_wave[4];
  __shared__ uint32_t s_tile, s_prefix;
  const uint32_t num = level == 0 ? (uint32_t)num_rays : ctl->dnum[level];
  const uint32_t ntiles = (num + RTL_TILE - 1) / RTL_TILE;
  const unsigned long long tag_agg = (unsigned long long)(2 * level + 2) << 32,
                           tag_inc = (unsigned long long)(2 * level + 3) << 32;
  const int dd = with_exit ? 2 : 1;
  const float r = (float)(1.0 / (double)(float)(1u << level));
  for (;;) {
    if (threadIdx.x == 0) s_tile = atomicAdd(&ctl->ticket[level], 1u);
    __syncthreads();
    const uint32_t t = s_tile;
    if (t >= ntiles) break;
    // ---- decide this thread's RTL_PER consecutive nuggets
    uint32_t cnt[RTL_PER];
    int2 nug[RTL_PER];
    float dv0[RTL_PER], dv1[RTL_PER];
    int local = 0;
#pragma unroll
    for (int k = 0; k < RTL_PER; k++) {
      const uint32_t i = t * RTL_TILE + threadIdx.x * RTL_PER + k;
      cnt[k] = 0;
      dv0[k] = dv1[k] = 0.0f;
      nug[k] = make_int2(0, 0);
      if (i < num) {
        nug[k] = level == 0 ? make_int2((int)i, 0) : nin[i];
        const int ridx = nug[k].x, pidx = nug[k].y;
        const int16_t *p = in.points + (int64_t)pidx * 3;
        const float o[3] = {in.ro[ridx * 3], in.ro[ridx * 3 + 1], in.ro[ridx * 3 + 2]};
        const float d[3] = {in.rd[ridx * 3], in.rd[ridx * 3 + 1], in.rd[ridx * 3 + 2]};
        const float vc[3] = {fmaf(r, fmaf(2.0f, (float)p[0], 1.0f), -1.0f), fmaf(r, fmaf(2.0f, (float)p[1], 1.0f), -1.0f),
                             fmaf(r, fmaf(2.0f, (float)p[2], 1.0f), -1.0f)};
        const float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f, signbit(d[2]) ? 1.0f : -1.0f};
        const float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
        if (last && with_depth && with_exit) {
          const float xs[3] = {signbit(-d[0]) ? 1.0f : -1.0f, signbit(-d[1]) ? 1.0f : -1.0f,
                               signbit(-d[2]) ? 1.0f : -1.0f};
          dv0[k] = ray_aabb(o, d, inv, sgn, vc, r);
          dv1[k] = ray_aabb(o, d, inv, xs, vc, r);
          cnt[k] = (dv0[k] > 0.0f && dv1[k] > 0.0f) ? 1u : 0u;
        } else {
          dv0[k] = ray_aabb(o, d, inv, sgn, vc, r);
          if (!last)
            cnt[k] = dv0[k] != 0.0f ? (uint32_t)__popc(in.octree[pidx]) : 0u;
          else
            cnt[k] = dv0[k] > 0.0f ? 1u : 0u;
        }
      }
      local += (int)cnt[k];
    }
    int agg = 0;
    const int ex = block_exclusive_scan(local, s_wave, &agg);
    // ---- the tile's offset: publish the aggregate, look back over earlier tiles (wave 0)
    if (threadIdx.x < 64) {
      uint32_t prefix = 0;
      if (t == 0) {
        if (threadIdx.x == 0)
          __hip_atomic_store(status, tag_inc | (uint32_t)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        if (threadIdx.x == 0)
          __hip_atomic_store(status + t, tag_agg | (uint32_t)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int64_t end = t;  // lane i reads tile end - 1 - i (before tile 0: an inclusive 0)
        for (;;) {
          const int64_t k = end - 1 - (int64_t)threadIdx.x;
          const unsigned long long v =
              k >= 0 ? __hip_atomic_load(status + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag_inc;
          const unsigned long long tg = v & 0xffffffff00000000ull;
          const uint64_t inc = ballot(tg == tag_inc), any = ballot(tg == tag_inc || tg == tag_agg);
          if (inc) {  // the nearest inclusive tile, once every tile after it has published
            const int f = __builtin_ctzll(inc);
            const uint64_t need = f == 63 ? ~0ull : ((2ull << f) - 1);
            if ((any & need) == need) {
              uint32_t x = (int)threadIdx.x <= f ? (uint32_t)v : 0u;
#pragma unroll
              for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
              prefix += x;
              break;
            }
          } else if (any == ~0ull) {  // 64 aggregates: add them, look further back
            uint32_t x = (uint32_t)v;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
            prefix += x;
            end -= 64;
            continue;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (threadIdx.x == 0)
          __hip_atomic_store(status + t, tag_inc | (prefix + (uint32_t)agg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (threadIdx.x == 0) s_prefix = prefix;
    }
    __syncthreads();
    const uint32_t prefix = s_prefix;
    uint32_t base = prefix + (uint32_t)ex;
    // ---- the outputs at their final positions (a prefix of `cap` of them)
#pragma unroll
    for (int k = 0; k < RTL_PER; k++) {
      if (!cnt[k]) continue;
      if (!last) {
        rt_children(in, nug[k].x, nug[k].y, level, base, nout, cap);
      } else if (base < cap) {
        nout[base] = nug[k];
        if (dout && with_depth) {
          dout[(int64_t)base * dd] = dv0[k];
          if (with_exit) dout[(int64_t)base * dd + 1] = dv1[k];
        }
      }
      base += cnt[k];
    }
    if (t + 1 == ntiles && threadIdx.x == 0) {
      const uint32_t total = prefix + (uint32_t)agg;
      ctl->total[level + 1] = total;
      ctl->dnum[level + 1] = total < cap ? total : cap;
      if (total > cap) ctl->truncated = 1;
    }
    __syncthreads();  // s_tile / s_prefix are rewritten for the next tile
  }
}

// the fused march over levels 0..target_level; ctl and status zeroed here; n0 / n1 ping-pong
// buffers of `cap` rows; the target level's nuggets / depths go to out / dout (`cap` rows)
static int rt_fused_levels(const RayIn &in, int64_t num_rays, uint32_t target_level, int return_depth, int with_exit,
                           uint32_t cap, RtlCtl *ctl, unsigned long long *status, int2 *n0, int2 *n1, int2 *out,
                           float *dout, hipStream_t st) {
  const int64_t ntiles_max = cdiv(std::max<int64_t>((int64_t)cap, num_rays), (int64_t)RTL_TILE);
  KL_CHECK_RC(fill_async(ctl, 0, sizeof(RtlCtl), st));
  KL_CHECK_RC(fill_async(status, 0, (size_t)std::max<int64_t>(ntiles_max, 1) * 8, st));
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ntiles_max, RTL_GRID));
  const int2 *src = nullptr;
  for (uint32_t l = 0; l <= target_level; l++) {
    const int last = l == target_level;
    int2 *dst = last ? out : ((l & 1) ? n1 : n0);
    hipLaunchKernelGGL(rt_level_kernel, dim3(grid), dim3(256), 0, st, in, ctl, src, dst, last ? dout : nullptr, status,
                       num_rays, l, last, return_depth, with_exit, cap);
    KL_CHECK_LAUNCH();
    src = dst;
  }
  return KL_OK;
}
#endif  // KL_DEV


// ---- Hit-list level march (r05, the default of both entries): level l's list holds the nuggets
// that HIT at level l (not the candidates).  Per level, one count pass decides every listed node's
// children at l + 1 together (their points are contiguous: points[s + 1 .. s + popc]), leaving a
// byte of hit children per node; the write pass lists the hit children in front-to-back order
// (rt_children's order) -- at the target level with their depths.  Against the per-level march
// (decide every candidate, scan, then subdivide every hit into its untested children): the
// candidates are never written or re-read, the ray is read once per hit node instead of once per
// candidate, and no count goes back to the host until the end.
// Each pass's workgroup takes a contiguous run of 256-node tiles (rth_span), so the list offsets
// need only the workgroups' totals: each workgroup publishes its total (agent-scope store), and
// the workgroup that finishes last (a ticket: MI355X_MICROARCH.md's hand-off -- vmcnt(0), barrier,
// one agent-scope add; agent-scope loads) scans them for the next pass -- two launches per level.
// Fixed-capacity mode (kl_raytrace_fixed): the per-level march keeps each level's first `cap`
// candidates (a hit node's children, untested) and drops the rest with their subtrees; here a child
// is kept when its candidate index -- the node's candidate base (the listed nodes' child counts
// `pc` summed over the list before it) plus its front-to-back rank -- is below `cap`, so the lists
// are exactly the hits among the per-level march's kept candidates.  The candidate bases' workgroup
// totals are added up by the previous write pass (per next-list workgroup) and scanned by its last
// workgroup (level 0: rth_root_kernel).
constexpr int RTH_TILE = 256;      // nodes per tile = threads per workgroup
#ifndef RTH_MIN_WAVES  // rth_count_kernel's minimum waves per SIMD (A/B builds)
#define RTH_MIN_WAVES 8  // r06: 63 VGPRs, 8 waves (66 and 7 unbounded): the kernel 6.7 % faster
#endif
constexpr int RTH_SCAN_PT = 8;     // the last workgroup's scan: 8 totals per thread, 2,048 workgroups
constexpr int RTH_PW = 32;         // the write pass's LDS sums of the next list's workgroup totals
static_assert(RTF_GRID <= RTH_TILE * RTH_SCAN_PT, "one pass of the last workgroup's scan");

__device__ __forceinline__ void rth_node(const int2 *__restrict__ list, int64_t i, int &ridx, int &pidx) {
  const int2 nu = list[i];
  ridx = nu.x;
  pidx = nu.y;
}

// The front-to-back rank of each child of node pidx (index order k -> rank nibble), from the ray's
// octant code at the node (rt_children's order)
__device__ __forceinline__ uint32_t rth_fb_ranks(const RayIn &in, int ridx, int pidx, uint32_t level, uint32_t ob) {
  const int16_t *p = in.points + (int64_t)pidx * 3;
  const float *org = in.ro + (int64_t)ridx * 3;
  const float scale = (float)(1.0 / (double)(float)(1u << level));
  const float x = (float)((double)(0.5f * org[0] + 0.5f) - (double)scale * ((double)(float)p[0] + 0.5));
  const float y = (float)((double)(0.5f * org[1] + 0.5f) - (double)scale * ((double)(float)p[1] + 0.5));
  const float z = (float)((double)(0.5f * org[2] + 0.5f) - (double)scale * ((double)(float)p[2] + 0.5));
  const uint32_t perm = c_rt_perm[(x > 0 ? 4u : 0u) + (y > 0 ? 2u : 0u) + (z > 0 ? 1u : 0u)];
  uint32_t ranks = 0;
  int rk = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t j = (perm >> (4 * q)) & 15u;
    if (ob & (1u << j)) {
      const int k = __popc(ob & ((1u << j) - 1));  // index-order position of child j
      ranks |= (uint32_t)rk << (4 * k);
      rk++;
    }
  }
  return ranks;
}

// this workgroup's tiles [t0, t1) of a list of n nodes: contiguous runs, balanced (every workgroup
// of the grid gets floor or ceil of tiles / grid, so all of them are in flight; the grid is a power
// of two); rth_owner inverts it
__device__ __forceinline__ int64_t rth_tile0(int64_t w, int64_t nt) {  // workgroup w's first tile
  return (w * nt) >> __builtin_ctz(gridDim.x);
}
__device__ __forceinline__ void rth_span(int64_t n, int64_t &t0, int64_t &t1) {
  const int64_t nt = (n + RTH_TILE - 1) / RTH_TILE;
  t0 = rth_tile0(blockIdx.x, nt);
  t1 = rth_tile0((int64_t)blockIdx.x + 1, nt);
}
// the workgroup whose run holds tile T of a list of nt tiles
__device__ __forceinline__ uint32_t rth_owner(int64_t T, int64_t nt) {
  const int64_t G = gridDim.x;
  return (uint32_t)((T * G + G - 1) / nt);
}

// 64-bit exclusive scan over the RTH_TILE threads; *total = the sum
__device__ __forceinline__ uint64_t rth_scan64(uint64_t v, uint64_t *s_w, uint64_t *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < RTH_TILE / 64; w++) {
    const uint64_t t = s_w[w];
    before += w < wid ? t : 0;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + inc - v;
}

// the hand-off of common.h (grid_last); its tickets for the largest grid
constexpr int RTH_TICKET_WORDS = (int)gl_ticket_words(RTF_GRID);
__device__ __forceinline__ bool rth_last(unsigned *tk, int *s_flag) { return grid_last(tk, s_flag); }

// The last workgroup: the exclusive scan of vals[0, gridDim.x) in place (agent-scope loads), each
// prefix clamped to clampv (rows at or past `cap` are never written); returns the total.
__device__ __forceinline__ uint64_t rth_scan_totals(uint32_t *vals, uint32_t clampv, uint64_t *s_w) {
  const int G = (int)gridDim.x, i0 = (int)threadIdx.x * RTH_SCAN_PT;
  uint32_t v[RTH_SCAN_PT];
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < RTH_SCAN_PT; k++) {
    v[k] = i0 + k < G ? __hip_atomic_load(vals + i0 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    sum += v[k];
  }
  uint64_t total;
  uint64_t ex = rth_scan64(sum, s_w, &total);
#pragma unroll
  for (int k = 0; k < RTH_SCAN_PT; k++) {
    if (i0 + k < G) vals[i0 + k] = (uint32_t)(ex < clampv ? ex : clampv);
    ex += v[k];
  }
  return total;
}

// count pass: hmask[i] = the hit (fixed mode: and kept) children of listed node i in index order;
// wsum[w] = their total over workgroup w's tiles.  root: level 0, the root's own test first (eager
// mode; in fixed mode pc == 0 marks a missed root).  Fixed mode: cwoff = the workgroups' exclusive
// candidate offsets.  The last workgroup scans wsum into the write pass's offsets; the total past
// cap sets result[1]; *next = min(total, cap) (the next list's count), at the last level result[0]
// = it; pcw_zero (fixed, not the last level): the next candidate totals, zeroed for the write pass.
__global__ void __launch_bounds__(RTH_TILE, RTH_MIN_WAVES) rth_count_kernel(RayIn in, const uint32_t *__restrict__ dnum,
                                                             const int2 *__restrict__ list, uint32_t level,
                                                             uint32_t target_level, int root, int with_depth,
                                                             int with_exit, uint8_t *__restrict__ hmask,
                                                             uint32_t *__restrict__ wsum, const uint32_t *__restrict__ pc,
                                                             const uint32_t *__restrict__ cwoff, uint32_t cap,
                                                             unsigned *__restrict__ ticket, uint32_t *__restrict__ next,
                                                             int64_t *__restrict__ result, int last,
                                                             uint32_t *__restrict__ pcw_zero) {
  __shared__ int s_wave[RTH_TILE / 64];
  __shared__ uint64_t s_w64[RTH_TILE / 64];
  __shared__ int s_flag;
  const int64_t num = *dnum;
  int64_t t0, t1;
  rth_span(num, t0, t1);
  uint32_t wt = 0;                                     // the workgroup's hit children
  uint32_t cb_run = cwoff ? cwoff[blockIdx.x] : 0u;    // (fixed) the candidate base of its next tile
  for (int64_t t = t0; t < t1; t++) {  // workgroup-uniform
    const int64_t i = t * RTH_TILE + threadIdx.x;
    const bool in_list = i < num;
    uint32_t cb = 0;
    if (cwoff) {  // the node's candidate base: the tile's base + the scan of pc within the tile
      int tot;
      cb = cb_run + (uint32_t)block_exclusive_scan(in_list ? (int)pc[i] : 0, s_wave, &tot);
      cb_run += (uint32_t)tot;
    }
    uint32_t m = 0;
    if (in_list && !(cwoff && pc[i] == 0)) {
      int ridx, pidx;
      rth_node(list, i, ridx, pidx);
      const float o[3] = {in.ro[ridx * 3], in.ro[ridx * 3 + 1], in.ro[ridx * 3 + 2]};
      const float d[3] = {in.rd[ridx * 3], in.rd[ridx * 3 + 1], in.rd[ridx * 3 + 2]};
      const float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f,
                            signbit(d[2]) ? 1.0f : -1.0f};
      const float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
      bool self = true;
      if (root && !cwoff) {  // the root's own test (rt_decide_one at level 0, not the target)
        const float vc[3] = {fmaf(1.0f, fmaf(2.0f, (float)in.points[0], 1.0f), -1.0f),
                             fmaf(1.0f, fmaf(2.0f, (float)in.points[1], 1.0f), -1.0f),
                             fmaf(1.0f, fmaf(2.0f, (float)in.points[2], 1.0f), -1.0f)};
        self = ray_aabb(o, d, inv, sgn, vc, 1.0f) != 0.0f;
      }
      if (self) {
        const uint32_t ob = in.octree[pidx];
        const int32_t s = in.exsum[pidx];
        const int nk = __popc(ob);
        const uint32_t lc = level + 1;
        const bool last = lc == target_level;
        const float r = (float)(1.0 / (double)(float)(1u << lc));
        uint32_t kept = 0xffu;  // (fixed mode: children whose candidate index is below cap)
        if (cwoff) {
          const uint32_t ranks = rth_fb_ranks(in, ridx, pidx, level, ob);
#pragma unroll
          for (int k = 0; k < 8; k++)
            if (cb + ((ranks >> (4 * k)) & 15u) >= cap) kept &= ~(1u << k);
        }
        int16_t cp[8][3];
#pragma unroll
        for (int k = 0; k < 8; k++) {  // children k = 0..nk-1 at points[s + 1 + k] (index order)
          const int64_t c = (int64_t)s + 1 + (k < nk ? k : 0);
          cp[k][0] = in.points[c * 3];
          cp[k][1] = in.points[c * 3 + 1];
          cp[k][2] = in.points[c * 3 + 2];
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if (k < nk) {
            const float vc[3] = {fmaf(r, fmaf(2.0f, (float)cp[k][0], 1.0f), -1.0f),
                                 fmaf(r, fmaf(2.0f, (float)cp[k][1], 1.0f), -1.0f),
                                 fmaf(r, fmaf(2.0f, (float)cp[k][2], 1.0f), -1.0f)};
            const float en = ray_aabb(o, d, inv, sgn, vc, r);
            bool hit;
            if (!last) {
              hit = en != 0.0f;
            } else if (with_depth && with_exit) {
              const float xs[3] = {signbit(-d[0]) ? 1.0f : -1.0f, signbit(-d[1]) ? 1.0f : -1.0f,
                                   signbit(-d[2]) ? 1.0f : -1.0f};
              hit = en > 0.0f && ray_aabb(o, d, inv, xs, vc, r) > 0.0f;
            } else {
              hit = en > 0.0f;
            }
            if (hit) m |= 1u << k;
          }
        }
        m &= kept;
      }
    }
    if (in_list) hmask[i] = (uint8_t)m;
    int tot;
    (void)block_exclusive_scan(__popc(m), s_wave, &tot);
    wt += (uint32_t)tot;
  }
  if (threadIdx.x == 0) __hip_atomic_store(wsum + blockIdx.x, wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (rth_last(ticket, &s_flag)) {
    const uint64_t total = rth_scan_totals(wsum, cap, s_w64);
    if (threadIdx.x == 0) {
      if (total > cap) result[1] = 1;
      const uint32_t c = total < cap ? (uint32_t)total : cap;
      *next = c;
      if (last) result[0] = c;
    }
    if (pcw_zero)
      for (int k = threadIdx.x; k < (int)gridDim.x; k += blockDim.x) pcw_zero[k] = 0u;
  }
}

// write pass: workgroup w's hit children from woff[w] on (its tiles' scans of the hit counts), in
// front-to-back order; at the target level with depths.  pc_out (fixed mode, not the last level):
// each listed child's own child count, and pcw (zeroed by the count pass) their totals per
// workgroup of the next list's partition -- summed in LDS for the RTH_PW workgroups from the
// first one this workgroup writes into, global atomics past them; the last workgroup scans pcw
// into the next count pass's candidate offsets (the candidate total past cap sets result[1]).
__global__ void __launch_bounds__(RTH_TILE) rth_write_kernel(RayIn in, const uint32_t *__restrict__ dnum,
                                                             const int2 *__restrict__ list, uint32_t level,
                                                             uint32_t target_level, int with_depth, int with_exit,
                                                             const uint8_t *__restrict__ hmask,
                                                             const uint32_t *__restrict__ woff, uint32_t cap,
                                                             int2 *__restrict__ nout, float *__restrict__ dout,
                                                             uint32_t *__restrict__ pc_out, uint32_t *__restrict__ pcw,
                                                             const uint32_t *__restrict__ dnext,
                                                             unsigned *__restrict__ ticket, int64_t *__restrict__ result) {
  __shared__ int s_wave[RTH_TILE / 64];
  __shared__ uint64_t s_w64[RTH_TILE / 64];
  __shared__ uint32_t s_pw[RTH_PW];
  __shared__ int s_flag;
  const int64_t num = *dnum;
  const int dd = with_exit ? 2 : 1;
  int64_t t0, t1;
  rth_span(num, t0, t1);
  uint32_t run = woff[blockIdx.x];
  int64_t nt2 = 1;   // (pcw) the next list's tiles
  uint32_t pw0 = 0;  // (pcw) the next list's workgroup of this workgroup's first row
  if (pcw) {
    nt2 = max((int64_t)1, ((int64_t)*dnext + RTH_TILE - 1) / RTH_TILE);
    pw0 = rth_owner(run / RTH_TILE, nt2);
    if (threadIdx.x < RTH_PW) s_pw[threadIdx.x] = 0u;  // (ordered by the scans' barriers / the one below)
  }
  for (int64_t t = t0; t < t1; t++) {  // workgroup-uniform
    const int64_t i = t * RTH_TILE + threadIdx.x;
    const uint32_t m = i < num ? hmask[i] : 0u;
    int tot;
    uint32_t base = run + (uint32_t)block_exclusive_scan(__popc(m), s_wave, &tot);
    run += (uint32_t)tot;
    if (m) {
      int ridx, pidx;
      rth_node(list, i, ridx, pidx);
      const uint32_t ob = in.octree[pidx];
      const int32_t s = in.exsum[pidx];
      const int16_t *p = in.points + (int64_t)pidx * 3;
      const float *org = in.ro + (int64_t)ridx * 3;
      const float scale = (float)(1.0 / (double)(float)(1u << level));
      const float x = (float)((double)(0.5f * org[0] + 0.5f) - (double)scale * ((double)(float)p[0] + 0.5));
      const float y = (float)((double)(0.5f * org[1] + 0.5f) - (double)scale * ((double)(float)p[1] + 0.5));
      const float z = (float)((double)(0.5f * org[2] + 0.5f) - (double)scale * ((double)(float)p[2] + 0.5));
      const uint32_t perm = c_rt_perm[(x > 0 ? 4u : 0u) + (y > 0 ? 2u : 0u) + (z > 0 ? 1u : 0u)];
      const uint32_t lc = level + 1;
      const bool depth_out = dout != nullptr && with_depth && lc == target_level;
      // (pcw) the next list's workgroup of row `base` and the row its successor starts at: one
      // division per node, then steps as `base` advances
      uint32_t ko = 0;
      int64_t knext = INT64_MAX;
      if (pcw && base < cap) {
        ko = rth_owner(base / RTH_TILE, nt2);
        knext = rth_tile0((int64_t)ko + 1, nt2) * RTH_TILE;
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {  // front to back: the code's permutation of the child indices
        const uint32_t j = (perm >> (4 * q)) & 15u;
        if (!(ob & (1u << j))) continue;
        const int c = __popc(ob & ((2u << j) - 1));  // 1..popc: the child's rank among the node's children
        if (!((m >> (c - 1)) & 1u)) continue;
        if (base < cap) {
          nout[base] = make_int2(ridx, s + c);
          if (pc_out) {
            const uint32_t pcv = (uint32_t)__popc(in.octree[s + c]);
            pc_out[base] = pcv;
            if (pcw) {
              while ((int64_t)base >= knext) knext = rth_tile0((int64_t)(++ko) + 1, nt2) * RTH_TILE;
              const uint32_t k = ko - pw0;
              if (k < (uint32_t)RTH_PW) atomicAdd(&s_pw[k], pcv);
              else atomicAdd(&pcw[pw0 + k], pcv);
            }
          }
          if (depth_out) {
            const int16_t *cp = in.points + (int64_t)(s + c) * 3;
            const float o[3] = {org[0], org[1], org[2]};
            const float d[3] = {in.rd[ridx * 3], in.rd[ridx * 3 + 1], in.rd[ridx * 3 + 2]};
            const float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f,
                                  signbit(d[2]) ? 1.0f : -1.0f};
            const float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
            const float r = (float)(1.0 / (double)(float)(1u << lc));
            const float vc[3] = {fmaf(r, fmaf(2.0f, (float)cp[0], 1.0f), -1.0f),
                                 fmaf(r, fmaf(2.0f, (float)cp[1], 1.0f), -1.0f),
                                 fmaf(r, fmaf(2.0f, (float)cp[2], 1.0f), -1.0f)};
            dout[(int64_t)base * dd] = ray_aabb(o, d, inv, sgn, vc, r);
            if (with_exit) {
              const float xs[3] = {signbit(-d[0]) ? 1.0f : -1.0f, signbit(-d[1]) ? 1.0f : -1.0f,
                                   signbit(-d[2]) ? 1.0f : -1.0f};
              dout[(int64_t)base * dd + 1] = ray_aabb(o, d, inv, xs, vc, r);
            }
          }
        }
        base++;
      }
    }
  }
  if (pcw) {  // workgroup-uniform
    __syncthreads();
    if (threadIdx.x < RTH_PW && s_pw[threadIdx.x]) atomicAdd(&pcw[pw0 + threadIdx.x], s_pw[threadIdx.x]);
    if (rth_last(ticket, &s_flag)) {
      const uint64_t total = rth_scan_totals(pcw, cap, s_w64);
      if (threadIdx.x == 0 && total > cap) result[1] = 1;
    }
  }
}

// fixed mode, after the march: the rows past the result's count -- nuggets -1, depths 0 (the rows
// below it are the march's own writes)
__global__ void rth_tail_fill_kernel(const int64_t *__restrict__ result, int64_t capacity, int2 *__restrict__ nuggets,
                                     float *__restrict__ depth, int dd) {
  const int64_t r0 = result[0];
  for (int64_t i = r0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < capacity;
       i += (int64_t)gridDim.x * blockDim.x) {
    nuggets[i] = make_int2(-1, -1);
    if (depth)
      for (int k = 0; k < dd; k++) depth[i * dd + k] = 0.0f;
  }
}

// fixed mode, level 0: each ray's candidate count at level 1 -- the root's children when the root
// is hit (rt_decide_one at level 0, not the target), else none -- their workgroup totals over the
// count pass's partition of the rays, scanned by the last workgroup (past cap: result[1])
__global__ void __launch_bounds__(RTH_TILE) rth_root_kernel(RayIn in, int64_t num_rays, uint32_t *__restrict__ pc,
                                                            uint32_t *__restrict__ pcw, uint32_t cap,
                                                            unsigned *__restrict__ ticket, int64_t *__restrict__ result) {
  __shared__ int s_wave[RTH_TILE / 64];
  __shared__ uint64_t s_w64[RTH_TILE / 64];
  __shared__ int s_flag;
  int64_t t0, t1;
  rth_span(num_rays, t0, t1);
  uint32_t wt = 0;
  for (int64_t t = t0; t < t1; t++) {
    const int64_t i = t * RTH_TILE + threadIdx.x;
    uint32_t v = 0;
    if (i < num_rays) {
      const float o[3] = {in.ro[i * 3], in.ro[i * 3 + 1], in.ro[i * 3 + 2]};
      const float d[3] = {in.rd[i * 3], in.rd[i * 3 + 1], in.rd[i * 3 + 2]};
      const float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f, signbit(d[2]) ? 1.0f : -1.0f};
      const float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
      const float vc[3] = {fmaf(1.0f, fmaf(2.0f, (float)in.points[0], 1.0f), -1.0f),
                           fmaf(1.0f, fmaf(2.0f, (float)in.points[1], 1.0f), -1.0f),
                           fmaf(1.0f, fmaf(2.0f, (float)in.points[2], 1.0f), -1.0f)};
      v = ray_aabb(o, d, inv, sgn, vc, 1.0f) != 0.0f ? (uint32_t)__popc(in.octree[0]) : 0u;
      pc[i] = v;
    }
    int tot;
    (void)block_exclusive_scan((int)v, s_wave, &tot);
    wt += (uint32_t)tot;
  }
  if (threadIdx.x == 0) __hip_atomic_store(pcw + blockIdx.x, wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (rth_last(ticket, &s_flag)) {
    const uint64_t total = rth_scan_totals(pcw, cap, s_w64);
    if (threadIdx.x == 0 && total > cap) result[1] = 1;
  }
}

// The levels of the hit-list march.  lists a / b (`cap` rows each), hm (cap bytes), tsA / tsB
// (>= the grid's workgroups each: the candidate / hit totals), dn[2] (the current / next list's
// count), tk (rth_last's tickets), result (rows, truncated) zeroed by the caller; list a holds level
// 0 (ray i at the root) and dn[0] = num_rays.  Fixed mode: pc (cap), cap = the capacity the
// candidates are truncated at.
struct RthBufs {
  int2 *a, *b;
  uint8_t *hm;
  uint32_t *tsA, *tsB, *dn, *pc;
  unsigned *tk;
  int64_t *result;
};
static unsigned rth_grid(int64_t cap, int64_t num_rays) {  // a power of two (rth_tile0)
  const int64_t want = std::min<int64_t>(cdiv(std::max(cap, num_rays), (int64_t)RTH_TILE), RTF_GRID);
  unsigned g = 1;
  while ((int64_t)g * 2 <= want) g *= 2;
  return g;
}
static int rth_levels(const RayIn &in, int64_t num_rays, uint32_t target_level, int return_depth, int with_exit,
                      int64_t cap, bool fixed, const RthBufs &bf, int2 *out, float *dout, hipStream_t st) {
  const unsigned g = rth_grid(cap, num_rays);
  unsigned *ticket = bf.tk;
  int2 *cur = bf.a, *nxt = bf.b;
  if (fixed) {
    hipLaunchKernelGGL(rth_root_kernel, dim3(g), dim3(RTH_TILE), 0, st, in, num_rays, bf.pc, bf.tsA, (uint32_t)cap,
                       ticket, bf.result);
    KL_CHECK_LAUNCH();
  }
  for (uint32_t l = 0; l < target_level; l++) {
    const int last = l + 1 == target_level;
    const uint32_t *dcur = bf.dn + (l & 1);
    uint32_t *dnext = bf.dn + ((l + 1) & 1);
    const bool pc_next = fixed && !last;
    hipLaunchKernelGGL(rth_count_kernel, dim3(g), dim3(RTH_TILE), 0, st, in, dcur, (const int2 *)cur, l, target_level,
                       (int)(l == 0), return_depth, with_exit, bf.hm, bf.tsB,
                       fixed ? (const uint32_t *)bf.pc : (const uint32_t *)nullptr,
                       fixed ? (const uint32_t *)bf.tsA : (const uint32_t *)nullptr, (uint32_t)cap, ticket, dnext,
                       bf.result, last, pc_next ? bf.tsA : (uint32_t *)nullptr);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(rth_write_kernel, dim3(g), dim3(RTH_TILE), 0, st, in, dcur, (const int2 *)cur, l, target_level,
                       return_depth, with_exit, (const uint8_t *)bf.hm, (const uint32_t *)bf.tsB, (uint32_t)cap,
                       last ? out : nxt, last ? dout : nullptr, pc_next ? bf.pc : (uint32_t *)nullptr,
                       pc_next ? bf.tsA : (uint32_t *)nullptr, (const uint32_t *)dnext, ticket, bf.result);
    KL_CHECK_LAUNCH();
    std::swap(cur, nxt);
  }
  return KL_OK;
}

__global__ void rth_init_kernel(int64_t n, int2 *__restrict__ list, uint32_t *__restrict__ dn,
                                int64_t *__restrict__ result, unsigned *__restrict__ tk) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < n) list[t] = make_int2((int)t, 0);
  if (tk)  // the hit-list passes' tickets (rth_last): all of them, whatever the grid of this launch
    for (int64_t k = t; k < RTH_TICKET_WORDS; k += (int64_t)gridDim.x * blockDim.x) tk[k] = 0u;
  if (t == 0) {
    dn[0] = (uint32_t)n;
    dn[1] = 0;
    result[0] = 0;
    result[1] = 0;
  }
}

// the eager march over the hit lists; returns 1 when some level outgrew `cap` (the caller falls back)
static int rt_hitlist(const RayIn &in, int64_t num_rays, uint32_t target_level, int return_depth, int with_exit,
                      Scratch &sc, int32_t **nuggets, float **depth, int64_t *num_hits, hipStream_t st) {
  if (target_level == 0 || num_rays == 0) return 1;  // (the per-level march: the root alone, or nothing)
  const int dd = with_exit ? 2 : 1;
  const int64_t cap = std::max<int64_t>(std::max<int64_t>(16 * num_rays, num_rays), 1 << 16);
  if (cap >= ((int64_t)1 << 31)) return 1;
  const int64_t ntiles = cdiv(cap, (int64_t)RTH_TILE);
  const size_t lb = al256b((size_t)cap * sizeof(int2)), mb = al256b((size_t)cap), tb = al256b((size_t)ntiles * 4);
  const size_t kb = (size_t)RTH_TICKET_WORDS * 4;
  char *w = (char *)sc.get(256 + 2 * lb + mb + tb + kb);
  // (r06) the two outputs from ONE allocation (each is a host callback into the caller's allocator
  // before the first launch, the GPU idle meanwhile): nuggets | depths
  const size_t ob = al256b((size_t)cap * sizeof(int2));
  char *ob_p = (char *)sc.get(ob + (return_depth ? (size_t)cap * dd * sizeof(float) : 0));
  int2 *out = (int2 *)ob_p;
  float *dout = return_depth && ob_p ? (float *)(ob_p + ob) : nullptr;
  if (!w || !out) return KL_E_ALLOC;
  RthBufs bf{};
  bf.dn = (uint32_t *)w;
  bf.result = (int64_t *)(w + 64);  // (rows, truncated)
  bf.a = (int2 *)(w + 256);
  bf.b = (int2 *)(w + 256 + lb);
  bf.hm = (uint8_t *)(w + 256 + 2 * lb);
  bf.tsB = (uint32_t *)(w + 256 + 2 * lb + mb);
  bf.tk = (unsigned *)(w + 256 + 2 * lb + mb + tb);
  hipLaunchKernelGGL(rth_init_kernel, dim3((unsigned)cdiv(num_rays, 256)), dim3(256), 0, st, num_rays, bf.a, bf.dn,
                     bf.result, bf.tk);
  KL_CHECK_LAUNCH();
  KL_CHECK_RC(rth_levels(in, num_rays, target_level, return_depth, with_exit, cap, false, bf, out, dout, st));
  int64_t h[2] = {0, 0};
  KL_CHECK_RC(host_read(h, bf.result, sizeof(h), st));
  if (h[1]) return 1;
  *nuggets = (int32_t *)out;
  *depth = dout;
  *num_hits = h[0];
  return KL_OK;
}

#if KL_DEV  // the fused march
// the fixed-capacity entry's result from the fused march: (rows, truncated)
__global__ void rt_fused_result_kernel(const RtlCtl *__restrict__ ctl, uint32_t target_level,
                                       int64_t *__restrict__ result) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    result[0] = ctl->dnum[target_level + 1];
    result[1] = ctl->truncated ? 1 : 0;
  }
}
#endif  // KL_DEV


#if KL_DEV  // the depth-first march (dev param 15 = 4): a measured dead end, DESIGN.md 3.5
// ---- Per-ray depth-first march (r05, the eager entry): the level march's output is ray-major, and
// within a ray each nugget's children follow it in front-to-back order, level by level -- which is
// exactly the order of a depth-first walk that visits a node's children front to back (every level's
// list restricted to one ray is that ray's walk order at that level, and a leaf's position is its
// rank in the walk).  So each lane walks its own ray through the octree with the same per-node
// decision (rt_decide_one's ray_aabb and keep rules, the same front-to-back child order as
// rt_children): no nugget lists in HBM, no per-level scans or host reads.  A hit node is expanded
// in two dependent loads: its point, octree byte and exsum, then ALL its children's points together,
// whose decisions are made at once -- the hit ones pushed (a per-level LDS stack of child offsets),
// or at the target level emitted.  Two passes: hits per ray (COUNT), then, after a scan over the
// rays, the same walk writing each hit at its ray's offset.
// Measured (cfg4, 512^2 rays, level 9): 1.22 ms against the per-level march's 1.20 -- each lane's
// walk is a chain of ~40 dependent load round trips (two per expanded node) and all 4,096 waves are
// resident at once, so the time is the longest chain, not the bytes.  A variant with each node's
// children's octree bytes / exsums loaded with their points (one round trip on the way down) and a
// slot buffer instead of the count pass measured 2.6 ms (102 VGPRs; rays past the 32 slots walked
// again).  Kept as dev param 15 = 4, tested equal to the other marches.
constexpr int RTD_THREADS = 64;
constexpr int RTD_MAXL = SPC_MAX_LEVELS + 1;


template <bool WRITE>
__global__ void __launch_bounds__(RTD_THREADS) rt_dfs_kernel(RayIn in, int64_t num_rays, uint32_t target_level,
                                                             int with_depth, int with_exit,
                                                             uint32_t *__restrict__ cnt,
                                                             const uint32_t *__restrict__ off,
                                                             int2 *__restrict__ nout, float *__restrict__ dout) {
  __shared__ uint32_t s_list[RTD_MAXL][RTD_THREADS];  // pending hit nodes of a level (offsets 1..8)
  __shared__ int32_t s_base[RTD_MAXL][RTD_THREADS];   // their parent's exsum
  const int64_t ridx = blockIdx.x * (int64_t)RTD_THREADS + threadIdx.x;
  if (ridx >= num_rays) return;
  const int tx = threadIdx.x;
  const float o[3] = {in.ro[ridx * 3], in.ro[ridx * 3 + 1], in.ro[ridx * 3 + 2]};
  const float d[3] = {in.rd[ridx * 3], in.rd[ridx * 3 + 1], in.rd[ridx * 3 + 2]};
  const float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f, signbit(d[2]) ? 1.0f : -1.0f};
  const float xs[3] = {signbit(-d[0]) ? 1.0f : -1.0f, signbit(-d[1]) ? 1.0f : -1.0f, signbit(-d[2]) ? 1.0f : -1.0f};
  const float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
  const float oh[3] = {0.5f * o[0] + 0.5f, 0.5f * o[1] + 0.5f, 0.5f * o[2] + 0.5f};
  const int dd = with_exit ? 2 : 1;
  uint32_t n = 0;
  uint32_t pos = WRITE ? off[ridx] : 0u;
  // a node's decision at level lv (rt_decide_one): keep flag at the target level, else dv != 0
  auto decide = [&](int16_t qx, int16_t qy, int16_t qz, uint32_t lv, float &en, float &ex) -> bool {
    const float r = (float)(1.0 / (double)(float)(1u << lv));
    const float vc[3] = {fmaf(r, fmaf(2.0f, (float)qx, 1.0f), -1.0f), fmaf(r, fmaf(2.0f, (float)qy, 1.0f), -1.0f),
                         fmaf(r, fmaf(2.0f, (float)qz, 1.0f), -1.0f)};
    en = ray_aabb(o, d, inv, sgn, vc, r);
    if (lv != target_level) return en != 0.0f;
    if (with_depth && with_exit) {
      ex = ray_aabb(o, d, inv, xs, vc, r);
      return en > 0.0f && ex > 0.0f;
    }
    return en > 0.0f;
  };
  auto emit = [&](int pidx, float en, float ex) {
    if (WRITE) {
      nout[pos] = make_int2((int)ridx, pidx);
      if (dout && with_depth) {
        dout[(int64_t)pos * dd] = en;
        if (with_exit) dout[(int64_t)pos * dd + 1] = ex;
      }
      pos++;
    } else {
      n++;
    }
  };
  {  // the root (level 0)
    float en, ex = 0.0f;
    const bool hit = decide(in.points[0], in.points[1], in.points[2], 0, en, ex);
    if (target_level == 0) {
      if (hit) emit(0, en, ex);
    } else if (hit) {
      int pidx = 0;
      uint32_t l = 0;
      for (;;) {
        // ---- expand hit node pidx of level l < target: its point, octree byte and exsum
        const int16_t *pp = in.points + (int64_t)pidx * 3;
        const float px = (float)pp[0], py = (float)pp[1], pz = (float)pp[2];
        const uint32_t ob = in.octree[pidx];
        const int32_t s = in.exsum[pidx];
        const float r = (float)(1.0 / (double)(float)(1u << l));
        const float x = (float)((double)oh[0] - (double)r * ((double)px + 0.5));
        const float y = (float)((double)oh[1] - (double)r * ((double)py + 0.5));
        const float z = (float)((double)oh[2] - (double)r * ((double)pz + 0.5));
        const uint32_t perm = c_rt_perm[(x > 0 ? 4u : 0u) + (y > 0 ? 2u : 0u) + (z > 0 ? 1u : 0u)];
        // the children in front-to-back order (offsets 1..8 from s) and all their points at once
        // (packed in nibbles: a register array indexed by a running count would live in scratch)
        uint32_t cl = 0;
        int nk = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t j = (perm >> (4 * q)) & 15u;
          if (ob & (1u << j)) {
            cl |= (uint32_t)__popc(ob & ((2u << j) - 1)) << (4 * nk);
            nk++;
          }
        }
        int16_t cp[8][3];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const int16_t *c = in.points + (int64_t)(k < nk ? s + (int)((cl >> (4 * k)) & 15u) : pidx) * 3;
          cp[k][0] = c[0];
          cp[k][1] = c[1];
          cp[k][2] = c[2];
        }
        const uint32_t lc = l + 1;
        uint32_t hits = 0;
        int nh = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if (k < nk) {
            const uint32_t ck = (cl >> (4 * k)) & 15u;
            float en, ex = 0.0f;
            if (decide(cp[k][0], cp[k][1], cp[k][2], lc, en, ex)) {
              if (lc == target_level) {
                emit(s + (int)ck, en, ex);
              } else {
                hits |= ck << (4 * nh);
                nh++;
              }
            }
          }
        }
        uint32_t m = l;  // the deepest level with pending nodes
        if (nh) {
          s_list[lc][tx] = hits;
          s_base[lc][tx] = s;
          m = lc;
        }
        while (m > 0 && s_list[m][tx] == 0u) m--;
        if (m == 0) break;
        const uint32_t lst = s_list[m][tx];
        s_list[m][tx] = lst >> 4;
        pidx = s_base[m][tx] + (int)(lst & 15u);
        l = m;
      }
    }
  }
  if (!WRITE) cnt[ridx] = n;
}

// host-sized raytrace by the depth-first march: counts, scan (one host read of the total), writes
static int rt_dfs(const RayIn &in, int64_t num_rays, uint32_t target_level, int return_depth, int with_exit,
                  Scratch &sc, int32_t **nuggets, float **depth, int64_t *num_hits, hipStream_t st) {
  const int dd = with_exit ? 2 : 1;
  const size_t cb = al256b((size_t)(num_rays + 1) * sizeof(uint32_t));
  uint32_t *cnt = (uint32_t *)sc.get(cb + (size_t)(num_rays + 2) * sizeof(uint32_t));
  if (!cnt) return KL_E_ALLOC;
  uint32_t *off = (uint32_t *)((char *)cnt + cb);
  KL_CHECK_RC(fill_async(cnt + num_rays, 0, sizeof(uint32_t), st));  // the scan's (n + 1)-th input
  const unsigned grid = (unsigned)cdiv(num_rays, RTD_THREADS);
  hipLaunchKernelGGL(rt_dfs_kernel<false>, dim3(grid), dim3(RTD_THREADS), 0, st, in, num_rays, target_level,
                     return_depth, with_exit, cnt, (const uint32_t *)nullptr, (int2 *)nullptr, (float *)nullptr);
  KL_CHECK_LAUNCH();
  uint32_t total = 0;
  KL_CHECK_RC(exclusive_scan(cnt, off, num_rays, sc, st, &total));
  int2 *out = (int2 *)sc.get((size_t)total * sizeof(int2));
  float *dout = return_depth ? (float *)sc.get(std::max<size_t>((size_t)total * dd * sizeof(float), 16)) : nullptr;
  if (!out || (return_depth && !dout)) return KL_E_ALLOC;
  if (total) {
    hipLaunchKernelGGL(rt_dfs_kernel<true>, dim3(grid), dim3(RTD_THREADS), 0, st, in, num_rays, target_level,
                       return_depth, with_exit, (uint32_t *)nullptr, (const uint32_t *)off, out, dout);
    KL_CHECK_LAUNCH();
  }
  *nuggets = (int32_t *)out;
  *depth = dout;
  *num_hits = total;
  return KL_OK;
}
#endif  // KL_DEV


template <typename S>
__global__ void pack_bounds_kernel(int64_t n, const S *__restrict__ ids, int32_t *__restrict__ out) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < n) out[t] = (t == 0 || ids[t - 1] != ids[t]) ? 1 : 0;
}

}  // namespace kl

using namespace kl;

extern "C" int kl_mesh_to_spc(int64_t num_faces, const float *fv, uint32_t level, kl_alloc_fn alloc, void *ctx,
                              uint8_t **octree, int64_t *num_nodes, int64_t **face_idx, float **bary,
                              int64_t *num_leaves, kl_stream stream) {
  KL_REQUIRE(level < (uint32_t)SPC_MAX_LEVELS, "mesh_to_spc: level must be < 15");
  KL_REQUIRE(alloc != nullptr, "mesh_to_spc: allocator required");
  Scratch sc{alloc, ctx};
  KL_DEV_STAT(0, 1);
  if (!(g_dev_flags & (1 << 10))) {  // dev bit 10: the per-level path
    const int rc = mesh_to_spc_nodes(num_faces, fv, level, sc, octree, num_nodes, face_idx, bary, num_leaves,
                                     S(stream));
    if (rc != 1) {
      KL_DEV_STAT(0, 0);
      return rc;
    }
  }
  return mesh_to_spc_impl(num_faces, fv, level, sc, octree, num_nodes, face_idx, bary, num_leaves, S(stream));
}

extern "C" size_t kl_mesh_to_spc_fixed_workspace_bytes(int64_t num_faces) {
  M2sNodes w;
  return num_faces >= 0 && w.plan(num_faces) ? w.total : 0;
}

extern "C" int kl_mesh_to_spc_fixed(int64_t num_faces, const float *fv, uint32_t level, int64_t node_capacity,
                                    int64_t leaf_capacity, uint8_t *octree, int64_t *face_idx, float *bary,
                                    int64_t *result, void *workspace, size_t workspace_bytes, kl_stream stream) {
  KL_REQUIRE(level >= 1 && level < (uint32_t)SPC_MAX_LEVELS, "mesh_to_spc: level must be in [1, 15) with a capacity");
  KL_REQUIRE(num_faces >= 0 && node_capacity >= 0 && leaf_capacity >= 0, "mesh_to_spc: negative size");
  M2sNodes w;
  KL_REQUIRE(w.plan(num_faces), "mesh_to_spc: too many faces for the fixed-capacity form");
  KL_REQUIRE(workspace != nullptr && workspace_bytes >= w.total, "mesh_to_spc: workspace too small");
  hipStream_t st = S(stream);
  w.place((char *)workspace);
  if (node_capacity) KL_CHECK_RC(fill_async(octree, 0, (size_t)node_capacity, st));
  if (leaf_capacity) {
    KL_CHECK_RC(fill_async(face_idx, 0xff, (size_t)leaf_capacity * 8, st));
    KL_CHECK_RC(fill_async(bary, 0, (size_t)leaf_capacity * 8, st));
  }
  KL_CHECK_RC(m2s_nodes_levels(num_faces, fv, level, w, st));
  const int b = (int)((level - 1) & 1);
  hipLaunchKernelGGL(m2s_fixed_final_kernel, dim3(1024), dim3(256), 0, st, w.ctl, level, w.arena, w.S[b], w.M[b],
                     w.fmin8(level), fv, node_capacity, leaf_capacity, octree, face_idx, bary, result);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

extern "C" int kl_mesh_to_spc_level_counts(int64_t *counts, int capacity) {
  const int n = t_m2s_levels < capacity ? t_m2s_levels : capacity;
  for (int i = 0; i < n; i++) counts[i] = t_m2s_counts[i];
  return t_m2s_levels;
}

extern "C" int kl_morton_to_octree(int64_t n, const uint64_t *morton, uint32_t level, kl_alloc_fn alloc, void *ctx,
                                   uint8_t **octree, int64_t *num_nodes, kl_stream stream) {
  KL_REQUIRE(alloc != nullptr, "morton_to_octree: allocator required");
  Scratch sc{alloc, ctx};
  return morton_to_octree_impl(n, morton, level, sc, octree, num_nodes, S(stream));
}

extern "C" int kl_scan_octrees(int batch, const uint8_t *octrees, const int32_t *lengths_host, int32_t *exsum,
                               int32_t *pyramid_host, int *level, kl_stream stream) {
  hipStream_t st = S(stream);
  const int STR = SPC_MAX_LEVELS + 2;
  int64_t maxlen = 0;
  for (int b = 0; b < batch; b++) maxlen = std::max<int64_t>(maxlen, lengths_host[b]);
  uint32_t *cnt = nullptr;
  int32_t *dpyr = nullptr;
  void *tmp = nullptr;
  size_t tb = 0;
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                (int)maxlen + 1, st));
  KL_CHECK_HIP(hipMallocAsync((void **)&cnt, (maxlen + 1) * sizeof(uint32_t), st));
  KL_CHECK_HIP(hipMallocAsync((void **)&dpyr, (size_t)batch * (2 * STR + 1) * sizeof(int32_t), st));
  KL_CHECK_HIP(hipMallocAsync(&tmp, tb > 0 ? tb : 16, st));
  int64_t off = 0;
  for (int b = 0; b < batch; b++) {
    const int64_t osize = lengths_host[b];
    hipLaunchKernelGGL(popc_kernel, dim3((unsigned)cdiv(osize + 1, 256)), dim3(256), 0, st, osize, octrees + off,
                       cnt);
    KL_CHECK_LAUNCH();
    // exsum segment b: [off + b, off + b + osize] = exclusive sum over osize+1 entries
    KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, (uint32_t *)(exsum + off + b), (int)osize + 1, st));
    hipLaunchKernelGGL(pyramid_kernel, dim3(1), dim3(64), 0, st, exsum + off + b, (uint32_t)osize,
                       dpyr + (size_t)b * (2 * STR + 1), dpyr + (size_t)b * (2 * STR + 1) + 2 * STR);
    KL_CHECK_LAUNCH();
    off += osize;
  }
  std::vector<int32_t> h((size_t)batch * (2 * STR + 1));
  KL_CHECK_HIP(hipMemcpyAsync(h.data(), dpyr, h.size() * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  KL_CHECK_HIP(hipStreamSynchronize(st));
  KL_CHECK_HIP(hipFreeAsync(cnt, st));
  KL_CHECK_HIP(hipFreeAsync(dpyr, st));
  KL_CHECK_HIP(hipFreeAsync(tmp, st));
  int lvl = 0;
  for (int b = 0; b < batch; b++) {
    for (int i = 0; i < 2 * STR; i++) pyramid_host[(size_t)b * 2 * STR + i] = h[(size_t)b * (2 * STR + 1) + i];
    lvl = h[(size_t)b * (2 * STR + 1) + 2 * STR];
  }
  *level = lvl;
  return KL_OK;
}

extern "C" int kl_generate_points(int batch, int max_level, const uint8_t *octrees, const int32_t *pyramids_host,
                                  const int32_t *exsum, int16_t *points, kl_stream stream) {
  hipStream_t st = S(stream);
  const int L = max_level;
  int64_t pmax = 1;
  for (int b = 0; b < batch; b++) pmax = std::max<int64_t>(pmax, pyramids_host[(size_t)b * 2 * (L + 2) + (L + 2) + L + 1]);
  uint64_t *mort = nullptr;
  KL_CHECK_HIP(hipMallocAsync((void **)&mort, pmax * sizeof(uint64_t), st));
  const uint8_t *oct = octrees;
  const int32_t *ex = exsum;
  int16_t *pts = points;
  for (int b = 0; b < batch; b++) {
    const int32_t *pyr = pyramids_host + (size_t)b * 2 * (L + 2);
    const int32_t *pyrsum = pyr + L + 2;
    const int32_t osize = pyrsum[L];
    const int32_t total = pyrsum[L + 1];
    KL_CHECK_RC(fill_async(mort, 0, sizeof(uint64_t), st));
    const uint8_t *co = oct;
    const int32_t *cs = ex + 1;
    const uint64_t *cm = mort;
    for (int l = 0; l < L; l++) {
      const int n = pyr[l];
      if (n > 0) {
        hipLaunchKernelGGL(nodes_to_morton_kernel, dim3((unsigned)cdiv(n, 64)), dim3(64), 0, st, co, cs, cm, mort, n);
        KL_CHECK_LAUNCH();
      }
      co += n;
      cs += n;
      cm += n;
    }
    if (total > 0) {
      hipLaunchKernelGGL(morton_to_points_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, mort, pts,
                         (int64_t)total);
      KL_CHECK_LAUNCH();
    }
    pts += (size_t)total * 3;
    oct += osize;
    ex += osize + 1;
  }
  KL_CHECK_HIP(hipFreeAsync(mort, st));
  return KL_OK;
}

extern "C" int kl_raytrace(const uint8_t *octree, int64_t octree_size, const int16_t *points, int64_t num_points,
                           const int32_t *exsum, int max_level, const float *ray_o, const float *ray_d,
                           int64_t num_rays, uint32_t target_level, int return_depth, int with_exit,
                           kl_alloc_fn alloc, void *ctx, int32_t **nuggets, float **depth, int64_t *num_hits,
                           kl_stream stream) {
  (void)octree_size;
  (void)num_points;
  (void)max_level;
  KL_REQUIRE(alloc != nullptr, "raytrace: allocator required");
  hipStream_t st = S(stream);
  Scratch sc{alloc, ctx};
  RayIn in{octree, points, exsum, ray_o, ray_d};
  const int dd = with_exit ? 2 : 1;
  // the fused march (rt_level_kernel), every level's count on the device and ONE host read at the
  // end, with buffers of 16 nuggets per ray; a level with more falls back to the per-level march
  // below (dev param 15 = 2: that march always, for A/B)
  KL_DEV_STAT(1, 0);
  // default: the hit-list march (rt_hitlist), falling back to the per-level march below when a level
  // outgrows its buffers.  Dev param 15 = 2: the per-level march; 4: the per-ray depth-first march
  // (rt_dfs); 3: the fused level march first (kept for A/B, tested equal: at cfg4 1.22 and 2.8 ms
  // against the per-level march's 1.20)
  if (g_dev_param[15] == 0 && num_rays < ((int64_t)1 << 31)) {
    const int rc = rt_hitlist(in, num_rays, target_level, return_depth, with_exit, sc, nuggets, depth, num_hits, st);
    if (rc <= 0) {
      KL_DEV_STAT(1, 4);
      return rc;
    }
    KL_DEV_STAT(1, 5);  // the lists outgrew their buffers: the per-level march below
  }
#if KL_DEV  // the depth-first and fused marches (A/B)
  if (num_rays > 0 && num_rays < ((int64_t)1 << 31) && g_dev_param[15] == 4 && target_level < (uint32_t)RTD_MAXL) {
    KL_DEV_STAT(1, 3);
    return rt_dfs(in, num_rays, target_level, return_depth, with_exit, sc, nuggets, depth, num_hits, st);
  }
  const int64_t fcap = std::max<int64_t>(16 * num_rays, 1 << 16);
  if (num_rays > 0 && fcap < ((int64_t)1 << 31) && g_dev_param[15] == 3) {
    const int64_t ntiles_max = cdiv(fcap, (int64_t)RTL_TILE);
    const size_t buf = al256b((size_t)fcap * sizeof(int2));
    char *w = (char *)sc.get(al256b(sizeof(RtlCtl)) + al256b((size_t)ntiles_max * 8) + 2 * buf);
    int2 *out = (int2 *)sc.get((size_t)fcap * sizeof(int2));
    float *dout = return_depth ? (float *)sc.get((size_t)fcap * dd * sizeof(float)) : nullptr;
    if (!w || !out || (return_depth && !dout)) return KL_E_ALLOC;
    RtlCtl *ctl = (RtlCtl *)w;
    unsigned long long *status = (unsigned long long *)(w + al256b(sizeof(RtlCtl)));
    int2 *b0 = (int2 *)(w + al256b(sizeof(RtlCtl)) + al256b((size_t)ntiles_max * 8)), *b1 = (int2 *)((char *)b0 + buf);
    KL_CHECK_RC(rt_fused_levels(in, num_rays, target_level, return_depth, with_exit, (uint32_t)fcap, ctl, status, b0,
                                b1, out, dout, st));
    RtlCtl h;
    KL_CHECK_RC(host_read(&h, ctl, sizeof(RtlCtl), st));
    KL_DEV_STAT(1, h.truncated ? 2 : 1);
    if (!h.truncated) {
      *nuggets = (int32_t *)out;
      *depth = dout;
      *num_hits = h.total[target_level + 1];
      return KL_OK;
    }
  }
#endif

  int64_t num = num_rays;
  int2 *n0 = (int2 *)sc.get(num * sizeof(int2));
  if (!n0) return KL_E_ALLOC;
  if (num > 0) {
    hipLaunchKernelGGL(rt_init_kernel, dim3((unsigned)cdiv(num, 256)), dim3(256), 0, st, num, n0, (uint32_t *)nullptr,
                       (int64_t *)nullptr);
    KL_CHECK_LAUNCH();
  }
  *depth = nullptr;
  for (uint32_t l = 0; l <= target_level; l++) {
    const int last = l == target_level;
    uint32_t *info = (uint32_t *)sc.get((num + 1) * sizeof(uint32_t));
    uint32_t *psum = (uint32_t *)sc.get((num + 2) * sizeof(uint32_t));
    float *d0 = nullptr;
    if (last && return_depth) d0 = (float *)sc.get(num * dd * sizeof(float));
    if (!info || !psum || (last && return_depth && !d0)) return KL_E_ALLOC;
    hipLaunchKernelGGL(rt_decide_kernel, dim3((unsigned)cdiv(num + 1, 256)), dim3(256), 0, st, in, num, n0, info, d0,
                       l, last, return_depth, with_exit);
    KL_CHECK_LAUNCH();
    uint32_t cnt = 0;
    int rc = exclusive_scan(info, psum, num, sc, st, &cnt);
    if (rc) return rc;
    int2 *n1 = (int2 *)sc.get((size_t)cnt * sizeof(int2));
    if (!n1) return KL_E_ALLOC;
    if (cnt == 0) {
      *nuggets = (int32_t *)n1;
      if (return_depth) *depth = (float *)sc.get(16);
      *num_hits = 0;
      return KL_OK;
    }
    if (!last) {
      hipLaunchKernelGGL(rt_subdivide_kernel, dim3((unsigned)cdiv(num, 256)), dim3(256), 0, st, in, num, n0, n1, info,
                         psum, l, (int64_t)INT64_MAX);
      KL_CHECK_LAUNCH();
    } else {
      float *d1 = nullptr;
      if (return_depth) {
        d1 = (float *)sc.get((size_t)cnt * dd * sizeof(float));
        if (!d1) return KL_E_ALLOC;
        *depth = d1;
      }
      hipLaunchKernelGGL(rt_compact_kernel, dim3((unsigned)cdiv(num, 256)), dim3(256), 0, st, num, n0, d0, n1, d1, dd,
                         info, psum, (int64_t)INT64_MAX);
      KL_CHECK_LAUNCH();
    }
    n0 = n1;
    num = cnt;
  }
  *nuggets = (int32_t *)n0;
  *num_hits = num;
  return KL_OK;
}

// Fixed-capacity raytrace: the same levels with every count kept on the device, so the call
// reads nothing back and can be captured into a graph.  Each level's nugget list lives in a
// workspace buffer of max(num_rays, capacity) rows; past `capacity` a level keeps its first
// `capacity` nuggets (a prefix of the full list) and result[1] is set.  Output rows past
// result[0] hold nugget (-1, -1) and depth 0.
namespace {
struct RtfWs {
  size_t a, b, info, psum, dtmp, dnum, tsum, hm, tsa, tsb, tk, total;
  int64_t cap0, ntiles;
};
RtfWs rtf_layout(int64_t num_rays, int64_t capacity, int with_exit) {
  RtfWs w{};
  w.cap0 = std::max<int64_t>(std::max<int64_t>(num_rays, capacity), 1);
  w.ntiles = cdiv(w.cap0, (int64_t)DSCAN_TILE);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  w.a = o; o += al(w.cap0 * sizeof(int2));
  w.b = o; o += al(w.cap0 * sizeof(int2));
  w.info = o; o += al((w.cap0 + 1) * 4);
  w.psum = o; o += al((w.cap0 + 2) * 4);
  w.dtmp = o; o += al(w.cap0 * (with_exit ? 2 : 1) * 4);
  w.dnum = o; o += 256;
  // the per-level scan's tile sums, or the fused march's tile status words (8 B per RTL_TILE rows)
  w.tsum = o; o += al(std::max<int64_t>(w.ntiles * 4, cdiv(w.cap0, (int64_t)RTL_TILE) * 8));
  // the hit-list march: child masks per listed node, the candidate / hit tile totals (pc, the listed
  // nodes' child counts, lives in dtmp)
  w.hm = o; o += al(w.cap0);
  w.tsa = o; o += al(cdiv(w.cap0, (int64_t)RTH_TILE) * 4);
  w.tsb = o; o += al(cdiv(w.cap0, (int64_t)RTH_TILE) * 4);
  w.tk = o; o += al((size_t)RTH_TICKET_WORDS * 4);  // the hit-list passes' tickets
  w.total = o;
  return w;
}
}  // namespace

extern "C" size_t kl_raytrace_fixed_workspace_bytes(int64_t num_rays, int64_t capacity, int with_exit) {
  return rtf_layout(num_rays, capacity, with_exit).total;
}

extern "C" int kl_raytrace_fixed(const uint8_t *octree, const int16_t *points, const int32_t *exsum,
                                 const float *ray_o, const float *ray_d, int64_t num_rays, uint32_t target_level,
                                 int return_depth, int with_exit, int64_t capacity, int32_t *nuggets, float *depth,
                                 int64_t *result, void *workspace, size_t workspace_bytes, kl_stream stream) {
  KL_REQUIRE(num_rays >= 0 && capacity >= 0, "raytrace: negative size");
  KL_REQUIRE(target_level < (uint32_t)SPC_MAX_LEVELS, "raytrace: level must be < 15");
  const RtfWs L = rtf_layout(num_rays, capacity, with_exit);
  KL_REQUIRE(L.cap0 < ((int64_t)1 << 28), "raytrace: num_rays and capacity must be < 2^28");
  KL_REQUIRE(workspace && workspace_bytes >= L.total, "raytrace: workspace too small");
  hipStream_t st = S(stream);
  const int dd = with_exit ? 2 : 1;
  uint8_t *w = (uint8_t *)workspace;
  int2 *n0 = (int2 *)(w + L.a), *n1 = (int2 *)(w + L.b);
  uint32_t *info = (uint32_t *)(w + L.info), *psum = (uint32_t *)(w + L.psum), *dnum = (uint32_t *)(w + L.dnum);
  float *d0 = return_depth ? (float *)(w + L.dtmp) : nullptr;
  // the hit-list march (default) fills the rows past its count afterwards (dev param 25 = 1: all rows
  // first, as the other marches do)
  const bool hitlist = g_dev_param[15] != 2 && g_dev_param[15] != 3 && target_level > 0 && num_rays > 0;
  const bool tail_fill = hitlist && g_dev_param[25] != 1;
  if (capacity > 0 && !tail_fill) {
    KL_CHECK_RC(fill_async(nuggets, 0xff, (size_t)capacity * 2 * 4, st));
    if (return_depth) KL_CHECK_RC(fill_async(depth, 0, (size_t)capacity * dd * 4, st));
  }
  RayIn in{octree, points, exsum, ray_o, ray_d};
  const int64_t cap0 = L.cap0;
#if KL_DEV  // the fused march (A/B)
  if (g_dev_param[15] == 3 && capacity > 0) {  // dev param 15 = 3: the fused march (2.2 against 1.09 ms at cfg4)
    RtlCtl *ctl = (RtlCtl *)dnum;
    static_assert(sizeof(RtlCtl) <= 256, "RtlCtl fits the dnum slot");
    KL_CHECK_RC(rt_fused_levels(in, num_rays, target_level, return_depth, with_exit, (uint32_t)capacity, ctl,
                                (unsigned long long *)(w + L.tsum), n0, n1, (int2 *)nuggets,
                                return_depth ? depth : nullptr, st));
    hipLaunchKernelGGL(rt_fused_result_kernel, dim3(1), dim3(64), 0, st, (const RtlCtl *)ctl, target_level, result);
    KL_CHECK_LAUNCH();
    return KL_OK;
  }
#endif

  // default: the hit-list march with the per-level march's truncation (rth_count_kernel's fixed
  // mode); dev param 15 = 2: the per-level march below
  if (hitlist && capacity > 0) {
    RthBufs bf{};
    bf.a = n0;
    bf.b = n1;
    bf.hm = (uint8_t *)(w + L.hm);
    bf.tsA = (uint32_t *)(w + L.tsa);
    bf.tsB = (uint32_t *)(w + L.tsb);
    bf.dn = dnum;
    bf.pc = (uint32_t *)(w + L.dtmp);
    bf.tk = (unsigned *)(w + L.tk);
    bf.result = result;
    hipLaunchKernelGGL(rth_init_kernel, dim3((unsigned)cdiv(num_rays, 256)), dim3(256), 0, st, num_rays, n0, dnum,
                       result, bf.tk);
    KL_CHECK_LAUNCH();
    KL_CHECK_RC(rth_levels(in, num_rays, target_level, return_depth, with_exit, capacity, true, bf, (int2 *)nuggets,
                           return_depth ? depth : nullptr, st));
    if (tail_fill) {
      hipLaunchKernelGGL(rth_tail_fill_kernel, dim3((unsigned)std::min<int64_t>(cdiv(capacity, 256), 2048)), dim3(256), 0,
                         st, (const int64_t *)result, capacity, (int2 *)nuggets, return_depth ? depth : nullptr, dd);
      KL_CHECK_LAUNCH();
    }
    return KL_OK;
  }
  hipLaunchKernelGGL(rt_init_kernel, dim3((unsigned)cdiv(std::max<int64_t>(num_rays, 1), 256)), dim3(256), 0, st,
                     num_rays, n0, dnum, result);
  KL_CHECK_LAUNCH();
  const unsigned g = (unsigned)std::min<int64_t>(cdiv(cap0, 256), RTF_GRID);
  const unsigned gt = (unsigned)L.ntiles;
  uint32_t *tsum = (uint32_t *)(w + L.tsum);
  for (uint32_t l = 0; l <= target_level; l++) {
    const int last = l == target_level;
    hipLaunchKernelGGL(rtf_decide_kernel, dim3(g), dim3(256), 0, st, in, (const uint32_t *)dnum, n0, info,
                       last ? d0 : nullptr, l, last, return_depth, with_exit);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(dscan_tile_sum_kernel, dim3(gt), dim3(256), 0, st, (const uint32_t *)info,
                       (const uint32_t *)dnum, tsum);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(dscan_tile_offset_kernel, dim3(1), dim3(1024), 0, st, tsum, (const uint32_t *)dnum, psum);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(dscan_apply_kernel, dim3(gt), dim3(256), 0, st, (const uint32_t *)info, (const uint32_t *)dnum,
                       (const uint32_t *)tsum, psum);
    KL_CHECK_LAUNCH();
    if (!last) {
      hipLaunchKernelGGL(rtf_subdivide_kernel, dim3(g), dim3(256), 0, st, in, (const uint32_t *)dnum, n0, n1, info,
                         psum, l, (int64_t)capacity);
    } else {
      hipLaunchKernelGGL(rtf_compact_kernel, dim3(g), dim3(256), 0, st, (const uint32_t *)dnum, n0, d0,
                         (int2 *)nuggets, return_depth ? depth : nullptr, dd, info, psum, (int64_t)capacity);
    }
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(rt_count_kernel, dim3(1), dim3(64), 0, st, psum, (uint32_t)capacity, dnum, result, last);
    KL_CHECK_LAUNCH();
    std::swap(n0, n1);
  }
  return KL_OK;
}

extern "C" int kl_points_to_morton(int64_t num_points, const int16_t *points, int64_t *morton, kl_stream stream) {
  KL_REQUIRE(num_points >= 0, "points_to_morton: negative size");
  if (num_points == 0) return KL_OK;
  hipLaunchKernelGGL(points_to_morton_kernel, dim3((unsigned)cdiv(num_points, 256)), dim3(256), 0, S(stream), points,
                     morton, num_points);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

extern "C" int kl_morton_to_points(int64_t num_points, const int64_t *morton, int16_t *points, kl_stream stream) {
  KL_REQUIRE(num_points >= 0, "morton_to_points: negative size");
  if (num_points == 0) return KL_OK;
  hipLaunchKernelGGL(morton_to_points_kernel, dim3((unsigned)cdiv(num_points, 256)), dim3(256), 0, S(stream),
                     (const uint64_t *)morton, points, num_points);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

extern "C" int kl_mark_pack_boundaries(kl_dtype dtype, int64_t num, const void *ids, int32_t *out, kl_stream stream) {
  if (num == 0) return KL_OK;
  const dim3 g((unsigned)cdiv(num, 256));
  switch (dtype) {
    case KL_I32:
      hipLaunchKernelGGL(pack_bounds_kernel<int32_t>, g, dim3(256), 0, S(stream), num, (const int32_t *)ids, out);
      break;
    case KL_I64:
      hipLaunchKernelGGL(pack_bounds_kernel<int64_t>, g, dim3(256), 0, S(stream), num, (const int64_t *)ids, out);
      break;
    case KL_I16:
      hipLaunchKernelGGL(pack_bounds_kernel<int16_t>, g, dim3(256), 0, S(stream), num, (const int16_t *)ids, out);
      break;
    case KL_I8:
      hipLaunchKernelGGL(pack_bounds_kernel<int8_t>, g, dim3(256), 0, S(stream), num, (const int8_t *)ids, out);
      break;
    case KL_U8:
      hipLaunchKernelGGL(pack_bounds_kernel<uint8_t>, g, dim3(256), 0, S(stream), num, (const uint8_t *)ids, out);
      break;
    default:
      set_error("mark_pack_boundaries: unsupported dtype");
      return KL_E_INVALID;
  }
  KL_CHECK_LAUNCH();
  return KL_OK;
}
