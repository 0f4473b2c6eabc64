// checksign.hip -- point-in-mesh test by ray-crossing parity.
//
// Reference: kaolin/ops/mesh/check_sign.py:25-154 (check_sign, _unbatched_check_sign_cuda) over
// mesh_intersection.cpp:33-68 (unbatched_mesh_intersection_cuda) and
// mesh_intersection_cuda.cu:40-233 (kernel and helpers).
//
// Per (point q, face p1 p2 p3): skip when q's (y, z) lies outside the face's (y, z) bbox (the
// bounds rounded to float, as the reference's `float y_min = min(...)`); the face separates q
// from q + (10, 0, 0) when the signed volumes of the two ends differ in sign; then q's (y, z)
// projection must be inside the projected triangle (three edge signed areas, each computed in
// a direction-independent way), and a projection on an edge or a vertex counts only for the
// face "below" it (mesh_intersection_cuda.cu:150-200), so that one crossing is one count.
// `contains` = odd count.  Every operation in the reference's order, no contraction: the
// counts are bit-identical.
//
// MI355X mapping: one lane per point, a register count per lane (the reference adds 1.0 with
// a global atomicAdd per crossing).
// * Batched entry (check_sign): the faces are binned into a G x G grid over the mesh's (y, z)
//   box (count, scan, fill), and each lane walks only its point's cell list.  Points are
//   visited in the Morton order of their (y, z) so that a wave's lanes share cells.  Face
//   corners are gathered from (vertices, faces) once, with check_sign's 1 / maxlen
//   normalisation applied on load (the IEEE division the reference does in torch).
// * Unbatched _C entry (unbatched_mesh_intersection_cuda): the same grid path on the given
//   corner arrays, writing the crossing counts.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace kl {

constexpr int kCsTile = 256;

template <typename T>
struct CsFaces {
  const T *v1, *v2, *v3;   // (F,3) corner arrays (unbatched _C entry), or
  const T *verts;          // (B,V,3) vertices with
  const int64_t *faces;    // (F,3) indices (batched entry)
  const T *maxlen;         // (B) divisor applied on load, or null
  int64_t V;
  int *bad;                // set to 1 when a face index is outside [0, V) (batched entry)
};

// mesh_intersection_cuda.cu:71-82 (signed_area on the (y, z) projection)
template <typename T>
__device__ __forceinline__ T cs_signed_area(T ax, T ay, T bx, T by, T cx, T cy) {
  if (cx > bx || (bx == cx && cy < by)) return -((by - cy) * (ax - cx) + (cx - bx) * (ay - cy));
  return (cy - by) * (ax - bx) + (bx - cx) * (ay - by);
}

// mesh_intersection_cuda.cu:84-98
template <typename T>
__device__ __forceinline__ bool cs_above(T vx, T vy, T lx, T ly, T rx, T ry) {
  const T v1x = rx - lx, v1y = ry - ly;
  const T v2x = vx - lx, v2y = vy - ly;
  return (v1x * v2y - v1y * v2x) > (T)0;
}

// mesh_intersection_cuda.cu:60-66: dot(cross(b - a, c - a), d - a)
template <typename T>
__device__ __forceinline__ T cs_signed_volume(T ax, T ay, T az, const T *b, const T *c, const T *d) {
  const T ux = b[0] - ax, uy = b[1] - ay, uz = b[2] - az;
  const T vx = c[0] - ax, vy = c[1] - ay, vz = c[2] - az;
  const T nx = uy * vz - uz * vy, ny = uz * vx - ux * vz, nz = ux * vy - uy * vx;
  return nx * (d[0] - ax) + ny * (d[1] - ay) + nz * (d[2] - az);
}

// one (point, face) pair: 1 when the ray from q crosses the face once (mesh_intersection_cuda.cu:120-205)
template <typename T>
__device__ __forceinline__ int cs_cross(T qx, T qy, T qz, const T *p1, const T *p2, const T *p3, const float *bb) {
  // bbox_check (:45-55): the bounds are float
  if (qy < (T)bb[0] || (T)bb[1] < qy || qz < (T)bb[2] || (T)bb[3] < qz) return 0;
  const bool c1 = cs_signed_volume(qx, qy, qz, p1, p2, p3) > (T)0;
  const bool c2 = cs_signed_volume(qx + (T)10., qy, qz, p1, p2, p3) > (T)0;
  if (c1 == c2) return 0;
  const T d1 = cs_signed_area(qy, qz, p1[1], p1[2], p2[1], p2[2]);
  const T d2 = cs_signed_area(qy, qz, p2[1], p2[2], p3[1], p3[2]);
  if (!(d1 * d2 >= (T)0)) return 0;
  const T d3 = cs_signed_area(qy, qz, p3[1], p3[2], p1[1], p1[2]);
  if (!(d3 * d1 >= (T)0 && d2 * d3 >= (T)0)) return 0;
  bool on_edge = false, on_vertex = false;
  T v1x = 0, v1y = 0, v2x = 0, v2y = 0, ox = 0, oy = 0;
  if (qy == p1[1] && qz == p1[2]) {
    on_vertex = true; v1x = p2[1]; v1y = p2[2]; v2x = p3[1]; v2y = p3[2];
  } else if (qy == p2[1] && qz == p2[2]) {
    on_vertex = true; v1x = p1[1]; v1y = p1[2]; v2x = p3[1]; v2y = p3[2];
  } else if (qy == p3[1] && qz == p3[2]) {
    on_vertex = true; v1x = p1[1]; v1y = p1[2]; v2x = p2[1]; v2y = p2[2];
  } else if (d1 == (T)0) {
    on_edge = true; v1x = p1[1]; v1y = p1[2]; v2x = p2[1]; v2y = p2[2]; ox = p3[1]; oy = p3[2];
  } else if (d2 == (T)0) {
    on_edge = true; v1x = p2[1]; v1y = p2[2]; v2x = p3[1]; v2y = p3[2]; ox = p1[1]; oy = p1[2];
  } else if (d3 == (T)0) {
    on_edge = true; v1x = p3[1]; v1y = p3[2]; v2x = p1[1]; v2y = p1[2]; ox = p2[1]; oy = p2[2];
  }
  if (!on_edge && !on_vertex) return 1;
  if (v1x > v2x || (v1x == v2x && v1y > v2y)) {
    T tx = v1x, ty = v1y;
    v1x = v2x; v1y = v2y; v2x = tx; v2y = ty;
  }
  if (on_edge) return cs_above(ox, oy, v1x, v1y, v2x, v2y) ? 0 : 1;
  // is_valid_overlap_vertice (:93-98)
  return (cs_above(qy, qz, v1x, v1y, v2x, v2y) && (v1x < qy) && (v2x >= qy)) ? 1 : 0;
}

template <typename T>
__device__ __forceinline__ void cs_load_face(const CsFaces<T> &src, int64_t b, int64_t f, T *v) {
  if (src.faces) {
    const T *vb = src.verts + b * src.V * 3;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      int64_t vi = src.faces[f * 3 + c];
      if (vi < 0 || vi >= src.V) {  // torch.index_select raises here (check_sign.py:29-31)
        *src.bad = 1;
        vi = 0;
      }
#pragma unroll
      for (int k = 0; k < 3; k++) v[c * 3 + k] = vb[vi * 3 + k];
    }
    if (src.maxlen) {
      const T m = src.maxlen[b];
#pragma unroll
      for (int k = 0; k < 9; k++) v[k] = v[k] / m;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      v[k] = src.v1[f * 3 + k];
      v[3 + k] = src.v2[f * 3 + k];
      v[6 + k] = src.v3[f * 3 + k];
    }
  }
}

// Float-bit order key of v (monotone), for the point ordering below.
__device__ __forceinline__ uint32_t cs_order_bits(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint32_t cs_spread16(uint32_t x) {
  x &= 0xffffu;
  x = (x | (x << 8)) & 0x00ff00ffu;
  x = (x | (x << 4)) & 0x0f0f0f0fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

// Sort keys: 2D Morton code of the top 16 order bits of (y, z), so that the 256 points of a
// workgroup share a small (y, z) box and the face culling below removes most of the mesh.
// The order only changes which lane tests which point; every count is unchanged.
template <typename T>
__global__ void __launch_bounds__(256)
    cs_key_kernel(int64_t n, int64_t P, const T *__restrict__ points, uint32_t *__restrict__ keys,
                  int32_t *__restrict__ vals) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t ky = cs_order_bits((float)points[i * 3 + 1]) >> 16;
  const uint32_t kz = cs_order_bits((float)points[i * 3 + 2]) >> 16;
  keys[i] = (cs_spread16(ky) << 1) | cs_spread16(kz);
  vals[i] = (int32_t)(i % P);  // point index within its mesh
}

// ---- batched entry: a (y, z) grid of face lists ------------------------------------------
// A ray toward +x can only cross faces whose (y, z) bounds hold the point, so the mesh's (y, z)
// box is cut into G x G cells and every face is listed in the cells its float bounds overlap.
// The cell of a value is a monotone function of it (the same float expression for faces and
// points), so every face that passes a point's bbox_check is in the point's cell list.  The
// counts do not depend on the order of a list.  Points outside the box cross nothing.

// Per face: normalised corners (9 x T) and float (y, z) bounds (4), written once; plus the
// per-tile union bounds (reduced to the mesh box below).
template <typename T>
__global__ void __launch_bounds__(kCsTile)
    cs_prep_kernel(int64_t F, CsFaces<T> src, T *__restrict__ fc, float *__restrict__ fb, float *__restrict__ tbox) {
  __shared__ float s_r[4][kCsTile / 64];
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.y, f = (int64_t)blockIdx.x * kCsTile + tid;
  float r0 = INFINITY, r1 = -INFINITY, r2 = INFINITY, r3 = -INFINITY;
  if (f < F) {
    T v[9];
    cs_load_face(src, b, f, v);
    const int64_t o = b * F + f;
#pragma unroll
    for (int k = 0; k < 9; k++) fc[o * 9 + k] = v[k];
    const float bb[4] = {(float)fmin(v[1], fmin(v[4], v[7])), (float)fmax(v[1], fmax(v[4], v[7])),
                         (float)fmin(v[2], fmin(v[5], v[8])), (float)fmax(v[2], fmax(v[5], v[8]))};
#pragma unroll
    for (int k = 0; k < 4; k++) fb[o * 4 + k] = bb[k];
    r0 = bb[0]; r1 = bb[1]; r2 = bb[2]; r3 = bb[3];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    r0 = fminf(r0, __shfl_xor(r0, o));
    r1 = fmaxf(r1, __shfl_xor(r1, o));
    r2 = fminf(r2, __shfl_xor(r2, o));
    r3 = fmaxf(r3, __shfl_xor(r3, o));
  }
  if ((tid & 63) == 0) {
    s_r[0][tid >> 6] = r0; s_r[1][tid >> 6] = r1; s_r[2][tid >> 6] = r2; s_r[3][tid >> 6] = r3;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kCsTile / 64; w++) {
      r0 = fminf(r0, s_r[0][w]); r1 = fmaxf(r1, s_r[1][w]); r2 = fminf(r2, s_r[2][w]); r3 = fmaxf(r3, s_r[3][w]);
    }
    float *o = tbox + (b * gridDim.x + blockIdx.x) * 4;
    o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3;
  }
}

// mesh box (y0, y1, z0, z1) and cell scales (G / extent, 0 for an empty or infinite extent);
// one workgroup per mesh
__global__ void __launch_bounds__(256)
    cs_meshbox_kernel(int64_t ntiles, int G, const float *__restrict__ tbox, float *__restrict__ mbox) {
  __shared__ float s_r[4][4];
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  float r0 = INFINITY, r1 = -INFINITY, r2 = INFINITY, r3 = -INFINITY;
  for (int64_t t = tid; t < ntiles; t += 256) {
    const float *tb = tbox + (b * ntiles + t) * 4;
    r0 = fminf(r0, tb[0]); r1 = fmaxf(r1, tb[1]); r2 = fminf(r2, tb[2]); r3 = fmaxf(r3, tb[3]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    r0 = fminf(r0, __shfl_xor(r0, o));
    r1 = fmaxf(r1, __shfl_xor(r1, o));
    r2 = fminf(r2, __shfl_xor(r2, o));
    r3 = fmaxf(r3, __shfl_xor(r3, o));
  }
  if ((tid & 63) == 0) {
    s_r[0][tid >> 6] = r0; s_r[1][tid >> 6] = r1; s_r[2][tid >> 6] = r2; s_r[3][tid >> 6] = r3;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; w++) {
      r0 = fminf(r0, s_r[0][w]); r1 = fmaxf(r1, s_r[1][w]); r2 = fminf(r2, s_r[2][w]); r3 = fmaxf(r3, s_r[3][w]);
    }
    const float ey = r1 - r0, ez = r3 - r2;
    float *o = mbox + b * 8;
    o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3;
    o[4] = (ey > 0.f && ey < INFINITY) ? (float)G / ey : 0.f;
    o[5] = (ez > 0.f && ez < INFINITY) ? (float)G / ez : 0.f;
  }
}

// monotone cell coordinate of v in [0, G)
__device__ __forceinline__ int cs_cell(float v, float v0, float inv, int G) {
  const float c = fminf(fmaxf((v - v0) * inv, 0.f), (float)(G - 1));
  return (int)c;
}

// fill == false: count the list entries of each cell, and their total in 64 bits (the int32
// scan below is used only when that total is < 2^31); fill == true: write them
template <bool FILL>
__global__ void __launch_bounds__(256)
    cs_bin_kernel(int64_t F, int G, const float *__restrict__ fb, const float *__restrict__ mbox,
                  int *__restrict__ cnt, const int *__restrict__ offs, int *__restrict__ list,
                  unsigned long long *__restrict__ total) {
  const int64_t b = blockIdx.y, f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int cy0 = 0, cy1 = -1, cz0 = 0, cz1 = -1;
  if (f < F) {
    const float *bb = fb + (b * F + f) * 4;
    const float y0 = bb[0], y1 = bb[1], z0 = bb[2], z1 = bb[3];
    if (y0 <= y1 && z0 <= z1) {  // NaN bounds never pass bbox_check
      const float *m = mbox + b * 8;
      cy0 = cs_cell(y0, m[0], m[4], G);
      cy1 = cs_cell(y1, m[0], m[4], G);
      cz0 = cs_cell(z0, m[2], m[5], G);
      cz1 = cs_cell(z1, m[2], m[5], G);
    }
  }
  if (!FILL) wave_add_u64(total, (unsigned long long)(cy1 - cy0 + 1) * (unsigned long long)(cz1 - cz0 + 1));
  int *c = cnt + b * (int64_t)G * G;
  for (int cz = cz0; cz <= cz1; cz++)
    for (int cy = cy0; cy <= cy1; cy++) {
      const int64_t cell = (int64_t)cz * G + cy;
      const int slot = atomicAdd(c + cell, 1);
      if (FILL) list[offs[b * (int64_t)G * G + cell] + slot] = (int)f;
    }
}

// one lane per point (Morton order through perm): walk the point's cell list
template <typename T>
__global__ void __launch_bounds__(256)
    cs_grid_check_kernel(int64_t P, int64_t F, int G, const T *__restrict__ points, const T *__restrict__ maxlen,
                         const int32_t *__restrict__ perm, const float *__restrict__ mbox, const int *__restrict__ cnt,
                         const int *__restrict__ offs, const int *__restrict__ list, const T *__restrict__ fc,
                         const float *__restrict__ fb, T *__restrict__ counts, uint8_t *__restrict__ contains) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= P) return;
  const int64_t p = perm ? (int64_t)perm[b * P + i] : i;
  const int64_t row = b * P + p;
  T qx = points[row * 3 + 0], qy = points[row * 3 + 1], qz = points[row * 3 + 2];
  if (maxlen) {
    const T m = maxlen[b];
    qx = qx / m; qy = qy / m; qz = qz / m;
  }
  const float *mb = mbox + b * 8;
  int count = 0;
  // outside the union of the face bounds (or NaN): no face passes bbox_check
  if (qy >= (T)mb[0] && qy <= (T)mb[1] && qz >= (T)mb[2] && qz <= (T)mb[3]) {
    const int cy = cs_cell((float)qy, mb[0], mb[4], G), cz = cs_cell((float)qz, mb[2], mb[5], G);
    const int64_t cell = b * (int64_t)G * G + (int64_t)cz * G + cy;
    const int n = cnt[cell], o = offs[cell];
    for (int k = 0; k < n; k++) {
      const int64_t f = b * F + list[o + k];
      const T *v = fc + f * 9;
      const T p1[3] = {v[0], v[1], v[2]}, p2[3] = {v[3], v[4], v[5]}, p3[3] = {v[6], v[7], v[8]};
      const float *bb = fb + f * 4;
      const float bbj[4] = {bb[0], bb[1], bb[2], bb[3]};
      count += cs_cross(qx, qy, qz, p1, p2, p3, bbj);
    }
  }
  if (counts) counts[row] = (T)count;
  if (contains) contains[row] = (uint8_t)(count & 1);
}

static int cs_grid_dim(int64_t F) {
  int G = 1;
  while (G < 1024 && (int64_t)G * G < F) G++;
  return G;
}

// workspace layout of the batched entry (byte offsets, 256-aligned); the face lists come from
// the allocator callback once their total is known
struct CsWs {
  size_t keys_in, keys_out, vals_in, vals_out, tbox, mbox, ctl, fc, fb, cnt, offs, temp, temp_bytes, total;
  int G;
};
static size_t cs_align(size_t x) { return (x + 255) & ~(size_t)255; }
static CsWs cs_ws_layout(int64_t B, int64_t F, int64_t P, size_t tsize) {
  CsWs w{};
  w.G = cs_grid_dim(F);
  const int64_t cells = B * (int64_t)w.G * w.G;
  size_t t1 = 0, t2 = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t1, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (const int32_t *)nullptr, (int32_t *)nullptr, (int)(P > 0 ? P : 1));
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (const int *)nullptr, (int *)nullptr, (int)cells);
  size_t o = 0;
  w.keys_in = o; o += cs_align((size_t)(B * P) * 4);
  w.keys_out = o; o += cs_align((size_t)(B * P) * 4);
  w.vals_in = o; o += cs_align((size_t)(B * P) * 4);
  w.vals_out = o; o += cs_align((size_t)(B * P) * 4);
  w.tbox = o; o += cs_align((size_t)(B * cdiv(F, kCsTile)) * 16);
  w.mbox = o; o += cs_align((size_t)B * 32);
  w.ctl = o; o += cs_align(16);  // u64 list total, int bad-index flag
  w.fc = o; o += cs_align((size_t)(B * F) * 9 * tsize);
  w.fb = o; o += cs_align((size_t)(B * F) * 16);
  w.cnt = o; o += cs_align((size_t)cells * 4);
  w.offs = o; o += cs_align((size_t)cells * 4);
  w.temp = o; w.temp_bytes = cs_align(t1 > t2 ? t1 : (t2 > 0 ? t2 : 1)); o += w.temp_bytes;
  w.total = o;
  return w;
}

// counts (B,P) in T (the _C contract) and/or contains (B,P) bool bytes
template <typename T>
static int check_sign_grid(int64_t B, int64_t F, int64_t P, const void *points, const CsFaces<T> &src,
                           const void *maxlen, void *counts, uint8_t *contains, void *ws, size_t ws_bytes,
                           kl_alloc_fn alloc, void *alloc_ctx, hipStream_t st) {
  if (B == 0 || P == 0) return KL_OK;
  if (F == 0) {
    if (counts) KL_CHECK_RC(fill_async(counts, 0, (size_t)(B * P) * sizeof(T), st));
    if (contains) KL_CHECK_RC(fill_async(contains, 0, (size_t)(B * P), st));
    return KL_OK;
  }
  const CsWs L = cs_ws_layout(B, F, P, sizeof(T));
  KL_REQUIRE(ws && ws_bytes >= L.total, "check_sign: workspace too small");
  KL_REQUIRE(alloc != nullptr, "check_sign: allocator callback required");
  int G = L.G;
  uint8_t *w = (uint8_t *)ws;
  uint32_t *kin = (uint32_t *)(w + L.keys_in), *kout = (uint32_t *)(w + L.keys_out);
  int32_t *vin = (int32_t *)(w + L.vals_in), *vout = (int32_t *)(w + L.vals_out);
  float *tbox = (float *)(w + L.tbox), *mbox = (float *)(w + L.mbox), *fb = (float *)(w + L.fb);
  T *fc = (T *)(w + L.fc);
  int *cnt = (int *)(w + L.cnt), *offs = (int *)(w + L.offs);
  unsigned long long *d_total = (unsigned long long *)(w + L.ctl);
  CsFaces<T> fsrc = src;
  fsrc.bad = (int *)(w + L.ctl + 8);
  const int64_t ntiles = cdiv(F, kCsTile);
  KL_CHECK_RC(fill_async(w + L.ctl, 0, 16, st));
  hipLaunchKernelGGL(cs_prep_kernel<T>, dim3((unsigned)ntiles, (unsigned)B), dim3(kCsTile), 0, st, F, fsrc, fc, fb,
                     tbox);
  KL_CHECK_LAUNCH();
  const dim3 fgrid((unsigned)cdiv(F, 256), (unsigned)B);
  // The list total is F * (cells per face); many large faces can take it past the int32 scan.
  // Then the grid is coarsened (G = 1 lists every face once: total <= F < 2^31).
  struct {
    unsigned long long total;
    int bad, pad;
  } ctl{};
  for (;;) {
    hipLaunchKernelGGL(cs_meshbox_kernel, dim3((unsigned)B), dim3(256), 0, st, ntiles, G, (const float *)tbox, mbox);
    KL_CHECK_LAUNCH();
    KL_CHECK_RC(fill_async(cnt, 0, (size_t)B * G * G * 4, st));
    hipLaunchKernelGGL(cs_bin_kernel<false>, fgrid, dim3(256), 0, st, F, G, (const float *)fb, (const float *)mbox,
                       cnt, (const int *)nullptr, (int *)nullptr, d_total);
    KL_CHECK_LAUNCH();
    KL_CHECK_HIP(hipMemcpyAsync(&ctl, d_total, 16, hipMemcpyDeviceToHost, st));
    KL_CHECK_HIP(hipStreamSynchronize(st));
    KL_REQUIRE(!ctl.bad, "check_sign: index out of range in self (a face index is outside [0, num_vertices))");
    // (dev flag 1 << 24: a 2^10 cap, so that tests reach the coarsening on small meshes)
    const unsigned long long cap = (g_dev_flags & (1 << 24)) ? (1ull << 10) : (1ull << 31);
    if (ctl.total < cap || G == 1) break;
    G = G / 2 > 1 ? G / 2 : 1;
    KL_CHECK_RC(fill_async(d_total, 0, 8, st));
  }
  const int64_t total = (int64_t)ctl.total;
  KL_REQUIRE(total < ((int64_t)1 << 31), "check_sign: face lists too long");
  const int64_t ncells = B * (int64_t)G * G;
  size_t tb = L.temp_bytes;
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(w + L.temp, tb, cnt, offs, (int)ncells, st));
  int *list = (int *)alloc(alloc_ctx, (size_t)(total > 0 ? total : 1) * 4);
  if (!list) {
    set_error("check_sign: allocator returned NULL");
    return KL_E_ALLOC;
  }
  KL_CHECK_RC(fill_async(cnt, 0, (size_t)ncells * 4, st));
  hipLaunchKernelGGL(cs_bin_kernel<true>, fgrid, dim3(256), 0, st, F, G, (const float *)fb, (const float *)mbox, cnt,
                     (const int *)offs, list, (unsigned long long *)nullptr);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL(cs_key_kernel<T>, dim3((unsigned)cdiv(B * P, 256)), dim3(256), 0, st, B * P, P,
                     (const T *)points, kin, vin);
  KL_CHECK_LAUNCH();
  for (int64_t b = 0; b < B; b++) {  // each mesh's points sorted on their own
    size_t ts = L.temp_bytes;
    KL_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(w + L.temp, ts, kin + b * P, kout + b * P, vin + b * P,
                                                    vout + b * P, (int)P, 0, 32, st));
  }
  hipLaunchKernelGGL(cs_grid_check_kernel<T>, dim3((unsigned)cdiv(P, 256), (unsigned)B), dim3(256), 0, st, P, F, G,
                     (const T *)points, (const T *)maxlen, (const int32_t *)vout, (const float *)mbox,
                     (const int *)cnt, (const int *)offs, (const int *)list, (const T *)fc, (const float *)fb,
                     (T *)counts, contains);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
static int mesh_intersection_unbatched(int64_t P, int64_t F, const void *points, const void *v1, const void *v2,
                                       const void *v3, void *counts, void *ws, size_t ws_bytes, kl_alloc_fn alloc,
                                       void *alloc_ctx, hipStream_t st) {
  CsFaces<T> src{(const T *)v1, (const T *)v2, (const T *)v3, nullptr, nullptr, nullptr, 0, nullptr};
  return check_sign_grid<T>(1, F, P, points, src, nullptr, counts, nullptr, ws, ws_bytes, alloc, alloc_ctx, st);
}

template <typename T>
static int check_sign_batched(int64_t B, int64_t V, int64_t F, int64_t P, const void *verts, const int64_t *faces,
                              const void *points, const void *maxlen, uint8_t *contains, void *ws, size_t ws_bytes,
                              kl_alloc_fn alloc, void *alloc_ctx, hipStream_t st) {
  CsFaces<T> src{nullptr, nullptr, nullptr, (const T *)verts, faces, (const T *)maxlen, V, nullptr};
  return check_sign_grid<T>(B, F, P, points, src, maxlen, nullptr, contains, ws, ws_bytes, alloc, alloc_ctx, st);
}

}  // namespace kl

using namespace kl;

#define KL_CS_DISPATCH(dtype, FN, ...)                          \
  switch (dtype) {                                              \
    case KL_F32: return FN<float>(__VA_ARGS__);                 \
    case KL_F64: return FN<double>(__VA_ARGS__);                \
    default: set_error("expected a Float or Double tensor");    \
      return KL_E_INVALID;                                      \
  }

extern "C" int kl_unbatched_mesh_intersection(kl_dtype dtype, int64_t num_points, int64_t num_faces, const void *points,
                                              const void *verts_1, const void *verts_2, const void *verts_3,
                                              void *result, void *workspace, size_t workspace_bytes,
                                              kl_alloc_fn alloc, void *alloc_ctx, kl_stream stream) {
  KL_REQUIRE(num_points >= 0 && num_faces >= 0, "unbatched_mesh_intersection: negative size");
  KL_REQUIRE(num_points < ((int64_t)1 << 31) && num_faces < ((int64_t)1 << 31),
             "unbatched_mesh_intersection: num_points and num_faces must be < 2^31");
  KL_CS_DISPATCH(dtype, mesh_intersection_unbatched, num_points, num_faces, points, verts_1, verts_2, verts_3, result,
                 workspace, workspace_bytes, alloc, alloc_ctx, S(stream));
}

extern "C" size_t kl_check_sign_workspace_bytes(kl_dtype dtype, int64_t batch_size, int64_t num_faces,
                                                int64_t num_points) {
  return cs_ws_layout(batch_size, num_faces, num_points, dtype == KL_F64 ? 8 : 4).total;
}

extern "C" int kl_check_sign(kl_dtype dtype, int64_t batch_size, int64_t num_vertices, int64_t num_faces,
                             int64_t num_points, const void *verts, const int64_t *faces, const void *points,
                             const void *maxlen, uint8_t *contains, void *workspace, size_t workspace_bytes,
                             kl_alloc_fn alloc, void *alloc_ctx, kl_stream stream) {
  KL_REQUIRE(batch_size >= 0 && num_vertices >= 0 && num_faces >= 0 && num_points >= 0, "check_sign: negative size");
  KL_REQUIRE(batch_size < 65536, "check_sign: batch_size must be < 65536");
  KL_REQUIRE(num_points < ((int64_t)1 << 31) && num_faces < ((int64_t)1 << 31),
             "check_sign: num_points and num_faces must be < 2^31");
  KL_CS_DISPATCH(dtype, check_sign_batched, batch_size, num_vertices, num_faces, num_points, verts, faces, points,
                 maxlen, contains, workspace, workspace_bytes, alloc, alloc_ctx, S(stream));
}
