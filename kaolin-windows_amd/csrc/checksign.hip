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

#ifndef KCS_STAGE
#define KCS_STAGE 16
#endif
#ifndef KCS_GROUP
#define KCS_GROUP 32
#endif

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

// ---- batched entry: a (y, z) grid of face lists ------------------------------------------
// A ray toward +x can only cross faces whose (y, z) bounds hold the point, so the mesh's (y, z)
// box is cut into G x G cells and every face is listed in the cells its float bounds overlap.
// The cell of a value is a monotone function of it (the same float expression for faces and
// points), so every face that passes a point's bbox_check is in the point's cell list.  The
// counts do not depend on the order of a list.  Points outside the box cross nothing.
//
// The lists hold the face records themselves (no index to chase), and the points are put in
// cell order by a counting sort over the same grid, so that the lanes of a wave walk the same
// list: every count is unchanged by either.

// Face record: float (y, z) bounds first (one 16-byte load), then the normalised corners.
template <typename T>
struct alignas(16) CsRec {
  float bb[4];
  T p[9];
};
// A point in cell order: normalised coordinates and its index within its mesh.
template <typename T>
struct alignas(16) CsPt {
  T q[3];
  int32_t p;
};

// Per face: the record, written once; plus the per-tile union bounds (reduced to the mesh box
// below).
template <typename T>
__global__ void __launch_bounds__(kCsTile)
    cs_prep_kernel(int64_t F, CsFaces<T> src, CsRec<T> *__restrict__ rec, float *__restrict__ tbox) {
  __shared__ float s_r[4][kCsTile / 64];
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.y, f = (int64_t)blockIdx.x * kCsTile + tid;
  float r0 = INFINITY, r1 = -INFINITY, r2 = INFINITY, r3 = -INFINITY;
  if (f < F) {
    CsRec<T> r;
    cs_load_face(src, b, f, r.p);
    const T *v = r.p;
    r.bb[0] = (float)fmin(v[1], fmin(v[4], v[7]));
    r.bb[1] = (float)fmax(v[1], fmax(v[4], v[7]));
    r.bb[2] = (float)fmin(v[2], fmin(v[5], v[8]));
    r.bb[3] = (float)fmax(v[2], fmax(v[5], v[8]));
    rec[b * F + f] = r;
    r0 = r.bb[0]; r1 = r.bb[1]; r2 = r.bb[2]; r3 = r.bb[3];
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

// fill == false: count the list entries of each cell, and their total in 64 bits (the grid is
// coarsened when it passes 2^31); fill == true: write the records.  A workgroup's faces are
// neighbours in a mesh, so their cells usually fit one LDS window: the entries are counted
// there and each touched cell takes one global atomic per workgroup (device atomics to
// scattered words run at ~20 per ns chip-wide, a few hundred thousand of them were the cost);
// a workgroup whose window is larger takes one global atomic per entry.
constexpr int kCsWin = 4096;
template <bool FILL, typename T>
__global__ void __launch_bounds__(256)
    cs_bin_kernel(int64_t F, int G, const CsRec<T> *__restrict__ rec, const float *__restrict__ mbox,
                  int *__restrict__ cnt, const int64_t *__restrict__ offs, CsRec<T> *__restrict__ list,
                  unsigned long long *__restrict__ total, const int *__restrict__ ovf) {
  __shared__ int s_c[kCsWin];
  __shared__ int s_r[4][4];
  if (FILL && ovf && *ovf) return;  // capturable entry: the lists did not fit (cs_brute_kernel answers)
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.y, f = (int64_t)blockIdx.x * 256 + tid;
  int cy0 = 0, cy1 = -1, cz0 = 0, cz1 = -1;
  CsRec<T> r;
  if (f < F) {
    const float4 bb = *reinterpret_cast<const float4 *>(rec[b * F + f].bb);
    if (FILL) r = rec[b * F + f];
    if (bb.x <= bb.y && bb.z <= bb.w) {  // NaN bounds never pass bbox_check
      const float *m = mbox + b * 8;
      cy0 = cs_cell(bb.x, m[0], m[4], G);
      cy1 = cs_cell(bb.y, m[0], m[4], G);
      cz0 = cs_cell(bb.z, m[2], m[5], G);
      cz1 = cs_cell(bb.w, m[2], m[5], G);
    }
  }
  __shared__ unsigned long long s_t[4];
  if (!FILL) block_add_u64(total, (unsigned long long)(cy1 - cy0 + 1) * (unsigned long long)(cz1 - cz0 + 1), s_t);
  // the workgroup's cell window
  const bool any = cy1 >= cy0;
  int w0 = any ? cy0 : INT_MAX, w1 = any ? cy1 : INT_MIN, w2 = any ? cz0 : INT_MAX, w3 = any ? cz1 : INT_MIN;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    w0 = min(w0, __shfl_xor(w0, o));
    w1 = max(w1, __shfl_xor(w1, o));
    w2 = min(w2, __shfl_xor(w2, o));
    w3 = max(w3, __shfl_xor(w3, o));
  }
  if ((tid & 63) == 0) {
    s_r[tid >> 6][0] = w0; s_r[tid >> 6][1] = w1; s_r[tid >> 6][2] = w2; s_r[tid >> 6][3] = w3;
  }
  __syncthreads();
  w0 = min(min(s_r[0][0], s_r[1][0]), min(s_r[2][0], s_r[3][0]));
  w1 = max(max(s_r[0][1], s_r[1][1]), max(s_r[2][1], s_r[3][1]));
  w2 = min(min(s_r[0][2], s_r[1][2]), min(s_r[2][2], s_r[3][2]));
  w3 = max(max(s_r[0][3], s_r[1][3]), max(s_r[2][3], s_r[3][3]));
  if (w1 < w0) return;  // no face of the workgroup is listed (uniform)
  const int64_t base = b * (int64_t)G * G;
  const int ww = w1 - w0 + 1;
  const int64_t area = (int64_t)ww * (w3 - w2 + 1);
  if (area > kCsWin) {
    for (int cz = cz0; cz <= cz1; cz++)
      for (int cy = cy0; cy <= cy1; cy++) {
        const int64_t cell = base + (int64_t)cz * G + cy;
        if (FILL) {
          const int slot = atomicAdd(cnt + cell, 1);
          list[offs[cell] + slot] = r;
        } else {
          atomicAdd(cnt + cell, 1);
        }
      }
    return;
  }
  const int na = (int)area;
  for (int i = tid; i < na; i += 256) s_c[i] = 0;
  __syncthreads();
  for (int cz = cz0; cz <= cz1; cz++)
    for (int cy = cy0; cy <= cy1; cy++) atomicAdd(s_c + (cz - w2) * ww + (cy - w0), 1);
  __syncthreads();
  for (int i = tid; i < na; i += 256) {
    const int c = s_c[i];
    if (!c) continue;
    const int64_t cell = base + (int64_t)(w2 + i / ww) * G + (w0 + i % ww);
    if (FILL)
      s_c[i] = atomicAdd(cnt + cell, c);  // the workgroup's first slot in the cell
    else
      atomicAdd(cnt + cell, c);
  }
  if (!FILL) return;
  __syncthreads();
  for (int cz = cz0; cz <= cz1; cz++)
    for (int cy = cy0; cy <= cy1; cy++) {
      const int slot = atomicAdd(s_c + (cz - w2) * ww + (cy - w0), 1);
      list[offs[base + (int64_t)cz * G + cy] + slot] = r;
    }
}

// a point's normalised coordinates (check_sign.py:146: points / maxlen)
template <typename T>
__device__ __forceinline__ void cs_load_point(const T *__restrict__ points, const T *__restrict__ maxlen, int64_t b,
                                              int64_t row, T *q) {
  q[0] = points[row * 3 + 0]; q[1] = points[row * 3 + 1]; q[2] = points[row * 3 + 2];
  if (maxlen) {
    const T m = maxlen[b];
    q[0] = q[0] / m; q[1] = q[1] / m; q[2] = q[2] / m;
  }
}

// inside the union of the face bounds (a point outside it, or NaN, passes no bbox_check)
template <typename T>
__device__ __forceinline__ bool cs_in_box(const T *q, const float *mb) {
  return q[1] >= (T)mb[0] && q[1] <= (T)mb[1] && q[2] >= (T)mb[2] && q[2] <= (T)mb[3];
}
template <typename T>
__device__ __forceinline__ int cs_point_cell(const T *q, const float *mb, int G) {
  return cs_cell((float)q[2], mb[2], mb[5], G) * G + cs_cell((float)q[1], mb[0], mb[4], G);
}

// Counting sort of the points by cell, pass 1: each in-box point takes a slot in its cell;
// the others are answered here (no crossing).
template <typename T>
__global__ void __launch_bounds__(256)
    cs_pcount_kernel(int64_t P, int G, const T *__restrict__ points, const T *__restrict__ maxlen,
                     const float *__restrict__ mbox, int *__restrict__ pcnt, int32_t *__restrict__ pslot,
                     T *__restrict__ counts, uint8_t *__restrict__ contains) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= P) return;
  const int64_t row = b * P + i;
  T q[3];
  cs_load_point(points, maxlen, b, row, q);
  const float *mb = mbox + b * 8;
  int slot = -1;
  if (cs_in_box(q, mb)) {
    slot = atomicAdd(pcnt + b * (int64_t)G * G + cs_point_cell(q, mb, G), 1);
  } else {
    if (counts) counts[row] = (T)0;
    if (contains) contains[row] = 0;
  }
  pslot[row] = slot;
}

// pass 2: the in-box points to their cell-ordered places.  poffs: per cell, the scan of the
// point counts (offset by poffs[0], the face list total that precedes them in the same scan).
template <typename T>
__global__ void __launch_bounds__(256)
    cs_pscatter_kernel(int64_t P, int G, const T *__restrict__ points, const T *__restrict__ maxlen,
                       const float *__restrict__ mbox, const int32_t *__restrict__ pslot,
                       const int64_t *__restrict__ poffs, CsPt<T> *__restrict__ sorted) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= P) return;
  const int64_t row = b * P + i;
  const int slot = pslot[row];
  if (slot < 0) return;
  CsPt<T> pt;
  cs_load_point(points, maxlen, b, row, pt.q);
  const int64_t cell = b * (int64_t)G * G + cs_point_cell(pt.q, mbox + b * 8, G);
  pt.p = (int32_t)i;
  sorted[poffs[cell] - poffs[0] + slot] = pt;
}

// (dev flag 1 << 25) one lane per point in input order: walk the point's cell list, eight
// records' bounds loaded together, the corners only of the faces whose bounds hold the point
template <typename T>
__global__ void __launch_bounds__(256)
    cs_grid_check_kernel(int64_t P, int G, const T *__restrict__ points, const T *__restrict__ maxlen,
                         const float *__restrict__ mbox, const int *__restrict__ cnt, const int64_t *__restrict__ offs,
                         const CsRec<T> *__restrict__ list, T *__restrict__ counts, uint8_t *__restrict__ contains) {
  const int64_t b = blockIdx.y, GG = (int64_t)G * G;
  const float *mb = mbox + b * 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const int64_t row = b * P + i;
  T q[3];
  cs_load_point(points, maxlen, b, row, q);
  int count = 0;
  if (cs_in_box(q, mb)) {
    const int64_t cell = b * GG + cs_point_cell(q, mb, G);
    const int n = cnt[cell];
    const CsRec<T> *L = list + offs[cell];
    const T qx = q[0], qy = q[1], qz = q[2];
    for (int k0 = 0; k0 < n; k0 += 8) {
      float4 bb[8];
#pragma unroll
      for (int u = 0; u < 8; u++)
        bb[u] = (k0 + u < n) ? *reinterpret_cast<const float4 *>(L[k0 + u].bb)
                             : make_float4(INFINITY, -INFINITY, INFINITY, -INFINITY);
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const float b4[4] = {bb[u].x, bb[u].y, bb[u].z, bb[u].w};
        if (qy < (T)b4[0] || (T)b4[1] < qy || qz < (T)b4[2] || (T)b4[3] < qz) continue;
        const T *v = L[k0 + u].p;
        const T p1[3] = {v[0], v[1], v[2]}, p2[3] = {v[3], v[4], v[5]}, p3[3] = {v[6], v[7], v[8]};
        count += cs_cross(qx, qy, qz, p1, p2, p3, b4);
      }
    }
  }
  if (counts) counts[row] = (T)count;
  if (contains) contains[row] = (uint8_t)(count & 1);
}

// Work units of the cell check: a cell with points takes one unit per kCsStage records of its
// list (at least one), so that no wave walks a long list alone (a few cells of the bench's
// sphere hold ~350 faces: walking them took half the check's time).  ucnt per cell, their
// total in ctl.  (KCS_STAGE / KCS_GROUP: compile-time overrides for A/B runs.)
constexpr int kCsStage = KCS_STAGE, kCsGroup = KCS_GROUP;  // records per unit, lanes per unit
__global__ void __launch_bounds__(256)
    cs_units_kernel(int64_t ncells, const int *__restrict__ cnt, int *__restrict__ ucnt,
                    unsigned long long *__restrict__ units) {
  __shared__ unsigned long long s_t[4];
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int u = 0;
  if (c < ncells) {
    u = cnt[ncells + c] > 0 ? max(1, (cnt[c] + kCsStage - 1) / kCsStage) : 0;
    ucnt[c] = u;
  }
  block_add_u64(units, (unsigned long long)u, s_t);
}
// unit -> cell (uoffs: the units' scan, offset by uoffs[0])
__global__ void __launch_bounds__(256)
    cs_unitmap_kernel(int64_t ncells, const int *__restrict__ ucnt, const int64_t *__restrict__ uoffs,
                      int64_t *__restrict__ unit_cell, const int *__restrict__ ovf) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= ncells || (ovf && *ovf)) return;
  const int u = ucnt[c];
  const int64_t o = uoffs[c] - uoffs[0];
  for (int s = 0; s < u; s++) unit_cell[o + s] = c;
}

// Two units per wave, 32 lanes each: the unit's cell's points (cell order, 32 a pass) against
// the unit's <= 16 records, staged through LDS with coalesced loads; the lanes of a unit then
// read the same record (an LDS broadcast).  The kernel is VALU-bound (counters: ~1000 VALU
// instructions per 64-lane wave at 64-record units, ~27 % of lanes busy since a cell holds
// ~17 points), so lanes are what to save: 64-record units one per wave took 112 us, two per
// wave (twice the LDS per wave, half the occupancy) 113, 32-record units two per wave 85,
// 16-record units two per wave 75.
// Per-lane gathers of records, or scalar loads of them, measured 1.1-1.8x slower.  A one-unit
// cell writes its points' answers; the units of a longer list add their counts into acc,
// answered by cs_finalize_kernel.
__device__ __forceinline__ void cs_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <typename T>
__global__ void __launch_bounds__(256)
    cs_cell_check_kernel(int64_t nunits, int64_t P, int64_t GG, const int64_t *__restrict__ unit_cell,
                         const int64_t *__restrict__ uoffs, const int *__restrict__ ucnt,
                         const int64_t *__restrict__ poffs, const CsPt<T> *__restrict__ sorted,
                         const int *__restrict__ cnt, const int64_t *__restrict__ offs,
                         const CsRec<T> *__restrict__ list, int *__restrict__ acc, T *__restrict__ counts,
                         uint8_t *__restrict__ contains, const unsigned long long *__restrict__ dunits,
                         const int *__restrict__ ovf) {
  constexpr int NG = 256 / kCsGroup;
  // capturable entry: the grid covers the workspace's unit room, the unit count is on the device
  if (ovf) {
    if (*ovf) return;
    nunits = (int64_t)*dunits;
  }
  __shared__ CsRec<T> s_rec[NG][kCsStage];
  const int g = threadIdx.x / kCsGroup, gl = threadIdx.x % kCsGroup;
  const int64_t u = (int64_t)blockIdx.x * NG + g;
  int64_t np = 0, s0 = 0, b = 0, c = 0;
  int m = 0;
  bool whole = true;
  CsRec<T> *S = s_rec[g];
  if (u < nunits) {
    c = unit_cell[u];
    const int seg = (int)(u - (uoffs[c] - uoffs[0]));
    whole = ucnt[c] == 1;
    np = poffs[c + 1] - poffs[c];
    s0 = poffs[c] - poffs[0];
    b = c / GG;
    const int k0 = seg * kCsStage;
    m = min(kCsStage, cnt[c] - k0);
    const CsRec<T> *L = list + offs[c] + k0;
    for (int v = gl; v < m; v += kCsGroup) S[v] = L[v];
  }
  cs_wave_sync();
  for (int64_t p0 = 0; p0 < np; p0 += kCsGroup) {
    const bool act = p0 + gl < np;
    T qx = (T)INFINITY, qy = (T)INFINITY, qz = (T)INFINITY;  // an idle lane passes no bbox_check
    int32_t p = 0;
    if (act) {
      const CsPt<T> pt = sorted[s0 + p0 + gl];
      qx = pt.q[0]; qy = pt.q[1]; qz = pt.q[2];
      p = pt.p;
    }
    int count = 0;
    for (int j = 0; j < m; j++) {
      const CsRec<T> r = S[j];
      count += cs_cross(qx, qy, qz, r.p, r.p + 3, r.p + 6, r.bb);
    }
    if (act) {
      const int64_t row = b * P + p;
      if (whole) {
        if (counts) counts[row] = (T)count;
        if (contains) contains[row] = (uint8_t)(count & 1);
      } else if (count) {
        atomicAdd(acc + row, count);
      }
    }
  }
}

// the answers of the points of multi-unit cells (one lane per in-box point, cell order)
template <typename T>
__global__ void __launch_bounds__(256)
    cs_finalize_kernel(int64_t P, int G, const int64_t *__restrict__ poffs, const CsPt<T> *__restrict__ sorted,
                       const float *__restrict__ mbox, const int *__restrict__ ucnt, const int *__restrict__ acc,
                       T *__restrict__ counts, uint8_t *__restrict__ contains, const int *__restrict__ ovf) {
  if (ovf && *ovf) return;
  const int64_t b = blockIdx.y, GG = (int64_t)G * G;
  const int64_t s0 = poffs[b * GG] - poffs[0], s1 = poffs[(b + 1) * GG] - poffs[0];
  const int64_t j = s0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= s1) return;
  const CsPt<T> pt = sorted[j];
  if (ucnt[b * GG + cs_point_cell(pt.q, mbox + b * 8, G)] <= 1) return;
  const int64_t row = b * P + pt.p;
  const int count = acc[row];
  if (counts) counts[row] = (T)count;
  if (contains) contains[row] = (uint8_t)(count & 1);
}

// Capturable entry (no allocator): the face lists and the unit map must fit the workspace's
// fixed room, known only on the device.  ovf = 1 when they do not; the list kernels then exit and
// cs_brute_kernel answers every point against every face record instead -- the same cs_cross
// tests over a superset of each point's cell list, so the same counts, at O(P F) cost.
__global__ void cs_capacity_kernel(unsigned long long *__restrict__ ctl, unsigned long long list_cap,
                                   unsigned long long unit_cap) {
  if (threadIdx.x == 0) ((int *)(ctl + 2))[1] = (ctl[0] > list_cap || ctl[1] > unit_cap) ? 1 : 0;
}
template <typename T>
__global__ void __launch_bounds__(256)
    cs_brute_kernel(int64_t P, int64_t F, const T *__restrict__ points, const T *__restrict__ maxlen,
                    const CsRec<T> *__restrict__ rec, T *__restrict__ counts, uint8_t *__restrict__ contains,
                    const int *__restrict__ ovf) {
  if (!*ovf) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= P) return;
  const int64_t row = b * P + i;
  T q[3];
  cs_load_point(points, maxlen, b, row, q);
  int count = 0;
  for (int64_t f = 0; f < F; f++) {
    const CsRec<T> &r = rec[b * F + f];
    count += cs_cross(q[0], q[1], q[2], r.p, r.p + 3, r.p + 6, r.bb);
  }
  if (counts) counts[row] = (T)count;
  if (contains) contains[row] = (uint8_t)(count & 1);
}

static int cs_grid_dim(int64_t F) {
  int G = 1;
  while (G < 1024 && (int64_t)G * G < F) G++;
  return G;
}

struct CsToI64 {
  __host__ __device__ int64_t operator()(int v) const { return (int64_t)v; }
};
using CsCountIt = hipcub::TransformInputIterator<int64_t, CsToI64, const int *>;

// workspace layout of the batched entry (byte offsets, 256-aligned); the face lists come from
// the allocator callback once their total is known.  cnt / offs: [face counts per cell |
// point counts per cell | check units per cell | 0] and their exclusive scan in 64 bits.
struct CsWs {
  size_t pslot, acc, sorted, tbox, mbox, ctl, rec, cnt, offs, macc, morg, mlen, temp, temp_bytes, list, list_cap, total;
  int G;
};
static size_t cs_align(size_t x) { return (x + 255) & ~(size_t)255; }
static CsWs cs_ws_layout(int64_t B, int64_t F, int64_t P, size_t tsize) {
  CsWs w{};
  w.G = cs_grid_dim(F);
  const int64_t cells = B * (int64_t)w.G * w.G;
  size_t t1 = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t1, CsCountIt((const int *)nullptr, CsToI64()), (int64_t *)nullptr,
                                         (int)(3 * cells + 1));
  const size_t psz = tsize == 8 ? sizeof(CsPt<double>) : sizeof(CsPt<float>);
  const size_t rsz = tsize == 8 ? sizeof(CsRec<double>) : sizeof(CsRec<float>);
  size_t o = 0;
  w.pslot = o; o += cs_align((size_t)(B * P) * 4);
  w.acc = o; o += cs_align((size_t)(B * P) * 4);
  w.sorted = o; o += cs_align((size_t)(B * P) * psz);
  w.tbox = o; o += cs_align((size_t)(B * cdiv(F, kCsTile)) * 16);
  w.mbox = o; o += cs_align((size_t)B * 32);
  w.ctl = o; o += cs_align(32);  // u64 list total, u64 check units, int bad-index flag
  w.rec = o; o += cs_align((size_t)(B * F) * rsz);
  w.cnt = o; o += cs_align((size_t)(3 * cells + 1) * 4);
  w.offs = o; o += cs_align((size_t)(3 * cells + 1) * 8);
  w.macc = o; o += cs_align((size_t)B * 9 * 8);  // maxlen from the vertices (kl_voxelgrid_bounds)
  w.morg = o; o += cs_align((size_t)B * 3 * tsize);
  w.mlen = o; o += cs_align((size_t)B * tsize);
  w.temp = o; w.temp_bytes = cs_align(t1 > 0 ? t1 : 1); o += w.temp_bytes;
  // room for 16 list entries per face (up to 256 MiB) and a unit per cell, so that a typical
  // mesh's lists need no allocator call (a host round trip); longer lists come from the callback
  w.list = o; w.list_cap = std::min<size_t>((size_t)(16 * B * F), ((size_t)256 << 20) / rsz); o += w.list_cap * rsz;
  o += cs_align((size_t)(2 * cells) * 8);
  w.total = o;
  return w;
}

struct CsCtl {
  unsigned long long total, units;
  int bad, pad;
};
// pinned, so that the list-total read is one small DMA (one per host thread)
static CsCtl *cs_host_ctl() {
  thread_local CsCtl *p = nullptr;
  thread_local bool tried = false;
  if (!tried) {
    tried = true;
    if (hipHostMalloc((void **)&p, sizeof(CsCtl), hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
    }
  }
  return p;
}

// counts (B,P) in T (the _C contract) and/or contains (B,P) bool bytes.  The batched entry with
// maxlen == null takes check_sign.py:140-146's maxlen from the vertices on the device.
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
  // alloc == null: the capturable entry -- no host round trip (fixed room in the workspace,
  // cs_brute_kernel past it; a bad face index is clamped, not reported)
  const bool capturable = alloc == nullptr;
  int G = L.G;
  uint8_t *w = (uint8_t *)ws;
  int32_t *pslot = (int32_t *)(w + L.pslot);
  CsPt<T> *sorted = (CsPt<T> *)(w + L.sorted);
  float *tbox = (float *)(w + L.tbox), *mbox = (float *)(w + L.mbox);
  CsRec<T> *rec = (CsRec<T> *)(w + L.rec);
  int *cnt = (int *)(w + L.cnt);
  int64_t *offs = (int64_t *)(w + L.offs);
  unsigned long long *d_total = (unsigned long long *)(w + L.ctl);
  CsFaces<T> fsrc = src;
  fsrc.bad = (int *)(w + L.ctl + 16);
  int *acc = (int *)(w + L.acc);
  int *d_ovf = (int *)(w + L.ctl + 20);
  const T *ml = (const T *)maxlen;
  if (src.faces && !maxlen) {
    KL_REQUIRE(src.V > 0, "check_sign: verts has no vertices");
    T *mlen = (T *)(w + L.mlen);
    KL_CHECK_RC(kl_voxelgrid_bounds(sizeof(T) == 8 ? KL_F64 : KL_F32, (int)B, src.V, src.verts, w + L.morg, mlen,
                                    w + L.macc, (size_t)B * 9 * 8, (kl_stream)st));
    ml = mlen;
  }
  if (src.faces) fsrc.maxlen = ml;
  const int64_t ntiles = cdiv(F, kCsTile);
  // (dev flag 1 << 25: points in input order, no counting sort)
  const bool sort_points = capturable || !(g_dev_flags & (1 << 25));
  KL_CHECK_RC(fill_async(w + L.ctl, 0, 32, st));
  hipLaunchKernelGGL(cs_prep_kernel<T>, dim3((unsigned)ntiles, (unsigned)B), dim3(kCsTile), 0, st, F, fsrc, rec,
                     tbox);
  KL_CHECK_LAUNCH();
  const dim3 fgrid((unsigned)cdiv(F, 256), (unsigned)B), pgrid((unsigned)cdiv(P, 256), (unsigned)B);
  // The list total is F * (cells per face); many large faces can take it past 2^31 entries.
  // Then the grid is coarsened (G = 1 lists every face once: total <= F < 2^31).
  CsCtl local{}, *ctl = cs_host_ctl();
  if (!ctl) ctl = &local;
  for (;;) {
    const int64_t ncells = B * (int64_t)G * G;
    hipLaunchKernelGGL(cs_meshbox_kernel, dim3((unsigned)B), dim3(256), 0, st, ntiles, G, (const float *)tbox, mbox);
    KL_CHECK_LAUNCH();
    KL_CHECK_RC(fill_async(cnt, 0, (size_t)(3 * ncells + 1) * 4, st));
    hipLaunchKernelGGL((cs_bin_kernel<false, T>), fgrid, dim3(256), 0, st, F, G, (const CsRec<T> *)rec,
                       (const float *)mbox, cnt, (const int64_t *)nullptr, (CsRec<T> *)nullptr, d_total,
                       (const int *)nullptr);
    KL_CHECK_LAUNCH();
    if (sort_points) {
      hipLaunchKernelGGL(cs_pcount_kernel<T>, pgrid, dim3(256), 0, st, P, G, (const T *)points, ml,
                         (const float *)mbox, cnt + ncells, pslot, (T *)counts, contains);
      KL_CHECK_LAUNCH();
    }
    if (sort_points) {
      hipLaunchKernelGGL(cs_units_kernel, dim3((unsigned)cdiv(ncells, 256)), dim3(256), 0, st, ncells,
                         (const int *)cnt, cnt + 2 * ncells, d_total + 1);
      KL_CHECK_LAUNCH();
    }
    if (capturable) break;
    KL_CHECK_HIP(hipMemcpyAsync(ctl, d_total, sizeof(CsCtl), hipMemcpyDeviceToHost, st));
    KL_CHECK_HIP(hipStreamSynchronize(st));
    KL_REQUIRE(!ctl->bad, "check_sign: index out of range in self (a face index is outside [0, num_vertices))");
    // (dev flag 1 << 24: a 2^10 cap, so that tests reach the coarsening on small meshes)
    const unsigned long long cap = (g_dev_flags & (1 << 24)) ? (1ull << 10) : (1ull << 31);
    if (ctl->total < cap || G == 1) break;
    G = G / 2 > 1 ? G / 2 : 1;
    KL_CHECK_RC(fill_async(d_total, 0, 16, st));
  }
  const int64_t ncells = B * (int64_t)G * G;
  const int64_t unit_room = 2 * ncells;
  if (capturable) {
    // (dev flag 1 << 26: no list room, so that tests reach cs_brute_kernel on small meshes)
    hipLaunchKernelGGL(cs_capacity_kernel, dim3(1), dim3(64), 0, st, d_total,
                       (unsigned long long)((g_dev_flags & (1 << 26)) ? 0 : L.list_cap),
                       (unsigned long long)unit_room);
    KL_CHECK_LAUNCH();
  }
  const int64_t total = capturable ? 0 : (int64_t)ctl->total;
  KL_REQUIRE(total < ((int64_t)1 << 31), "check_sign: face lists too long");
  size_t tb = L.temp_bytes;
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(w + L.temp, tb, CsCountIt(cnt, CsToI64()), offs, (int)(3 * ncells + 1),
                                                st));
  // (capturable: an upper bound for the grid, the count itself is read on the device)
  const int64_t nunits = capturable ? unit_room : sort_points ? (int64_t)ctl->units : 0;
  // the lists, then the unit -> cell map: in the workspace when both fit (its unit room is
  // 2 * ncells of the initial grid: units <= ncells + total / kCsStage, and total <= list_cap =
  // 16 entries per face <= kCsStage * ncells when kCsStage >= 16), else from the allocator
  static_assert(kCsStage >= 16, "check_sign: the workspace's unit room assumes >= 16 records per unit");
  const size_t list_bytes = (size_t)(total > 0 ? total : 1) * sizeof(CsRec<T>);
  const bool in_ws = capturable || ((size_t)total <= L.list_cap && nunits <= 2 * B * (int64_t)L.G * L.G);
  uint8_t *lbuf = in_ws ? w + L.list
                        : (uint8_t *)alloc(alloc_ctx, cs_align(list_bytes) + (size_t)(nunits > 0 ? nunits : 1) * 8);
  if (!lbuf) {
    set_error("check_sign: allocator returned NULL");
    return KL_E_ALLOC;
  }
  CsRec<T> *list = (CsRec<T> *)lbuf;
  int64_t *unit_cell = (int64_t *)(lbuf + (in_ws ? L.list_cap * sizeof(CsRec<T>) : cs_align(list_bytes)));
  KL_CHECK_RC(fill_async(cnt, 0, (size_t)ncells * 4, st));
  hipLaunchKernelGGL((cs_bin_kernel<true, T>), fgrid, dim3(256), 0, st, F, G, (const CsRec<T> *)rec,
                     (const float *)mbox, cnt, (const int64_t *)offs, list, (unsigned long long *)nullptr,
                     capturable ? (const int *)d_ovf : nullptr);
  KL_CHECK_LAUNCH();
  if (sort_points) {
    const int64_t *poffs = offs + ncells, *uoffs = offs + 2 * ncells;
    const int *ucnt = cnt + 2 * ncells;
    hipLaunchKernelGGL(cs_pscatter_kernel<T>, pgrid, dim3(256), 0, st, P, G, (const T *)points, ml,
                       (const float *)mbox, (const int32_t *)pslot, poffs, sorted);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(cs_unitmap_kernel, dim3((unsigned)cdiv(ncells, 256)), dim3(256), 0, st, ncells, ucnt, uoffs,
                       unit_cell, capturable ? (const int *)d_ovf : nullptr);
    KL_CHECK_LAUNCH();
    KL_CHECK_RC(fill_async(acc, 0, (size_t)(B * P) * 4, st));
    if (nunits > 0) {
      hipLaunchKernelGGL(cs_cell_check_kernel<T>, dim3((unsigned)cdiv(nunits, 256 / kCsGroup)), dim3(256), 0, st, nunits, P,
                         (int64_t)G * G, (const int64_t *)unit_cell, uoffs, ucnt, poffs, (const CsPt<T> *)sorted,
                         (const int *)cnt, (const int64_t *)offs, (const CsRec<T> *)list, acc, (T *)counts, contains,
                         (const unsigned long long *)(d_total + 1), capturable ? (const int *)d_ovf : nullptr);
      KL_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(cs_finalize_kernel<T>, pgrid, dim3(256), 0, st, P, G, poffs, (const CsPt<T> *)sorted,
                       (const float *)mbox, ucnt, (const int *)acc, (T *)counts, contains,
                       capturable ? (const int *)d_ovf : nullptr);
    if (capturable) {
      KL_CHECK_LAUNCH();
      hipLaunchKernelGGL(cs_brute_kernel<T>, pgrid, dim3(256), 0, st, P, F, (const T *)points, ml,
                         (const CsRec<T> *)rec, (T *)counts, contains, (const int *)d_ovf);
    }
  } else {
    hipLaunchKernelGGL(cs_grid_check_kernel<T>, pgrid, dim3(256), 0, st, P, G, (const T *)points, ml,
                       (const float *)mbox, (const int *)cnt, (const int64_t *)offs, (const CsRec<T> *)list,
                       (T *)counts, contains);
  }
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
