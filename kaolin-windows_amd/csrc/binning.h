// binning.h -- screen-space face bins shared by the rasterizer and the soft mask.
//
// The reference walks EVERY face of a mesh for every pixel (rasterization_cuda.cu:88-171,
// dibr_soft_mask_cuda.cu:80-172).  Both walks depend on face ORDER (max-z with lowest
// index on ties; first `knum` hits in index order), so bins must preserve it.  Here a
// bin is a bitmap over 64-face chunks (chunk c = faces [64c, 64c+64) of one mesh):
//   word c/32 of (mesh b, tile), bit c%32  set  <=>  some face of chunk c may touch the tile.
// Consumers iterate set chunks in ascending order and, inside a chunk, faces in lane
// order, so the walk order is exactly the reference's, restricted to candidate faces.
// Layout: word-major, word w of tile t (tiles of all meshes numbered b * tiles_y * tiles_x + ...)
// at bitmap[w * ntiles + t] (bm_index): the order kernels count a tile per lane with coalesced
// loads; a tile walk reads its <= 32 words once per work item.
// Bit setting is an idempotent atomicOr, so bins are deterministic.
//
// Tiles are TILE_W x TILE_H pixels (one wave = one 64-pixel row segment).
//
// Face sources (how a consumer obtains a face's bbox in multiplied coordinates):
//   BboxSrc     explicit (N,4) bboxes (the reference's packed / soft-mask _C inputs);
//   RastSrc     min/max of face_vertices_image * m, optional valid mask (fused path);
//   SoftSrc     min/max of face_vertices_image * m -/+ boxlen*m (fused path).
// The fused sources evaluate exactly the reference front-end's torch expressions
// (rasterization.py:337-344, dibr.py:31-39), so bins and walks see identical values.
#pragma once

#include "common.h"

namespace kl {

constexpr int TILE_W = 64;
constexpr int TILE_H = 8;

struct BinGeom {
  int batch, height, width;
  int tiles_x, tiles_y;
  int chunks;          // chunks per mesh (upper bound)
  int words;           // uint32 words per tile
  __host__ __device__ size_t ntiles() const { return (size_t)batch * tiles_x * tiles_y; }
  size_t bytes() const { return ntiles() * words * sizeof(uint32_t); }
};
__host__ __device__ inline size_t bm_index(size_t ntiles, size_t tile, int word) { return (size_t)word * ntiles + tile; }

inline BinGeom make_bin_geom(int batch, int height, int width, int64_t max_faces_per_mesh) {
  BinGeom g;
  g.batch = batch;
  g.height = height;
  g.width = width;
  g.tiles_x = (int)cdiv(width, TILE_W);
  g.tiles_y = (int)cdiv(height, TILE_H);
  g.chunks = (int)cdiv(max_faces_per_mesh > 0 ? max_faces_per_mesh : 1, 64);
  g.words = (int)cdiv(g.chunks, 32);
  return g;
}

template <typename T>
struct BboxSrc {
  const T *bbox;  // (N,4)
  const T *fvi;   // (N,3,2) already x multiplier
  __device__ __forceinline__ bool valid(int64_t) const { return true; }
  __device__ __forceinline__ void verts(int64_t f, T v[6]) const {
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[f * 6 + q];
  }
  __device__ __forceinline__ void get(int64_t f, T &x0, T &y0, T &x1, T &y1) const {
    const T *b = bbox + f * 4;
    x0 = b[0];
    y0 = b[1];
    x1 = b[2];
    y1 = b[3];
  }
};

// min / max over the three vertices as torch.min / torch.max(dim) (NaN propagates)
template <typename T>
__device__ __forceinline__ T tmin3(T a, T b, T c) {
  T r = a;
  if (b < r || b != b) r = (r != r) ? r : b;
  if (c < r || c != c) r = (r != r) ? r : c;
  return r;
}
template <typename T>
__device__ __forceinline__ T tmax3(T a, T b, T c) {
  T r = a;
  if (b > r || b != b) r = (r != r) ? r : b;
  if (c > r || c != c) r = (r != r) ? r : c;
  return r;
}

template <typename T>
struct RastSrc {
  const T *fvi;          // (B*F,3,2) unscaled
  const uint8_t *vmask;  // (B*F) valid faces, or nullptr = all valid
  T m;
  const T *nz;           // (B*F) face_normals_z: valid = nz >= 0 (NaN invalid), used when vmask is null
  __device__ __forceinline__ bool valid(int64_t f) const {
    if (vmask) return vmask[f] != 0;
    return nz == nullptr || nz[f] >= (T)0;
  }
  __device__ __forceinline__ void verts(int64_t f, T v[6]) const {
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[f * 6 + q] * m;
  }
  __device__ __forceinline__ void get(int64_t f, T &x0, T &y0, T &x1, T &y1) const {
    const T *v = fvi + f * 6;
    const T ax = v[0] * m, ay = v[1] * m, bx = v[2] * m, by = v[3] * m, cx = v[4] * m, cy = v[5] * m;
    x0 = tmin3(ax, bx, cx);
    y0 = tmin3(ay, by, cy);
    x1 = tmax3(ax, bx, cx);
    y1 = tmax3(ay, by, cy);
  }
};

template <typename T>
struct SoftSrc {
  const T *fvi;  // (B*F,3,2) unscaled
  T m;
  T pad;         // (T)(boxlen * multiplier), the python-float product cast to the tensor dtype
  __device__ __forceinline__ bool valid(int64_t) const { return true; }
  __device__ __forceinline__ void verts(int64_t f, T v[6]) const {
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = fvi[f * 6 + q] * m;
  }
  __device__ __forceinline__ void get(int64_t f, T &x0, T &y0, T &x1, T &y1) const {
    const T *v = fvi + f * 6;
    const T ax = v[0] * m, ay = v[1] * m, bx = v[2] * m, by = v[3] * m, cx = v[4] * m, cy = v[5] * m;
    x0 = tmin3(ax, bx, cx) - pad;
    y0 = tmin3(ay, by, cy) - pad;
    x1 = tmax3(ax, bx, cx) + pad;
    y1 = tmax3(ay, by, cy) + pad;
  }
};

// Conservative pixel-index interval [lo, hi] whose centres c(i) = s * (2i + 1 - N)
// (s = m / N, float) may satisfy  vmin <= c(i) < vmax  (x axis; the y axis calls it
// with the flipped centre formula).  Any NaN bound => the reference's comparisons are
// all false and never reject, so the whole axis is a candidate.
__device__ __forceinline__ void axis_range(double vmin, double vmax, double s, int n, bool flip,
                                           int &lo, int &hi) {
  if (!(vmin == vmin) || !(vmax == vmax) || !(s > 0.0) || !(s < 1e300)) {
    lo = 0;
    hi = n - 1;
    return;
  }
  // invert c = s*(2i+1-n)  ->  i = (c/s + n - 1)/2 ; y axis: c = s*(n-2j-1) -> j = (n-1-c/s)/2
  double a = vmin / s, b = vmax / s;
  double ia, ib;
  if (!flip) {
    ia = (a + n - 1) * 0.5;
    ib = (b + n - 1) * 0.5;
  } else {
    ia = (n - 1 - b) * 0.5;
    ib = (n - 1 - a) * 0.5;
  }
  if (!(ib >= -2.0) || !(ia <= (double)n + 1.0)) {  // entirely off screen (also +-inf)
    lo = 1;
    hi = 0;
    return;
  }
  double l = floor(ia) - 1.0, h = ceil(ib) + 1.0;
  if (l < 0.0) l = 0.0;
  if (h > (double)(n - 1)) h = (double)(n - 1);
  if (l > h) {
    lo = 1;
    hi = 0;
    return;
  }
  lo = (int)l;
  hi = (int)h;
}

// Sets chunk c's bit in every tile of mesh b that one of the wave's faces touches (the
// lane's face covers tiles [tx0,tx1] x [ty0,ty1]; empty when tx0 > tx1).  Small unions
// are walked by the wave with one atomicOr per tile, large ones per lane.
// Marks chunk c's bit in every tile of the lanes' tile ranges.  The chunk's union rectangle
// (<= 256 tiles) is flagged in the wave's LDS scratch `wf` (256 bytes) by every lane for its own
// tiles, then the flagged tiles are OR-ed in lane-parallel: one atomic per touched tile, no
// serial walk of the rectangle.  Larger rectangles: per-lane atomics.
__device__ __forceinline__ void bin_mark(const BinGeom &g, int b, int c, int lane, int tx0, int tx1, int ty0,
                                         int ty1, uint32_t *__restrict__ bitmap, uint8_t *wf) {
  const bool has = tx0 <= tx1;
  const int ux0 = wave_min(has ? tx0 : INT32_MAX), ux1 = wave_max(has ? tx1 : -1);
  const int uy0 = wave_min(has ? ty0 : INT32_MAX), uy1 = wave_max(has ? ty1 : -1);
  if (ux0 > ux1) return;
  const uint32_t bit = 1u << (c & 31);
  const size_t tile_base = (size_t)b * g.tiles_y * g.tiles_x;
  const int uw = ux1 - ux0 + 1;
  const int area = uw * (uy1 - uy0 + 1);
  if (area <= 256) {
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (q * 64 + lane < area) wf[q * 64 + lane] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (has)
      for (int ty = ty0; ty <= ty1; ty++)
        for (int tx = tx0; tx <= tx1; tx++) wf[(ty - uy0) * uw + (tx - ux0)] = 1;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int e = q * 64 + lane;
      if (e < area && wf[e]) {
        const int ty = uy0 + e / uw, tx = ux0 + e % uw;
        atomicOr(&bitmap[bm_index(g.ntiles(), tile_base + (size_t)ty * g.tiles_x + tx, c >> 5)], bit);
      }
    }
    __builtin_amdgcn_wave_barrier();  // wf is reused by the wave's next call
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  } else if (has) {
    for (int ty = ty0; ty <= ty1; ty++)
      for (int tx = tx0; tx <= tx1; tx++)
        atomicOr(&bitmap[bm_index(g.ntiles(), tile_base + (size_t)ty * g.tiles_x + tx, c >> 5)], bit);
  }
}

// The reference's float pixel pitches (m / W, m / H) and their inverses (estimates only),
// computed once on the host with the same float division.
struct PixPitch {
  float sx, sy, xinv, yinv;
};

// Exact pixel interval of one axis whose centres c pass the reference's bbox test
// (!(c < vlo) && !(c >= vhi), rasterization_cuda.cu:101-104) in float arithmetic: an
// index estimate corrected against the exact centre formula (monotone in the index).
// x: c(k) = (T)(s * (2k + 1 - n)) increasing; y (flip): c(k) = (T)(s * (n - 2k - 1))
// decreasing.  NaN bounds never reject.  Empty: a > b.
template <typename T>
__device__ __forceinline__ void exact_range(T vlo, T vhi, float s, float inv, int n, bool flip, int &a, int &b) {
  if (!(vlo == vlo)) vlo = (T)-INFINITY;  // a NaN bound passes every centre, as -inf / +inf do
  if (!(vhi == vhi)) vhi = (T)INFINITY;
  auto c = [&](int k) -> T { return flip ? (T)(s * (float)(n - 2 * k - 1)) : (T)(s * (float)(2 * k + 1 - n)); };
  auto est = [&](T v) -> int {  // index whose centre is near v, clamped to [0, n]
    const float t = flip ? ((float)(n - 1) - (float)v * inv) * 0.5f : ((float)v * inv + (float)(n - 1)) * 0.5f;
    if (!(t == t)) return 0;
    return t <= 0.0f ? 0 : (t >= (float)n ? n : (int)t);
  };
  // P(k) monotone false -> true in k: first k with P (n if none).  The estimate is the answer or
  // one below it but for rounding at the clamps or near-integer estimates, so P(e - 1), P(e) and
  // P(e + 1) settle it without branches; the walk runs only where they do not (rare, and a
  // divergent walk in every lane cost the binning kernel ~40 % of its VALU and SALU issue).
  auto first = [&](int e, auto P) {
    const bool pm = e > 0 && P(e - 1);
    const bool p0 = e >= n || P(e);
    const bool pp = e + 1 >= n || P(e + 1);
    if (!pm && p0) return e;
    if (!p0 && pp) return e + 1;
#pragma clang loop unroll(disable)
    while (e > 0 && P(e - 1)) e--;
#pragma clang loop unroll(disable)
    while (e < n && !P(e)) e++;
    return e;
  };
  if (!flip) {
    a = first(est(vlo), [&](int k) { return !(c(k) < vlo); });
    b = first(est(vhi), [&](int k) { return c(k) >= vhi; }) - 1;
  } else {
    a = first(est(vhi), [&](int k) { return !(c(k) >= vhi); });
    b = first(est(vlo), [&](int k) { return c(k) < vlo; }) - 1;
  }
}

// One wave per (mesh b, chunk c).  Mesh b owns faces [first(b), last(b)) of the source.
// first_idx == nullptr => uniform meshes of `faces_per_mesh` faces.
// bbox_out (optional): the face bboxes of the source, (N,4), for consumers that walk them.
template <typename T, typename Src>
__global__ void __launch_bounds__(256) bin_faces_kernel(Src src, const int64_t *__restrict__ first_idx,
                                                        int faces_per_mesh, BinGeom g, float m,
                                                        uint32_t *__restrict__ bitmap, T *__restrict__ bbox_out,
                                                        uint2 *__restrict__ rng_out) {
  __shared__ uint8_t s_bm[4][256];  // bin_mark scratch, one per wave
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.y;
  const int c = wave;
  if (c >= g.chunks) return;
  int64_t f0, f1;
  if (first_idx) {
    f0 = first_idx[b];
    f1 = first_idx[b + 1];
  } else {
    f0 = (int64_t)b * faces_per_mesh;
    f1 = f0 + faces_per_mesh;
  }
  const int64_t base = f0 + (int64_t)c * 64;
  if (base >= f1) return;
  const int64_t f = base + lane;
  int tx0 = 1, tx1 = 0, ty0 = 1, ty1 = 0;
  if (f < f1 && src.valid(f)) {
    T bx0, by0, bx1, by1;
    src.get(f, bx0, by0, bx1, by1);
    if (bbox_out) {
      bbox_out[f * 4 + 0] = bx0;
      bbox_out[f * 4 + 1] = by0;
      bbox_out[f * 4 + 2] = bx1;
      bbox_out[f * 4 + 3] = by1;
    }
    int ix0, ix1, iy0, iy1;
    if (rng_out) {  // exact pixel ranges (the consumer's bbox test), tiles from them
      const float sx = m / (float)g.width, sy = m / (float)g.height;
      exact_range(bx0, bx1, sx, (float)g.width / m, g.width, false, ix0, ix1);
      exact_range(by0, by1, sy, (float)g.height / m, g.height, true, iy0, iy1);
      const bool e = ix0 > ix1 || iy0 > iy1;
      rng_out[f] = e ? make_uint2(1u, 1u)
                     : make_uint2((uint32_t)ix0 | ((uint32_t)ix1 << 16), (uint32_t)iy0 | ((uint32_t)iy1 << 16));
    } else {
      const double sx = (double)(m / (float)g.width), sy = (double)(m / (float)g.height);
      axis_range((double)bx0, (double)bx1, sx, g.width, false, ix0, ix1);
      axis_range((double)by0, (double)by1, sy, g.height, true, iy0, iy1);
    }
    if (ix0 <= ix1 && iy0 <= iy1) {
      tx0 = ix0 / TILE_W;
      tx1 = ix1 / TILE_W;
      ty0 = iy0 / TILE_H;
      ty1 = iy1 / TILE_H;
    }
  }
  bin_mark(g, b, c, lane, tx0, tx1, ty0, ty1, bitmap, s_bm[threadIdx.x >> 6]);
}

// zero_bytes: bytes from `bitmap` zeroed first (0 = the bitmap's own g.bytes()).
template <typename T, typename Src>
inline int launch_binning(Src src, const int64_t *first_idx, int faces_per_mesh, const BinGeom &g, float m,
                          uint32_t *bitmap, hipStream_t st, T *bbox_out = nullptr, size_t zero_bytes = 0,
                          uint2 *rng_out = nullptr) {
  KL_CHECK_RC(fill_async(bitmap, 0, zero_bytes ? zero_bytes : g.bytes(), st));
  dim3 grid((unsigned)cdiv((int64_t)g.chunks * 64, 256), (unsigned)g.batch);
  hipLaunchKernelGGL((bin_faces_kernel<T, Src>), grid, dim3(256), 0, st, src, first_idx, faces_per_mesh, g, m,
                     bitmap, bbox_out, rng_out);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl
