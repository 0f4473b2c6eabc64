// binning.h -- screen-space face bins shared by the rasterizer and the soft mask.
//
// The reference walks EVERY face of a mesh for every pixel (rasterization_cuda.cu:88-171,
// dibr_soft_mask_cuda.cu:80-172).  Both walks depend on face ORDER (max-z with lowest
// index on ties; first `knum` hits in index order), so bins must preserve it.  Here a
// bin is a bitmap over 64-face chunks (chunk c = faces [64c, 64c+64) of one mesh):
//   bitmap[b][tile][c/32] bit c%32  set  <=>  some face of chunk c may touch the tile.
// Consumers iterate set chunks in ascending order and, inside a chunk, faces in lane
// order, so the walk order is exactly the reference's, restricted to candidate faces.
// Bit setting is an idempotent atomicOr, so bins are deterministic.
//
// Tiles are TILE_W x TILE_H pixels (one wave = one 64-pixel row segment).
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
  size_t bytes() const { return (size_t)batch * tiles_x * tiles_y * words * sizeof(uint32_t); }
};

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
  double l = floor(ia) - 1.0, h = ceil(ib) + 1.0;
  if (l < 0.0) l = 0.0;
  if (h > (double)(n - 1)) h = (double)(n - 1);
  if (l > h || ib < -2.0 || ia > (double)n + 1.0) {
    lo = 1;
    hi = 0;  // empty
    return;
  }
  lo = (int)l;
  hi = (int)h;
}

// One wave per (mesh b, chunk c).  bboxes: (total,4) [xmin,ymin,xmax,ymax] (x multiplier).
// Mesh b owns faces [first(b), last(b)).  first_idx == nullptr => uniform meshes of F faces.
template <typename T>
__global__ void __launch_bounds__(256) bin_faces_kernel(const T *__restrict__ bboxes,
                                                        const int64_t *__restrict__ first_idx,
                                                        int faces_per_mesh, BinGeom g, float m,
                                                        uint32_t *__restrict__ bitmap) {
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
  if (f < f1) {
    const T *bb = bboxes + f * 4;
    int ix0, ix1, iy0, iy1;
    const double sx = (double)(m / (float)g.width), sy = (double)(m / (float)g.height);
    axis_range((double)bb[0], (double)bb[2], sx, g.width, false, ix0, ix1);
    axis_range((double)bb[1], (double)bb[3], sy, g.height, true, iy0, iy1);
    if (ix0 <= ix1 && iy0 <= iy1) {
      tx0 = ix0 / TILE_W;
      tx1 = ix1 / TILE_W;
      ty0 = iy0 / TILE_H;
      ty1 = iy1 / TILE_H;
    }
  }
  const bool has = tx0 <= tx1;
  const int ux0 = wave_min(has ? tx0 : INT32_MAX), ux1 = wave_max(has ? tx1 : -1);
  const int uy0 = wave_min(has ? ty0 : INT32_MAX), uy1 = wave_max(has ? ty1 : -1);
  if (ux0 > ux1) return;
  const uint32_t bit = 1u << (c & 31);
  const size_t tile_base = (size_t)b * g.tiles_y * g.tiles_x;
  const int area = (ux1 - ux0 + 1) * (uy1 - uy0 + 1);
  if (area <= 256) {
    for (int ty = uy0; ty <= uy1; ty++)
      for (int tx = ux0; tx <= ux1; tx++) {
        const uint64_t hit = ballot(has && tx0 <= tx && tx <= tx1 && ty0 <= ty && ty <= ty1);
        if (hit && lane == 0)
          atomicOr(&bitmap[(tile_base + (size_t)ty * g.tiles_x + tx) * g.words + (c >> 5)], bit);
      }
  } else if (has) {
    for (int ty = ty0; ty <= ty1; ty++)
      for (int tx = tx0; tx <= tx1; tx++)
        atomicOr(&bitmap[(tile_base + (size_t)ty * g.tiles_x + tx) * g.words + (c >> 5)], bit);
  }
}

template <typename T>
inline int launch_binning(const T *bboxes, const int64_t *first_idx, int faces_per_mesh, const BinGeom &g,
                          float m, uint32_t *bitmap, hipStream_t st) {
  KL_CHECK_HIP(hipMemsetAsync(bitmap, 0, g.bytes(), st));
  dim3 grid((unsigned)cdiv((int64_t)g.chunks * 64, 256), (unsigned)g.batch);
  hipLaunchKernelGGL(bin_faces_kernel<T>, grid, dim3(256), 0, st, bboxes, first_idx, faces_per_mesh, g, m,
                     bitmap);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl
