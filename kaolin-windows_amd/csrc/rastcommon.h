// rastcommon.h -- the rasterizer's per-(pixel, face) arithmetic and face records, shared by the
// tile rasterizer (raster.hip) and the fused DIB-R tile kernel (dibrtile.hip).
#pragma once

#include "common.h"

namespace kl {

// Face records written by the binning pass: vertices x m (6), depths (3), pad (3); and
// the exact pixel ranges of the reference's bbox test (rasterization_cuda.cu:101-104),
// x0 | x1 << 16 and y0 | y1 << 16, empty (1, 0) for invalid faces.
constexpr int RT_REC = 12;

// The reference's per-(pixel, face) test, statement for statement: bbox reject, edge
// functions, copysign(eps) normalisation, barycentric sign test.  true => (w0,w1,w2)
// are the face's weights at the pixel centre (x0, y0).  tri_weights is the part after
// the bbox reject.
template <typename T>
__device__ __forceinline__ bool tri_weights(const T *v, T x0, T y0, float eps, T &w0, T &w1, T &w2) {
  const T aex = v[0] - x0, aey = v[1] - y0;
  const T bex = v[2] - x0, bey = v[3] - y0;
  const T cex = v[4] - x0, cey = v[5] - y0;
  w0 = bex * cey - bey * cex;
  w1 = cex * aey - cey * aex;
  w2 = aex * bey - aey * bex;
  T norm = w0 + w1 + w2;
  norm = (T)((double)norm + copysign((double)eps, (double)norm));
  w0 /= norm;
  w1 /= norm;
  w2 /= norm;
  return !(w0 < (T)0 || w1 < (T)0 || w2 < (T)0);
}

// Depth-ordered visibility through one 64-bit atomicMax per covered (face, pixel):
//   float : key = order(z0) << 32 | ~local_face   -> max depth, lowest index on ties,
//           which is exactly the reference's `if (z0 <= max_z0) continue` fold over
//           faces in index order;
//   double: pass 0 maxes order(z0) (64 bit), pass 1 mins the index among the faces
//           that reach it.
// order() maps floats to unsigned keys monotonically with -0 == +0.  z0 = -inf never
// wins in the reference (-inf <= -inf), so it is dropped.  A NaN z0 breaks the total
// order (the reference then keeps the LAST passing face); such pixels are flagged and
// re-walked sequentially by the resolve kernel.
__device__ __forceinline__ uint32_t order32(float z) {
  uint32_t u = __float_as_uint(z == 0.0f ? 0.0f : z);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint64_t order64(double z) {
  uint64_t u = (uint64_t)__double_as_longlong(z == 0.0 ? 0.0 : z);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

}  // namespace kl
