// dibrbwd.h -- the pixel-major dibr_rasterization backward (dibrbwd.hip), called by kl_dibr_backward.
#pragma once

#include "soft_common.h"

namespace kl {

// Workspace of db_backward for B*F faces (feature slots sized for feat_dim <= 8).
size_t db_ws_bytes(int B, int H, int W, int F, int K);

// The rasterizer's and the soft mask's face gradients of kl_dibr_backward in one pixel-major
// pass.  rng: the forward's exact raster ranges (B*F); srng: its soft-mask ranges (B*F).
// Writes grad_fvi (raster + soft, each rounded once) and grad_feat of every face except the
// faces whose raster range spans more than 2 x 2 tiles: those are listed in *big (count in
// *nbig, which must be zero on entry), with their soft sums left in *soft_sum (double, B*F*6;
// nullptr when grad_mask is null) for the per-face gather (rasterize_bwd_bigface_kernel).
template <typename T>
int db_backward(int B, int H, int W, int F, int D, int K, const T *grad_feat, const T *grad_mask,
                const int64_t *face_idx, const T *w, const T *fvi, const T *feat, const T *mask,
                const SoftState<T> &s, float sigmainv, float m, float eps, const uint2 *rng, const uint2 *srng,
                T *gfvi, T *gfeat, void *ws, size_t ws_bytes, int *nbig, hipStream_t st, int **big,
                const double **soft_sum);

}  // namespace kl
