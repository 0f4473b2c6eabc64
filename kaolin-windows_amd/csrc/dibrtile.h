// dibrtile.h -- the fused DIB-R tile kernel's interface (dibrtile.hip), launched by
// kl_dibr_forward (raster.hip) for f32 inputs.
#pragma once

#include "soft_common.h"
#include "tileorder.h"

namespace kl {

struct DibrTileArgs {
  const float *rec;        // (B*F) x RT_REC face records (binning pass)
  const uint2 *rng;        // (B*F) the rasterizer's exact pixel ranges (empty for invalid faces)
  const uint2 *srng;       // (B*F) the soft mask's (enlarged bbox)
  SoftSrc<float> src;      // unscaled face_vertices_image, multiplier (the soft evaluation)
  const float *feat;       // (B,F,3,D)
  const uint32_t *bitmap;  // the soft bins (binning.h, word-major)
  const int32_t *items;    // work items (tileorder.h, order_soft_items), heaviest first
  const int *nitems;
  BinGeom g;
  int F, D, K;
  float eps, sigmainv, m;
  float *out_feat;
  int64_t *out_idx;
  float *out_w;
  float *mask;
  uint8_t *hits;
  uint32_t *rec_face;
  float *rec_prob;
  int *seg_tot;
  int2 *bwd_items;
  int *bwd_cnt;
  int bwd_cap;
  int dev;  // dev param 12 (timing breakdowns; outputs invalid when set): 1 = stop after the
            // rasterizer's outputs, 2 = skip the pair ranking, 3 = stop after the expansion
};

// fewest rows per work item (lp >= 1) for knum (order_soft_items' lp_min)
int dt_lp_min(int K);
// the kernel over `grid` work items (soft_items_bound(nt, lp_min, soft_split()))
int dibr_tile_launch(const DibrTileArgs &a, int lp_min, int grid, hipStream_t st);

}  // namespace kl
