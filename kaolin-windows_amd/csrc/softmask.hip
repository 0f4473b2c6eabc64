// softmask.hip -- DIB-R soft silhouette (dibr_soft_mask forward / backward) for gfx950.
//
// Reference forward (dibr_soft_mask_cuda.cu:27-184): for every pixel NOT covered by a
// rasterized face, walk ALL faces of its mesh in index order, keep the first `knum`
// whose enlarged bbox contains the pixel centre, and store for each its probability
// exp(-sigmainv * d^2 / m^2), index and distance type; mask = 1 - prod(1 - p).
//
// Here: faces are binned to 64x8 tiles (binning.h, order-preserving 64-face chunks);
// one wave owns a 64-pixel row segment, walks only candidate chunks in ascending order
// and stops as soon as every lane is covered or has `knum` hits.  Hits are staged in
// LDS ([slot][lane] layout, conflict-free), then the wave writes its whole contiguous
// output range (64 pixels x knum slots of prob / idx / type, padding included) with
// lane-contiguous stores -- the K-slot tensors are ~95% of the op's HBM traffic, so
// they are written exactly once and coalesced.  Per-hit arithmetic is the reference's,
// including its float/double promotions (EPS = 1e-7 is a double literal there).
//
// Backward (dibr_soft_mask_cuda.cu:230-353): one thread per pixel, atomics into the
// face-vertex gradient.
#include "soft_common.h"

#include <hipcub/hipcub.hpp>

namespace kl {

// Forward, one wave per 64-pixel row segment, three phases:
//  1. selection: walk the candidate chunks of the tile in ascending order (the next
//     chunk's bboxes are loaded while the current one is tested).  Each lane takes one
//     face of the chunk and computes the exact lane interval its bbox covers on this
//     row; only faces whose interval meets a still-active pixel (uncovered, < knum
//     hits) are visited, in lane order, appending their id to the slot list of every
//     active pixel of the interval ([slot][lane] in LDS);
//  2. evaluation: the wave's hits, flattened, are evaluated 64 at a time with every
//     lane busy (distance, probability, type), written straight to their output slots
//     and the probabilities kept in LDS for the in-order product;
//  3. the unused slots (-1 / 0 / 0) are written with lane-contiguous stores.
// LDS per wave: K x 64 slots of sizeof(T) (face id, then its probability) + 2 x 64 ints.
template <typename T, typename Src>
__global__ void __launch_bounds__(256) soft_mask_fwd_kernel(
    Src src, const T *__restrict__ bbox, const int64_t *__restrict__ sel,
    const uint32_t *__restrict__ bitmap, BinGeom g, int F, int K, float sigmainv, float multiplier,
    T *__restrict__ out_mask, T *__restrict__ out_prob, int64_t *__restrict__ out_idx,
    uint8_t *__restrict__ out_type, uint8_t *__restrict__ out_hits, bool bbox_vec4,
    const int32_t *__restrict__ tile_order) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  const size_t per_wave = (size_t)K * 64 * sizeof(T) + 128 * sizeof(int);
  unsigned char *mine = smem + per_wave * wid;
  T *s_slot = reinterpret_cast<T *>(mine);                                    // [K][64]
  int *s_kid = reinterpret_cast<int *>(mine + (size_t)K * 64 * sizeof(T));   // [64]
  int *s_pre = s_kid + 64;                                                    // [64] exclusive prefix

  // work unit = (tile, row group): tiles in tile_order (heaviest first), else grid order
  const int groups = TILE_H / waves;
  const int tile = tile_order[blockIdx.x / groups];
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int b = tile / (g.tiles_x * g.tiles_y);
  const int j = ty * TILE_H + (blockIdx.x % groups) * waves + wid;
  const int H = g.height, W = g.width;
  if (j >= H) return;
  const int ibase = tx * TILE_W;
  const int i = ibase + lane;
  const bool px_valid = i < W;
  const size_t pix = ((size_t)b * H + j) * W + (px_valid ? i : W - 1);
  const bool covered = px_valid ? (sel[pix] >= 0) : true;
  const T y0 = pix_y<T>(multiplier, H, j);
  // phase 1 view: the id of slot (k, lane) lives in the first 4 bytes of s_slot[k*64 + lane]
  uint32_t *s_face = reinterpret_cast<uint32_t *>(s_slot);
  constexpr int ID_STEP = (int)(sizeof(T) / sizeof(uint32_t));

  // ---- phase 1: selection
  int kid = 0;
  bool active = !covered && K > 0;
  uint64_t amask = ballot(active);
  const uint32_t *words = bitmap + ((size_t)(b * g.tiles_y + j / TILE_H) * g.tiles_x + tx);  // word w: [w * ntiles]
  const int64_t f0 = (int64_t)b * F;
  const T *bb = bbox + f0 * 4;
  // candidate chunks: 64 bitmap words per vector load, non-empty words found by ballot
  int wg = 0;                 // word group (64 words)
  uint32_t wv = 0;            // this lane's word of the group
  uint64_t wmask = 0;         // non-empty words of the group
  uint32_t word = 0;          // word being consumed (uniform)
  int wbase = 0;              // chunk index of bit 0 of `word`
  auto next_chunk = [&]() -> int {
    while (!word) {
      while (!wmask) {
        if (wg * 64 >= g.words) return -1;
        const int w = wg * 64 + lane;
        wv = w < g.words ? words[(size_t)w * g.ntiles()] : 0u;
        wmask = ballot(wv != 0);
        wg++;
      }
      const int s = __builtin_ctzll(wmask);
      wmask &= wmask - 1;
      word = (uint32_t)__builtin_amdgcn_readlane((int)wv, s);
      wbase = ((wg - 1) * 64 + s) * 32;
    }
    const int c = wbase + __builtin_ctz(word);
    word &= word - 1;
    return c;
  };
  T nb0 = 0, nb1 = 0, nb2 = 0, nb3 = 0;
  auto load_chunk = [&](int c) {
    const int fl = c * 64 + lane;
    if (fl < F) {
      if (sizeof(T) == 4 && bbox_vec4) {
        const float4 q = reinterpret_cast<const float4 *>(bb)[fl];
        nb0 = (T)q.x;
        nb1 = (T)q.y;
        nb2 = (T)q.z;
        nb3 = (T)q.w;
      } else {
        nb0 = bb[fl * 4 + 0];
        nb1 = bb[fl * 4 + 1];
        nb2 = bb[fl * 4 + 2];
        nb3 = bb[fl * 4 + 3];
      }
    }
  };
  int cn = -1;
  if (amask) {
    cn = next_chunk();
    if (cn >= 0) load_chunk(cn);
  }
  while (cn >= 0 && amask) {
    const int c = cn;
    const T bx0 = nb0, by0 = nb1, bx1 = nb2, by1 = nb3;
    cn = next_chunk();
    if (cn >= 0) load_chunk(cn);  // in flight while chunk c is tested
    const int fl = c * 64 + lane;
    int lo = 64, hi = -1;
    if (fl < F && !(y0 < by0 || y0 >= by1)) seg_range<T>(bx0, bx1, multiplier, W, ibase, lo, hi);
    const uint64_t rm = lo <= hi ? ((~0ull >> (63 - hi)) & (~0ull << lo)) : 0ull;
    uint64_t mask = ballot((rm & amask) != 0);
    while (mask) {
      const int s = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int a = __builtin_amdgcn_readlane(lo, s), e = __builtin_amdgcn_readlane(hi, s);
      if (active && lane >= a && lane <= e) {
        s_face[(kid * 64 + lane) * ID_STEP] = (uint32_t)(c * 64 + s);
        kid++;
        if (kid >= K) active = false;
      }
      amask = ballot(active);
      if (!amask) break;
      // faces of this chunk whose interval no longer meets an active pixel are skipped
      mask &= ballot((rm & amask) != 0);
    }
  }
  if (!px_valid) kid = 0;
  if (out_hits && px_valid) out_hits[pix] = (uint8_t)kid;

  // ---- phase 2: dense evaluation of the wave's hits
  int pre = kid;  // inclusive scan over lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(pre, o);
    if (lane >= o) pre += u;
  }
  const int total = __shfl(pre, 63);
  s_kid[lane] = kid;
  s_pre[lane] = pre - kid;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const size_t rowpix0 = ((size_t)b * H + j) * W + (size_t)ibase;
  for (int e = lane; e < total; e += 64) {
    int lo = 0;  // owner lane p: last lane with s_pre[p] <= e (and a hit)
#pragma unroll
    for (int st = 32; st > 0; st >>= 1)
      if (s_pre[lo + st] <= e) lo += st;
    const int p = lo, k = e - s_pre[p];
    const uint32_t fl = s_face[(k * 64 + p) * ID_STEP];
    T v[6];
    src.verts(f0 + fl, v);
    T dsq;
    int edgeid;
    soft_dist<T>(pix_x<T>(multiplier, W, ibase + p), y0, v, multiplier, dsq, edgeid);
    const T z = (T)sigmainv * dsq / (T)multiplier / (T)multiplier;
    const T pr = kl_exp<T>(-z);
    const size_t o = (rowpix0 + p) * K + k;
    out_prob[o] = pr;
    out_idx[o] = (int64_t)fl;
    out_type[o] = (uint8_t)(edgeid + 1);
    s_slot[k * 64 + p] = pr;  // overwrites only this hit's own id
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

  // soft mask value: 1 - prod(1 - p) in double, slot order (dibr_soft_mask_cuda.cu:174-182)
  if (px_valid) {
    T res;
    if (covered) {
      res = (T)1.0;
    } else {
      T allprob = (T)1.0;
      for (int k = 0; k < kid; k++) allprob = (T)((double)allprob * (1.0 - (double)s_slot[k * 64 + lane]));
      res = (T)(1.0 - (double)allprob);
    }
    out_mask[pix] = res;
  }

  // ---- phase 3: the unused slots of this row segment, lane-contiguous
  if (K == 0) return;
  const int n = min(64, W - ibase);
  const int ne = n * K;
  int p = 0, k = lane;  // element e = p*K + k, advanced incrementally (no division)
  while (k >= K) {
    k -= K;
    p++;
  }
  const int dp = 64 / K, dk = 64 - dp * K;
  for (int e = lane; e < ne; e += 64) {
    if (k >= s_kid[p]) {
      const size_t o = rowpix0 * K + e;
      out_idx[o] = -1;
      out_prob[o] = (T)0;
      out_type[o] = 0;
    }
    p += dp;
    k += dk;
    if (k >= K) {
      k -= K;
      p++;
    }
  }
}

// Backward, aggregated: one 512-thread workgroup per 64x8 tile (one wave per row
// segment).  The wave's hits (the first kid slots of each uncovered pixel) are
// evaluated densely, 64 at a time, and the per-face vertex-gradient terms -- the
// reference's expressions, each already divided by the multiplier as it adds them --
// are summed in double in an LDS hash table keyed by face (faces of a tile are shared by
// many of its pixels); the table is flushed with one global double atomic per (face,
// coordinate) into a double accumulator, rounded once afterwards (acc_finalize).
// kid per pixel: `hits` from the fused forward, or the reference's scan of the slots
// up to the first -1 (hits == nullptr, the _C contract).
template <typename T, bool SCALE>
__global__ void __launch_bounds__(512) soft_mask_bwd_agg_kernel(
    const T *__restrict__ grad, const T *__restrict__ mask, const int64_t *__restrict__ sel,
    const T *__restrict__ prob, const int64_t *__restrict__ cidx, const uint8_t *__restrict__ ctype,
    const uint8_t *__restrict__ hits, const T *__restrict__ fvi, int B, int H, int W, int F, int K,
    float sigmainv, float multiplier, double *__restrict__ gacc) {
  __shared__ int s_key[SMB_HCAP];
  __shared__ double s_val[SMB_HCAP * 6];
  __shared__ double s_a[8][64];
  __shared__ int s_pre[8][64];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  FaceHash<T> hash{s_key, s_val};
  hash.init(threadIdx.x, blockDim.x);
  __syncthreads();

  const int b = blockIdx.z;
  const int j = blockIdx.y * 8 + wid;
  const int ibase = blockIdx.x * 64;
  const int i = ibase + lane;
  const T ms = (T)multiplier;
  const T *fb = fvi + (size_t)b * F * 6;  // this mesh's face vertices
  int kid = 0;
  size_t pk = 0;
  if (j < H && i < W) {
    const size_t p = ((size_t)b * H + j) * W + i;
    pk = p * K;
    if (sel[p] < 0) {
      if (hits) {
        kid = hits[p];
      } else {
        while (kid < K && cidx[pk + kid] >= 0) kid++;
      }
      // the reference's  -1.0 * sigmainv * dLdp * (1.0 - allprob), evaluated left to right
      s_a[wid][lane] = -1.0 * (double)sigmainv * (double)grad[p] * (1.0 - (double)mask[p]);
    }
  }
  int pre = kid;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(pre, o);
    if (lane >= o) pre += u;
  }
  const int total = __shfl(pre, 63);
  s_pre[wid][lane] = pre - kid;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

  const T y0 = pix_y<T>(multiplier, H, j < H ? j : 0);
  const size_t rowk = (((size_t)b * H + (j < H ? j : 0)) * W + ibase) * K;
  double *gb = gacc + (size_t)b * F * 6;
  for (int e = lane; e < total; e += 64) {
    int lo = 0;
#pragma unroll
    for (int st = 32; st > 0; st >>= 1)
      if (s_pre[wid][lo + st] <= e) lo += st;
    const int p = lo, k = e - s_pre[wid][p];
    const size_t o = rowk + (size_t)p * K + k;
    const int f = (int)cidx[o];
    const T pr = prob[o];
    const int edgeid = (int)ctype[o] - 1;
    const T x0 = pix_x<T>(multiplier, W, ibase + p);
    const T dLdz = (T)(s_a[wid][p] / (1.0 - (double)pr + SM_EPS) * (double)pr);
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = SCALE ? fb[(size_t)f * 6 + q] * ms : fb[(size_t)f * 6 + q];
    int c0, c1;
    T g0x, g0y, g1x, g1y;
    soft_hit_grad<T>(v, edgeid, x0, y0, dLdz, multiplier, c0, c1, g0x, g0y, g1x, g1y);
    hash.add(f, c0, c1, g0x, g0y, g1x, g1y, gb);
  }
  __syncthreads();
  hash.flush(threadIdx.x, blockDim.x, gb);
}

// Longest-first order of the tiles for the forward walk: a tile's cost grows with its
// candidate chunks (set bits of its bitmap words), and the heaviest tiles -- around the
// silhouette's tight spots -- would otherwise start last and set the kernel's tail.
__global__ void __launch_bounds__(256) tile_work_kernel(const uint32_t *__restrict__ bitmap, BinGeom g,
                                                         uint32_t *__restrict__ keys, int32_t *__restrict__ vals) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  if (t >= nt) return;
  uint32_t n = 0;
  for (int k = 0; k < g.words; k++) n += __popc(bitmap[bm_index(nt, t, k)]);
  keys[t] = 0xffffu - min(n, 0xffffu);  // ascending sort -> heaviest first
  vals[t] = t;
}

template <typename T>
static size_t sm_lds_per_wave(int K) {
  return (size_t)K * 64 * sizeof(T) + 128 * sizeof(int);
}

// workspace: bin bitmap | tile order (keys/vals in/out + sort temp) | per-face bboxes
// (fused path; sized for f64)
struct SmWs {
  size_t order, order_temp, order_temp_bytes, bbox, bytes;
  SmWs(const BinGeom &g, int F) {
    const int nt = g.batch * g.tiles_y * g.tiles_x;
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (const int32_t *)nullptr, (int32_t *)nullptr, nt, 0, 16);
    order = al256(g.bytes());
    order_temp = order + 4 * al256((size_t)nt * 4);
    order_temp_bytes = tb;
    bbox = order_temp + al256(tb);
    bytes = bbox + (size_t)g.batch * F * 4 * sizeof(double);
  }
};
static size_t sm_ws_bytes(int B, int H, int W, int F) { return SmWs(make_bin_geom(B, H, W, F), F).bytes; }

// bbox == nullptr: the source computes the bboxes (fused path) and binning stores them
template <typename T, typename Src>
static int soft_mask_fwd(Src src, const T *bbox, int B, int H, int W, int F, int K, const int64_t *sel,
                         float sigmainv, float m, void *mask, void *prob, int64_t *cidx, uint8_t *ctype,
                         uint8_t *hits, void *ws, size_t ws_bytes, hipStream_t st) {
  BinGeom g = make_bin_geom(B, H, W, F);
  const SmWs L(g, F);
  KL_REQUIRE(ws_bytes >= (bbox ? L.bbox : L.bytes), "dibr_soft_mask_forward: workspace too small");
  KL_REQUIRE(K >= 0, "dibr_soft_mask_forward: knum must be >= 0");
  KL_REQUIRE(F < (1 << 28), "dibr_soft_mask_forward: too many faces");
  KL_REQUIRE(hits == nullptr || K <= 255, "dibr_soft_mask_forward: per-pixel hit counts need knum <= 255");
  if (B == 0 || H == 0 || W == 0) return KL_OK;
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(ws);
  char *w = reinterpret_cast<char *>(ws);
  T *bbox_out = nullptr;
  if (!bbox) {
    bbox_out = reinterpret_cast<T *>(w + L.bbox);
    bbox = bbox_out;
  }
  int rc = launch_binning<T, Src>(src, nullptr, F, g, m, bitmap, st, bbox_out);
  if (rc) return rc;
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  const size_t ob = al256((size_t)nt * 4);
  uint32_t *kin = reinterpret_cast<uint32_t *>(w + L.order), *kout = reinterpret_cast<uint32_t *>(w + L.order + ob);
  int32_t *vin = reinterpret_cast<int32_t *>(w + L.order + 2 * ob);
  int32_t *vout = reinterpret_cast<int32_t *>(w + L.order + 3 * ob);
  hipLaunchKernelGGL(tile_work_kernel, dim3((unsigned)cdiv(nt, 256)), dim3(256), 0, st, bitmap, g, kin, vin);
  KL_CHECK_LAUNCH();
  size_t tb = L.order_temp_bytes;
  KL_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(w + L.order_temp, tb, kin, kout, vin, vout, nt, 0, 16, st));
  const size_t pw = sm_lds_per_wave<T>(K);
  int waves = 4;
  while (waves > 1 && pw * waves > 64 * 1024) waves--;
  KL_REQUIRE(pw * waves <= 160 * 1024, "dibr_soft_mask_forward: knum too large for the LDS slot lists");
  while (TILE_H % waves) waves--;
  const unsigned units = (unsigned)(nt * (TILE_H / waves));
  hipLaunchKernelGGL((soft_mask_fwd_kernel<T, Src>), dim3(units), dim3(64 * waves), pw * waves, st, src, bbox, sel,
                     bitmap, g, F, K, sigmainv, m, (T *)mask, (T *)prob, cidx, ctype, hits,
                     ((uintptr_t)bbox & 15) == 0, (const int32_t *)vout);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

// workspace: the (B,F,3,2) double accumulator
static size_t sm_bwd_ws_bytes(int B, int F) { return al256((size_t)B * F * 6 * sizeof(double)); }

template <typename T, bool SCALE>
static int soft_mask_bwd(int B, int H, int W, int F, int K, const void *grad, const void *mask,
                         const int64_t *sel, const void *prob, const int64_t *cidx, const uint8_t *ctype,
                         const uint8_t *hits, const void *fvi, float sigmainv, float m, void *gfvi, void *ws,
                         size_t ws_bytes, hipStream_t st) {
  KL_REQUIRE(F < (1 << 28), "dibr_soft_mask_backward: too many faces");
  const size_t n = (size_t)B * F * 6;
  if ((int64_t)B * H * W == 0 || K <= 0 || n == 0) return fill_async(gfvi, 0, sizeof(T) * n, st);
  KL_REQUIRE(ws && ws_bytes >= sm_bwd_ws_bytes(B, F), "dibr_soft_mask_backward: workspace too small");
  double *acc = reinterpret_cast<double *>(ws);
  KL_CHECK_RC(fill_async(acc, 0, n * sizeof(double), st));
  dim3 grid((unsigned)cdiv(W, 64), (unsigned)cdiv(H, 8), B);
  hipLaunchKernelGGL((soft_mask_bwd_agg_kernel<T, SCALE>), grid, dim3(512), 0, st, (const T *)grad, (const T *)mask,
                     sel, (const T *)prob, cidx, ctype, hits, (const T *)fvi, B, H, W, F, K, sigmainv, m, acc);
  KL_CHECK_LAUNCH();
  return acc_finalize<T>(acc, (T *)gfvi, n, false, st);
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_soft_mask_workspace_bytes(int batch, int height, int width, int num_faces) {
  return std::max(sm_ws_bytes(batch, height, width, num_faces), soft_tile_slots_ws_bytes(batch, height, width, num_faces));
}

extern "C" int kl_dibr_soft_mask_forward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                         int knum, const void *fvi, const void *bbox, const int64_t *sel,
                                         float sigmainv, float multiplier, void *mask, void *prob,
                                         int64_t *cidx, uint8_t *ctype, void *ws, size_t ws_bytes,
                                         kl_stream stream) {
  // f32 with knum <= 255: the tile path (softtile.hip, soft_tile_forward_slots: multi-wave heavy rows,
  // padding in 16-byte stores); else the per-row-wave kernel above.  Dev param 30 = 1: that kernel for
  // f32 too (A/B).
  if (dtype == KL_F32 && knum >= 0 && knum <= 255 && num_faces < (1 << 28) && g_dev_param[30] != 1)
    return soft_tile_forward_slots(batch, height, width, num_faces, knum, (const float *)fvi, (const float *)bbox, sel,
                                   sigmainv, multiplier, (float *)mask, (float *)prob, cidx, ctype, ws, ws_bytes,
                                   S(stream));
  if (dtype == KL_F32)
    return soft_mask_fwd<float>(BboxSrc<float>{(const float *)bbox, (const float *)fvi}, (const float *)bbox, batch,
                                height, width, num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype,
                                nullptr, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_mask_fwd<double>(BboxSrc<double>{(const double *)bbox, (const double *)fvi}, (const double *)bbox,
                                 batch, height, width, num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx,
                                 ctype, nullptr, ws, ws_bytes, S(stream));
  set_error("dibr_soft_mask_forward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_soft_mask_forward_fused(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                               int knum, const void *fvi, const int64_t *sel, float sigmainv,
                                               double pad, float multiplier, void *mask, void *prob,
                                               int64_t *cidx, uint8_t *ctype, uint8_t *hits, void *ws,
                                               size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_fwd<float>(SoftSrc<float>{(const float *)fvi, (float)multiplier, (float)pad}, nullptr, batch,
                                height, width, num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype,
                                hits, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_mask_fwd<double>(SoftSrc<double>{(const double *)fvi, (double)multiplier, pad}, nullptr, batch,
                                 height, width, num_faces, knum, sel, sigmainv, multiplier, mask, prob, cidx, ctype,
                                 hits, ws, ws_bytes, S(stream));
  set_error("dibr_soft_mask_forward not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_soft_mask_backward_workspace_bytes(int batch, int num_faces) {
  return sm_bwd_ws_bytes(batch, num_faces);
}

extern "C" int kl_dibr_soft_mask_backward(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                          int knum, const void *grad, const void *mask, const int64_t *sel,
                                          const void *prob, const int64_t *cidx, const uint8_t *ctype,
                                          const void *fvi, float sigmainv, float multiplier, void *gfvi, void *ws,
                                          size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_bwd<float, false>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype,
                                       nullptr, fvi, sigmainv, multiplier, gfvi, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_mask_bwd<double, false>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype,
                                        nullptr, fvi, sigmainv, multiplier, gfvi, ws, ws_bytes, S(stream));
  set_error("dibr_soft_mask_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_soft_mask_backward_fused(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                                int knum, const void *grad, const void *mask, const int64_t *sel,
                                                const void *prob, const int64_t *cidx, const uint8_t *ctype,
                                                const uint8_t *hits, const void *fvi, float sigmainv,
                                                float multiplier, void *gfvi, void *ws, size_t ws_bytes,
                                                kl_stream stream) {
  if (dtype == KL_F32)
    return soft_mask_bwd<float, true>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype, hits,
                                      fvi, sigmainv, multiplier, gfvi, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_mask_bwd<double, true>(batch, height, width, num_faces, knum, grad, mask, sel, prob, cidx, ctype,
                                       hits, fvi, sigmainv, multiplier, gfvi, ws, ws_bytes, S(stream));
  set_error("dibr_soft_mask_backward not implemented for this dtype");
  return KL_E_INVALID;
}
