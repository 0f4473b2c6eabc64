// softtile.hip -- DIB-R soft mask with a compact saved state (the fused front-end path).
//
// The reference's dibr_soft_mask returns only the soft mask (dibr.py:27-55); its four
// (B,H,W,knum) slot tensors -- prob f32, idx int64 (-1 padded), type u8 -- exist only
// to be saved for its backward (dibr.py:58-73), and at 13 B x knum per pixel they are
// ~95% of the op's HBM traffic (414 MB at the bench config, almost all padding).  The
// fused path saves instead, per pixel, the number of filled slots (u8) and, per hit, a
// record (face | type << 28, prob) packed contiguously per 64-pixel row segment in
// (pixel, slot) order: the same values as the filled slots, nothing for the padding.
// The soft mask and the gradients are computed with the reference's arithmetic and
// hit order, so they equal the _C path's (tests/test_gpu_parity.py).
//
// Forward, per work item = a part of a 64x8 tile's rows (one 4-wave workgroup):
//  1. the tile's candidate 64-face chunks (binning.h bitmap) are expanded cooperatively,
//     one chunk per wave and step: each face's exact lane interval on the tile's columns and
//     the item's rows its bbox spans, and faces that touch them are appended in index order
//     to an LDS face list (ordered compaction across the waves);
//  2. each row walks the list: faces whose interval meets a still-active pixel (uncovered,
//     < knum hits) are appended, in index order, to the [slot][lane] lists of the active
//     pixels they cover -- exactly the reference's "first knum faces whose enlarged bbox
//     contains the pixel centre";
//  3. the row's hits are evaluated densely, records written contiguously, and the mask is
//     1 - prod(1 - p) in slot order.
// Items run heaviest first (candidate-chunk counts, one counting-sort workgroup); the
// heaviest tiles (the silhouette's tight spots) are split into 4 or 8 items whose rows get
// 2 or 4 waves each, for the walk (blocks of the list round-robin, a per-pixel count prefix
// giving each wave its slots) and the evaluation.
//
// Backward, per tile: each row wave reads its records (coalesced), evaluates the
// reference's per-hit terms and sums them per face in an LDS hash (soft_common.h),
// flushed with global atomics -- into a zeroed gradient, or added onto the rasterizer
// backward's gradient (kl_dibr_backward).
#include "soft_common.h"
#include "tileorder.h"
#include "tilewalk.h"

#include <algorithm>

namespace kl {


template <typename T, typename Src = SoftSrc<T>>
struct SoftTileArgs {
  Src src;                   // SoftSrc: unscaled face_vertices_image, multiplier, bbox pad; BboxSrc (the
                             // _C contract): multiplied face_vertices_image and the caller's bboxes
  const uint2 *rng;          // (B*F) exact pixel ranges of the enlarged bboxes (binning pass)
  const int64_t *sel;        // (B,H,W) rasterized face index
  const uint32_t *bitmap;
  const int32_t *order;      // work items, heaviest first
  const int *nitems;         // their number
  BinGeom g;
  int F, K;
  float sigmainv, m;
  T *mask;                   // (B,H,W)
  uint8_t *hits;             // (B,H,W)
  uint32_t *rec_face;        // per row segment s: [s*64*K, s*64*K + hits of the segment)
  T *rec_prob;
  int *seg_tot;              // per row segment: its number of hits
  uint8_t *defer;            // per row segment: its hits are left to soft_tile_eval_kernel
  uint64_t *dbg;             // dev stamps (kl_dev_set_debug), 10 per wave, or nullptr
  int dev;                   // dev ablation flags (kl_dev_set_flags), 0 in the product path
  int prefilled;             // mask / hits / seg_tot / defer already written for pixels and rows
                             // without hits (kl_dibr_forward's rasterizer): only hits are written
  // kl_dibr_forward: the backward's work items, appended here (DibrState): a workgroup with hits
  // adds (item, piece) for each SB_PIECE of its rows' hits to shard blockIdx % DS_SHARDS with one
  // atomic; nullptr: not listed (the backward's plan kernel lists them from seg_tot)
  int2 *bwd_items = nullptr;
  int *bwd_cnt = nullptr;
  int bwd_cap = 0;
  // slot-list layout of soft_tile_fwd_kernel: slot k of lane p at k * 64 + ((p + (k & swz)) & 63).  The
  // rotation (swz = 63) spreads a pixel's consecutive slots, which the evaluation's consecutive threads
  // touch, over the banks; swz = 0 (dev param 19 = 1) is the plain [slot][lane] layout.
  int swz = 63;
  // (prefilled, r05) per work item: 1 when its rows hold an uncovered pixel (the rasterizer's flags,
  // raster_tile_kernel); an item without is done at once -- one load, not the order -> sel chain
  const uint8_t *live = nullptr;
  int live_n = 0;  // its length: items <= TILE_H per tile (the grid's bound can exceed it)
  // The _C contract (kl_dibr_soft_mask_forward, r06): the reference's (B,H,W,knum) prob / idx / type
  // slot tensors written directly.  Each item's rows are padded first (idx -1, prob 0, type 0: 16-byte
  // stores issued before the walk, in flight during it), then every hit is stored at its slot after
  // those stores completed; no compact records (rec_face == nullptr).
  T *slot_prob = nullptr;
  int64_t *slot_idx = nullptr;
  uint8_t *slot_type = nullptr;
};


// The workgroup's face list: the candidate chunks' faces touching its rows, in index order
// (face id; lane interval lo | hi << 6 and row bits << 12), refilled when full.
#ifndef ST_EVAL_U
#define ST_EVAL_U 2  // hits in flight per lane in the f32 evaluation: 89 VGPRs, 5 waves per SIMD (4: 115, 4)
#endif
#ifndef SB_MIN_WAVES  // the soft backward's minimum waves per SIMD (A/B builds)
#define SB_MIN_WAVES 1
#endif
#ifndef SB_HC  // the soft backward's hash: slots and copies per slot (A/B builds)
#define SB_HC 512
#define SB_NC 1
#endif
#ifndef SB_VS  // doubles per hash slot: the 6 sums (A/B builds; r06r: 7, spreading slots 16 apart over the banks, measured equal)
#define SB_VS 6
#endif
#ifndef ST_FC
#define ST_FC 2  // candidate chunks per wave and fill step (A/B builds: EXTRA=-DST_FC=3)
#endif
#ifndef ST_FWD_MIN_WAVES
#define ST_FWD_MIN_WAVES 1  // the forward kernel's minimum waves per SIMD (A/B builds)
#endif
constexpr int ST_LIST_CAP = 960;  // (40.6 KB of LDS at knum 30 with 4 rows: 4 workgroups per CU)
// list | per-wave scratch (16 ints) | the multi-wave walk's per-round counts ([Q][64] per row)
constexpr size_t st_head_lds() { return (size_t)ST_LIST_CAP * 8 + 16 * sizeof(int) + ST_WAVES * 64 * sizeof(int); }

// Forward, one work item (a part of a tile's rows) per 4-wave workgroup: fill and walk (1a,
// 1b below), the dense evaluation by the row's Q waves, the mask by its first wave.
template <typename T, typename Src = SoftSrc<T>>
__global__ void __launch_bounds__(256, ST_FWD_MIN_WAVES) soft_tile_fwd_kernel(SoftTileArgs<T, Src> a) {
  extern __shared__ __align__(16) unsigned char smem[];
  {
    const int ni = *a.nitems;
    // (the two loads in flight together; an index past the flags is past the items too)
    const bool lv = a.live ? a.live[min((int)blockIdx.x, a.live_n - 1)] != 0 : true;
    if ((int)blockIdx.x >= ni || !lv) return;
  }
  uint64_t *const dbg = kDevStamps ? a.dbg : nullptr;  // compiled out unless KL_DEV_STAMPS
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int K = a.K;
  const BinGeom &g = a.g;
  const int H = g.height, W = g.width;
  const int item = a.order[blockIdx.x];
  const int tile = item & 0xffffff, part = (item >> 24) & 15, lp = (item >> 28) & 7;
  if (kDevStamps && (a.dev & (1 << 16)) && lp < 2) return;  // dev: the heavy items alone
  const int RP = TILE_H >> lp;      // rows of this part
  const int Q = ST_WAVES / RP;      // waves per row (lp >= 1: RP <= 4)
  const int r = wid / Q, qi = wid - r * Q;
  uint32_t *L_face = reinterpret_cast<uint32_t *>(smem);
  uint32_t *L_pack = L_face + ST_LIST_CAP;
  int *s_wcnt = reinterpret_cast<int *>(L_pack + ST_LIST_CAP);  // [ST_WAVES] per-wave scratch
  unsigned char *rowmem = smem + st_head_lds() + st_row_lds(K) * r;
  uint32_t *s_face = reinterpret_cast<uint32_t *>(rowmem);                          // [K][64]
  int *s_pre = reinterpret_cast<int *>(rowmem + (size_t)K * 64 * sizeof(uint32_t));  // [64], then total
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int b = tile / (g.tiles_x * g.tiles_y);
  const int j = ty * TILE_H + part * RP + r;
  const bool row_ok = j < H;
  const int ibase = tx * TILE_W;
  const int i = ibase + lane;
  const bool px_valid = row_ok && i < W;
  const size_t pix = ((size_t)b * H + (row_ok ? j : H - 1)) * W + (i < W ? i : W - 1);
  const bool covered = px_valid ? (a.sel[pix] >= 0) : true;
  const int64_t f0 = (int64_t)b * a.F;
  const int F = a.F;
  const bool slots = a.slot_prob != nullptr;  // (launch-uniform)
  if (slots && qi == 0 && row_ok && K > 0) {  // the row's slot ranges as padding (see SoftTileArgs)
    const size_t e0 = ((size_t)b * H + j) * W + (size_t)ibase, ne = (size_t)min(64, W - ibase) * K;
    wave_fill(reinterpret_cast<uint8_t *>(a.slot_idx + e0 * K), ne * sizeof(int64_t), 0xffffffffu, lane);
    wave_fill(reinterpret_cast<uint8_t *>(a.slot_prob + e0 * K), ne * sizeof(T), 0u, lane);
    wave_fill(a.slot_type + e0 * K, ne, 0u, lane);
  }
  const int swz = a.swz;
  auto sl = [swz](int k, int p) { return k * 64 + ((p + (k & swz)) & 63); };
  uint64_t t0 = 0, w0 = 0, t1 = 0, c_fill = 0, tf = 0;
  int nchunks = 0;
  if (dbg) {
    t0 = stamp_clk();
    w0 = stamp_wall();
  }

  int kid = 0;
  bool active = !covered && K > 0;  // (every wave of a row tracks its pixels' state)
  uint64_t amask = ballot(active);
  const int j0 = ty * TILE_H + part * RP;  // the workgroup's first row
  // any active pixel in the workgroup's rows? (workgroup-uniform)
  if (lane == 0) s_wcnt[wid] = amask != 0;
  __syncthreads();
  int any = 0;
  for (int w = 0; w < ST_WAVES; w++) any |= s_wcnt[w];
  __syncthreads();
  if (!any && a.prefilled) return;  // no uncovered pixel: its outputs are written (workgroup-uniform)
  if (any) {
    ChunkSeq seq;
    seq.init(a.bitmap + ((size_t)(b * g.tiles_y + ty) * g.tiles_x + tx), g.words, g.ntiles(), lane);
    const uint2 *rg = a.rng + f0;
    // this wave's two chunks of the next fill step (ordinals pos + wid and pos + ST_WAVES + wid)
    // with their pixel ranges in flight: unconditional loads from clamped indices (a guarded load
    // is waited for at once), issued after the current step's ranges are tested.  Two chunks per
    // wave and step: the fill of a heavy tile (hundreds of candidate chunks) is a chain of steps
    // that each wait for their loads, so twice the chunks per step halves the chain.
    constexpr int FC = ST_FC;  // chunks per wave and step
    int pos = 0, nc[FC];
    bool nexists = false;
    uint2 nr[FC];
#pragma unroll
    for (int k = 0; k < FC; k++) {
      nc[k] = -1;
      nr[k] = make_uint2(1u, 1u);
    }
    auto pf_next = [&]() {
      nexists = seq.at(pos, lane) >= 0;
#pragma unroll
      for (int k = 0; k < FC; k++) nc[k] = nexists ? seq.at(pos + k * ST_WAVES + wid, lane) : -1;
      pos += FC * ST_WAVES;
#pragma unroll
      for (int k = 0; k < FC; k++) {
        int fl = nc[k] * 64 + lane;
        fl = fl < 0 ? 0 : (fl < F ? fl : F - 1);
        nr[k] = rg[fl];
      }
    };
    pf_next();
    bool more = nexists;
    while (true) {
      // ---- 1a. fill: the candidate chunks' faces that touch the workgroup's rows, in index
      //          order, with their lane interval and row bits, FC x ST_WAVES chunks per step
      int len = 0;
      if (dbg) tf = stamp_clk();
      while (more && len + FC * ST_WAVES * 64 <= ST_LIST_CAP) {
        bool keep[FC];
        int flk[FC];
        uint32_t pk[FC];
        uint64_t km[FC];
#pragma unroll
        for (int k = 0; k < FC; k++) {
          const int c = nc[k];
          flk[k] = c * 64 + lane;
          const int ix0 = (int)(nr[k].x & 0xffffu), ix1 = (int)(nr[k].x >> 16);
          const int iy0 = (int)(nr[k].y & 0xffffu), iy1 = (int)(nr[k].y >> 16);
          const int ya = max(iy0, j0) - j0, yb = min(iy1, j0 + RP - 1) - j0;
          const uint32_t rows = ya <= yb ? ((2u << yb) - 1u) & ~((1u << ya) - 1u) : 0u;
          const int lo = max(ix0 - ibase, 0), hi = min(ix1 - ibase, 63);
          keep[k] = c >= 0 && flk[k] < F && rows != 0 && lo <= hi;
          pk[k] = (uint32_t)lo | ((uint32_t)hi << 6) | (rows << 12);
        }
        pf_next();  // consumed by the next step, in this fill or after the walk
        more = nexists;
#pragma unroll
        for (int k = 0; k < FC; k++) {
          km[k] = ballot(keep[k]);
          if (lane == 0) s_wcnt[k * ST_WAVES + wid] = __popcll(km[k]);
        }
        __syncthreads();
        // list order = chunk order: every wave's first chunk (ordinals pos + w), then every wave's
        // second (pos + ST_WAVES + w)
        int tot = 0;
#pragma unroll
        for (int k = 0; k < FC; k++) {
          int pre = tot;
          for (int w = 0; w < ST_WAVES; w++) {
            const int v = s_wcnt[k * ST_WAVES + w];
            pre += w < wid ? v : 0;
            tot += v;
          }
          if (keep[k]) {
            const int p = len + pre + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(km[k] >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)km[k], 0u));
            L_face[p] = (uint32_t)flk[k];
            L_pack[p] = pk[k];
          }
        }
        len += tot;
        __syncthreads();
      }
      if (dbg) {
        nchunks += len;
        c_fill += stamp_clk() - tf;
      }
      // ---- 1b. walk: per row, the list in blocks of 64 entries; the entries' pixel masks are
      //          transposed so that every pixel lane holds the (ordered) entries covering it,
      //          and appends them until it has knum hits.  The Q waves of a row take the
      //          blocks round-robin, a prefix of their per-pixel counts giving each its slots.
      const int nb = (len + 63) >> 6;
      auto block_mask = [&](int blk) -> uint64_t {
        const int e = blk * 64 + lane;
        uint64_t rm = 0;
        if (e < len) {
          const uint32_t pk = L_pack[e];
          if ((pk >> (12 + r)) & 1u) {
            const int lo = (int)(pk & 63u), hi = (int)((pk >> 6) & 63u);
            rm = (~0ull >> (63 - hi)) & (~0ull << lo);
          }
        }
        return rm;
      };
      if (Q == 1) {
        for (int blk = 0; blk < nb && amask; blk++) {
          const uint64_t rm = block_mask(blk);
          if (!ballot((rm & amask) != 0)) continue;
          uint64_t cm = transpose64(rm, lane);
          if (!active) cm = 0;
          const int base = blk * 64;
          while (cm) {
            const int q = __builtin_ctzll(cm);
            cm &= cm - 1;
            s_face[sl(kid, lane)] = L_face[base + q];
            if (++kid >= K) {
              active = false;
              cm = 0;
            }
          }
          amask = ballot(active);
        }
      } else {
        // per-wave counts of this round ([Q][64] per row, in the head: with knum > 55 the rows
        // past RP are not allocated)
        int *s_cnt = reinterpret_cast<int *>(smem + (size_t)ST_LIST_CAP * 8 + 16 * sizeof(int)) + r * Q * 64;
        for (int b0 = 0; b0 < nb; b0 += Q) {  // workgroup-uniform rounds
          const int blk = b0 + qi;
          uint64_t cm = 0;
          if (amask && blk < nb) {
            const uint64_t rm = block_mask(blk);
            if (ballot((rm & amask) != 0)) {
              cm = transpose64(rm, lane);
              if (!active) cm = 0;
            }
          }
          s_cnt[qi * 64 + lane] = __popcll(cm);
          __syncthreads();
          int slot = kid, all = 0;
          for (int q = 0; q < Q; q++) {
            const int v = s_cnt[q * 64 + lane];
            slot += q < qi ? v : 0;
            all += v;
          }
          const int base = blk * 64;
          while (cm && slot < K) {
            s_face[sl(slot, lane)] = L_face[base + __builtin_ctzll(cm)];
            cm &= cm - 1;
            slot++;
          }
          kid = min(K, kid + all);
          active = active && kid < K;
          amask = ballot(active);
          if (lane == 0) s_wcnt[2 * ST_WAVES + wid] = amask != 0;
          __syncthreads();  // s_cnt is rewritten by the next round
          // every row of the workgroup saturated (knum hits or covered): the remaining blocks
          // cannot add a hit (workgroup-uniform exit; the pole tiles' rows fill in a few rounds)
          int live = 0;
          for (int w = 0; w < ST_WAVES; w++) live |= s_wcnt[2 * ST_WAVES + w];
          if (!live) break;
        }
      }
      if (lane == 0) s_wcnt[wid] = amask != 0;
      __syncthreads();
      any = 0;
      for (int w = 0; w < ST_WAVES; w++) any |= s_wcnt[w];
      __syncthreads();
      if (!any || !more) break;
    }
  }
  if (qi == 0) {
    if (!px_valid) kid = 0;
    const int pre = wave_incl_scan(kid);
    s_pre[lane] = pre - kid;
    if (lane == 63) s_pre[64] = pre;
  }
  if (dbg) t1 = stamp_clk();
  const bool inline_eval = sizeof(T) == 4 && K > 0;
  // every row's prefix and total are read by every wave of the workgroup below (f32); with slot
  // outputs the padding stores complete first, as any thread may store a hit over them
  if (slots) __builtin_amdgcn_s_waitcnt(0);
  if (Q > 1 || inline_eval) {
    __syncthreads();
  } else {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  const int total = s_pre[64];

  // ---- 2. the rows' hits ((pixel, slot) order) -> records, evaluated here for f32 by ALL the
  //         workgroup's waves over the item's rows together (a row of ~1,000 hits no longer sits on
  //         one wave while its neighbours' waves idle); f64 leaves face ids for
  //         soft_tile_eval_kernel and flags its rows for it.
  const size_t rbase = ((size_t)(b * H + (row_ok ? j : 0)) * g.tiles_x + tx) * 64 * (size_t)K;
  if (inline_eval) {
    // the rows' hit totals and their exclusive prefix (RP <= 8 rows)
    int rtot[8], rpre[9];
    rpre[0] = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      rtot[q] = q < RP ? *reinterpret_cast<const int *>(smem + st_head_lds() + st_row_lds(K) * q +
                                                          (size_t)K * 64 * sizeof(uint32_t) + 64 * sizeof(int))
                       : 0;
      rpre[q + 1] = rpre[q] + rtot[q];
    }
    const int all = rpre[8];
    const float m = a.m;
    const float sx = m / (float)W, sy = m / (float)H;
    constexpr int U = ST_EVAL_U;
    constexpr int S = 64 * ST_WAVES;
    for (int e0 = (int)threadIdx.x; e0 < all; e0 += S * U) {
      int pp[U], kk[U], rr[U], ee[U];
      uint32_t ff[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int g0 = e0 + S * u;
        int r0 = 0;  // the hit's row: last row with rpre <= g0
#pragma unroll
        for (int q = 1; q < 8; q++) r0 += (q < RP && rpre[q] <= g0) ? 1 : 0;
        const int e = g0 - rpre[r0];
        const int *pre_r = reinterpret_cast<const int *>(smem + st_head_lds() + st_row_lds(K) * r0 +
                                                         (size_t)K * 64 * sizeof(uint32_t));
        int lo = 0;  // owner lane p: last lane with s_pre[p] <= e
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
          if (pre_r[lo + st] <= e) lo += st;
        pp[u] = lo;
        kk[u] = e - pre_r[lo];
        rr[u] = r0;
        ee[u] = e;
        const uint32_t *face_r = reinterpret_cast<const uint32_t *>(smem + st_head_lds() + st_row_lds(K) * r0);
        ff[u] = g0 < all ? face_r[sl(kk[u], lo)] : 0u;
        if (kDevStamps && a.dev) ff[u] = min(ff[u], (uint32_t)(F - 1));  // dev ablations leave no face ids
      }
      T v[U][6];
#pragma unroll
      for (int u = 0; u < U; u++) a.src.verts(f0 + ff[u], v[u]);  // all in flight (ff = 0 past the end)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int g0 = e0 + S * u;
        if (g0 < all) {
          const int jr = ty * TILE_H + part * RP + rr[u];
          const T y0 = (T)(sy * (float)(H - 2 * jr - 1));  // == pix_y
          T dsq;
          int edgeid;
          soft_dist<T>((T)(sx * (float)(2 * (ibase + pp[u]) + 1 - W)), y0, v[u], m, dsq, edgeid);
          const T z = (T)a.sigmainv * dsq / (T)m / (T)m;
          const T pr = kl_exp<T>(-z);
          if (slots) {
            const size_t o = (((size_t)b * H + jr) * W + (size_t)(ibase + pp[u])) * K + kk[u];
            a.slot_prob[o] = pr;
            a.slot_idx[o] = (int64_t)ff[u];
            a.slot_type[o] = (uint8_t)(edgeid + 1);
          } else {
            const size_t rb = ((size_t)(b * H + jr) * g.tiles_x + tx) * 64 * (size_t)K;
            a.rec_face[rb + ee[u]] = ff[u] | ((uint32_t)(edgeid + 1) << 28);
            a.rec_prob[rb + ee[u]] = pr;
          }
          T *prob_r = reinterpret_cast<T *>(smem + st_head_lds() + st_row_lds(K) * rr[u]);
          prob_r[sl(kk[u], pp[u])] = pr;
        }
      }
    }
    __syncthreads();
    T *s_prob = reinterpret_cast<T *>(s_face);
    if (qi == 0 && px_valid && kid > 0) {
      // 1 - prod(1 - p) in double, slot order (dibr_soft_mask_cuda.cu:174-182); slots read
      // eight at a time so that their LDS reads overlap
      T allprob = (T)1.0;
      for (int k0 = 0; k0 < kid; k0 += 8) {
        T pk[8];
#pragma unroll
        for (int u = 0; u < 8; u++) pk[u] = s_prob[sl(min(k0 + u, kid - 1), lane)];
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (k0 + u < kid) allprob = (T)((double)allprob * (1.0 - (double)pk[u]));
      }
      a.mask[pix] = (T)(1.0 - (double)allprob);
    }
  } else if (qi == 0) {
    for (int e = lane; e < total; e += 64) {
      int lo = 0;  // owner lane p: last lane with s_pre[p] <= e
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (s_pre[lo + st] <= e) lo += st;
      a.rec_face[rbase + e] = s_face[sl(e - s_pre[lo], lo)];
    }
  }
  if (qi == 0 && (!a.prefilled || total > 0)) {
    if (px_valid && (!a.prefilled || kid > 0)) {
      a.hits[pix] = (uint8_t)kid;
      if (kid == 0) a.mask[pix] = covered ? (T)1.0 : (T)0.0;  // 1 - prod over no slots = 0
    }
    if (row_ok && lane == 0) {
      a.seg_tot[(size_t)(b * H + j) * g.tiles_x + tx] = total;
      a.defer[(size_t)(b * H + j) * g.tiles_x + tx] = inline_eval ? 0 : 1;
    }
  }
  if (a.bwd_items) {  // workgroup-uniform; the rows' totals through LDS (s_wcnt is free by now)
    if (qi == 0 && lane == 0) s_wcnt[r] = total;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int k = 0; k < RP; k++) tot += s_wcnt[k];
      const int n = (tot + SB_PIECE - 1) / SB_PIECE;
      if (n) {
        const int sh = (int)(blockIdx.x & (DS_SHARDS - 1));
        int2 *dst = a.bwd_items + (size_t)sh * a.bwd_cap + atomicAdd(&a.bwd_cnt[sh * DS_CNT_STRIDE], n);
        for (int k = 0; k < n; k++) dst[k] = make_int2(item, k);
      }
    }
  }
  if (dbg && lane == 0) {
    uint64_t *d = dbg + ((size_t)blockIdx.x * ST_WAVES + wid) * 10;
    d[8] = c_fill;
    d[0] = t0;
    d[1] = t1;
    d[2] = stamp_clk();
    d[3] = w0;
    d[4] = stamp_wall();
    d[5] = (uint64_t)total;
    d[6] = ((uint64_t)nchunks << 32) | (uint32_t)(qi | (Q << 8));
    d[7] = ((uint64_t)(uint32_t)j << 32) | (uint32_t)tile;
  }
}

// Evaluation of the selected hits (f64): one wave per row segment (4 per workgroup, tiles in
// grid order), the hits evaluated densely U x 64 at a time with
// their vertex loads in flight together, the reference's per-(pixel, face) distance and
// probability, then 1 - prod(1 - p) in slot order for the pixels with hits.
template <typename T>
__global__ void __launch_bounds__(256) soft_tile_eval_kernel(SoftTileArgs<T> a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int R = blockDim.x >> 6;
  const int K = a.K;
  const BinGeom &g = a.g;
  const int H = g.height, W = g.width;
  unsigned char *mine = smem + ((size_t)K * 64 * sizeof(T) + 64 * sizeof(int)) * wid;
  T *s_prob = reinterpret_cast<T *>(mine);                                  // [K][64]
  int *s_pre = reinterpret_cast<int *>(mine + (size_t)K * 64 * sizeof(T));  // [64]
  const int per_tile = TILE_H / R;
  const int tile = blockIdx.x / per_tile;
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int b = tile / (g.tiles_x * g.tiles_y);
  const int j = ty * TILE_H + (blockIdx.x % per_tile) * R + wid;
  if (j >= H) return;
  if (!a.defer[(size_t)(b * H + j) * g.tiles_x + tx]) return;  // evaluated by the selection kernel
  const int ibase = tx * TILE_W;
  const int i = ibase + lane;
  const bool px_valid = i < W;
  const size_t pix = ((size_t)b * H + j) * W + (px_valid ? i : W - 1);
  const int kid = px_valid ? (int)a.hits[pix] : 0;
  const int pre = wave_incl_scan(kid);
  const int total = __builtin_amdgcn_readlane(pre, 63);
  if (total == 0) return;
  s_pre[lane] = pre - kid;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const float m = a.m;
  const float sx = m / (float)W, sy = m / (float)H;
  const T y0 = (T)(sy * (float)(H - 2 * j - 1));  // == pix_y
  const int64_t f0 = (int64_t)b * a.F;
  const size_t rbase = ((size_t)(b * H + j) * g.tiles_x + tx) * 64 * (size_t)K;
  constexpr int U = 4;
  for (int e0 = lane; e0 < total; e0 += 64 * U) {
    int pp[U], kk[U];
    uint32_t ff[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = e0 + 64 * u;
      int lo = 0;  // owner lane p: last lane with s_pre[p] <= e
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (s_pre[lo + st] <= e) lo += st;
      pp[u] = lo;
      kk[u] = e - s_pre[lo];
      ff[u] = e < total ? a.rec_face[rbase + e] : 0u;
    }
    T v[U][6];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (e0 + 64 * u < total) a.src.verts(f0 + ff[u], v[u]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = e0 + 64 * u;
      if (e < total) {
        T dsq;
        int edgeid;
        soft_dist<T>((T)(sx * (float)(2 * (ibase + pp[u]) + 1 - W)), y0, v[u], m, dsq, edgeid);
        const T z = (T)a.sigmainv * dsq / (T)m / (T)m;
        const T pr = kl_exp<T>(-z);
        a.rec_face[rbase + e] = ff[u] | ((uint32_t)(edgeid + 1) << 28);
        a.rec_prob[rbase + e] = pr;
        s_prob[kk[u] * 64 + pp[u]] = pr;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (kid > 0) {
    // 1 - prod(1 - p) in double, slot order (dibr_soft_mask_cuda.cu:174-182)
    T allprob = (T)1.0;
    for (int k = 0; k < kid; k++) allprob = (T)((double)allprob * (1.0 - (double)s_prob[k * 64 + lane]));
    a.mask[pix] = (T)(1.0 - (double)allprob);
  }
}

// ---------------------------------------------------------------- backward
// Work items of the backward: (forward item code, piece): the hits of a tile's rows (all 8, or a
// part of them) taken row-major in pieces of SB_PIECE (one hit per thread of a workgroup), so that
// the heavy tiles (the silhouette's tight spots, ~10^4 hits) spread over many workgroups.  The
// fused forward (kl_dibr_forward) lists them as it writes the hits (SoftTileArgs::bwd_items,
// DS_SHARDS shards); for the standalone soft mask the plan kernel (one workgroup) lists whole
// tiles from the forward's per-row-segment hit totals.  The backward kernel is persistent and
// takes the items round-robin.

// Block 0 plans; blocks 1.. zero the backward's double accumulator (n doubles) meanwhile -- one
// launch instead of a fill followed by the one-workgroup plan (5.4 + 7.8 us at cfg3).
constexpr int SB_ZERO_BLOCKS = 128;
__global__ void __launch_bounds__(1024) soft_bwd_plan_kernel(const int *__restrict__ seg_tot, BinGeom g,
                                                             int2 *__restrict__ items, int *__restrict__ ctl,
                                                             double *__restrict__ acc, size_t n) {
  __shared__ int s_wave[16];
  if (blockIdx.x > 0) {
    for (size_t i = (blockIdx.x - 1) * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)(gridDim.x - 1) * blockDim.x)
      acc[i] = 0.0;
    return;
  }
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  int carry = 0;
  for (int t0 = 0; t0 < nt; t0 += blockDim.x) {
    const int t = t0 + threadIdx.x;
    int np = 0;
    if (t < nt) {
      const int tx = t % g.tiles_x, ty = (t / g.tiles_x) % g.tiles_y, b = t / (g.tiles_x * g.tiles_y);
      int v[TILE_H];
#pragma unroll
      for (int r = 0; r < TILE_H; r++) {  // the tile's row totals, loads in flight together
        const int j = ty * TILE_H + r;
        v[r] = j < g.height ? seg_tot[((size_t)b * g.height + j) * g.tiles_x + tx] : 0;
      }
      int tot = 0;
#pragma unroll
      for (int r = 0; r < TILE_H; r++) tot += v[r];
      np = (tot + SB_PIECE - 1) / SB_PIECE;
    }
    int all;
    const int excl = carry + block_exclusive_scan(np, s_wave, &all);
    for (int q = 0; q < np; q++) items[excl + q] = make_int2(t, q);  // code = tile: all 8 rows
    carry += all;
  }
  if (threadIdx.x < DS_SHARDS) ctl[threadIdx.x * DS_CNT_STRIDE] = threadIdx.x == 0 ? carry : 0;  // one shard
}

// Per-face accumulation for one work item: LDS hash on the mesh-local face index with
// the list of used slots, so the flush and the reset touch only those.  Sums are in
// double (see FaceHash, soft_common.h): HC = 512 slots keep the workgroup near 34 KB of LDS.
template <typename T, int HC, int NC = 1>
struct ItemHash {
  int *key;     // [HC], -1 = empty
  double *val;  // [HC * NC * SB_VS]: NC copies of a face's sums, copy = lane % NC (fewer lanes of an
                // instruction on one address: a piece's neighbouring hits share faces)
  int *used;    // [HC]
  int *nused;
  __device__ __forceinline__ int slot(int f) {
    unsigned h = ((unsigned)f * 2654435761u) >> (32 - __builtin_ctz(HC));
#pragma unroll 1
    for (int t = 0; t < 32; t++) {
      const int cur = key[h];
      if (cur == f) return (int)h;
      if (cur == -1) {
        const int prev = atomicCAS(&key[h], -1, f);
        if (prev == -1) {
          used[atomicAdd(nused, 1)] = (int)h;
          return (int)h;
        }
        if (prev == f) return (int)h;
      }
      h = (h + 1) & (HC - 1);
    }
    return -1;
  }
  // flags (kl_dibr_backward's soft accumulator, or nullptr): byte f set for every face whose sums
  // this item adds to, so the gather reads (and re-zeroes) only those
  __device__ __forceinline__ void add(int f, int c0, int c1, T g0x, T g0y, T g1x, T g1y, double *gmesh, int ast,
                                      uint8_t *flags) {
    const int s = slot(f);
    if (s >= 0) {
      double *v = val + (s * NC + (int)(threadIdx.x & (NC - 1))) * SB_VS;
      atomicAdd(&v[c0 * 2], (double)g0x);
      atomicAdd(&v[c0 * 2 + 1], (double)g0y);
      if (c1 >= 0) {
        atomicAdd(&v[c1 * 2], (double)g1x);
        atomicAdd(&v[c1 * 2 + 1], (double)g1y);
      }
    } else {  // no free slot within the probe bound
      global_add_pair<double>(gmesh + (size_t)f * ast, c0, c1, g0x, g0y, g1x, g1y);
      if (flags) flags[f] = 1;
    }
  }
  // one thread per (used slot, coordinate), coordinate fastest: a face's 6 sums go out from 6
  // consecutive lanes to 48 contiguous bytes, so a wave's double atomics leave L2 as a few
  // 64-B requests per face instead of one request per lane (memory-side atomics,
  // MI355X_MICROARCH.md: one lane per row is an order of magnitude slower).  Every thread of the
  // workgroup calls it (barrier before the key reset).
  __device__ __forceinline__ void flush_reset(int tid, int nthreads, double *gmesh, int ast, uint8_t *flags) {
    const int n = *nused;
    for (int u = tid; u < n * 6; u += nthreads) {
      const int sl = used[u / 6], c = u % 6;
      double v = 0.0;  // the copies in copy order (each sum is exact: the order does not matter)
#pragma unroll
      for (int k = 0; k < NC; k++) {
        v += val[(sl * NC + k) * SB_VS + c];
        val[(sl * NC + k) * SB_VS + c] = 0.0;
      }
      if (v != 0.0) atomicAdd(gmesh + (size_t)key[sl] * ast + c, v);
      if (c == 0 && flags) flags[key[sl]] = 1;
    }
    __syncthreads();
    for (int u = tid; u < n; u += nthreads) key[used[u]] = -1;
  }
};

// Backward (persistent): one work item (tile, piece) at a time per 512-thread workgroup;
// each wave prepares one row of the tile (filled-slot prefix, the reference's
// a = -sigmainv * dLdp * (1 - allprob)), then every thread takes one hit of the piece:
// its record, the reference's terms (soft_hit_grad), summed per face in the item hash.
template <typename T>
__global__ void __launch_bounds__(512, SB_MIN_WAVES) soft_tile_bwd_kernel(
    const T *__restrict__ grad, const T *__restrict__ mask, const uint8_t *__restrict__ hits,
    const uint32_t *__restrict__ rec_face, const T *__restrict__ rec_prob, const T *__restrict__ fvi, BinGeom g,
    int F, int K, float sigmainv, float multiplier, double *__restrict__ gacc, const int2 *__restrict__ items,
    const int *__restrict__ ctl, int cap, int *__restrict__ scratch, int dev, int ast, uint8_t *__restrict__ sflag) {
  constexpr int HC = SB_HC, NC = SB_NC;
  __shared__ int s_key[HC];
  __shared__ double s_val[HC * NC * SB_VS];
  __shared__ int s_used[HC];
  __shared__ int s_nused;
  __shared__ double s_a[TILE_H][64];
  __shared__ int s_pre[TILE_H][65];
  __shared__ int s_rowpre[TILE_H + 1];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;  // the item's row
  const int H = g.height, W = g.width;
  for (int q = threadIdx.x; q < HC; q += blockDim.x) s_key[q] = -1;
  for (int q = threadIdx.x; q < HC * NC * SB_VS; q += blockDim.x) s_val[q] = 0.0;
  if (threadIdx.x == 0) s_nused = 0;
  if (scratch && threadIdx.x == 0 && blockIdx.x == 0) *scratch = 0;
  ItemHash<T, HC, NC> hash{s_key, s_val, s_used, &s_nused};
  // the shards' item counts (ctl[s * DS_CNT_STRIDE]) and their prefix
  int nsh[DS_SHARDS], nitems = 0;
#pragma unroll
  for (int k = 0; k < DS_SHARDS; k++) {
    nsh[k] = ctl[k * DS_CNT_STRIDE];
    nitems += nsh[k];
  }
  const T ms = (T)multiplier;
  const float sx = multiplier / (float)W, sy = multiplier / (float)H;
  // items are taken round-robin (a claim counter's returning atomic costs more than the
  // imbalance it removes: the items are pieces of at most SB_PIECE hits)
  for (int q = (int)blockIdx.x;; q += (int)gridDim.x) {
    __syncthreads();  // the previous item's hash reset is done
    if (q >= nitems) return;
    // the item's shard and index in it (unrolled over the shards: nsh stays in registers, no scratch)
    int sh = 0, qq = q;
#pragma unroll
    for (int k = 0; k < DS_SHARDS - 1; k++)
      if (sh == k && qq >= nsh[k]) {
        qq -= nsh[k];
        sh = k + 1;
      }
    const int2 it = items[(size_t)sh * cap + qq];
    const int tile = it.x & 0xffffff, part = (it.x >> 24) & 15, lp = (it.x >> 28) & 7;
    const int RP = TILE_H >> lp;  // rows of the item
    const int tx = tile % g.tiles_x, ty = (tile / g.tiles_x) % g.tiles_y, b = tile / (g.tiles_x * g.tiles_y);
    const int j0 = ty * TILE_H + part * RP;
    const int ibase = tx * TILE_W;
    if (wid < RP) {  // row `wid` of the item
      const int j = j0 + wid, i = ibase + lane;
      int kid = 0;
      if (j < H && i < W) {
        const size_t p = ((size_t)b * H + j) * W + i;
        kid = hits[p];
        // the reference's  -1.0 * sigmainv * dLdp * (1.0 - allprob), evaluated left to right
        if (kid) s_a[wid][lane] = -1.0 * (double)sigmainv * (double)grad[p] * (1.0 - (double)mask[p]);
      }
      const int pre = wave_incl_scan(kid);
      s_pre[wid][lane] = pre - kid;
      if (lane == 63) s_rowpre[wid + 1] = pre;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_rowpre[0] = 0;
      for (int r = 1; r <= RP; r++) s_rowpre[r] += s_rowpre[r - 1];
    }
    __syncthreads();
    const int f = it.y * SB_PIECE + (int)threadIdx.x;
    if (f < s_rowpre[RP] && !(dev & 8)) {
      int r = 0;
      for (int k = 1; k < RP; k++) r += s_rowpre[k] <= f ? 1 : 0;
      const int e = f - s_rowpre[r];
      int lo = 0;  // owner lane: last lane with s_pre[r][lo] <= e
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (s_pre[r][lo + st] <= e) lo += st;
      const int j = j0 + r;
      const size_t o = ((size_t)(b * H + j) * g.tiles_x + tx) * 64 * (size_t)K + e;
      const uint32_t rr = rec_face[o];
      const T pr = rec_prob[o];
      const int face = (int)(rr & 0x0fffffffu);
      const int edgeid = (int)(rr >> 28) - 1;
      const T x0 = (T)(sx * (float)(2 * (ibase + lo) + 1 - W));  // == pix_x
      const T y0 = (T)(sy * (float)(H - 2 * j - 1));               // == pix_y
      const T dLdz = (T)(s_a[r][lo] / (1.0 - (double)pr + SM_EPS) * (double)pr);
      const T *fb = fvi + ((size_t)b * F + face) * 6;
      T v[6];
#pragma unroll
      for (int c = 0; c < 6; c++) v[c] = fb[c] * ms;
      int c0, c1;
      T g0x, g0y, g1x, g1y;
      soft_hit_grad<T>(v, edgeid, x0, y0, dLdz, multiplier, c0, c1, g0x, g0y, g1x, g1y);
      if (dev & 2)
        asm volatile("" : : "v"(g0x), "v"(g0y), "v"(g1x), "v"(g1y), "v"(c0), "v"(c1));
      else
        hash.add(face, c0, c1, g0x, g0y, g1x, g1y, gacc + (size_t)b * F * ast, ast,
                 sflag ? sflag + (size_t)b * F : nullptr);
    }
    __syncthreads();
    hash.flush_reset(threadIdx.x, blockDim.x, gacc + (size_t)b * F * ast, ast, sflag ? sflag + (size_t)b * F : nullptr);
    __syncthreads();
    if (threadIdx.x == 0) s_nused = 0;
  }
}

// workspace: bitmap | ghist[32], gdone (zeroed with the bitmap) | tile buckets | work items |
// item count | pixel ranges | defer flags
struct StWs {
  size_t hist, zero, bk, order, nitems, rng, defer, bytes;
  StWs(const BinGeom &g, int F) {
    const size_t nt = (size_t)g.batch * g.tiles_y * g.tiles_x;
    hist = g.bytes();
    zero = hist + (ORD_HIST + 1) * sizeof(int);
    bk = (zero + 255) & ~(size_t)255;
    order = (bk + nt + 255) & ~(size_t)255;
    nitems = order + nt * TILE_H * sizeof(int32_t);
    rng = (nitems + sizeof(int) + 255) & ~(size_t)255;
    defer = (rng + (size_t)g.batch * F * sizeof(uint2) + 255) & ~(size_t)255;
    bytes = defer + (size_t)g.batch * g.height * g.tiles_x;
  }
};

SoftSplit soft_split() {
  SoftSplit sp = ST_SPLIT;
  if (g_dev_param[0]) sp.b4 = g_dev_param[0];
  if (g_dev_param[1]) sp.b8 = g_dev_param[1];
  if (g_dev_param[2]) sp.cap4 = g_dev_param[2];
  if (g_dev_param[3]) sp.cap8 = g_dev_param[3];
  return sp;
}

int soft_lp_min(int K) {
  // the fewest row halvings (at most 4 rows per workgroup) whose slot lists fit in 64 KB of LDS;
  // knum near 255 takes one row per workgroup.  r05z: at knum 30, 2-row items (LDS for 5 workgroups
  // per CU, the kernel's VGPR occupancy at ST_EVAL_U = 2) against these 4-row ones: cfg3 5,609-5,649
  // against 5,618-5,646 Mpixels/s, cfg5 9,394-9,425 against 9,875-9,906 -- kept at 4 rows
  int lp = 1;
  while (lp < 3 && st_head_lds() + (size_t)(TILE_H >> lp) * st_row_lds(K) > 64 * 1024) lp++;
  // dev param 20 = 1..3: that many halvings where the LDS fits 64 KB (A/B)
  const int dp = g_dev_param[20];
  if (dp >= 1 && dp <= 3 && st_head_lds() + (size_t)(TILE_H >> dp) * st_row_lds(K) <= 64 * 1024) lp = dp;
  return lp;
}

template <typename T>
int soft_tile_forward(int B, int H, int W, int F, int K, const T *fvi, const int64_t *sel, float sigmainv, double pad,
                      float m, T *mask, const SoftState<T> &s, void *ws, size_t ws_bytes, hipStream_t st) {
  int *scratch = s.scratch;
  const BinGeom g = make_bin_geom(B, H, W, F);
  const StWs L(g, F);
  KL_REQUIRE(ws_bytes >= L.bytes, "dibr_soft_mask: workspace too small");
  KL_REQUIRE(K >= 0 && K <= 255, "dibr_soft_mask: the compact path needs 0 <= knum <= 255");
  KL_REQUIRE(F < (1 << 28), "dibr_soft_mask: too many faces");
  if ((int64_t)B * H * W == 0) return scratch ? fill_async(scratch, 0, sizeof(int), st) : KL_OK;
  char *w = reinterpret_cast<char *>(ws);
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(w);
  int *ghist = reinterpret_cast<int *>(w + L.hist);
  uint8_t *bk = reinterpret_cast<uint8_t *>(w + L.bk);
  int32_t *order = reinterpret_cast<int32_t *>(w + L.order);
  uint2 *rng = reinterpret_cast<uint2 *>(w + L.rng);
  const SoftSrc<T> src{fvi, (T)m, (T)pad};
  const int rc = launch_binning<T, SoftSrc<T>>(src, nullptr, F, g, m, bitmap, st, nullptr, L.zero, rng);
  if (rc) return rc;
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  int *nitems = reinterpret_cast<int *>(w + L.nitems);
  hipLaunchKernelGGL(tile_bucket_kernel, dim3((unsigned)cdiv(nt, 4)), dim3(256), 0, st, (const uint32_t *)bitmap,
                     g.words, nt, bk, ghist, scratch);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL(soft_order_kernel, dim3(1), dim3(1024), 0, st, (const uint8_t *)bk, (const int *)ghist, nt, order,
                     soft_lp_min(K), nitems, soft_split());
  KL_CHECK_LAUNCH();
  uint8_t *defer = reinterpret_cast<uint8_t *>(w + L.defer);
  return soft_tile_forward_main<T>(B, H, W, F, K, fvi, sel, sigmainv, pad, m, mask, s, bitmap, order, nitems, rng,
                                   defer, st, false, nullptr, nullptr, 0);
}

// The selection and evaluation kernels on bins made by the caller: bitmap (SoftSrc bins),
// work items (order_soft_items with lp_min = soft_lp_min(K)) and their count, and the exact
// pixel ranges of the enlarged bboxes; s.scratch already zeroed.
template <typename T>
int soft_tile_forward_main(int B, int H, int W, int F, int K, const T *fvi, const int64_t *sel, float sigmainv,
                           double pad, float m, T *mask, const SoftState<T> &s, const uint32_t *bitmap,
                           const int32_t *order, const int *nitems, const uint2 *rng, uint8_t *defer,
                           hipStream_t st, bool prefilled, int2 *bwd_items, int *bwd_cnt, int bwd_cap,
                           const uint8_t *live) {
  const BinGeom g = make_bin_geom(B, H, W, F);
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  if (nt == 0) return KL_OK;
  const int lp_min = soft_lp_min(K);
  const size_t lds = st_head_lds() + (size_t)(TILE_H >> lp_min) * st_row_lds(K);
  KL_REQUIRE(lds <= 160 * 1024, "dibr_soft_mask: knum too large for the LDS slot lists");
  const SoftSrc<T> src{fvi, (T)m, (T)pad};
  SoftTileArgs<T> args{src, rng,  sel,    bitmap, order,      nitems,     g,         F,     K,
                       sigmainv, m, mask, s.hits, s.rec_face, s.rec_prob, s.seg_tot, defer, (uint64_t *)g_dev_debug,
                       g_dev_flags, prefilled ? 1 : 0};
  args.bwd_items = bwd_items;
  args.bwd_cnt = bwd_cnt;
  args.bwd_cap = bwd_cap;
  args.swz = g_dev_param[19] == 1 ? 0 : 63;
  args.live = prefilled ? live : nullptr;
  args.live_n = nt * TILE_H;
  hipLaunchKernelGGL((soft_tile_fwd_kernel<T>), dim3((unsigned)soft_items_bound(nt, lp_min, soft_split())), dim3(64 * ST_WAVES), lds,
                     st, args);
  KL_CHECK_LAUNCH();
  if (K > 0 && sizeof(T) != 4) {  // f64: the rows left for the evaluation kernel
    const size_t ew = (size_t)K * 64 * sizeof(T) + 64 * sizeof(int);
    int RE = 4;
    while (RE > 1 && ew * RE > 64 * 1024) RE >>= 1;
    hipLaunchKernelGGL((soft_tile_eval_kernel<T>), dim3((unsigned)(nt * (TILE_H / RE))), dim3(64 * RE), ew * RE, st,
                       args);
    KL_CHECK_LAUNCH();
  }
  return KL_OK;
}

// persistent backward workgroups per CU (dev param 27 overrides; 4 fit by LDS and registers)
static int sb_wgs_per_cu() { return g_dev_param[27] > 0 ? g_dev_param[27] : 3; }

// workspace: item counters (DS_SHARDS, one used) | items | the (B,F,3,2) double accumulator
constexpr size_t SB_CTL_BYTES = DS_SHARDS * DS_CNT_STRIDE * sizeof(int);
static size_t soft_bwd_acc_offset(int B, int H, int W, int K) {
  const BinGeom g = make_bin_geom(B, H, W, 1);
  const size_t nt = (size_t)g.batch * g.tiles_y * g.tiles_x;
  return al256(SB_CTL_BYTES + nt * (size_t)(K + 2) * sizeof(int2));
}

int soft_bwd_item_cap(int B, int H, int W, int K) {
  const BinGeom g = make_bin_geom(B, H, W, 1);
  const int64_t nt = (int64_t)g.batch * g.tiles_y * g.tiles_x;
  const int64_t parts = soft_items_bound((int)nt, soft_lp_min(K), soft_split());
  const int64_t hits = (int64_t)B * H * g.tiles_x * 64 * (K > 0 ? K : 0);
  return (int)(parts + hits / SB_PIECE + 1);
}
size_t soft_tile_bwd_ws_bytes(int B, int H, int W, int F, int K) {
  return soft_bwd_acc_offset(B, H, W, K) + al256((size_t)B * F * 6 * sizeof(double));
}

// acc_out == nullptr: the sums are rounded into gfvi (overwritten, or added with accumulate);
// otherwise they are left in acc_out (B*F*6 doubles, zeroed here; gfvi unused) for a caller
// that rounds them itself (kl_dibr_backward's gather) -- *has_sum tells whether any was made.
template <typename T>
int soft_tile_backward(int B, int H, int W, int F, int K, const T *grad, const T *mask, const SoftState<T> &s,
                       const T *fvi, float sigmainv, float m, T *gfvi, bool accumulate, void *ws, size_t ws_bytes,
                       hipStream_t st, double *acc_out, bool *has_sum) {
  KL_REQUIRE(F < (1 << 28), "dibr_soft_mask backward: too many faces");
  const size_t n = (size_t)B * F * 6;
  if (has_sum) *has_sum = false;
  if ((int64_t)B * H * W == 0 || K <= 0 || grad == nullptr || n == 0) {
    if (!accumulate && !acc_out) KL_CHECK_RC(fill_async(gfvi, 0, sizeof(T) * n, st));
    return s.scratch ? fill_async(s.scratch, 0, sizeof(int), st) : KL_OK;
  }
  KL_REQUIRE(ws_bytes >= (acc_out ? soft_bwd_acc_offset(B, H, W, K) : soft_tile_bwd_ws_bytes(B, H, W, F, K)),
             "dibr_soft_mask backward: workspace too small");
  const BinGeom g = make_bin_geom(B, H, W, F);
  int *ctl = reinterpret_cast<int *>(ws);
  int2 *items = reinterpret_cast<int2 *>(reinterpret_cast<char *>(ws) + SB_CTL_BYTES);
  double *acc = acc_out ? acc_out
                        : reinterpret_cast<double *>(reinterpret_cast<char *>(ws) + soft_bwd_acc_offset(B, H, W, K));
  hipLaunchKernelGGL(soft_bwd_plan_kernel, dim3(1 + SB_ZERO_BLOCKS), dim3(1024), 0, st, (const int *)s.seg_tot, g,
                     items, ctl, acc, n);
  KL_CHECK_LAUNCH();
  int dev_id = 0, ncu = 256;
  if (hipGetDevice(&dev_id) == hipSuccess)
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev_id);
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  const unsigned grid = (unsigned)std::max(1, std::min(nt * (K + 1), ncu * sb_wgs_per_cu()));
  hipLaunchKernelGGL((soft_tile_bwd_kernel<T>), dim3(grid), dim3(512), 0, st, grad, mask, (const uint8_t *)s.hits,
                     (const uint32_t *)s.rec_face, (const T *)s.rec_prob, fvi, g, F, K, sigmainv, m, acc,
                     (const int2 *)items, (const int *)ctl, 0, s.scratch, g_dev_flags, 6, (uint8_t *)nullptr);
  KL_CHECK_LAUNCH();
  if (acc_out) {
    if (has_sum) *has_sum = true;
    return KL_OK;
  }
  return acc_finalize<T>(acc, gfvi, n, accumulate, st);
}
size_t soft_tile_bwd_items_bytes(int B, int H, int W, int K) { return soft_bwd_acc_offset(B, H, W, K); }

template <typename T>
int soft_tile_backward_listed(int B, int H, int W, int F, int K, const T *grad, const T *mask, const SoftState<T> &s,
                              const T *fvi, float sigmainv, float m, const int2 *items, const int *cnt, int cap,
                              double *acc, uint8_t *sflag, hipStream_t st) {
  if ((int64_t)B * H * W == 0 || K <= 0 || grad == nullptr || (int64_t)B * F == 0) return KL_OK;
  const BinGeom g = make_bin_geom(B, H, W, F);
  int dev_id = 0, ncu = 256;
  if (hipGetDevice(&dev_id) == hipSuccess)
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev_id);
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  const unsigned grid = (unsigned)std::max(1, std::min(nt * (K + 1), ncu * sb_wgs_per_cu()));
  hipLaunchKernelGGL((soft_tile_bwd_kernel<T>), dim3(grid), dim3(512), 0, st, grad, mask, (const uint8_t *)s.hits,
                     (const uint32_t *)s.rec_face, (const T *)s.rec_prob, fvi, g, F, K, sigmainv, m, acc, items, cnt,
                     cap, (int *)nullptr, g_dev_flags, DS_ACC_STRIDE, sflag);
  KL_CHECK_LAUNCH();
  return KL_OK;
}
template int soft_tile_backward_listed<float>(int, int, int, int, int, const float *, const float *,
                                              const SoftState<float> &, const float *, float, float, const int2 *,
                                              const int *, int, double *, uint8_t *, hipStream_t);
template int soft_tile_backward_listed<double>(int, int, int, int, int, const double *, const double *,
                                               const SoftState<double> &, const double *, float, float, const int2 *,
                                               const int *, int, double *, uint8_t *, hipStream_t);

template int soft_tile_forward<float>(int, int, int, int, int, const float *, const int64_t *, float, double, float,
                                      float *, const SoftState<float> &, void *, size_t, hipStream_t);
template int soft_tile_forward<double>(int, int, int, int, int, const double *, const int64_t *, float, double,
                                       float, double *, const SoftState<double> &, void *, size_t, hipStream_t);
template int soft_tile_forward_main<float>(int, int, int, int, int, const float *, const int64_t *, float, double,
                                           float, float *, const SoftState<float> &, const uint32_t *,
                                           const int32_t *, const int *, const uint2 *, uint8_t *, hipStream_t,
                                           bool, int2 *, int *, int, const uint8_t *);
template int soft_tile_forward_main<double>(int, int, int, int, int, const double *, const int64_t *, float, double,
                                            float, double *, const SoftState<double> &, const uint32_t *,
                                            const int32_t *, const int *, const uint2 *, uint8_t *, hipStream_t,
                                            bool, int2 *, int *, int, const uint8_t *);
template int soft_tile_backward<float>(int, int, int, int, int, const float *, const float *,
                                       const SoftState<float> &, const float *, float, float, float *, bool, void *,
                                       size_t, hipStream_t, double *, bool *);
template int soft_tile_backward<double>(int, int, int, int, int, const double *, const double *,
                                        const SoftState<double> &, const double *, float, float, double *, bool,
                                        void *, size_t, hipStream_t, double *, bool *);

size_t soft_tile_ws_bytes(int B, int H, int W, int F) { return StWs(make_bin_geom(B, H, W, F), F).bytes; }

// ---- The _C contract soft-mask forward on the tile machinery (r06; kl_dibr_soft_mask_forward, f32,
// knum <= 255).  The reference's dibr_soft_mask_forward_cuda writes, per pixel, knum slots of prob /
// idx / type -- 13 B x knum, 409 MB at cfg3, ~97 % of it padding.  softmask.hip's kernel walks every
// row with ONE wave (a heavy pole row takes the whole kernel's time on its own, 140 us at cfg3); here
// the caller's bboxes go through the same binning, heavy-first item order and multi-wave rows as the
// compact path, and the kernel stores the slot tensors directly (SoftTileArgs::slot_*).  Workspace:
// the compact path's (StWs) + hits (B*H*W bytes) + segment totals; no compact records.
struct StSlotWs {
  size_t hits, seg, scratch, whist, tk, bytes;
  StSlotWs(int B, int H, int W, int F) {
    const BinGeom g = make_bin_geom(B, H, W, F);
    hits = al256(StWs(g, F).bytes);
    seg = hits + al256((size_t)B * H * W);
    scratch = seg + al256((size_t)B * H * g.tiles_x * sizeof(int));
    // (r06) the chip order kernel's per-workgroup histograms and its tickets (zeroed by the binning)
    whist = scratch + 256;
    tk = whist + al256((size_t)cdiv((int64_t)g.batch * g.tiles_y * g.tiles_x, CO_THREADS) * ORD_HIST * sizeof(int));
    bytes = tk + 256;
  }
};

// (r06) The caller's bboxes binned without global atomics and without a zero fill (raster_bin_word_kernel's
// scheme, soft bitmap only): workgroup (grp, b) bins mesh b's faces [512 grp, 512 grp + 512) -- 8 chunks,
// one byte of every tile's bitmap word -- marking its tiles in LDS (8 mark bytes per tile) with the exact
// pixel ranges of bin_faces_kernel, then stores that byte of every tile.  zero: ints zeroed by workgroup
// (0, 0).
constexpr int ST_BIN_THREADS = 512;
inline bool st_bin_word_ok(const BinGeom &g) { return (size_t)g.tiles_x * g.tiles_y * 8 <= 64 * 1024; }
__global__ void __launch_bounds__(ST_BIN_THREADS) bbox_bin_word_kernel(BboxSrc<float> src, int F, BinGeom g, float m,
                                                                      uint32_t *__restrict__ bitmap,
                                                                      uint2 *__restrict__ rng, int *__restrict__ zero,
                                                                      int nzero) {
  extern __shared__ uint32_t s_words[];
  const int ntv = g.tiles_x * g.tiles_y;
  const int grp = blockIdx.x, b = blockIdx.y;
  if (grp == 0 && b == 0)
    for (int t = threadIdx.x; t < nzero; t += blockDim.x) zero[t] = 0;
  uint8_t *ms = reinterpret_cast<uint8_t *>(s_words);  // [tile][8] mark bytes
  for (int t = threadIdx.x; t < 2 * ntv; t += blockDim.x) s_words[t] = 0;
  __syncthreads();
  const int fl = grp * ST_BIN_THREADS + (int)threadIdx.x;
  if (fl < F) {
    const int64_t f = (int64_t)b * F + fl;
    float bx0, by0, bx1, by1;
    src.get(f, bx0, by0, bx1, by1);
    const float sx = m / (float)g.width, sy = m / (float)g.height;
    int ix0, ix1, iy0, iy1;
    exact_range(bx0, bx1, sx, (float)g.width / m, g.width, false, ix0, ix1);
    exact_range(by0, by1, sy, (float)g.height / m, g.height, true, iy0, iy1);
    const bool e = ix0 > ix1 || iy0 > iy1;
    rng[f] = e ? make_uint2(1u, 1u) : make_uint2((uint32_t)ix0 | ((uint32_t)ix1 << 16), (uint32_t)iy0 | ((uint32_t)iy1 << 16));
    if (!e) {
      const int w = (fl >> 6) & 7;
      for (int ty = iy0 / TILE_H; ty <= iy1 / TILE_H; ty++)
        for (int tx = ix0 / TILE_W; tx <= ix1 / TILE_W; tx++) ms[(ty * g.tiles_x + tx) * 8 + w] = 1;
    }
  }
  __syncthreads();
  const size_t base = (size_t)b * ntv;
  const int word = grp >> 2, byte = grp & 3;
  uint8_t *sb = reinterpret_cast<uint8_t *>(bitmap);
  for (int t = threadIdx.x; t < ntv; t += blockDim.x)
    sb[bm_index(g.ntiles(), base + t, word) * 4 + byte] =
        (uint8_t)((reinterpret_cast<const uint64_t *>(ms)[t] * 0x0102040810204080ull) >> 56);
}

// (dev param 31 = 1: the r06e preamble -- atomic binning, bucket and one-workgroup order kernels -- for A/B)
size_t soft_tile_slots_ws_bytes(int B, int H, int W, int F) { return StSlotWs(B, H, W, F).bytes; }

int soft_tile_forward_slots(int B, int H, int W, int F, int K, const float *fvi, const float *bbox, const int64_t *sel,
                            float sigmainv, float m, float *mask, float *prob, int64_t *cidx, uint8_t *ctype, void *ws,
                            size_t ws_bytes, hipStream_t st) {
  const BinGeom g = make_bin_geom(B, H, W, F);
  const StWs L(g, F);
  const StSlotWs SL(B, H, W, F);
  KL_REQUIRE(ws_bytes >= SL.bytes, "dibr_soft_mask_forward: workspace too small");
  KL_REQUIRE(K >= 0 && K <= 255 && F < (1 << 28), "dibr_soft_mask_forward: tile path needs knum <= 255");
  if ((int64_t)B * H * W == 0) return KL_OK;
  char *w = reinterpret_cast<char *>(ws);
  uint32_t *bitmap = reinterpret_cast<uint32_t *>(w);
  int *ghist = reinterpret_cast<int *>(w + L.hist);
  uint8_t *bk = reinterpret_cast<uint8_t *>(w + L.bk);
  int32_t *order = reinterpret_cast<int32_t *>(w + L.order);
  uint2 *rng = reinterpret_cast<uint2 *>(w + L.rng);
  int *nitems = reinterpret_cast<int *>(w + L.nitems);
  int *scratch = reinterpret_cast<int *>(w + SL.scratch);
  const BboxSrc<float> src{bbox, fvi};
  const int nt = g.batch * g.tiles_y * g.tiles_x;
  const int lp_min = soft_lp_min(K);
  const int nb = (int)cdiv(nt, CO_THREADS);
  if (nt <= ORD_LDS_TILES && st_bin_word_ok(g) && g_dev_param[31] != 1 && chip_order_resident(nb)) {
    // (r06) word binning + the chip-wide order kernel on the soft bitmap alone: 12.4 + ~7 us against the
    // r06e chain's atomic binning (with its zero fill), bucket and one-workgroup order kernels (12.7 +
    // 4.8 + 7.9 us)
    unsigned *tk = reinterpret_cast<unsigned *>(w + SL.tk);
    hipLaunchKernelGGL(bbox_bin_word_kernel, dim3((unsigned)(g.words * 4), (unsigned)g.batch), dim3(ST_BIN_THREADS),
                       (size_t)g.tiles_x * g.tiles_y * 8, st, src, F, g, m, bitmap, rng, reinterpret_cast<int *>(tk), 16);
    KL_CHECK_LAUNCH();
    CountOrderArgs ca{};
    ca.bm[0] = ca.bm[1] = bitmap;
    ca.words = g.words;
    ca.nt = nt;
    ca.nb = nb;
    ca.whist[0] = ca.whist[1] = reinterpret_cast<int *>(w + SL.whist);
    ca.ticket = tk;
    ca.order[0] = ca.order[1] = order;
    ca.nitems[0] = ca.nitems[1] = nitems;
    ca.lp_min1 = lp_min;
    ca.skip_empty1 = 0;  // every tile gets its item: the kernel writes every pixel's slots and mask
    ca.noband = 2;       // plain heaviest-first (as kl_dibr_forward's soft items)
    ca.sp = soft_split();
    ca.only1 = 1;
    hipLaunchKernelGGL(tile_countorder_chip_kernel, dim3((unsigned)(nb + 1)), dim3(CO_THREADS),
                       (size_t)nb * ORD_HIST * sizeof(int), st, ca);
    KL_CHECK_LAUNCH();
  } else {
    KL_CHECK_RC((launch_binning<float, BboxSrc<float>>(src, nullptr, F, g, m, bitmap, st, nullptr, L.zero, rng)));
    hipLaunchKernelGGL(tile_bucket_kernel, dim3((unsigned)cdiv(nt, 4)), dim3(256), 0, st, (const uint32_t *)bitmap,
                       g.words, nt, bk, ghist, scratch);
    KL_CHECK_LAUNCH();
    hipLaunchKernelGGL(soft_order_kernel, dim3(1), dim3(1024), 0, st, (const uint8_t *)bk, (const int *)ghist, nt,
                       order, lp_min, nitems, soft_split());
    KL_CHECK_LAUNCH();
  }
  const size_t lds = st_head_lds() + (size_t)(TILE_H >> lp_min) * st_row_lds(K);
  KL_REQUIRE(lds <= 160 * 1024, "dibr_soft_mask: knum too large for the LDS slot lists");
  SoftTileArgs<float, BboxSrc<float>> a{};
  a.src = src;
  a.rng = rng;
  a.sel = sel;
  a.bitmap = bitmap;
  a.order = order;
  a.nitems = nitems;
  a.g = g;
  a.F = F;
  a.K = K;
  a.sigmainv = sigmainv;
  a.m = m;
  a.mask = mask;
  a.hits = reinterpret_cast<uint8_t *>(w + SL.hits);
  a.rec_face = nullptr;
  a.rec_prob = nullptr;  // (slot mode: the mask reads the probabilities from the LDS slots, as r05)
  a.seg_tot = reinterpret_cast<int *>(w + SL.seg);
  a.defer = reinterpret_cast<uint8_t *>(w + L.defer);
  a.dbg = (uint64_t *)g_dev_debug;
  a.dev = g_dev_flags;
  a.prefilled = 0;
  a.swz = g_dev_param[19] == 1 ? 0 : 63;
  a.slot_prob = prob;
  a.slot_idx = cidx;
  a.slot_type = ctype;
  const dim3 grid((unsigned)soft_items_bound(nt, lp_min, soft_split()));
  hipLaunchKernelGGL((soft_tile_fwd_kernel<float, BboxSrc<float>>), grid, dim3(64 * ST_WAVES), lds, st, a);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_soft_mask_compact_workspace_bytes(int batch, int height, int width, int num_faces) {
  return soft_tile_ws_bytes(batch, height, width, num_faces);
}

extern "C" size_t kl_soft_mask_compact_records(int batch, int height, int width, int knum) {
  return (size_t)batch * height * cdiv(width, TILE_W) * TILE_W * (size_t)(knum > 0 ? knum : 0);
}

extern "C" size_t kl_soft_mask_compact_segments(int batch, int height, int width) {
  return (size_t)batch * height * cdiv(width, TILE_W);
}

extern "C" size_t kl_soft_mask_compact_bwd_workspace_bytes(int batch, int height, int width, int num_faces,
                                                         int knum) {
  return soft_tile_bwd_ws_bytes(batch, height, width, num_faces, knum);
}

extern "C" int kl_dibr_soft_mask_forward_compact(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                                 int knum, const void *fvi, const int64_t *sel, float sigmainv,
                                                 double pad, float multiplier, void *mask, uint8_t *hits,
                                                 uint32_t *rec_face, void *rec_prob, int *seg_tot, int *scratch,
                                                 void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32)
    return soft_tile_forward<float>(batch, height, width, num_faces, knum, (const float *)fvi, sel, sigmainv, pad,
                                    multiplier, (float *)mask,
                                    SoftState<float>{hits, rec_face, (float *)rec_prob, seg_tot, scratch}, ws,
                                    ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_tile_forward<double>(batch, height, width, num_faces, knum, (const double *)fvi, sel, sigmainv, pad,
                                     multiplier, (double *)mask,
                                     SoftState<double>{hits, rec_face, (double *)rec_prob, seg_tot, scratch}, ws,
                                     ws_bytes, S(stream));
  set_error("dibr_soft_mask not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_dibr_soft_mask_backward_compact(kl_dtype dtype, int batch, int height, int width, int num_faces,
                                                  int knum, const void *grad, const void *mask, const uint8_t *hits,
                                                  const uint32_t *rec_face, const void *rec_prob, const int *seg_tot,
                                                  const void *fvi, float sigmainv, float multiplier, void *gfvi,
                                                  int accumulate, int *scratch, void *ws, size_t ws_bytes,
                                                  kl_stream stream) {
  if (dtype == KL_F32)
    return soft_tile_backward<float>(
        batch, height, width, num_faces, knum, (const float *)grad, (const float *)mask,
        SoftState<float>{(uint8_t *)hits, (uint32_t *)rec_face, (float *)rec_prob, (int *)seg_tot, scratch},
        (const float *)fvi, sigmainv, multiplier, (float *)gfvi, accumulate != 0, ws, ws_bytes, S(stream));
  if (dtype == KL_F64)
    return soft_tile_backward<double>(
        batch, height, width, num_faces, knum, (const double *)grad, (const double *)mask,
        SoftState<double>{(uint8_t *)hits, (uint32_t *)rec_face, (double *)rec_prob, (int *)seg_tot, scratch},
        (const double *)fvi, sigmainv, multiplier, (double *)gfvi, accumulate != 0, ws, ws_bytes, S(stream));
  set_error("dibr_soft_mask backward not implemented for this dtype");
  return KL_E_INVALID;
}
