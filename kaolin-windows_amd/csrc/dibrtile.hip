// dibrtile.hip -- dibr_rasterization's forward (f32) as ONE tile kernel: the rasterizer and the
// compact soft mask of a part of a 64x8 tile's rows in one 4-wave workgroup, over ONE expansion
// of the tile's candidate chunks (the fused path of kl_dibr_forward).
//
// The soft mask's candidates (every face whose enlarged bbox reaches the tile: the soft bins,
// dibr.py:31-39) are a superset of the rasterizer's (valid faces whose bbox reaches it,
// rasterization.py:337-344): the enlarged bbox contains the bbox whenever boxlen >= 0, and the
// float subtraction / addition of the pad is monotone.  So one walk over the soft bins serves
// both, in the reference's face order:
//   1. steps of 4 candidate chunks (one per wave; the faces' records and both exact ranges
//      loaded a step ahead): faces whose exact pixel range touches the item's rows go to the
//      step's rasterizer list (with their records) and, by their enlarged range, to the item's
//      soft list (kept in LDS for step 3); the rows then rank the step's (pixel, face) pairs in
//      per-pixel depth keys -- raster_tile_kernel's f32 pair walk (raster.hip);
//   2. each pixel's winner -> face_idx, weights, features; uncovered pixels are the soft mask's;
//   3. the soft walk (soft_tile_fwd_kernel, softtile.hip) over the soft list (over a second
//      expansion of the chunks if the list overflowed), the hits' evaluation, records and mask;
//   4. the backward's work items are listed (SoftTileArgs::bwd_items).
// Each stage is the two-kernel path's arithmetic in the same order, so the outputs equal it bit
// for bit (tests/test_gpu_parity.py); what is gone is the second chunk expansion, the
// rasterizer's own bins / order / launch, and the soft mask's read of face_idx.
#include "dibrtile.h"
#include "rastcommon.h"
#include "tilewalk.h"

#if KL_DEV  // the whole fused tile kernel: built into the dev library only (make dev)
namespace kl {

constexpr int DT_WAVES = 4;
constexpr int DT_STEP = DT_WAVES * 64;  // rasterizer list entries per step: one chunk per wave
constexpr int DT_VS = 12;               // LDS stride of a rasterizer entry: 6 coordinates, 3 depths, pad
constexpr int DT_LCAP = 960;            // soft list entries kept from the expansion

// LDS: head (counts, masks, the multi-wave walk's per-round counts) | soft list |
//      union(step buffers + depth keys ; the rows' slot lists)
constexpr size_t DT_HEAD = 128 + DT_WAVES * 64 * sizeof(int);
constexpr size_t DT_UNI = DT_HEAD + (size_t)DT_LCAP * 8;
constexpr size_t DT_STEP_BYTES = (size_t)DT_STEP * 8 + (size_t)DT_STEP * DT_VS * 4 + DT_WAVES * 64 * 4 +
                                 DT_WAVES * 64 * 8;
// LDS bytes for items of at most 8 >> lp_min rows
inline size_t dt_lds_bytes(int K, int lp_min) {
  const size_t rows = (size_t)(TILE_H >> lp_min) * st_row_lds(K);
  return DT_UNI + (rows > DT_STEP_BYTES ? rows : DT_STEP_BYTES);
}
// fewest rows per item (lp >= 1) whose LDS lets 4 workgroups share a CU; knum near 255: 1 row
int dt_lp_min(int K) {
  int lp = 1;
  while (lp < 3 && dt_lds_bytes(K, lp) > 40 * 1024) lp++;
  return lp;
}


__global__ void __launch_bounds__(256) dibr_tile_kernel(DibrTileArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  if ((int)blockIdx.x >= *a.nitems) return;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const BinGeom &g = a.g;
  const int H = g.height, W = g.width, F = a.F, K = a.K;
  const int item = a.items[blockIdx.x];
  const int tile = item & 0xffffff, part = (item >> 24) & 15, lp = (item >> 28) & 7;
  const int RP = TILE_H >> lp;      // rows of this item (lp >= 1: RP <= 4)
  const int Q = DT_WAVES / RP;      // waves per row
  const int r = wid / Q, qi = wid - r * Q;
  int *s_cnt = reinterpret_cast<int *>(smem);                                      // [4] per-wave counts
  unsigned long long *s_nan = reinterpret_cast<unsigned long long *>(smem + 32);   // [4] NaN-depth pixels
  unsigned long long *s_cov = reinterpret_cast<unsigned long long *>(smem + 64);   // [4] covered pixels
  uint32_t *SL_face = reinterpret_cast<uint32_t *>(smem + DT_HEAD);
  uint32_t *SL_pack = SL_face + DT_LCAP;
  unsigned char *U = smem + DT_UNI;
  uint32_t *L_face = reinterpret_cast<uint32_t *>(U);
  uint32_t *L_pack = L_face + DT_STEP;
  float *L_v = reinterpret_cast<float *>(L_pack + DT_STEP);
  int *s_pre = reinterpret_cast<int *>(L_v + DT_STEP * DT_VS);                           // [4][64]
  unsigned long long *s_key = reinterpret_cast<unsigned long long *>(s_pre + DT_WAVES * 64);  // [4][64]
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int b = tile / (g.tiles_x * g.tiles_y);
  const int j0 = ty * TILE_H + part * RP;  // the item's first row
  const int j = j0 + r;
  const bool row_ok = j < H;
  const int ibase = tx * TILE_W;
  const int i = ibase + lane;
  const bool px_valid = row_ok && i < W;
  const size_t pix = ((size_t)b * H + (row_ok ? j : H - 1)) * W + (i < W ? i : W - 1);
  const float m = a.m;
  const float sx = m / (float)W, sy = m / (float)H;
  const float x0 = sx * (float)(2 * i + 1 - W);                        // == pix_x<float>(m, W, i)
  const float y0 = sy * (float)(H - 2 * (row_ok ? j : H - 1) - 1);     // == pix_y<float>(m, H, j)
  const int64_t f0 = (int64_t)b * F;
  const float *rec = a.rec + f0 * RT_REC;
  const uint2 *rng = a.rng + f0;
  const uint2 *srng = a.srng + f0;
  if ((int)threadIdx.x < RP * 64) s_key[threadIdx.x] = 0;
  if ((int)threadIdx.x < DT_WAVES) s_nan[threadIdx.x] = 0;
  __syncthreads();

  // ---- 1. one expansion of the candidate chunks: rasterizer steps + the soft list
  ChunkSeq seq;
  seq.init(a.bitmap + tile, g.words, g.ntiles(), lane);
  struct Pref {
    float v[9];
    uint2 r, s;
    int c;
  };
  int pos = 0;
  bool more = false;
  auto issue = [&](Pref &P) {
    more = seq.at(pos, lane) >= 0;
    P.c = more ? seq.at(pos + wid, lane) : -1;
    pos += DT_WAVES;
    // unconditional loads from a clamped index: a guarded load would be waited for at once
    int fl = P.c * 64 + lane;
    fl = fl < 0 ? 0 : (fl < F ? fl : F - 1);
#pragma unroll
    for (int q = 0; q < 9; q++) P.v[q] = rec[(size_t)fl * RT_REC + q];
    P.r = rng[fl];
    P.s = srng[fl];
  };
  // a face's exact range against the item's rows and the tile's columns: row bits, lane interval
  auto clip = [&](uint2 rr, uint32_t &rows, int &lo, int &hi) {
    const int ix0 = (int)(rr.x & 0xffffu), ix1 = (int)(rr.x >> 16);
    const int iy0 = (int)(rr.y & 0xffffu), iy1 = (int)(rr.y >> 16);
    const int ya = max(iy0, j0) - j0, yb = min(iy1, j0 + RP - 1) - j0;
    rows = ya <= yb ? ((2u << yb) - 1u) & ~((1u << ya) - 1u) : 0u;
    lo = max(ix0 - ibase, 0);
    hi = min(ix1 - ibase, 63);
  };
  int slen = 0;  // soft candidates seen (the list keeps the first DT_LCAP)
  auto step = [&](Pref &cur, Pref &nxt) {
    const int c = cur.c;
    issue(nxt);
    const int fl = c * 64 + lane;
    const bool live = c >= 0 && fl < F;
    uint32_t rrows, srows;
    int rlo, rhi, slo, shi;
    clip(cur.r, rrows, rlo, rhi);
    clip(cur.s, srows, slo, shi);
    const bool rkeep = live && rrows != 0 && rlo <= rhi;
    const bool skeep = live && srows != 0 && slo <= shi;
    const uint64_t rkm = ballot(rkeep), skm = ballot(skeep);
    if (lane == 0) s_cnt[wid] = __popcll(rkm) | (__popcll(skm) << 16);
    __syncthreads();
    int rpre = 0, rlen = 0, spre = 0, stot = 0;
#pragma unroll
    for (int w = 0; w < DT_WAVES; w++) {
      const int v = s_cnt[w];
      rpre += w < wid ? (v & 0xffff) : 0;
      rlen += v & 0xffff;
      spre += w < wid ? (v >> 16) : 0;
      stot += v >> 16;
    }
    if (rkeep) {
      const int p = rpre + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(rkm >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)rkm, 0u));
      L_face[p] = (uint32_t)fl;
      L_pack[p] = (uint32_t)rlo | ((uint32_t)rhi << 6) | (rrows << 12);
#pragma unroll
      for (int q = 0; q < 9; q++) L_v[p * DT_VS + q] = cur.v[q];
    }
    if (skeep) {
      const int p = slen + spre + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(skm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)skm, 0u));
      if (p < DT_LCAP) {
        SL_face[p] = (uint32_t)fl;
        SL_pack[p] = (uint32_t)slo | ((uint32_t)shi << 6) | (srows << 12);
      }
    }
    slen += stot;
    __syncthreads();
    if (a.dev >= 2) {
      __syncthreads();
      return;
    }
    // this row's (pixel, face) pairs of the step, 64 entries at a time, evaluated densely by the
    // row's Q waves: pair t belongs to the entry whose exclusive width prefix is the last <= t.
    // Each pair ranks its depth in the pixel's key (max depth, lowest index on ties: the
    // reference's strict fold for non-NaN depths); a NaN depth flags the pixel for the replay.
    for (int base = 0; base < rlen; base += 64) {
      const int e = base + lane;
      int lo = 0, wdt = 0;
      if (e < rlen) {
        const uint32_t pk = L_pack[e];
        if ((pk >> (12 + r)) & 1u) {
          lo = (int)(pk & 63u);
          wdt = (int)((pk >> 6) & 63u) - lo + 1;
        }
      }
      int inc = wdt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
      }
      const int total = __shfl(inc, 63);
      if (total == 0) continue;
      s_pre[wid * 64 + lane] = ((inc - wdt) << 8) | lo;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (int t = lane + 64 * qi; t < total; t += 64 * Q) {
        int q = 0;  // owner entry: last q with prefix <= t
#pragma unroll
        for (int stp = 32; stp > 0; stp >>= 1)
          if ((s_pre[wid * 64 + q + stp] >> 8) <= t) q += stp;
        const int pq = s_pre[wid * 64 + q];
        const int px = (pq & 255) + t - (pq >> 8);
        const float *v = L_v + (base + q) * DT_VS;
        const float xp = sx * (float)(2 * (ibase + px) + 1 - W);
        float w0, w1, w2;
        if (!tri_weights<float>(v, xp, y0, a.eps, w0, w1, w2)) continue;
        const float z0 = w0 * v[6] + w1 * v[7] + w2 * v[8];
        if (z0 != z0)
          atomicOr(&s_nan[r], 1ull << px);
        else if (z0 != -INFINITY)
          atomicMax(&s_key[r * 64 + px], ((unsigned long long)order32(z0) << 32) |
                                               (unsigned long long)(~L_face[base + q]));
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    __syncthreads();  // the step buffers are rewritten by the next step
  };
  Pref PA, PB;
  issue(PA);
  while (more) {
    step(PA, PB);
    if (!more) break;
    step(PB, PA);
  }
  if (a.dev == 3) return;

  // ---- 2. the rasterizer's outputs; the covered pixels of each row
  int win = -1;
  if (qi == 0 && px_valid) {
    float mw0 = 0, mw1 = 0, mw2 = 0;
    const unsigned long long key = s_key[r * 64 + lane];
    if ((s_nan[r] >> lane) & 1ull) {
      // a NaN depth breaks the total order: replay the reference's fold over every face
      float max_z0 = -INFINITY;
      for (int f = 0; f < F; f++) {
        const uint2 rr = rng[f];  // exact bbox test (and validity)
        if (i < (int)(rr.x & 0xffffu) || i > (int)(rr.x >> 16) || j < (int)(rr.y & 0xffffu) ||
            j > (int)(rr.y >> 16))
          continue;
        const float *v = rec + (size_t)f * RT_REC;
        float w0, w1, w2;
        if (!tri_weights<float>(v, x0, y0, a.eps, w0, w1, w2)) continue;
        const float z0 = w0 * v[6] + w1 * v[7] + w2 * v[8];
        if (z0 <= max_z0) continue;
        max_z0 = z0;
        win = f;
        mw0 = w0;
        mw1 = w1;
        mw2 = w2;
      }
    } else if (key != 0) {
      win = (int)(~(uint32_t)key);
      tri_weights<float>(rec + (size_t)win * RT_REC, x0, y0, a.eps, mw0, mw1, mw2);  // the arithmetic that ranked it
    }
    const int D = a.D;
    a.out_idx[pix] = win;
    a.out_w[pix * 3 + 0] = mw0;
    a.out_w[pix * 3 + 1] = mw1;
    a.out_w[pix * 3 + 2] = mw2;
    if (win >= 0) {
      const float *c = a.feat + (size_t)(f0 + win) * 3 * D;
      for (int d = 0; d < D; d++) a.out_feat[pix * D + d] = mw0 * c[d] + mw1 * c[D + d] + mw2 * c[2 * D + d];
    } else {
      for (int d = 0; d < D; d++) a.out_feat[pix * D + d] = 0.0f;
    }
  }
  if (qi == 0) {
    const uint64_t cm = ballot(!px_valid || win >= 0);
    if (lane == 0) s_cov[r] = cm;
  }
  __syncthreads();  // s_cov written; the step buffers and keys are dead from here on
  if (a.dev == 1) return;

  // ---- 3. the soft mask's selection: per row, the first knum candidates (index order) of each
  //         uncovered pixel, over the soft list (softtile.hip, soft_tile_fwd_kernel 1b)
  const bool covered = (s_cov[r] >> lane) & 1ull;
  unsigned char *rowmem = U + st_row_lds(K) * r;
  uint32_t *s_face = reinterpret_cast<uint32_t *>(rowmem);                            // [K][64]
  int *s_rpre = reinterpret_cast<int *>(rowmem + (size_t)K * 64 * sizeof(uint32_t));  // [64], then total
  int kid = 0;
  bool active = !covered && K > 0;
  uint64_t amask = ballot(active);
  auto walk = [&](int len) {
    const int nb = (len + 63) >> 6;
    auto block_mask = [&](int blk) -> uint64_t {
      const int e = blk * 64 + lane;
      uint64_t rm = 0;
      if (e < len) {
        const uint32_t pk = SL_pack[e];
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
          s_face[kid * 64 + lane] = SL_face[base + q];
          if (++kid >= K) {
            active = false;
            cm = 0;
          }
        }
        amask = ballot(active);
      }
    } else {
      // per-wave counts of this round ([Q][64] per row)
      int *s_rc = reinterpret_cast<int *>(smem + 128) + r * Q * 64;
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
        s_rc[qi * 64 + lane] = __popcll(cm);
        __syncthreads();
        int slot = kid, all = 0;
        for (int q = 0; q < Q; q++) {
          const int v = s_rc[q * 64 + lane];
          slot += q < qi ? v : 0;
          all += v;
        }
        const int base = blk * 64;
        while (cm && slot < K) {
          s_face[slot * 64 + lane] = SL_face[base + __builtin_ctzll(cm)];
          cm &= cm - 1;
          slot++;
        }
        kid = min(K, kid + all);
        active = active && kid < K;
        amask = ballot(active);
        __syncthreads();  // s_rc is rewritten by the next round
      }
    }
  };
  auto any_active = [&]() -> bool {  // workgroup-uniform
    if (lane == 0) s_cnt[wid] = amask != 0;
    __syncthreads();
    int any = 0;
    for (int w = 0; w < DT_WAVES; w++) any |= s_cnt[w];
    __syncthreads();
    return any != 0;
  };
  if (any_active()) {
    if (slen <= DT_LCAP) {
      walk(slen);
    } else {
      // the list overflowed: a second expansion of the chunks, filling the list DT_LCAP entries
      // at a time (soft_tile_fwd_kernel 1a-1b)
      ChunkSeq sq;
      sq.init(a.bitmap + tile, g.words, g.ntiles(), lane);
      int pos2 = 0, nc = -1;
      bool nexists = false;
      uint2 nr = make_uint2(1u, 1u);
      auto pf_next = [&]() {
        nexists = sq.at(pos2, lane) >= 0;
        nc = nexists ? sq.at(pos2 + wid, lane) : -1;
        pos2 += DT_WAVES;
        int fl = nc * 64 + lane;
        fl = fl < 0 ? 0 : (fl < F ? fl : F - 1);
        nr = srng[fl];
      };
      pf_next();
      bool more2 = nexists;
      while (true) {
        int len = 0;
        while (more2 && len + DT_WAVES * 64 <= DT_LCAP) {
          const int c = nc;
          const int fl = c * 64 + lane;
          uint32_t rows;
          int lo, hi;
          clip(nr, rows, lo, hi);
          const bool keep = c >= 0 && fl < F && rows != 0 && lo <= hi;
          pf_next();
          more2 = nexists;
          const uint64_t km = ballot(keep);
          if (lane == 0) s_cnt[wid] = __popcll(km);
          __syncthreads();
          int pre = 0, tot = 0;
          for (int w = 0; w < DT_WAVES; w++) {
            const int v = s_cnt[w];
            pre += w < wid ? v : 0;
            tot += v;
          }
          if (keep) {
            const int p = len + pre + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0u));
            SL_face[p] = (uint32_t)fl;
            SL_pack[p] = (uint32_t)lo | ((uint32_t)hi << 6) | (rows << 12);
          }
          len += tot;
          __syncthreads();
        }
        walk(len);
        if (!any_active() || !more2) break;
      }
    }
  }
  if (qi == 0) {
    if (!px_valid) kid = 0;
    int pre = kid;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(pre, o);
      if (lane >= o) pre += u;
    }
    s_rpre[lane] = pre - kid;
    if (lane == 63) s_rpre[64] = pre;
  }
  __syncthreads();
  const int total = s_rpre[64];

  // ---- 3b. the row's hits ((pixel, slot) order) -> records, then the mask (softtile.hip 2)
  const size_t rbase = ((size_t)(b * H + (row_ok ? j : 0)) * g.tiles_x + tx) * 64 * (size_t)K;
  float *s_prob = reinterpret_cast<float *>(s_face);
  {
    const float yy = sy * (float)(H - 2 * (row_ok ? j : 0) - 1);  // == pix_y
    constexpr int UU = 4;
    const int S = 64 * Q;
    for (int e0 = qi * 64 + lane; e0 < total; e0 += S * UU) {
      int pp[UU], kk[UU];
      uint32_t ff[UU];
#pragma unroll
      for (int u = 0; u < UU; u++) {
        const int e = e0 + S * u;
        int lo = 0;  // owner lane p: last lane with s_rpre[p] <= e
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
          if (s_rpre[lo + st] <= e) lo += st;
        pp[u] = lo;
        kk[u] = e - s_rpre[lo];
        ff[u] = e < total ? s_face[kk[u] * 64 + lo] : 0u;
      }
      float v[UU][6];
#pragma unroll
      for (int u = 0; u < UU; u++) a.src.verts(f0 + ff[u], v[u]);  // all in flight (ff = 0 past the end)
#pragma unroll
      for (int u = 0; u < UU; u++) {
        const int e = e0 + S * u;
        if (e < total) {
          float dsq;
          int edgeid;
          soft_dist<float>(sx * (float)(2 * (ibase + pp[u]) + 1 - W), yy, v[u], m, dsq, edgeid);
          const float z = a.sigmainv * dsq / m / m;
          const float pr = kl_exp<float>(-z);
          a.rec_face[rbase + e] = ff[u] | ((uint32_t)(edgeid + 1) << 28);
          a.rec_prob[rbase + e] = pr;
          s_prob[kk[u] * 64 + pp[u]] = pr;
        }
      }
    }
  }
  __syncthreads();
  if (qi == 0 && px_valid) {
    if (kid > 0) {
      // 1 - prod(1 - p) in double, slot order (dibr_soft_mask_cuda.cu:174-182); slots read eight
      // at a time so that their LDS reads overlap
      float allprob = 1.0f;
      for (int k0 = 0; k0 < kid; k0 += 8) {
        float pk[8];
#pragma unroll
        for (int u = 0; u < 8; u++) pk[u] = s_prob[min(k0 + u, kid - 1) * 64 + lane];
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (k0 + u < kid) allprob = (float)((double)allprob * (1.0 - (double)pk[u]));
      }
      a.mask[pix] = (float)(1.0 - (double)allprob);
    } else {
      a.mask[pix] = covered ? 1.0f : 0.0f;  // 1 - prod over no slots = 0
    }
    a.hits[pix] = (uint8_t)kid;
  }
  if (qi == 0 && row_ok && lane == 0) a.seg_tot[(size_t)(b * H + j) * g.tiles_x + tx] = total;

  // ---- 4. the backward's work items: (item, piece) per SB_PIECE hits of the item's rows
  if (qi == 0 && lane == 0) s_cnt[r] = row_ok ? total : 0;
  __syncthreads();
  if (threadIdx.x == 0 && a.bwd_items) {
    int tot = 0;
    for (int k = 0; k < RP; k++) tot += s_cnt[k];
    const int n = (tot + SB_PIECE - 1) / SB_PIECE;
    if (n) {
      const int sh = (int)(blockIdx.x & (DS_SHARDS - 1));
      int2 *dst = a.bwd_items + (size_t)sh * a.bwd_cap + atomicAdd(&a.bwd_cnt[sh * DS_CNT_STRIDE], n);
      for (int k = 0; k < n; k++) dst[k] = make_int2(item, k);
    }
  }
}

int dibr_tile_launch(const DibrTileArgs &a, int lp_min, int grid, hipStream_t st) {
  const size_t lds = dt_lds_bytes(a.K, lp_min);
  KL_REQUIRE(lds <= 160 * 1024, "dibr_rasterization: knum too large for the LDS slot lists");
  hipLaunchKernelGGL(dibr_tile_kernel, dim3((unsigned)grid), dim3(64 * DT_WAVES), lds, st, a);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

}  // namespace kl

#endif  // KL_DEV
