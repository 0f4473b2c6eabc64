// dibrbwd.hip -- dibr_rasterization's backward (kl_dibr_backward) as one pixel-major pass.
//
// Both gradients are sums over pixels: every pixel a face won adds the rasterizer's float terms
// to that face (rasterization_cuda.cu:238-402), every soft-mask hit adds its terms to its face
// (dibr_soft_mask_cuda.cu:230-353).  The reference scatters them with float atomics.  Here one
// workgroup takes one 64x8 tile (a thread per pixel):
//  1. its pixels' rasterizer terms, summed per face in double in an LDS hash;
//  2. its hits' soft-mask terms (the compact state's records, coalesced per row segment), summed
//     per face the same way;
// and each (face, tile) sum is stored -- no atomics -- in a slot of the face: slot k is the tile's
// place in the face's tile rectangle (its exact pixel range for the raster sums, up to 2 x 2
// tiles; its enlarged soft-mask range for the soft sums, up to 2 x 4), marked by a flag byte.
// One thread per face then adds its flagged slots, rounds each gradient once and writes
// (T)raster + (T)soft, as autograd adds the two gradients.
//
// f32 terms sum exactly in double whenever their magnitudes span less than ~2^29, so the result
// does not depend on the grouping of the adds: it equals the oracle's ordered double sums, as the
// per-face gather's did.  Faces whose rectangles are larger take per-face paths: the raster
// sums the range gather (rasterize_bwd_bigface_kernel, raster.hip), the soft sums double atomics
// into a per-face accumulator zeroed for those faces only.
#include "dibrbwd.h"
#include "rastgrad.h"

namespace kl {

constexpr int DB_NSR = 4;     // raster slots per face: the tiles of its exact range, up to 2 x 2
constexpr int DB_NSS = 8;     // soft slots per face: the tiles of its enlarged range, up to 2 x 4
constexpr int DB_MAXD = 8;    // widest feature dimension of the slots
constexpr int DB_HCR = 512;   // raster hash: a tile's 512 pixels win at most 512 faces
constexpr int DB_HCS = 1024;  // soft hash: flushed when it may not hold another round's faces
constexpr int DB_THREADS = TILE_W * TILE_H;

// workspace: flags (16 B per face: raster slot bytes [0, 4), soft slot bytes [8, 16)) |
// raster slots | soft slots | soft accumulators of the large faces | large-face list
struct DbWs {
  size_t flags, rslot, sslot, sacc, big, bytes;
  DbWs(int B, int F) {
    const size_t n = (size_t)B * F;
    flags = 0;
    rslot = al256(n * 16);
    sslot = rslot + al256(n * DB_NSR * (6 + 3 * DB_MAXD) * sizeof(double));
    sacc = sslot + al256(n * DB_NSS * 6 * sizeof(double));
    big = sacc + al256(n * 6 * sizeof(double));
    bytes = big + al256(n * sizeof(int));
  }
};
size_t db_ws_bytes(int B, int H, int W, int F, int K) {
  (void)H;
  (void)W;
  (void)K;
  return DbWs(B, F).bytes;
}

// A face's tile rectangle from its exact range (x0 | x1 << 16, y0 | y1 << 16); false if empty.
__device__ __forceinline__ bool db_rect(uint2 r, int &tx0, int &ty0, int &nx, int &ny) {
  const int ix0 = (int)(r.x & 0xffffu), ix1 = (int)(r.x >> 16);
  const int iy0 = (int)(r.y & 0xffffu), iy1 = (int)(r.y >> 16);
  if (ix0 > ix1 || iy0 > iy1) return false;
  tx0 = ix0 / TILE_W;
  ty0 = iy0 / TILE_H;
  nx = ix1 / TILE_W - tx0 + 1;
  ny = iy1 / TILE_H - ty0 + 1;
  return true;
}

__device__ __forceinline__ bool db_soft_big(uint2 r) {
  int tx0, ty0, nx, ny;
  return db_rect(r, tx0, ty0, nx, ny) && (nx > 2 || ny > 4);
}

// Slot flags zeroed; the soft accumulators of faces with more than 2 x 4 soft tiles zeroed.
__global__ void __launch_bounds__(256) db_prep_kernel(int64_t n, const uint2 *__restrict__ srng,
                                                      uint4 *__restrict__ flags, double *__restrict__ sacc,
                                                      int with_soft) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= n) return;
  flags[f] = make_uint4(0u, 0u, 0u, 0u);
  if (with_soft && db_soft_big(srng[f])) {
#pragma unroll
    for (int q = 0; q < 6; q++) sacc[f * 6 + q] = 0.0;
  }
}

// The LDS hash of a tile: linear probing on the mesh-local face index, unbounded (the callers
// keep the number of keys below HC), with the list of used entries.
template <int HC>
__device__ __forceinline__ int db_slot(int *key, int *used, int *nused, int f) {
  unsigned h = ((unsigned)f * 2654435761u) >> (32 - __builtin_ctz(HC));
#pragma unroll 1
  while (true) {
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
}

template <typename T>
struct DbArgs {
  const T *grad_feat;
  const T *grad_mask;  // nullptr: no soft-mask gradient
  const int64_t *face_idx;
  const T *w, *fvi, *feat, *mask;
  const uint8_t *hits;
  const uint32_t *rec_face;
  const T *rec_prob;
  const uint2 *rng, *srng;
  BinGeom g;
  int F, D, K;
  float sigmainv, m, eps;
  uint8_t *flags;
  double *rslot, *sslot, *sacc;
};

// One workgroup per 64x8 tile, a thread per pixel (wave = row).
template <typename T, int MAXD>
__global__ void __launch_bounds__(DB_THREADS) db_tile_kernel(DbArgs<T> a) {
  constexpr int NVR = 6 + 3 * MAXD;
  constexpr int NVAL = DB_HCR * NVR > DB_HCS * 6 ? DB_HCR * NVR : DB_HCS * 6;
  __shared__ double s_val[NVAL];
  __shared__ int s_key[DB_HCS];
  __shared__ int s_used[DB_HCS];
  __shared__ int s_dst[DB_HCS];
  __shared__ int s_nused, s_flushed;
  __shared__ double s_a[TILE_H][64];
  __shared__ int s_pre[TILE_H][65];
  __shared__ int s_rowpre[TILE_H + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const BinGeom &g = a.g;
  const int H = g.height, W = g.width;
  const int tile = blockIdx.x;
  const int tx = tile % g.tiles_x, ty = (tile / g.tiles_x) % g.tiles_y, b = tile / (g.tiles_x * g.tiles_y);
  const int64_t fb = (int64_t)b * a.F;
  const int j = ty * TILE_H + wid, i = tx * TILE_W + lane;
  const bool px = j < H && i < W;
  const size_t p = px ? ((size_t)b * H + j) * W + i : 0;

  // ---- 1. the rasterizer's terms of the pixels (rasterization_cuda.cu:262-399, BaryGrad)
  for (int q = tid; q < DB_HCR; q += DB_THREADS) s_key[q] = -1;
  for (int q = tid; q < DB_HCR * NVR; q += DB_THREADS) s_val[q] = 0.0;
  if (tid == 0) s_nused = 0;
  __syncthreads();
  const int64_t f = px ? a.face_idx[p] : -1;
  if (f >= 0) {
    const int64_t tf = fb + f;
    const int D = a.D;
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = a.fvi[tf * 6 + q];
    const T wa = a.w[p * 3 + 0], wb = a.w[p * 3 + 1], wc = a.w[p * 3 + 2];
    const T *c = a.feat + tf * 3 * D;
    const T *gp = a.grad_feat + p * D;
    double t[NVR];
#pragma unroll
    for (int q = 0; q < NVR; q++) t[q] = 0.0;
    BaryGrad<T> bg;
    bg.init(v, wa, wb, wc, a.eps);
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < D) {
        const T gd = gp[d];
        t[6 + d] = (double)(gd * wa);
        t[6 + MAXD + d] = (double)(gd * wb);
        t[6 + 2 * MAXD + d] = (double)(gd * wc);
        T o[6];
        bg.terms(gd, c[d], c[D + d], c[2 * D + d], o);
#pragma unroll
        for (int q = 0; q < 6; q++) t[q] += (double)o[q];
      }
    }
    const int h = db_slot<DB_HCR>(s_key, s_used, &s_nused, (int)f);
#pragma unroll
    for (int q = 0; q < NVR; q++)
      if (t[q] != 0.0) atomicAdd(&s_val[h * NVR + q], t[q]);  // a zero adds nothing
  }
  __syncthreads();
  {  // raster slots: (face, tile) sums of faces whose range spans at most 2 x 2 tiles
    const int n = s_nused;
    for (int e = tid; e < n; e += DB_THREADS) {
      int tx0, ty0, nx, ny, k = -1;
      if (db_rect(a.rng[fb + s_key[s_used[e]]], tx0, ty0, nx, ny) && nx <= 2 && ny <= 2)
        k = (ty - ty0) * 2 + (tx - tx0);
      s_dst[e] = k;  // -1: the per-face gather's face
    }
    __syncthreads();
    for (int t = tid; t < n * NVR; t += DB_THREADS) {
      const int e = t / NVR, v = t - e * NVR;
      const int k = s_dst[e];
      if (k < 0) continue;
      const int h = s_used[e];
      const int64_t tf = fb + s_key[h];
      a.rslot[((size_t)tf * DB_NSR + k) * NVR + v] = s_val[h * NVR + v];
      if (v == 0) a.flags[(size_t)tf * 16 + k] = 1;
    }
  }
  if (a.grad_mask == nullptr || a.K <= 0) return;  // workgroup-uniform

  // ---- 2. the soft mask's terms of the tile's hits (dibr_soft_mask_cuda.cu:262-340)
  __syncthreads();
  for (int q = tid; q < DB_HCS; q += DB_THREADS) s_key[q] = -1;
  for (int q = tid; q < DB_HCS * 6; q += DB_THREADS) s_val[q] = 0.0;
  if (tid == 0) {
    s_nused = 0;
    s_flushed = 0;
  }
  {  // row `wid`: filled-slot prefix, the reference's -sigmainv * dLdp * (1 - allprob)
    int kid = 0;
    if (px) {
      kid = a.hits[p];
      if (kid) s_a[wid][lane] = -1.0 * (double)a.sigmainv * (double)a.grad_mask[p] * (1.0 - (double)a.mask[p]);
    }
    int pre = kid;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(pre, o);
      if (lane >= o) pre += u;
    }
    s_pre[wid][lane] = pre - kid;
    if (lane == 63) s_rowpre[wid + 1] = pre;
  }
  __syncthreads();
  if (tid == 0) {
    s_rowpre[0] = 0;
    for (int r = 1; r <= TILE_H; r++) s_rowpre[r] += s_rowpre[r - 1];
  }
  __syncthreads();
  const int total = s_rowpre[TILE_H];
  const int K = a.K;
  const T ms = (T)a.m;
  const float sx = a.m / (float)W, sy = a.m / (float)H;

  // flush: (face, tile) soft sums into the faces' slots (added onto this workgroup's earlier
  // flush of the same slot, if any); faces with more than 2 x 4 soft tiles: double atomics
  auto flush = [&]() {
    const int n = s_nused;
    const bool again = s_flushed != 0;
    for (int e = tid; e < n; e += DB_THREADS) {
      const int64_t tf = fb + s_key[s_used[e]];
      int tx0, ty0, nx, ny, k = -1;
      if (db_rect(a.srng[tf], tx0, ty0, nx, ny) && nx <= 2 && ny <= 4) k = (ty - ty0) * 2 + (tx - tx0);
      int prev = 0;
      if (again && k >= 0)  // written by this workgroup's earlier flush? (L2 read: past this CU's L1)
        prev = __hip_atomic_load(a.flags + (size_t)tf * 16 + 8 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_dst[e] = k < 0 ? -1 : (k | (prev ? 256 : 0));
    }
    __syncthreads();
    for (int t = tid; t < n * 6; t += DB_THREADS) {
      const int e = t / 6, v = t - e * 6;
      const int d = s_dst[e];
      const int h = s_used[e];
      const int64_t tf = fb + s_key[h];
      double val = s_val[h * 6 + v];
      if (d < 0) {
        if (val != 0.0) atomicAdd(a.sacc + tf * 6 + v, val);
      } else {
        const int k = d & 255;
        double *dst = a.sslot + ((size_t)tf * DB_NSS + k) * 6 + v;
        if (d & 256) val += __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *dst = val;
        if (v == 0) a.flags[(size_t)tf * 16 + 8 + k] = 1;
      }
    }
    __threadfence();  // visible to a later flush of this workgroup
    __syncthreads();
  };

  for (int base = 0; base < total; base += DB_THREADS) {
    if (s_nused > DB_HCS - DB_THREADS) {  // workgroup-uniform (read after the round's barrier)
      flush();
      const int n = s_nused;
      for (int e = tid; e < n; e += DB_THREADS) {
        const int h = s_used[e];
        s_key[h] = -1;
#pragma unroll
        for (int v = 0; v < 6; v++) s_val[h * 6 + v] = 0.0;
      }
      __syncthreads();
      if (tid == 0) {
        s_nused = 0;
        s_flushed = 1;
      }
      __syncthreads();
    }
    const int ea = base + tid;
    if (ea < total) {
      int r = 0;
#pragma unroll
      for (int k = 1; k < TILE_H; k++) r += s_rowpre[k] <= ea ? 1 : 0;
      const int e = ea - s_rowpre[r];
      int lo = 0;  // owner lane: last lane with s_pre[r][lo] <= e
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (s_pre[r][lo + st] <= e) lo += st;
      const int jj = ty * TILE_H + r;
      const size_t o = ((size_t)(b * H + jj) * g.tiles_x + tx) * 64 * (size_t)K + e;
      const uint32_t rr = a.rec_face[o];
      const T pr = a.rec_prob[o];
      const int face = (int)(rr & 0x0fffffffu);
      const int edgeid = (int)(rr >> 28) - 1;
      const T x0 = (T)(sx * (float)(2 * (tx * TILE_W + lo) + 1 - W));  // == pix_x
      const T y0 = (T)(sy * (float)(H - 2 * jj - 1));                    // == pix_y
      const T dLdz = (T)(s_a[r][lo] / (1.0 - (double)pr + SM_EPS) * (double)pr);
      const T *fv = a.fvi + (fb + face) * 6;
      T v[6];
#pragma unroll
      for (int c = 0; c < 6; c++) v[c] = fv[c] * ms;
      int c0, c1;
      T g0x, g0y, g1x, g1y;
      soft_hit_grad<T>(v, edgeid, x0, y0, dLdz, a.m, c0, c1, g0x, g0y, g1x, g1y);
      const int h = db_slot<DB_HCS>(s_key, s_used, &s_nused, face);
      atomicAdd(&s_val[h * 6 + c0 * 2], (double)g0x);
      atomicAdd(&s_val[h * 6 + c0 * 2 + 1], (double)g0y);
      if (c1 >= 0) {
        atomicAdd(&s_val[h * 6 + c1 * 2], (double)g1x);
        atomicAdd(&s_val[h * 6 + c1 * 2 + 1], (double)g1y);
      }
    }
    __syncthreads();
  }
  if (s_nused > 0) flush();
}

// One thread per face: its flagged slots added, each gradient rounded once; faces whose raster
// range spans more than 2 x 2 tiles are listed for the per-face gather, their soft sums left
// in sacc.
template <typename T, int MAXD>
__global__ void __launch_bounds__(256) db_combine_kernel(int64_t n, int D, const uint4 *__restrict__ flags,
                                                         const uint2 *__restrict__ rng, const uint2 *__restrict__ srng,
                                                         const double *__restrict__ rslot,
                                                         const double *__restrict__ sslot, double *__restrict__ sacc,
                                                         int with_soft, T *__restrict__ gfvi, T *__restrict__ gfeat,
                                                         int *__restrict__ big, int *__restrict__ nbig) {
  constexpr int NVR = 6 + 3 * MAXD;
  const int64_t tf = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (tf >= n) return;
  const uint4 fl = flags[tf];
  double sv[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (with_soft) {
    if (db_soft_big(srng[tf])) {
#pragma unroll
      for (int q = 0; q < 6; q++) sv[q] = sacc[tf * 6 + q];
    } else {
#pragma unroll
      for (int k = 0; k < DB_NSS; k++) {
        const uint32_t word = k < 4 ? fl.z : fl.w;
        if ((word >> (8 * (k & 3))) & 0xffu) {
          const double *sl = sslot + ((size_t)tf * DB_NSS + k) * 6;
#pragma unroll
          for (int q = 0; q < 6; q++) sv[q] += sl[q];
        }
      }
    }
  }
  int tx0, ty0, nx, ny;
  if (db_rect(rng[tf], tx0, ty0, nx, ny) && (nx > 2 || ny > 2)) {
    if (with_soft) {
#pragma unroll
      for (int q = 0; q < 6; q++) sacc[tf * 6 + q] = sv[q];
    }
    big[atomicAdd(nbig, 1)] = (int)tf;
    return;
  }
  double r[NVR];
#pragma unroll
  for (int v = 0; v < NVR; v++) r[v] = 0.0;
#pragma unroll
  for (int k = 0; k < DB_NSR; k++) {
    if ((fl.x >> (8 * k)) & 0xffu) {
      const double *sl = rslot + ((size_t)tf * DB_NSR + k) * NVR;
#pragma unroll
      for (int v = 0; v < NVR; v++) r[v] += sl[v];
    }
  }
#pragma unroll
  for (int q = 0; q < 6; q++) gfvi[tf * 6 + q] = with_soft ? (T)r[q] + (T)sv[q] : (T)r[q];
#pragma unroll
  for (int v = 6; v < NVR; v++) {
    const int rr = v - 6, ii = rr / MAXD, d = rr % MAXD;
    if (d < D) gfeat[tf * 3 * D + ii * D + d] = (T)r[v];
  }
}

template <typename T, int MAXD>
static void db_launch(int64_t n, int ntiles, const DbArgs<T> &a, const uint4 *flags, bool with_soft, T *gfvi,
                      T *gfeat, int *big, int *nbig, hipStream_t st) {
  if (ntiles > 0) hipLaunchKernelGGL((db_tile_kernel<T, MAXD>), dim3((unsigned)ntiles), dim3(DB_THREADS), 0, st, a);
  hipLaunchKernelGGL((db_combine_kernel<T, MAXD>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, n, a.D, flags,
                     a.rng, a.srng, (const double *)a.rslot, (const double *)a.sslot, a.sacc, with_soft ? 1 : 0,
                     gfvi, gfeat, big, nbig);
}

template <typename T>
int db_backward(int B, int H, int W, int F, int D, int K, const T *grad_feat, const T *grad_mask,
                const int64_t *face_idx, const T *w, const T *fvi, const T *feat, const T *mask,
                const SoftState<T> &s, float sigmainv, float m, float eps, const uint2 *rng, const uint2 *srng,
                T *gfvi, T *gfeat, void *ws, size_t ws_bytes, int *nbig, hipStream_t st, int **big,
                const double **soft_sum) {
  const DbWs L(B, F);
  KL_REQUIRE(ws_bytes >= L.bytes, "dibr_rasterization backward: workspace too small");
  KL_REQUIRE(D <= DB_MAXD, "dibr_rasterization backward: feature dimension > 8");
  KL_REQUIRE(H < 65536 && W < 65536 && F < (1 << 28), "dibr_rasterization backward: sizes out of range");
  const int64_t n = (int64_t)B * F;
  char *w8 = reinterpret_cast<char *>(ws);
  uint4 *flags = reinterpret_cast<uint4 *>(w8 + L.flags);
  double *sacc = reinterpret_cast<double *>(w8 + L.sacc);
  const bool with_soft = grad_mask != nullptr && K > 0 && (int64_t)B * H * W > 0;
  *big = reinterpret_cast<int *>(w8 + L.big);
  *soft_sum = with_soft ? sacc : nullptr;
  if (n == 0) return KL_OK;
  hipLaunchKernelGGL(db_prep_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, n, srng, flags, sacc,
                     with_soft ? 1 : 0);
  KL_CHECK_LAUNCH();
  const BinGeom g = make_bin_geom(B, H, W, F);
  DbArgs<T> a{grad_feat, with_soft ? grad_mask : nullptr, face_idx, w, fvi, feat, mask, s.hits, s.rec_face,
              s.rec_prob, rng, srng, g, F, D, K, sigmainv, m, eps, reinterpret_cast<uint8_t *>(flags),
              reinterpret_cast<double *>(w8 + L.rslot), reinterpret_cast<double *>(w8 + L.sslot), sacc};
  const int ntiles = (int64_t)B * H * W > 0 ? g.batch * g.tiles_y * g.tiles_x : 0;
  if (D <= 2)
    db_launch<T, 2>(n, ntiles, a, flags, with_soft, gfvi, gfeat, *big, nbig, st);
  else if (D == 3)
    db_launch<T, 3>(n, ntiles, a, flags, with_soft, gfvi, gfeat, *big, nbig, st);
  else if (D <= 4)
    db_launch<T, 4>(n, ntiles, a, flags, with_soft, gfvi, gfeat, *big, nbig, st);
  else
    db_launch<T, 8>(n, ntiles, a, flags, with_soft, gfvi, gfeat, *big, nbig, st);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template int db_backward<float>(int, int, int, int, int, int, const float *, const float *, const int64_t *,
                                const float *, const float *, const float *, const float *, const SoftState<float> &,
                                float, float, float, const uint2 *, const uint2 *, float *, float *, void *, size_t,
                                int *, hipStream_t, int **, const double **);
template int db_backward<double>(int, int, int, int, int, int, const double *, const double *, const int64_t *,
                                 const double *, const double *, const double *, const double *,
                                 const SoftState<double> &, float, float, float, const uint2 *, const uint2 *,
                                 double *, double *, void *, size_t, int *, hipStream_t, int **, const double **);

}  // namespace kl
