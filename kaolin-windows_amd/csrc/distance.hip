// distance.hip -- point->triangle distance and point-cloud sided distance for gfx950.
//
// point_to_mesh (unbatched_triangle_distance_cuda.cu:237-317): brute force over faces,
// one point per lane.  Faces are staged through LDS in tiles; per face the quantities
// that do not depend on the point (edges, normal, squared edge lengths, unit normal,
// edge normals) are computed ONCE while staging -- with exactly the reference's
// expressions, so every per-pair value is bit-identical to the oracle -- and the
// per-pair classification (types 1..6, 0) is evaluated branch-free with selects
// (no wave divergence across the seven cases).  The reference's 512-face tile
// argmin semantics (first face of a tile taken unconditionally, strict '>' inside a
// tile, strict '>' across tiles) are kept independently of the LDS tile size.
//
// sided_distance (sided_distance_cuda.cu:52-201): one p1 point per lane, p2 staged in
// LDS, 512-point argmin tiles as in the reference; the grid covers (batch, points)
// instead of the reference's fixed 32x16 grid.
#include "common.h"

#include <hip/hip_fp16.h>

#include <hipcub/hipcub.hpp>

#include <limits>
#include <type_traits>

namespace kl {

template <typename T>
struct V3 {
  T x, y, z;
};
template <typename T>
__device__ __forceinline__ V3<T> mk(T x, T y, T z) { return V3<T>{x, y, z}; }
template <typename T>
__device__ __forceinline__ V3<T> operator-(V3<T> a, V3<T> b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
template <typename T>
__device__ __forceinline__ V3<T> operator+(V3<T> a, V3<T> b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
template <typename T>
__device__ __forceinline__ V3<T> operator*(V3<T> a, T s) { return mk(a.x * s, a.y * s, a.z * s); }
template <typename T>
__device__ __forceinline__ V3<T> operator/(V3<T> a, T s) { return mk(a.x / s, a.y / s, a.z / s); }
template <typename T>
__device__ __forceinline__ T dot(V3<T> a, V3<T> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename T>
__device__ __forceinline__ V3<T> cross(V3<T> a, V3<T> b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
template <typename T>
__device__ __forceinline__ V3<T> sel3(bool c, V3<T> a, V3<T> b) {
  return mk(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z);
}

// Per-face precomputed record (all point-independent subexpressions of the reference).
template <typename T>
struct FaceRec {
  V3<T> v1, v2, v3, e12, e23, e31, un, en12, en23, en31;
  T l12, l23, l31;
  T thick;  // pruning only: max |dot(x - v1, un)| over the triangle (+ rounding slack)
  T hmax;   // pruning only: max |coordinate| of the vertices
};

template <typename T>
__device__ __forceinline__ void make_face(const T *v, FaceRec<T> &r) {
  r.v1 = mk(v[0], v[1], v[2]);
  r.v2 = mk(v[3], v[4], v[5]);
  r.v3 = mk(v[6], v[7], v[8]);
  r.e12 = r.v2 - r.v1;
  r.e23 = r.v3 - r.v2;
  r.e31 = r.v1 - r.v3;
  const V3<T> normal = cross(r.v1 - r.v2, r.e31);
  r.l12 = dot(r.e12, r.e12);
  r.l23 = dot(r.e23, r.e23);
  r.l31 = dot(r.e31, r.e31);
  const T inv_len = (T)1 / kl_sqrt<T>(dot(normal, normal));
  r.un = normal * inv_len;
  r.en12 = cross(normal, r.e12);
  r.en23 = cross(normal, r.e23);
  r.en31 = cross(normal, r.e31);
  const T hm = fmax(fmax(fmax(fabs(r.v1.x), fabs(r.v1.y)), fmax(fabs(r.v1.z), fabs(r.v2.x))),
                    fmax(fmax(fabs(r.v2.y), fabs(r.v2.z)), fmax(fmax(fabs(r.v3.x), fabs(r.v3.y)), fabs(r.v3.z))));
  r.hmax = hm;
  // the triangle lies within +-thick of the computed plane {x : dot(x - v1, un) = 0}
  r.thick = fmax(fabs(dot(r.e12, r.un)), fabs(dot(r.e31, r.un))) + (T)(64.0 / 16777216.0) * hm;
}

// The evaluation half of FaceRec as a global record (p2m_fwd_grec_kernel): a wave reads one
// face's record with a wave-uniform index, so it comes through scalar loads into SGPRs.
template <typename T>
struct alignas(16) FaceRecS {
  V3<T> v1, v2, v3, e12, e23, e31, un, en12, en23, en31;
  T l12, l23, l31, pad0, pad1, pad2;
};

// squared distance (as float, :302) + type of one point to one face (R = FaceRec / FaceRecS)
template <typename T, typename R>
__device__ __forceinline__ float point_face(const V3<T> &p, const R &f, int &type) {
  const V3<T> pv1 = p - f.v1, pv2 = p - f.v2, pv3 = p - f.v3;
  const T uab = dot(pv1, f.e12) / f.l12;
  const T uca = dot(pv3, f.e31) / f.l31;
  const T ubc = dot(pv2, f.e23) / f.l23;
  const bool t1 = uca > (T)1 && uab < (T)0;
  const bool t2 = !t1 && uab > (T)1 && ubc < (T)0;
  const bool t3 = !t1 && !t2 && ubc > (T)1 && uca < (T)0;
  const bool rest = !t1 && !t2 && !t3;
  const bool t4 = rest && (uab <= (T)1 && uab >= (T)0) && dot(f.en12, pv1) <= (T)0;
  const bool t5 = rest && !t4 && (ubc <= (T)1 && ubc >= (T)0) && dot(f.en23, pv2) <= (T)0;
  const bool t6 = rest && !t4 && !t5 && (uca <= (T)1 && uca >= (T)0) && dot(f.en31, pv3) <= (T)0;
  // point_at(vertex, edge, float t) -- the reference passes the parameter as float
  const T tp = t4 ? (T)(float)uab : (t5 ? (T)(float)ubc : (T)(float)uca);
  const V3<T> ev = t4 ? f.e12 : (t5 ? f.e23 : f.e31);
  const V3<T> vv = t4 ? f.v1 : (t5 ? f.v2 : f.v3);
  const V3<T> cp_edge = vv + ev * tp;
  const T dist = (p.x - f.v1.x) * f.un.x + (p.y - f.v1.y) * f.un.y + (p.z - f.v1.z) * f.un.z;
  const V3<T> cp_plane = p - f.un * dist;
  V3<T> cp = sel3(t4 || t5 || t6, cp_edge, cp_plane);
  cp = sel3(t3, f.v3, cp);
  cp = sel3(t2, f.v2, cp);
  cp = sel3(t1, f.v1, cp);
  type = t1 ? 1 : t2 ? 2 : t3 ? 3 : t4 ? 4 : t5 ? 5 : t6 ? 6 : 0;
  const V3<T> dv = p - cp;
  return (float)dot(dv, dv);
}

#ifdef KL_P2M_PROBE  // dev probe (scripts/dev/p2m_probe.hip): counts skipped / evaluated (wave, face) pairs
__device__ unsigned long long g_p2m_skipped, g_p2m_evaluated, g_p2m_pairs;  // pairs: per-point tests passed
#define KL_P2M_COUNT(v) v++
#else
#define KL_P2M_COUNT(v)
#endif

constexpr int P2M_TILE = 128;  // faces per LDS tile (a divisor of the reference's 512)
constexpr float P2M_E = 1.0f / 16777216.0f;  // float unit roundoff (d is stored as float for both dtypes)

// Lane-parallel pruning record of one face (LDS, structure of arrays): unit normal un and
// the plane offset dv = dot(v1, un) with the slab half-thickness thick (FaceRec), plus, per
// edge e, a unit vector o_e in the plane pointing away from the triangle and the offset
// off_e such that dot(x, o_e) <= off_e for every point x of the triangle (max over the
// three vertices, plus rounding slack).
template <typename T>
struct PruneTile {
  T o[9][P2M_TILE];
  T off[3][P2M_TILE];
  T dv[P2M_TILE];
};

// out[0..8] = o_e (3 per edge), out[9..11] = off_e, out[12] = dv
template <typename T>
__device__ __forceinline__ void make_prune_vals(const FaceRec<T> &r, T *out) {
  const V3<T> e[3] = {r.e12, r.e23, r.e31};
  const V3<T> a[3] = {r.v1, r.v2, r.v3};
  const V3<T> b[3] = {r.v2, r.v3, r.v1};
  const V3<T> opp[3] = {r.v3, r.v1, r.v2};
  const T slack = (T)(64.0 / 16777216.0) * r.hmax;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    V3<T> o = cross(r.un, e[k]);
    const T inv = (T)1 / kl_sqrt<T>(dot(o, o));
    o = o * inv;
    if (dot(opp[k] - a[k], o) > (T)0) o = mk(-o.x, -o.y, -o.z);
    const T d0 = dot(a[k], o), d1 = dot(b[k], o), d2 = dot(opp[k], o);
    out[3 * k] = o.x;
    out[3 * k + 1] = o.y;
    out[3 * k + 2] = o.z;
    out[9 + k] = fmax(fmax(d0, d1), d2) + slack;
  }
  out[12] = dot(r.v1, r.un);
}

template <typename T>
__device__ __forceinline__ void make_prune(const FaceRec<T> &r, PruneTile<T> &pt, int s) {
  T v[13];
  make_prune_vals<T>(r, v);
#pragma unroll
  for (int k = 0; k < 9; k++) pt.o[k][s] = v[k];
#pragma unroll
  for (int k = 0; k < 3; k++) pt.off[k][s] = v[9 + k];
  pt.dv[s] = v[12];
}

// Face skipping.  The reference's fold (first face of each 512-face tile taken
// unconditionally, then strict '<' inside a tile, strict '<' across tiles) gives every
// point the minimum float distance over all faces, earliest face on ties (NaN aside).
// A face whose computed distance d satisfies d >= min(best of earlier tiles, current
// tile best) can never change the outcome, so it need not be evaluated.  Points are
// processed in Morton order, so a wave's 64 points form a cluster (centre c, radius R).
// Every point x of a triangle satisfies |dot(x, un) - dv| <= thick (its plane slab) and
// dot(x, o_e) <= off_e for each edge (its in-plane edge half-planes); with
//   A = |dot(c, un) - dv| - thick,  B = max_e dot(c, o_e) - off_e   (each clamped at 0)
// un _|_ o_e gives |p - x| >= sqrt(A^2 + B^2) - R for every point p of the cluster.  The
// computed d is within 64 E M of the true squared-distance geometry (M = |c|inf + R +
// hmax, E = 2^-24 as d is truncated to float) and A, B within 16 E M of their exact
// values, so with s = 256 E M subtracted from A and B and the (1 +- 32 E) factors for the
// float evaluation and the near-orthogonality of the computed unit vectors,
//   (A^2 + B^2)(1 - 32E) > ((R + sqrt(thr))(1 + 16E) + s)^2 (1 + 32E)
// proves d > thr.  The test runs lane-parallel: each lane bounds one face of a 64-face
// chunk against the wave's cluster, a ballot gives the chunk's faces to evaluate, and the
// wave walks them in face order.  The first face of each reference tile is always
// evaluated.  Skipped or not, every evaluated value is the reference's, so results are
// unchanged; non-finite inputs give NaN / infinite bounds, which never skip (the
// comparisons are false, and a non-finite cluster disables the test).
// grid: (point blocks, face splits).  A split covers whole 512-face reference tiles
// [f_begin, f_end); with more than one split each writes its partial (dist, idx, type)
// at part + split * P (sorted point order) for p2m_combine_kernel.  The reference fold
// restricted to a split: only split 0 takes its first tile unconditionally; later
// splits start from +inf, so, as in the global fold, a NaN tile never replaces.
#ifndef KL_P2M_WAVES_PER_EU
#define KL_P2M_WAVES_PER_EU 5
#endif
// occupancy: the float kernel is latency-bound at 4 waves per SIMD (113 VGPRs); asking
// for 5 (96 VGPRs, 4 spilled) measured 3-5 % faster on cfg2, 6 (22 spills) no better
// PAIRS (r05): with shared thresholds on (all faces proper, a finite bounded cluster -- the fold is
// then the plain (distance, index) minimum, so pairs may be evaluated in any order), each (point,
// face) pair the wave's test keeps goes through a second, per-point test -- the same bound with the
// lane's own point and its own running best -- and the pairs that pass are queued per wave (LDS ring
// of (face slot, lane)) and evaluated 64 at a time, one pair per lane, the point fetched from its
// lane; each result is folded into its point's packed (distance bits, face << 3 | type) minimum with
// an LDS 64-bit atomic min.  The wave-level walk evaluated every kept face for all 64 points, most of
// them far from it; this evaluates ~one lane-slot per useful pair.  The minimum face itself is
// never skipped (every threshold is a computed distance, and skipping needs d > thr strictly), so
// the (distance, index) minimum -- the reference's result -- is exact.
constexpr int P2M_QCAP = 128;  // per-wave pair ring (a face adds <= 64 pairs; batches of 64 drain it)

// SUBC (r06): the pairs path's per-point test only for (face, 8-lane sub-cluster) pairs a sub-cluster
// bound keeps, 8 such pairs per wave instruction (p2m_fwd_kernel's pairs branch)
// (r06 A/B at cfg2: the sub-cluster kernel 0.818 ms at 4 waves per SIMD -- no spills -- against 0.85-0.89
// at 5 with 54 VGPRs spilled; the r05 pairs kernel 0.85-0.92 at 5, 0.94 at 4)
template <typename T, bool PAIRS, bool SUBC = true>
__global__ void __launch_bounds__(256, (sizeof(T) == 4 ? (PAIRS && SUBC ? 4 : KL_P2M_WAVES_PER_EU) : 1)) p2m_fwd_kernel(const T *__restrict__ pts, const T *__restrict__ fv,
                                                       const int32_t *__restrict__ order, int64_t P, int64_t F,
                                                       int64_t split_faces, T *__restrict__ out_dist,
                                                       int64_t *__restrict__ out_idx, int32_t *__restrict__ out_type,
                                                       T *__restrict__ part_dist, int64_t *__restrict__ part_idx,
                                                       int32_t *__restrict__ part_type,
                                                       const int32_t *__restrict__ bounds, uint32_t *gbest) {
  __shared__ FaceRec<T> sf[P2M_TILE];
  __shared__ PruneTile<T> sp;
  const int64_t si = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool valid = si < P;
  const int64_t pi = valid ? (order ? (int64_t)order[si] : si) : 0;
  const bool first_split = blockIdx.y == 0;
  const int64_t f_begin = (int64_t)blockIdx.y * split_faces;
  const int64_t f_end = min(F, f_begin + split_faces);
  const int lane = threadIdx.x & 63;
  V3<T> p = mk((T)0, (T)0, (T)0);
  if (valid) p = mk(pts[pi * 3], pts[pi * 3 + 1], pts[pi * 3 + 2]);
  // cluster of the wave's points (padding lanes repeat lane 0's point)
  const V3<T> p0 = mk(__shfl(p.x, 0), __shfl(p.y, 0), __shfl(p.z, 0));
  const V3<T> q = valid ? p : p0;
  const bool fin = isfinite(q.x) && isfinite(q.y) && isfinite(q.z);
  const bool all_fin = __all(fin);
  V3<T> c = mk((T)0, (T)0, (T)0), ext = mk((T)0, (T)0, (T)0);
  T R = (T)INFINITY, cinf = (T)0;
  if (all_fin) {
    c = mk((wave_min(q.x) + wave_max(q.x)) * (T)0.5, (wave_min(q.y) + wave_max(q.y)) * (T)0.5,
           (wave_min(q.z) + wave_max(q.z)) * (T)0.5);
    const V3<T> dq = q - c;
    R = wave_max(kl_sqrt<T>(dot(dq, dq))) * (T)(1.0 + 16.0 * P2M_E);
    // the cluster's box half-extents about c (>= |p - c| per axis for every point of the wave)
    ext = mk(wave_max(fabs(dq.x)), wave_max(fabs(dq.y)), wave_max(fabs(dq.z))) * (T)(1.0 + 4.0 * P2M_E);
    cinf = fmax(fmax(fabs(c.x), fabs(c.y)), fabs(c.z));
  }
  // (SUBC) this lane's 8-lane sub-cluster (lanes 8j .. 8j + 7, Morton-consecutive points): centre and
  // radius, the wave cluster's construction over the group (xor shuffles 1, 2, 4 stay in the group)
  V3<T> cj = mk((T)0, (T)0, (T)0);
  T Rj = (T)INFINITY;
  if (PAIRS && SUBC && all_fin) {
    auto gmin = [](T v) {
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) v = fmin(v, __shfl_xor(v, o));
      return v;
    };
    auto gmax = [](T v) {
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) v = fmax(v, __shfl_xor(v, o));
      return v;
    };
    cj = mk((gmin(q.x) + gmax(q.x)) * (T)0.5, (gmin(q.y) + gmax(q.y)) * (T)0.5, (gmin(q.z) + gmax(q.z)) * (T)0.5);
    const V3<T> dj = q - cj;
    Rj = gmax(kl_sqrt<T>(dot(dj, dj))) * (T)(1.0 + 16.0 * P2M_E);
  }
  // Shared thresholds (all faces proper, finite bounded cluster): the fold is then the plain
  // (distance, index) minimum, so the best distance any split has found for a point bounds
  // its result and is as good a threshold as this split's own.  gbest holds them as float
  // bits (distances are >= +0, so integer order is float order); reads may be stale, which
  // only weakens the bound.
  const bool share = gbest != nullptr && all_fin && bounds[6] != 0 && cinf + R < (T)1e15;
  // the per-point pair path (wave-uniform); face ids and types packed in 32 bits
  const bool pairs = PAIRS && share && F < ((int64_t)1 << 29);
  constexpr unsigned long long KEY_NONE = 0x7f800000ull << 32 | 0xffffffffull;  // +inf, no face
  __shared__ uint16_t s_q[PAIRS ? 4 : 1][P2M_QCAP];
  __shared__ unsigned long long s_best[PAIRS ? 256 : 1];
  __shared__ uint8_t s_sp[PAIRS && SUBC ? 4 : 1][64];  // (SUBC) a batch's kept (face, sub-cluster) pairs
  const int wid = threadIdx.x >> 6;
  uint32_t qhead = 0, qcnt = 0;  // the wave's ring (wave-uniform)
  T pthr = (T)INFINITY, psq = (T)INFINITY;  // pairs: the lane's best distance so far and its root
  if (pairs) s_best[threadIdx.x] = KEY_NONE;
  float published = INFINITY;
#ifdef KL_P2M_PROBE
  unsigned long long g_p2m_skipped = 0, g_p2m_evaluated = 0, g_p2m_pairs = 0;
#endif
  T best = (T)INFINITY, tbest = (T)INFINITY;
  int64_t best_f = 0, tbest_f = 0;
  int best_t = 0, tbest_t = 0;
  for (int64_t start = f_begin; start < f_end; start += P2M_TILE) {
    const int n = (int)min((int64_t)P2M_TILE, f_end - start);
    float shared_thr = INFINITY;
    if (share && valid)
      shared_thr = __uint_as_float(__hip_atomic_load(gbest + si, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (pairs && (T)shared_thr < pthr) {
      pthr = (T)shared_thr;
      psq = kl_sqrt<T>(pthr) * (T)(1.0 + 16.0 * P2M_E);
    }
    __syncthreads();
    for (int s = threadIdx.x; s < n; s += blockDim.x) {
      make_face<T>(fv + (start + s) * 9, sf[s]);
      make_prune<T>(sf[s], sp, s);
    }
    __syncthreads();
    // pairs: evaluate the ring's first nb pairs, one per lane, folding into s_best; then every lane
    // re-reads its own minimum as its threshold
    auto run_batch = [&](int nb) {
      const bool act = lane < nb;
      const uint32_t e = s_q[wid][(qhead + (act ? lane : 0)) & (P2M_QCAP - 1)];
      const int owner = (int)(e & 63u), sj = (int)(e >> 6);
      const V3<T> pp = mk(__shfl(p.x, owner), __shfl(p.y, owner), __shfl(p.z, owner));
      int t;
      const float d = point_face<T>(pp, sf[sj], t);
      if (act)
        atomicMin(&s_best[wid * 64 + owner],
                  (unsigned long long)__float_as_uint(d) << 32 | (uint32_t)(((start + sj) << 3) | t));
      qhead += nb;
      qcnt -= nb;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const unsigned long long mine = s_best[threadIdx.x];
      const T bd = (T)__uint_as_float((uint32_t)(mine >> 32));
      if (bd < pthr) {
        pthr = bd;
        psq = kl_sqrt<T>(pthr) * (T)(1.0 + 16.0 * P2M_E);
      }
    };
    for (int s0 = 0; s0 < n; s0 += 64) {
      // thresholds only decrease, so a stale maximum over the lanes is a safe upper bound
      T thr = fmin(best, tbest);
      if (thr != thr || !valid) thr = valid ? (T)INFINITY : (T)0;
      if (share) thr = fmin(thr, (T)shared_thr);
      if (pairs) thr = valid ? pthr : (T)0;
      const T thr_max = wave_max_all(thr);  // (every lane active: the chunk loop is wave-uniform)
      const int s = s0 + lane;
      bool eval = s < n;
      if (eval && all_fin && (pairs || ((start + s) & 511) != 0) && thr_max < (T)INFINITY) {
        const FaceRec<T> &fr = sf[s];
        const T M = cinf + R + fr.hmax;
        const T sl = (T)(256.0 * P2M_E) * M;
        const T A = fmax(fabs(dot(c, fr.un) - sp.dv[s]) - fr.thick - sl, (T)0);
        T b = dot(c, mk(sp.o[0][s], sp.o[1][s], sp.o[2][s])) - sp.off[0][s];
        b = fmax(b, dot(c, mk(sp.o[3][s], sp.o[4][s], sp.o[5][s])) - sp.off[1][s]);
        b = fmax(b, dot(c, mk(sp.o[6][s], sp.o[7][s], sp.o[8][s])) - sp.off[2][s]);
        const T B = fmax(b - sl, (T)0);
        const T K = (R + kl_sqrt<T>(thr_max)) * (T)(1.0 + 16.0 * P2M_E) + sl;
        if ((A * A + B * B) * (T)(1.0 - 32.0 * P2M_E) > K * K * (T)(1.0 + 32.0 * P2M_E)) eval = false;
        // The same bound over the cluster's box instead of its sphere: for every point p of the box,
        // |dot(p, u) - dot(c, u)| <= ext . |u| for the plane normal and each edge normal, so
        // with those subtracted from A and B per direction (and no R) the distance bound holds for
        // all points at once -- tighter than the sphere's single R for faces seen face-on or
        // edge-on; either proof skips.
        if (eval) {
          auto sup = [&](T ux, T uy, T uz) {  // ext . |u|, rounded up
            return (ext.x * fabs(ux) + ext.y * fabs(uy) + ext.z * fabs(uz)) * (T)(1.0 + 16.0 * P2M_E);
          };
          const T A2 = fmax(fabs(dot(c, fr.un) - sp.dv[s]) - fr.thick - sl - sup(fr.un.x, fr.un.y, fr.un.z), (T)0);
          T b2 = dot(c, mk(sp.o[0][s], sp.o[1][s], sp.o[2][s])) - sp.off[0][s] - sup(sp.o[0][s], sp.o[1][s], sp.o[2][s]);
          b2 = fmax(b2, dot(c, mk(sp.o[3][s], sp.o[4][s], sp.o[5][s])) - sp.off[1][s] -
                            sup(sp.o[3][s], sp.o[4][s], sp.o[5][s]));
          b2 = fmax(b2, dot(c, mk(sp.o[6][s], sp.o[7][s], sp.o[8][s])) - sp.off[2][s] -
                            sup(sp.o[6][s], sp.o[7][s], sp.o[8][s]));
          const T B2 = fmax(b2 - sl, (T)0);
          const T K2 = kl_sqrt<T>(thr_max) * (T)(1.0 + 16.0 * P2M_E) + sl;
          if ((A2 * A2 + B2 * B2) * (T)(1.0 - 32.0 * P2M_E) > K2 * K2 * (T)(1.0 + 32.0 * P2M_E)) eval = false;
        }
      }
      uint64_t mask = __ballot(eval);
#ifdef KL_P2M_PROBE
      g_p2m_evaluated += __popcll(mask);
      g_p2m_skipped += (uint64_t)min(64, n - s0) - __popcll(mask);
#endif
      if (pairs && SUBC) {
        // r06: the kept faces 8 at a time.  Lane L bounds face L & 7 of the batch against its own
        // sub-cluster (lanes 8 (L >> 3) ..; the wave test's sphere bound with the group's centre,
        // radius and largest per-point threshold); the passing (face, sub-cluster) pairs are listed
        // and take the per-point test 8 at a time -- lane l tests pair l >> 3 with the point of lane
        // 8 j + (l & 7), fetched by ds_bpermute with its threshold -- so the per-point test is issued
        // for the pairs some point of a sub-cluster can need, not for all 64 lanes per kept face.
        // Each bound is conservative (a skip is proven, R and the thresholds only overestimate), so
        // every pair the r05 per-point test passes still passes: the queued pairs and the minimum
        // are unchanged.
        const T gpsq = [&]() {
          T v = valid ? psq : (T)INFINITY;
#pragma unroll
          for (int o = 1; o < 8; o <<= 1) v = fmax(v, __shfl_xor(v, o));
          return v;
        }();
        while (mask) {
          int myf = 0, nbf = 0;  // lane k < 8: the batch's k-th kept face slot
#pragma unroll
          for (int k = 0; k < 8; k++) {
            if (mask) {
              const int sj = s0 + __builtin_ctzll(mask);
              mask &= mask - 1;
              if (lane == k) myf = sj;
              nbf++;
            }
          }
          const int kf = lane & 7;
          const int fk = __shfl(myf, kf);
          bool sub = kf < nbf;
          if (sub) {
            const FaceRec<T> &fr = sf[fk];
            const T sl = (T)(256.0 * P2M_E) * (cinf + R + fr.hmax);
            const T A = fmax(fabs(dot(cj, fr.un) - sp.dv[fk]) - fr.thick - sl, (T)0);
            T b = dot(cj, mk(sp.o[0][fk], sp.o[1][fk], sp.o[2][fk])) - sp.off[0][fk];
            b = fmax(b, dot(cj, mk(sp.o[3][fk], sp.o[4][fk], sp.o[5][fk])) - sp.off[1][fk]);
            b = fmax(b, dot(cj, mk(sp.o[6][fk], sp.o[7][fk], sp.o[8][fk])) - sp.off[2][fk]);
            const T B = fmax(b - sl, (T)0);
            const T K = (Rj + gpsq) * (T)(1.0 + 16.0 * P2M_E) + sl;
            if ((A * A + B * B) * (T)(1.0 - 32.0 * P2M_E) > K * K * (T)(1.0 + 32.0 * P2M_E)) sub = false;
          }
          const uint64_t sm = __ballot(sub);
          const int np = __popcll(sm);
          // the kept (face, sub-cluster) pairs of the batch, in lane order: lane index L per entry
          if (sub) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
            s_sp[wid][rank] = (uint8_t)lane;
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
          for (int c = 0; c < np; c += 8) {  // wave-uniform
            const int e = c + (lane >> 3);
            const bool on = e < np;
            const int L = on ? (int)s_sp[wid][e] : 0;
            const int sj = __shfl(myf, L & 7);
            const int owner = (L & ~7) | (lane & 7);
            const V3<T> pp = mk(__shfl(p.x, owner), __shfl(p.y, owner), __shfl(p.z, owner));
            const T opsq = __shfl(psq, owner);
            const bool ovalid = __shfl((int)valid, owner) != 0;
            const FaceRec<T> &fr = sf[sj];
            const T sl = (T)(256.0 * P2M_E) * (cinf + R + fr.hmax);
            const T A = fmax(fabs(dot(pp, fr.un) - sp.dv[sj]) - fr.thick - sl, (T)0);
            T b = dot(pp, mk(sp.o[0][sj], sp.o[1][sj], sp.o[2][sj])) - sp.off[0][sj];
            b = fmax(b, dot(pp, mk(sp.o[3][sj], sp.o[4][sj], sp.o[5][sj])) - sp.off[1][sj]);
            b = fmax(b, dot(pp, mk(sp.o[6][sj], sp.o[7][sj], sp.o[8][sj])) - sp.off[2][sj]);
            const T B = fmax(b - sl, (T)0);
            const T K = opsq + sl;
            const bool pass = on && ovalid && !((A * A + B * B) * (T)(1.0 - 32.0 * P2M_E) > K * K * (T)(1.0 + 32.0 * P2M_E));
            const uint64_t pm = __ballot(pass);
            if (pass) {
              const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
              s_q[wid][(qhead + qcnt + rank) & (P2M_QCAP - 1)] = (uint16_t)(owner | (sj << 6));
            }
            qcnt += (uint32_t)__popcll(pm);
#ifdef KL_P2M_PROBE
            g_p2m_pairs += __popcll(pm);
#endif
            if (qcnt >= 64) {
              __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
              __builtin_amdgcn_wave_barrier();
              run_batch(64);
            }
          }
        }
        continue;
      }
      if (pairs) {
        // the per-point test of each kept face (the wave test's bound with this lane's point, R = 0),
        // passing pairs appended to the ring
        while (mask) {
          const int sj = s0 + __builtin_ctzll(mask);
          mask &= mask - 1;
          const FaceRec<T> &fr = sf[sj];
          const T sl = (T)(256.0 * P2M_E) * (cinf + R + fr.hmax);
          const T A = fmax(fabs(dot(p, fr.un) - sp.dv[sj]) - fr.thick - sl, (T)0);
          T b = dot(p, mk(sp.o[0][sj], sp.o[1][sj], sp.o[2][sj])) - sp.off[0][sj];
          b = fmax(b, dot(p, mk(sp.o[3][sj], sp.o[4][sj], sp.o[5][sj])) - sp.off[1][sj]);
          b = fmax(b, dot(p, mk(sp.o[6][sj], sp.o[7][sj], sp.o[8][sj])) - sp.off[2][sj]);
          const T B = fmax(b - sl, (T)0);
          const T K = psq + sl;
          const bool pass = valid && !((A * A + B * B) * (T)(1.0 - 32.0 * P2M_E) > K * K * (T)(1.0 + 32.0 * P2M_E));
          const uint64_t pm = __ballot(pass);
          if (pass) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
            s_q[wid][(qhead + qcnt + rank) & (P2M_QCAP - 1)] = (uint16_t)(lane | (sj << 6));
          }
          qcnt += (uint32_t)__popcll(pm);
#ifdef KL_P2M_PROBE
          g_p2m_pairs += __popcll(pm);
#endif
          if (qcnt >= 64) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            run_batch(64);
          }
        }
        continue;
      }
      // fold one evaluated face into the reference's tile-wise running minimum
      auto fold = [&](int64_t f, float d, int t) {
        if ((f & 511) == 0) {  // a reference tile begins: merge the previous tile, restart
          if (f > f_begin && ((first_split && f == 512) || best > tbest)) {
            best = tbest; best_f = tbest_f; best_t = tbest_t;
          }
          tbest = (T)d; tbest_f = f; tbest_t = t;
        } else if (tbest > (T)d) {
          tbest = (T)d; tbest_f = f; tbest_t = t;
        }
      };
      // two faces per iteration: both records' LDS reads and both evaluations in flight together
      // (the fold still takes them in face order)
      while (mask) {
        const int sj = s0 + __builtin_ctzll(mask);
        mask &= mask - 1;
        if (mask) {
          const int sk = s0 + __builtin_ctzll(mask);
          mask &= mask - 1;
          int t0, t1;
          const float d0 = point_face<T>(p, sf[sj], t0);
          const float d1 = point_face<T>(p, sf[sk], t1);
          fold(start + sj, d0, t0);
          fold(start + sk, d1, t1);
        } else {
          int t;
          const float d = point_face<T>(p, sf[sj], t);
          fold(start + sj, d, t);
        }
      }
    }
    if (pairs && qcnt) {  // the tile's records are rewritten next: drain the ring
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      run_batch((int)qcnt);
    }
    if (share && valid) {
      const float cur = pairs ? (float)pthr : (float)fmin(best, tbest);
      if (cur < published) {
        atomicMin(gbest + si, __float_as_uint(cur));
        published = cur;
      }
    }
  }
#ifdef KL_P2M_PROBE
  if (lane == 0) {
    atomicAdd(&::kl::g_p2m_skipped, g_p2m_skipped);
    atomicAdd(&::kl::g_p2m_evaluated, g_p2m_evaluated);
    atomicAdd(&::kl::g_p2m_pairs, g_p2m_pairs);
  }
#endif
  if (!valid) return;
  if (pairs) {
    const unsigned long long key = s_best[threadIdx.x];
    // no pair of this split passed (another split holds a strictly better face): +inf, never chosen
    best = key == KEY_NONE ? (T)INFINITY : (T)__uint_as_float((uint32_t)(key >> 32));
    best_f = key == KEY_NONE ? 0 : (int64_t)((uint32_t)key >> 3);
    best_t = key == KEY_NONE ? 0 : (int)(key & 7u);
  } else if (f_end > f_begin && ((first_split && f_end <= 512) || best > tbest)) {
    best = tbest; best_f = tbest_f; best_t = tbest_t;
  }
  if (part_dist) {
    const int64_t o = (int64_t)blockIdx.y * P + si;
    part_dist[o] = best;
    part_idx[o] = best_f;
    part_type[o] = best_t;
  } else {
    out_dist[pi] = best;
    out_idx[pi] = best_f;
    out_type[pi] = best_t;
  }
}

// rows of the dev kernel's pruning records (the workspace keeps their room in every build)
constexpr int P2M_PR_ROWS = 18;
#if KL_DEV  // the scalar-record p2m kernel (dev param 11 = 2 / 3): a measured dead end, DESIGN.md 3.4
// ---- global face records (the sorted path): p2m_faces_kernel writes, once per call, each face's
// evaluation record (FaceRecS) and its pruning record as structure-of-arrays rows of length Fp:
// rows 0..12 = make_prune_vals, 13..15 = un, 16 = thick, 17 = hmax.

template <typename T>
__global__ void __launch_bounds__(256) p2m_faces_kernel(const T *__restrict__ fv, int64_t F, int64_t Fp,
                                                         FaceRecS<T> *__restrict__ rec, T *__restrict__ pr) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= F) return;
  FaceRec<T> r;
  make_face<T>(fv + f * 9, r);
  FaceRecS<T> g;
  g.v1 = r.v1; g.v2 = r.v2; g.v3 = r.v3;
  g.e12 = r.e12; g.e23 = r.e23; g.e31 = r.e31;
  g.un = r.un; g.en12 = r.en12; g.en23 = r.en23; g.en31 = r.en31;
  g.l12 = r.l12; g.l23 = r.l23; g.l31 = r.l31;
  g.pad0 = g.pad1 = g.pad2 = (T)0;
  rec[f] = g;
  T v[13];
  make_prune_vals<T>(r, v);
#pragma unroll
  for (int k = 0; k < 13; k++) pr[k * Fp + f] = v[k];
  pr[13 * Fp + f] = r.un.x;
  pr[14 * Fp + f] = r.un.y;
  pr[15 * Fp + f] = r.un.z;
  pr[16 * Fp + f] = r.thick;
  pr[17 * Fp + f] = r.hmax;
}

// p2m_fwd_kernel with the face records read from global memory instead of staged through LDS:
// each lane reads its face's pruning record (coalesced rows), and the evaluation loop reads the
// picked face's record with a wave-uniform index -- scalar loads, the record in SGPRs -- so
// the records take no VGPRs and no LDS, and the waves of a block never synchronise.  Same
// skipping test, same fold, same results.
template <typename T, bool PAIR>
__global__ void __launch_bounds__(256) p2m_fwd_grec_kernel(const T *__restrict__ pts,
                                                            const FaceRecS<T> *__restrict__ rec,
                                                            const T *__restrict__ pr, int64_t Fp,
                                                            const int32_t *__restrict__ order, int64_t P, int64_t F,
                                                            int64_t split_faces, T *__restrict__ out_dist,
                                                            int64_t *__restrict__ out_idx, int32_t *__restrict__ out_type,
                                                            T *__restrict__ part_dist, int64_t *__restrict__ part_idx,
                                                            int32_t *__restrict__ part_type,
                                                            const int32_t *__restrict__ bounds, uint32_t *gbest) {
  const int64_t si = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool valid = si < P;
  const int64_t pi = valid ? (int64_t)order[si] : 0;
  const bool first_split = blockIdx.y == 0;
  const int64_t f_begin = (int64_t)blockIdx.y * split_faces;
  const int64_t f_end = min(F, f_begin + split_faces);
  const int lane = threadIdx.x & 63;
  V3<T> p = mk((T)0, (T)0, (T)0);
  if (valid) p = mk(pts[pi * 3], pts[pi * 3 + 1], pts[pi * 3 + 2]);
  const V3<T> p0 = mk(__shfl(p.x, 0), __shfl(p.y, 0), __shfl(p.z, 0));
  const V3<T> q = valid ? p : p0;
  const bool fin = isfinite(q.x) && isfinite(q.y) && isfinite(q.z);
  const bool all_fin = __all(fin);
  V3<T> c = mk((T)0, (T)0, (T)0);
  T R = (T)INFINITY, cinf = (T)0;
  if (all_fin) {
    c = mk((wave_min(q.x) + wave_max(q.x)) * (T)0.5, (wave_min(q.y) + wave_max(q.y)) * (T)0.5,
           (wave_min(q.z) + wave_max(q.z)) * (T)0.5);
    const V3<T> dq = q - c;
    R = wave_max(kl_sqrt<T>(dot(dq, dq))) * (T)(1.0 + 16.0 * P2M_E);
    cinf = fmax(fmax(fabs(c.x), fabs(c.y)), fabs(c.z));
  }
  const bool share = gbest != nullptr && all_fin && bounds[6] != 0 && cinf + R < (T)1e15;
  float published = INFINITY;
  T best = (T)INFINITY, tbest = (T)INFINITY;
  int64_t best_f = 0, tbest_f = 0;
  int best_t = 0, tbest_t = 0;
  auto fold = [&](int64_t f, float d, int t) {
    if ((f & 511) == 0) {
      if (f > f_begin && ((first_split && f == 512) || best > tbest)) {
        best = tbest; best_f = tbest_f; best_t = tbest_t;
      }
      tbest = (T)d; tbest_f = f; tbest_t = t;
    } else if (tbest > (T)d) {
      tbest = (T)d; tbest_f = f; tbest_t = t;
    }
  };
  for (int64_t start = f_begin; start < f_end; start += 64) {
    const int n = (int)min((int64_t)64, f_end - start);
    T thr = fmin(best, tbest);
    if (thr != thr || !valid) thr = valid ? (T)INFINITY : (T)0;
    if (share && valid && (start & 127) == 0)
      thr = fmin(thr, (T)__uint_as_float(__hip_atomic_load(gbest + si, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    const T thr_max = wave_max_all(thr);  // (every lane active: the chunk loop is wave-uniform)
    const int64_t f = start + lane;
    bool eval = lane < n;
    if (eval && all_fin && (f & 511) != 0 && thr_max < (T)INFINITY) {
      const T *r = pr + f;
      const T hmax = r[17 * Fp], thick = r[16 * Fp];
      const V3<T> un = mk(r[13 * Fp], r[14 * Fp], r[15 * Fp]);
      const T M = cinf + R + hmax;
      const T sl = (T)(256.0 * P2M_E) * M;
      const T A = fmax(fabs(dot(c, un) - r[12 * Fp]) - thick - sl, (T)0);
      T b = dot(c, mk(r[0], r[Fp], r[2 * Fp])) - r[9 * Fp];
      b = fmax(b, dot(c, mk(r[3 * Fp], r[4 * Fp], r[5 * Fp])) - r[10 * Fp]);
      b = fmax(b, dot(c, mk(r[6 * Fp], r[7 * Fp], r[8 * Fp])) - r[11 * Fp]);
      const T B = fmax(b - sl, (T)0);
      const T K = (R + kl_sqrt<T>(thr_max)) * (T)(1.0 + 16.0 * P2M_E) + sl;
      if ((A * A + B * B) * (T)(1.0 - 32.0 * P2M_E) > K * K * (T)(1.0 + 32.0 * P2M_E)) eval = false;
    }
    uint64_t mask = __ballot(eval);
    while (mask) {
      const int sj = __builtin_ctzll(mask);
      mask &= mask - 1;
      if (PAIR && mask) {
        const int sk = __builtin_ctzll(mask);
        mask &= mask - 1;
        int t0, t1;
        const FaceRecS<T> fa = rec[start + sj], fb = rec[start + sk];
        const float d0 = point_face<T>(p, fa, t0);
        const float d1 = point_face<T>(p, fb, t1);
        fold(start + sj, d0, t0);
        fold(start + sk, d1, t1);
      } else {
        int t;
        const FaceRecS<T> fa = rec[start + sj];
        const float d = point_face<T>(p, fa, t);
        fold(start + sj, d, t);
      }
    }
    if (share && valid && ((start + 64) & 127) == 0) {
      const float cur = (float)fmin(best, tbest);
      if (cur < published) {
        atomicMin(gbest + si, __float_as_uint(cur));
        published = cur;
      }
    }
  }
  if (!valid) return;
  if (f_end > f_begin && ((first_split && f_end <= 512) || best > tbest)) {
    best = tbest; best_f = tbest_f; best_t = tbest_t;
  }
  if (part_dist) {
    const int64_t o = (int64_t)blockIdx.y * P + si;
    part_dist[o] = best;
    part_idx[o] = best_f;
    part_type[o] = best_t;
  } else {
    out_dist[pi] = best;
    out_idx[pi] = best_f;
    out_type[pi] = best_t;
  }
}
#endif  // KL_DEV

// folds the splits' partials in face order with the reference's strict '<'
template <typename T>
__global__ void __launch_bounds__(256) p2m_combine_kernel(const int32_t *__restrict__ order, int64_t P, int splits,
                                                           const T *__restrict__ part_dist,
                                                           const int64_t *__restrict__ part_idx,
                                                           const int32_t *__restrict__ part_type,
                                                           T *__restrict__ out_dist, int64_t *__restrict__ out_idx,
                                                           int32_t *__restrict__ out_type) {
  const int64_t si = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (si >= P) return;
  T best = part_dist[si];
  int64_t bi = part_idx[si];
  int32_t bt = part_type[si];
  for (int k = 1; k < splits; k++) {
    const T d = part_dist[(int64_t)k * P + si];
    if (best > d) {
      best = d;
      bi = part_idx[(int64_t)k * P + si];
      bt = part_type[(int64_t)k * P + si];
    }
  }
  const int64_t pi = order ? (int64_t)order[si] : si;
  out_dist[pi] = best;
  out_idx[pi] = bi;
  out_type[pi] = bt;
}

// ---- Morton ordering of the points (the clusters the skipping test works on)
__device__ __forceinline__ int32_t f2ord(float v) {  // order-preserving float -> int
  const int32_t b = __float_as_int(v);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int32_t b) { return __int_as_float(b >= 0 ? b : b ^ 0x7fffffff); }

// one 1024-thread block: per-axis min / max of the finite point coordinates
// bounds[6] = 1 iff every face is proper (finite, |coordinates| < 1e15, edges and normal of
// nonzero length as make_face computes them): then no point--face distance of a finite,
// bounded point is NaN, the reference fold is the plain (distance, index) minimum, and any
// computed distance is an upper bound of the result (p2m_fwd_kernel's shared thresholds).
template <typename T>
__global__ void __launch_bounds__(1024) p2m_bounds_kernel(const T *__restrict__ pts, int64_t P,
                                                          const T *__restrict__ fv, int64_t F, int32_t *partial) {
  __shared__ float red[6][16];
  __shared__ int proper;
  if (threadIdx.x == 0) proper = 1;
  __syncthreads();
  bool ok = true;
  for (int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; f < F; f += (int64_t)gridDim.x * blockDim.x) {
    const T *v = fv + f * 9;
    const V3<T> v1 = mk(v[0], v[1], v[2]), v2 = mk(v[3], v[4], v[5]), v3 = mk(v[6], v[7], v[8]);
    const V3<T> e12 = v2 - v1, e23 = v3 - v2, e31 = v1 - v3;
    const V3<T> normal = cross(v1 - v2, e31);
    const T nn = dot(normal, normal), l12 = dot(e12, e12), l23 = dot(e23, e23), l31 = dot(e31, e31);
    const T hm = fmax(fmax(fmax(fabs(v1.x), fabs(v1.y)), fmax(fabs(v1.z), fabs(v2.x))),
                      fmax(fmax(fabs(v2.y), fabs(v2.z)), fmax(fmax(fabs(v3.x), fabs(v3.y)), fabs(v3.z))));
    ok = ok && hm < (T)1e15 && nn > (T)1e-30 && l12 > (T)1e-30 && l23 > (T)1e-30 && l31 > (T)1e-30 &&
         nn < (T)1e36;  // (hm < 1e15 also rejects NaN / inf)
  }
  if (!ok) proper = 0;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float v = (float)pts[i * 3 + a];
      if (isfinite(v)) {
        lo[a] = fminf(lo[a], v);
        hi[a] = fmaxf(hi[a], v);
      }
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < 3; a++) {
    const float l = wave_min(lo[a]), h = wave_max(hi[a]);
    if ((threadIdx.x & 63) == 0) {
      red[a][w] = l;
      red[3 + a][w] = h;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int a = threadIdx.x;
    float r = red[a][0];
    for (int k = 1; k < (int)(blockDim.x >> 6); k++) r = a < 3 ? fminf(r, red[a][k]) : fmaxf(r, red[a][k]);
    partial[blockIdx.x * 8 + a] = f2ord(r);
  }
  if (threadIdx.x == 6) partial[blockIdx.x * 8 + 6] = proper;
}

// folds the bound kernel's per-block partials (every block of the Morton kernel does it, into
// LDS; block 0 also stores the result for p2m_fwd_kernel)
__device__ __forceinline__ void fold_bounds(const int32_t *__restrict__ partial, int nblk, int32_t *sb,
                                            int32_t *bounds) {
  if (threadIdx.x < 7) {
    const int a = threadIdx.x;
    int32_t r = partial[a];
    for (int k = 1; k < nblk; k++) {
      const int32_t v = partial[k * 8 + a];
      r = a < 3 ? min(r, v) : a < 6 ? max(r, v) : (r & v);
    }
    sb[a] = r;
    if (blockIdx.x == 0) bounds[a] = r;
  }
  __syncthreads();
}

// 3-D Hilbert index of a 10-bit-per-axis grid cell (Skilling's transpose transform, then
// bit interleave).  Hilbert order keeps every run of 64 consecutive points spatially
// compact (no Morton jumps across octant boundaries): on cfg2 the mean cluster radius is
// 0.39 against 0.50 for Morton order, and the faces a wave must evaluate shrink with it.
__device__ __forceinline__ uint32_t hilbert3(uint32_t x0, uint32_t x1, uint32_t x2) {
  uint32_t X[3] = {x0, x1, x2};
  for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1) {
    const uint32_t P = Q - 1;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      if (X[i] & Q) {
        X[0] ^= P;
      } else {
        const uint32_t t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  uint32_t t = 0;
  for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1;
  X[0] ^= t;
  X[1] ^= t;
  X[2] ^= t;
  uint32_t h = 0;
  for (int b = 9; b >= 0; b--) h = (h << 3) | (((X[0] >> b) & 1) << 2) | (((X[1] >> b) & 1) << 1) | ((X[2] >> b) & 1);
  return h;
}

constexpr uint32_t P2M_KEY_BITS = 31;  // 30-bit Hilbert keys; non-finite points get 2^30 (last)

template <typename T>
__global__ void __launch_bounds__(256) p2m_morton_kernel(const T *__restrict__ pts, int64_t P,
                                                          const int32_t *__restrict__ partial, int nblk,
                                                          int32_t *out_bounds, uint32_t *keys, int32_t *vals) {
  __shared__ int32_t bounds[8];
  fold_bounds(partial, nblk, bounds, out_bounds);
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= P) return;
  uint32_t code = 1u << 30;  // non-finite points last
  const float x = (float)pts[i * 3], y = (float)pts[i * 3 + 1], z = (float)pts[i * 3 + 2];
  if (isfinite(x) && isfinite(y) && isfinite(z)) {
    uint32_t g[3];
    const float v[3] = {x, y, z};
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float lo = ord2f(bounds[a]), hi = ord2f(bounds[3 + a]);
      const float t = hi > lo ? (v[a] - lo) / (hi - lo) : 0.0f;
      g[a] = (uint32_t)fminf(fmaxf(t * 1024.0f, 0.0f), 1023.0f);
    }
    code = hilbert3(g[0], g[1], g[2]);
  }
  keys[i] = code;
  vals[i] = (int32_t)i;
}

#ifndef KL_P2M_MAX_SPLITS
#define KL_P2M_MAX_SPLITS 32
#endif
constexpr int P2M_MAX_SPLITS = KL_P2M_MAX_SPLITS;
// workgroups the (point block, face split) grid aims for (scripts/dev/p2m_probe.hip sweeps it)
constexpr int P2M_TARGET_BLOCKS = 10240;  // dev param 28 = N overrides (A/B)
constexpr int P2M_BOUND_BLOCKS = 64;  // blocks of p2m_bounds_kernel

struct P2MWs {
  size_t keys_in, keys_out, vals_in, vals_out, temp, temp_bytes, part, gbest, rec, pr, bytes;
  int64_t Fp;
  P2MWs(int64_t P, int64_t F, size_t esize) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                       (const int32_t *)nullptr, (int32_t *)nullptr, (int)P, 0, P2M_KEY_BITS);
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    keys_in = 256 + 32 * P2M_BOUND_BLOCKS;  // [0, 28): bounds + flag; [256, ...): per-block partials
    keys_out = keys_in + al(4 * (size_t)P);
    vals_in = keys_out + al(4 * (size_t)P);
    vals_out = vals_in + al(4 * (size_t)P);
    temp = vals_out + al(4 * (size_t)P);
    temp_bytes = tb;
    part = temp + al(tb);  // P2M_MAX_SPLITS x P x (dist 8 + idx 8 + type 4)
    gbest = part + al((size_t)P2M_MAX_SPLITS * P * 20);  // P x float bits (shared thresholds)
    Fp = (F + 63) & ~(int64_t)63;
    rec = gbest + al(4 * (size_t)P);  // F x FaceRecS (36 values), then P2M_PR_ROWS rows of Fp
    pr = rec + al((size_t)F * 36 * esize);
    bytes = pr + al((size_t)P2M_PR_ROWS * Fp * esize);
  }
};

// below this many pairs the Morton sort is not worth its launches
constexpr int64_t P2M_SORT_MIN_PAIRS = (int64_t)1 << 24;

template <typename T, typename A>
__device__ __forceinline__ void edge_bwd(V3<T> vab, V3<T> pb, A *ga, A *gb, T *gp, T grad) {
  const T l = dot(vab, pb);
  const T m = dot(vab, vab);
  const T k = l / m;
  const T j = (T)fmax(0.0, fmin(1.0, (double)k));
  const V3<T> i = vab * j - pb;
  const V3<T> i_bar = i * grad;
  const T j_bar = dot(i_bar, vab);
  const T dj_dk = (k > 0 && k < 1) ? (T)1 : (T)0;
  const T k_bar = j_bar * dj_dk;
  const T m_bar = k_bar * (-l / (m * m));
  const T l_bar = k_bar * ((T)1 / m);
  const V3<T> di_dpb = mk(-i_bar.x, -i_bar.y, -i_bar.z);
  const V3<T> pb_bar = vab * l_bar + di_dpb;
  const V3<T> dm_dvab = vab * (T)2.;
  const V3<T> di_dvab = i_bar * j;
  const V3<T> vab_bar = (dm_dvab * m_bar + pb * l_bar) + di_dvab;
  const V3<T> vb_bar = mk(-vab_bar.x - pb_bar.x, -vab_bar.y - pb_bar.y, -vab_bar.z - pb_bar.z);
  gp[0] = pb_bar.x; gp[1] = pb_bar.y; gp[2] = pb_bar.z;
  atomicAdd(ga + 0, (A)vab_bar.x); atomicAdd(ga + 1, (A)vab_bar.y); atomicAdd(ga + 2, (A)vab_bar.z);
  atomicAdd(gb + 0, (A)vb_bar.x); atomicAdd(gb + 1, (A)vb_bar.y); atomicAdd(gb + 2, (A)vb_bar.z);
}

// A = double: the per-point terms summed per face coordinate in double (rounded once by
// acc_finalize), so the gradient does not depend on the atomics' order; A = T: the reference's
// float atomics (no workspace).
template <typename T, typename A>
__global__ void __launch_bounds__(256) p2m_bwd_kernel(const T *__restrict__ grad_dist, const T *__restrict__ pts,
                                                       const T *__restrict__ fv, const int64_t *__restrict__ fidx,
                                                       const int32_t *__restrict__ ftype, int64_t P,
                                                       T *__restrict__ gpts, A *__restrict__ gfv) {
  const int64_t pi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pi >= P) return;
  const int type = ftype[pi];
  const int64_t f = fidx[pi];
  const V3<T> p = mk(pts[pi * 3], pts[pi * 3 + 1], pts[pi * 3 + 2]);
  const T *v = fv + f * 9;
  const V3<T> v1 = mk(v[0], v[1], v[2]), v2 = mk(v[3], v[4], v[5]), v3 = mk(v[6], v[7], v[8]);
  const V3<T> e12 = v2 - v1, e23 = v3 - v2, e31 = v1 - v3;
  const T go = (T)(2. * (double)grad_dist[pi]);
  A *g = gfv + f * 9;
  T *gp = gpts + pi * 3;
  if (type == 0) {
    const V3<T> pv = p - v1;
    const V3<T> e21 = v1 - v2;
    const V3<T> normal = cross(e21, e31);
    const T len = kl_sqrt<T>(dot(normal, normal));
    const V3<T> un = normal / len;
    const T dist = dot(pv, un);
    const V3<T> gdv = un * (dist * go);
    const T gd = dot(un, gdv);
    const V3<T> gpv = un * gd;
    const V3<T> gun = gdv * dist + pv * gd;
    const T glen = -dot(normal, gun) / (len * len);
    const T gd2 = glen / ((T)2 * kl_sqrt<T>(dot(normal, normal)));
    const V3<T> gn = gun / len + normal * (gd2 * (T)2.);
    const V3<T> ge31 = cross(gn, e21);
    const V3<T> ge21 = cross(e31, gn);
    gp[0] = gpv.x; gp[1] = gpv.y; gp[2] = gpv.z;
    const V3<T> tmp = (ge31 + ge21) - gpv;
    atomicAdd(g + 0, (A)tmp.x); atomicAdd(g + 1, (A)tmp.y); atomicAdd(g + 2, (A)tmp.z);
    atomicAdd(g + 3, (A)-ge21.x); atomicAdd(g + 4, (A)-ge21.y); atomicAdd(g + 5, (A)-ge21.z);
    atomicAdd(g + 6, (A)-ge31.x); atomicAdd(g + 7, (A)-ge31.y); atomicAdd(g + 8, (A)-ge31.z);
  } else if (type >= 1 && type <= 3) {
    const V3<T> vv = type == 1 ? v1 : (type == 2 ? v2 : v3);
    const V3<T> gdv = (p - vv) * go;
    A *gg = g + (type - 1) * 3;
    atomicAdd(gg + 0, (A)-gdv.x); atomicAdd(gg + 1, (A)-gdv.y); atomicAdd(gg + 2, (A)-gdv.z);
    gp[0] = gdv.x; gp[1] = gdv.y; gp[2] = gdv.z;
  } else if (type == 4) {
    edge_bwd<T, A>(e12, p - v1, g + 3, g + 0, gp, go);
  } else if (type == 5) {
    edge_bwd<T, A>(e23, p - v2, g + 6, g + 3, gp, go);
  } else {
    edge_bwd<T, A>(e31, p - v3, g + 0, g + 6, gp, go);
  }
}

// ---------------------------------------------------------------- sided distance
// Arithmetic happens in the storage type itself (half in half, integers in their own
// type), as the reference's scalar_t arithmetic does.
constexpr int SD_TILE = 512;

// The largest value of S: a split's starting best (no tile best exceeds it; NaN never replaces it)
template <typename S>
__device__ __forceinline__ S sd_top() {
  if constexpr (std::is_same<S, __half>::value) return __float2half(INFINITY);
  else if constexpr (std::is_floating_point<S>::value) return (S)INFINITY;
  else return std::numeric_limits<S>::max();
}

// grid (point blocks, batch, splits): split z takes the 512-point tiles [z tps, (z + 1) tps) of p2.
// Split 0 folds as the reference (its first tile unconditional, then strict '>'); a later split
// starts from sd_top(), so it takes its first non-NaN tile best, and sided_combine_kernel folds the
// splits' results in order with the reference's strict '>' -- the reference's fold over all tiles,
// NaN tile bests included (a NaN best never replaces, and a first NaN tile stays).  With one split
// (part == nullptr) the result goes straight to dist / idx.
template <typename S>
__global__ void __launch_bounds__(256) sided_fwd_kernel(const S *__restrict__ p1, const S *__restrict__ p2,
                                                         int64_t N, int64_t M, S *__restrict__ dist,
                                                         int64_t *__restrict__ idx, int64_t tps,
                                                         S *__restrict__ part_d, int64_t *__restrict__ part_i) {
  __shared__ S buf[SD_TILE * 3];
  const int b = blockIdx.y;
  const int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool valid = n < N;
  const S *a = p1 + ((int64_t)b * N + (valid ? n : 0)) * 3;
  const S x1 = a[0], y1 = a[1], z1 = a[2];
  const bool first_split = blockIdx.z == 0;
  S best_all = first_split ? S(0) : sd_top<S>();
  int64_t best_all_i = 0;
  const int64_t kb = (int64_t)blockIdx.z * tps * SD_TILE, ke = min(M, kb + tps * SD_TILE);
  for (int64_t k2 = kb; k2 < ke; k2 += SD_TILE) {
    const int end_k = (int)min((int64_t)SD_TILE, M - k2);
    __syncthreads();
    for (int t = threadIdx.x; t < end_k * 3; t += blockDim.x) buf[t] = p2[((int64_t)b * M + k2) * 3 + t];
    __syncthreads();
    S best = S(0);
    int64_t best_i = 0;
    for (int k = 0; k < end_k; k++) {
      const S dx = buf[k * 3 + 0] - x1;
      const S dy = buf[k * 3 + 1] - y1;
      const S dz = buf[k * 3 + 2] - z1;
      const S d = dx * dx + dy * dy + dz * dz;
      if (k == 0 || d < best) {
        best = d;
        best_i = k + k2;
      }
    }
    if ((first_split && k2 == 0) || best_all > best) {
      best_all = best;
      best_all_i = best_i;
    }
  }
  if (!valid) return;
  if (part_d) {
    const int64_t o = ((int64_t)blockIdx.z * gridDim.y + b) * N + n;
    part_d[o] = best_all;
    part_i[o] = best_all_i;
  } else {
    dist[(int64_t)b * N + n] = best_all;
    idx[(int64_t)b * N + n] = best_all_i;
  }
}

template <typename S>
__global__ void __launch_bounds__(256) sided_combine_kernel(int64_t BN, int splits, const S *__restrict__ part_d,
                                                             const int64_t *__restrict__ part_i, S *__restrict__ dist,
                                                             int64_t *__restrict__ idx) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= BN) return;
  S best = part_d[t];
  int64_t bi = part_i[t];
  for (int z = 1; z < splits; z++) {
    const S d = part_d[(int64_t)z * BN + t];
    if (best > d) {
      best = d;
      bi = part_i[(int64_t)z * BN + t];
    }
  }
  dist[t] = best;
  idx[t] = bi;
}

template <typename S>
__device__ __forceinline__ void atomic_add_any(S *p, S v) { atomicAdd(p, v); }
template <>
__device__ __forceinline__ void atomic_add_any<__half>(__half *p, __half v) {
  // emulate with a 32-bit CAS on the containing word
  uintptr_t addr = reinterpret_cast<uintptr_t>(p);
  unsigned int *w = reinterpret_cast<unsigned int *>(addr & ~(uintptr_t)3);
  const bool hi = (addr & 2) != 0;
  unsigned int old = *w, assumed;
  do {
    assumed = old;
    unsigned short h = hi ? (unsigned short)(assumed >> 16) : (unsigned short)(assumed & 0xffff);
    __half cur = __ushort_as_half(h);
    unsigned short nh = __half_as_ushort(__hadd(cur, v));
    unsigned int nw = hi ? ((assumed & 0xffffu) | ((unsigned int)nh << 16)) : ((assumed & 0xffff0000u) | nh);
    old = atomicCAS(w, assumed, nw);
  } while (old != assumed);
}
template <typename S>
__device__ __forceinline__ void atomic_add_small_int(S *p, S v) {
  uintptr_t addr = reinterpret_cast<uintptr_t>(p);
  unsigned int *w = reinterpret_cast<unsigned int *>(addr & ~(uintptr_t)3);
  const int sh = (int)(addr & 3) * 8;
  const unsigned int msk = (sizeof(S) == 1 ? 0xffu : 0xffffu) << sh;
  unsigned int old = *w, assumed;
  do {
    assumed = old;
    S cur = (S)((assumed & msk) >> sh);
    S nv = (S)(cur + v);
    unsigned int nw = (assumed & ~msk) | (((unsigned int)(std::make_unsigned_t<S>)nv << sh) & msk);
    old = atomicCAS(w, assumed, nw);
  } while (old != assumed);
}
template <>
__device__ __forceinline__ void atomic_add_any<uint8_t>(uint8_t *p, uint8_t v) { atomic_add_small_int(p, v); }
template <>
__device__ __forceinline__ void atomic_add_any<int8_t>(int8_t *p, int8_t v) { atomic_add_small_int(p, v); }
template <>
__device__ __forceinline__ void atomic_add_any<int16_t>(int16_t *p, int16_t v) { atomic_add_small_int(p, v); }
template <>
__device__ __forceinline__ void atomic_add_any<int64_t>(int64_t *p, int64_t v) {
  atomicAdd(reinterpret_cast<unsigned long long *>(p), (unsigned long long)v);
}

template <typename S>
__global__ void __launch_bounds__(256) sided_bwd_kernel(const S *__restrict__ grad, const S *__restrict__ p1,
                                                         const S *__restrict__ p2, const int64_t *__restrict__ idx,
                                                         int64_t N, int64_t M, S *__restrict__ g1, S *__restrict__ g2) {
  const int b = blockIdx.y;
  const int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int64_t mi = (int64_t)b * N + n;
  const S x1 = p1[mi * 3], y1 = p1[mi * 3 + 1], z1 = p1[mi * 3 + 2];
  const int64_t j = (idx[mi] + (int64_t)b * M) * 3;
  const S x2 = p2[j], y2 = p2[j + 1], z2 = p2[j + 2];
  const S g = grad[mi];
  const S two = S(2);
  g1[mi * 3 + 0] = two * (x1 - x2) * g;
  g1[mi * 3 + 1] = two * (y1 - y2) * g;
  g1[mi * 3 + 2] = two * (z1 - z2) * g;
  atomic_add_any<S>(g2 + j + 0, two * (x2 - x1) * g);
  atomic_add_any<S>(g2 + j + 1, two * (y2 - y1) * g);
  atomic_add_any<S>(g2 + j + 2, two * (z2 - z1) * g);
}

template <typename T>
static int p2m_fwd(int64_t P, int64_t F, const void *pts, const void *fv, void *dist, int64_t *idx, int32_t *type,
                   void *ws, size_t ws_bytes, hipStream_t st) {
  if (P == 0) return KL_OK;
  KL_REQUIRE(F > 0, "unbatched_triangle_distance_forward: face_vertices must not be empty");
  KL_REQUIRE(P < ((int64_t)1 << 31), "unbatched_triangle_distance_forward: too many points");
  const int32_t *order = nullptr;
  T *pd = nullptr;
  int64_t *pidx = nullptr;
  int32_t *pt = nullptr;
  const int32_t *bounds_c = nullptr;
  uint32_t *gbest = nullptr;
  const unsigned pblocks = (unsigned)cdiv(P, 256);
  int splits = 1;
  int64_t split_faces = F;
  if (ws && P * F >= P2M_SORT_MIN_PAIRS) {
    const P2MWs L(P, F, sizeof(T));
    KL_REQUIRE(ws_bytes >= L.bytes, "unbatched_triangle_distance_forward: workspace too small");
    char *w = reinterpret_cast<char *>(ws);
    int32_t *bounds = reinterpret_cast<int32_t *>(w);
    int32_t *partial = bounds + 64;  // [256, 256 + 32 * nblk) bytes
    const int nblk = (int)std::min<int64_t>(P2M_BOUND_BLOCKS, std::max<int64_t>(1, cdiv(std::max(P, F), 4096)));
    hipLaunchKernelGGL(p2m_bounds_kernel<T>, dim3(nblk), dim3(1024), 0, st, (const T *)pts, P, (const T *)fv, F,
                       partial);
    KL_CHECK_LAUNCH();
    uint32_t *kin = reinterpret_cast<uint32_t *>(w + L.keys_in), *kout = reinterpret_cast<uint32_t *>(w + L.keys_out);
    int32_t *vin = reinterpret_cast<int32_t *>(w + L.vals_in), *vout = reinterpret_cast<int32_t *>(w + L.vals_out);
    hipLaunchKernelGGL(p2m_morton_kernel<T>, dim3(pblocks), dim3(256), 0, st, (const T *)pts, P, partial, nblk,
                       bounds, kin, vin);
    KL_CHECK_LAUNCH();
    size_t tb = L.temp_bytes;
    KL_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(w + L.temp, tb, kin, kout, vin, vout, (int)P, 0, P2M_KEY_BITS, st));
    order = vout;
    bounds_c = bounds;
    gbest = reinterpret_cast<uint32_t *>(w + L.gbest);
    KL_CHECK_RC(fill_async(gbest, 0x7f, 4 * (size_t)P, st));  // 0x7f7f7f7f = 3.4e38, above any proper distance
    // enough (point block, face split) workgroups to fill the chip ~10 times over (cfg2:
    // 20 splits of 1024 faces, 1.6 ms; 14 of 1536: 2.0 ms; 40 of 512: 2.1 ms);
    // splits cover whole 512-face reference tiles
    const int64_t tiles = cdiv(F, 512);
    const int64_t target = g_dev_param[28] > 0 ? g_dev_param[28] : P2M_TARGET_BLOCKS;
    const int64_t want = std::max<int64_t>(1, cdiv(target, pblocks));
    splits = (int)std::min<int64_t>(std::min<int64_t>(want, tiles), P2M_MAX_SPLITS);
    split_faces = cdiv(tiles, splits) * 512;
    splits = (int)cdiv(F, split_faces);
    if (splits > 1) {
      pd = reinterpret_cast<T *>(w + L.part);
      pidx = reinterpret_cast<int64_t *>(w + L.part + (size_t)P2M_MAX_SPLITS * P * 8);
      pt = reinterpret_cast<int32_t *>(w + L.part + (size_t)P2M_MAX_SPLITS * P * 16);
    }
  }
  // dev param 11 = 2 / 3: face records read from global memory through scalar loads
  // (p2m_fwd_grec_kernel, one / two faces per iteration) instead of staged through LDS -- measured
  // slower at cfg2 (1.70 against 1.51 ms for two faces per iteration), kept for A/B
#if KL_DEV
  if (order && (g_dev_param[11] == 2 || g_dev_param[11] == 3)) {
    char *w = reinterpret_cast<char *>(ws);
    const P2MWs L(P, F, sizeof(T));
    FaceRecS<T> *rec = reinterpret_cast<FaceRecS<T> *>(w + L.rec);
    T *pr = reinterpret_cast<T *>(w + L.pr);
    hipLaunchKernelGGL(p2m_faces_kernel<T>, dim3((unsigned)cdiv(F, 256)), dim3(256), 0, st, (const T *)fv, F, L.Fp,
                       rec, pr);
    KL_CHECK_LAUNCH();
    if (g_dev_param[11] == 2)  // one face per iteration
      hipLaunchKernelGGL((p2m_fwd_grec_kernel<T, false>), dim3(pblocks, (unsigned)splits), dim3(256), 0, st,
                         (const T *)pts, (const FaceRecS<T> *)rec, (const T *)pr, L.Fp, order, P, F, split_faces,
                         (T *)dist, idx, type, pd, pidx, pt, bounds_c, gbest);
    else
      hipLaunchKernelGGL((p2m_fwd_grec_kernel<T, true>), dim3(pblocks, (unsigned)splits), dim3(256), 0, st,
                         (const T *)pts, (const FaceRecS<T> *)rec, (const T *)pr, L.Fp, order, P, F, split_faces,
                         (T *)dist, idx, type, pd, pidx, pt, bounds_c, gbest);
  } else
#endif
  if (g_dev_param[11] == 4 || !order) {  // dev param 11 = 4: the wave-level walk alone (r04)
    hipLaunchKernelGGL((p2m_fwd_kernel<T, false>), dim3(pblocks, (unsigned)splits), dim3(256), 0, st, (const T *)pts,
                       (const T *)fv, order, P, F, split_faces, (T *)dist, idx, type, pd, pidx, pt, bounds_c, gbest);
  } else if (g_dev_param[11] == 5) {  // dev param 11 = 5: the r05 pairs path (per-point test per kept face)
    hipLaunchKernelGGL((p2m_fwd_kernel<T, true, false>), dim3(pblocks, (unsigned)splits), dim3(256), 0, st,
                       (const T *)pts, (const T *)fv, order, P, F, split_faces, (T *)dist, idx, type, pd, pidx, pt,
                       bounds_c, gbest);
  } else {
    hipLaunchKernelGGL((p2m_fwd_kernel<T, true>), dim3(pblocks, (unsigned)splits), dim3(256), 0, st, (const T *)pts,
                       (const T *)fv, order, P, F, split_faces, (T *)dist, idx, type, pd, pidx, pt, bounds_c, gbest);
  }
  KL_CHECK_LAUNCH();
  if (splits > 1) {
    hipLaunchKernelGGL(p2m_combine_kernel<T>, dim3(pblocks), dim3(256), 0, st, order, P, splits, pd, pidx, pt,
                       (T *)dist, idx, type);
    KL_CHECK_LAUNCH();
  }
  return KL_OK;
}

template <typename T>
static int p2m_bwd(int64_t P, int64_t F, const void *grad, const void *pts, const void *fv, const int64_t *idx,
                   const int32_t *type, void *gp, void *gf, void *ws, size_t ws_bytes, hipStream_t st) {
  const size_t n = (size_t)F * 9;
  if (ws == nullptr) {  // the reference's float atomics into the zeroed output
    KL_CHECK_RC(fill_async(gf, 0, sizeof(T) * n, st));
    if (P == 0) return KL_OK;
    hipLaunchKernelGGL((p2m_bwd_kernel<T, T>), dim3((unsigned)cdiv(P, 256)), dim3(256), 0, st, (const T *)grad,
                       (const T *)pts, (const T *)fv, idx, type, P, (T *)gp, (T *)gf);
    KL_CHECK_LAUNCH();
    return KL_OK;
  }
  KL_REQUIRE(ws_bytes >= n * sizeof(double), "unbatched_triangle_distance_backward: workspace too small");
  double *acc = reinterpret_cast<double *>(ws);
  KL_CHECK_RC(fill_async(acc, 0, n * sizeof(double), st));
  if (P > 0) {
    hipLaunchKernelGGL((p2m_bwd_kernel<T, double>), dim3((unsigned)cdiv(P, 256)), dim3(256), 0, st, (const T *)grad,
                       (const T *)pts, (const T *)fv, idx, type, P, (T *)gp, acc);
    KL_CHECK_LAUNCH();
  }
  return acc_finalize<T>(acc, (T *)gf, n, false, st);
}

// The face gradient's double sums, not rounded (the sharded backward adds every rank's sums, then
// rounds once: kaolin/distributed.py).
template <typename T>
static int p2m_bwd_sums(int64_t P, int64_t F, const void *grad, const void *pts, const void *fv, const int64_t *idx,
                        const int32_t *type, void *gp, double *sums, hipStream_t st) {
  KL_CHECK_RC(fill_async(sums, 0, (size_t)F * 9 * sizeof(double), st));
  if (P == 0) return KL_OK;
  hipLaunchKernelGGL((p2m_bwd_kernel<T, double>), dim3((unsigned)cdiv(P, 256)), dim3(256), 0, st, (const T *)grad,
                     (const T *)pts, (const T *)fv, idx, type, P, (T *)gp, sums);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename S>
static int sided_fwd(int B, int64_t N, int64_t M, const void *p1, const void *p2, void *dist, int64_t *idx,
                     hipStream_t st) {
  if (B == 0 || N == 0) return KL_OK;
  KL_REQUIRE(M > 0, "sided_distance_forward: p2 must not be empty");
  // few point blocks (cfg1: 2,048 points, 8 workgroups): split p2's tiles over a third grid
  // dimension so the chip fills, partials in a stream-ordered scratch, folded in split order
  const int64_t pblocks = cdiv(N, 256) * B, tiles = cdiv(M, (int64_t)SD_TILE);
  int splits = 1;
  if (pblocks < 256 && tiles > 1 && g_dev_param[23] != 1)  // dev param 23 = 1: one split (A/B)
    splits = (int)std::min<int64_t>(tiles, cdiv(512, pblocks));
  const int64_t tps = cdiv(tiles, (int64_t)splits);
  splits = (int)cdiv(tiles, tps);
  if (splits == 1) {
    hipLaunchKernelGGL(sided_fwd_kernel<S>, dim3((unsigned)cdiv(N, 256), B), dim3(256), 0, st, (const S *)p1,
                       (const S *)p2, N, M, (S *)dist, idx, tps, (S *)nullptr, (int64_t *)nullptr);
    KL_CHECK_LAUNCH();
    return KL_OK;
  }
  const int64_t BN = (int64_t)B * N;
  void *ws = nullptr;
  const size_t db = (((size_t)splits * BN * sizeof(S)) + 255) & ~(size_t)255;
  KL_CHECK_HIP(hipMallocAsync(&ws, db + (size_t)splits * BN * sizeof(int64_t), st));
  S *pd = (S *)ws;
  int64_t *pi = (int64_t *)((char *)ws + db);
  hipLaunchKernelGGL(sided_fwd_kernel<S>, dim3((unsigned)cdiv(N, 256), B, splits), dim3(256), 0, st, (const S *)p1,
                     (const S *)p2, N, M, (S *)dist, idx, tps, pd, pi);
  KL_CHECK_LAUNCH();
  hipLaunchKernelGGL(sided_combine_kernel<S>, dim3((unsigned)cdiv(BN, 256)), dim3(256), 0, st, BN, splits,
                     (const S *)pd, (const int64_t *)pi, (S *)dist, idx);
  KL_CHECK_LAUNCH();
  KL_CHECK_HIP(hipFreeAsync(ws, st));
  return KL_OK;
}

// The double-sum form (f32 / f64): grad_p2's terms -- the same float products as sided_bwd_kernel's
// -- added per coordinate in double and rounded once (acc_finalize), so the result does not
// depend on the order of the atomics (exact whenever the terms' magnitudes span < ~2^29) and a
// points-sharded caller (kaolin.distributed.sharded_sided_distance) can all-reduce the sums and
// round once to get the unsharded gradient bit for bit.
template <typename S>
__global__ void __launch_bounds__(256) sided_bwd_sums_kernel(const S *__restrict__ grad, const S *__restrict__ p1,
                                                              const S *__restrict__ p2,
                                                              const int64_t *__restrict__ idx, int64_t N, int64_t M,
                                                              S *__restrict__ g1, double *__restrict__ sums) {
  const int b = blockIdx.y;
  const int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int64_t mi = (int64_t)b * N + n;
  const S x1 = p1[mi * 3], y1 = p1[mi * 3 + 1], z1 = p1[mi * 3 + 2];
  const int64_t j = (idx[mi] + (int64_t)b * M) * 3;
  const S x2 = p2[j], y2 = p2[j + 1], z2 = p2[j + 2];
  const S g = grad[mi];
  const S two = S(2);
  g1[mi * 3 + 0] = two * (x1 - x2) * g;
  g1[mi * 3 + 1] = two * (y1 - y2) * g;
  g1[mi * 3 + 2] = two * (z1 - z2) * g;
  atomicAdd(sums + j + 0, (double)(two * (x2 - x1) * g));
  atomicAdd(sums + j + 1, (double)(two * (y2 - y1) * g));
  atomicAdd(sums + j + 2, (double)(two * (z2 - z1) * g));
}

template <typename S>
static int sided_bwd_sums(int B, int64_t N, int64_t M, const void *grad, const void *p1, const void *p2,
                          const int64_t *idx, void *g1, double *sums, void *g2, hipStream_t st) {
  const size_t n2 = (size_t)B * M * 3;
  KL_REQUIRE(sums != nullptr || n2 == 0, "sided_distance_backward: the double sums buffer is missing");
  KL_CHECK_RC(fill_async(sums, 0, sizeof(double) * n2, st));
  if (B > 0 && N > 0) {
    hipLaunchKernelGGL(sided_bwd_sums_kernel<S>, dim3((unsigned)cdiv(N, 256), B), dim3(256), 0, st, (const S *)grad,
                       (const S *)p1, (const S *)p2, idx, N, M, (S *)g1, sums);
    KL_CHECK_LAUNCH();
  }
  return g2 ? acc_finalize<S>(sums, (S *)g2, n2, false, st) : KL_OK;
}

template <typename S>
static int sided_bwd(int B, int64_t N, int64_t M, const void *grad, const void *p1, const void *p2,
                     const int64_t *idx, void *g1, void *g2, hipStream_t st) {
  KL_CHECK_RC(fill_async(g2, 0, sizeof(S) * (size_t)B * M * 3, st));
  if (B == 0 || N == 0) return KL_OK;
  hipLaunchKernelGGL(sided_bwd_kernel<S>, dim3((unsigned)cdiv(N, 256), B), dim3(256), 0, st, (const S *)grad,
                     (const S *)p1, (const S *)p2, idx, N, M, (S *)g1, (S *)g2);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

#define KL_DISPATCH_NUM(dt, FN, ...)                                   \
  switch (dt) {                                                        \
    case KL_F32: return FN<float>(__VA_ARGS__);                        \
    case KL_F64: return FN<double>(__VA_ARGS__);                       \
    case KL_F16: return FN<__half>(__VA_ARGS__);                       \
    case KL_U8: return FN<uint8_t>(__VA_ARGS__);                       \
    case KL_I8: return FN<int8_t>(__VA_ARGS__);                        \
    case KL_I16: return FN<int16_t>(__VA_ARGS__);                      \
    case KL_I32: return FN<int32_t>(__VA_ARGS__);                      \
    case KL_I64: return FN<int64_t>(__VA_ARGS__);                      \
    default: break;                                                    \
  }

}  // namespace kl

using namespace kl;

extern "C" size_t kl_unbatched_triangle_distance_workspace_bytes(int64_t P, int64_t F) {
  return P2MWs(P > 0 ? P : 1, F > 0 ? F : 1, sizeof(double)).bytes;
}

extern "C" int kl_unbatched_triangle_distance_forward(kl_dtype dtype, int64_t P, int64_t F, const void *pts,
                                                      const void *fv, void *dist, int64_t *idx, int32_t *type,
                                                      void *ws, size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32) return p2m_fwd<float>(P, F, pts, fv, dist, idx, type, ws, ws_bytes, S(stream));
  if (dtype == KL_F64) return p2m_fwd<double>(P, F, pts, fv, dist, idx, type, ws, ws_bytes, S(stream));
  set_error("unbatched_triangle_distance_forward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" size_t kl_unbatched_triangle_distance_bwd_workspace_bytes(int64_t F) {
  return (size_t)(F > 0 ? F : 1) * 9 * sizeof(double);
}

extern "C" int kl_unbatched_triangle_distance_backward(kl_dtype dtype, int64_t P, int64_t F, const void *grad,
                                                       const void *pts, const void *fv, const int64_t *idx,
                                                       const int32_t *type, void *gp, void *gf, void *ws,
                                                       size_t ws_bytes, kl_stream stream) {
  if (dtype == KL_F32) return p2m_bwd<float>(P, F, grad, pts, fv, idx, type, gp, gf, ws, ws_bytes, S(stream));
  if (dtype == KL_F64) return p2m_bwd<double>(P, F, grad, pts, fv, idx, type, gp, gf, ws, ws_bytes, S(stream));
  set_error("unbatched_triangle_distance_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_unbatched_triangle_distance_backward_sums(kl_dtype dtype, int64_t P, int64_t F, const void *grad,
                                                            const void *pts, const void *fv, const int64_t *idx,
                                                            const int32_t *type, void *gp, double *gf_sums,
                                                            kl_stream stream) {
  if (dtype == KL_F32) return p2m_bwd_sums<float>(P, F, grad, pts, fv, idx, type, gp, gf_sums, S(stream));
  if (dtype == KL_F64) return p2m_bwd_sums<double>(P, F, grad, pts, fv, idx, type, gp, gf_sums, S(stream));
  set_error("unbatched_triangle_distance_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_sided_distance_forward(kl_dtype dtype, int batch, int64_t n, int64_t m, const void *p1,
                                         const void *p2, void *dist, int64_t *idx, kl_stream stream) {
  KL_DISPATCH_NUM(dtype, sided_fwd, batch, n, m, p1, p2, dist, idx, S(stream));
  set_error("sided_distance_forward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_sided_distance_backward(kl_dtype dtype, int batch, int64_t n, int64_t m, const void *grad,
                                          const void *p1, const void *p2, const int64_t *idx, void *g1, void *g2,
                                          kl_stream stream) {
  KL_DISPATCH_NUM(dtype, sided_bwd, batch, n, m, grad, p1, p2, idx, g1, g2, S(stream));
  set_error("sided_distance_backward_cuda not implemented for this dtype");
  return KL_E_INVALID;
}

extern "C" int kl_sided_distance_backward_sums(kl_dtype dtype, int batch, int64_t n, int64_t m, const void *grad,
                                               const void *p1, const void *p2, const int64_t *idx, void *g1,
                                               double *g2_sums, void *g2, kl_stream stream) {
  if (dtype == KL_F32) return sided_bwd_sums<float>(batch, n, m, grad, p1, p2, idx, g1, g2_sums, g2, S(stream));
  if (dtype == KL_F64) return sided_bwd_sums<double>(batch, n, m, grad, p1, p2, idx, g1, g2_sums, g2, S(stream));
  set_error("sided_distance_backward_cuda (double sums) not implemented for this dtype");
  return KL_E_INVALID;
}
