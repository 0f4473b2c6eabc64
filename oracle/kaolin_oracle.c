/* kaolin_oracle.c -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * This library is the parity checker for the HIP product path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.  It is plain C,
 * compiled with -O2 -ffp-contract=off (see oracle/Makefile).  Single-threaded except two
 * loops over independent items (p2m forward per point, mesh_to_spc barycentrics per leaf),
 * which are OpenMP-parallel so that full-size parity checks finish in seconds; each item
 * writes only its own outputs, so results do not depend on the thread count.  The DIB-R loops
 * run on or_set_threads() threads (1 unless bench.py's all-threads CPU leg sets more).
 *
 * Floating-point kernels (rasterize, soft mask, point->triangle distance, sided
 * distance) live in oracle_typed.inc, instantiated for float and double.  This
 * file adds the integer / SPC paths:
 *   mesh_to_spc        kaolin/csrc/ops/conversions/mesh_to_spc/mesh_to_spc_cuda.cu:59-463
 *   morton_to_octree   kaolin/csrc/ops/spc/spc_cuda.cu:45-163
 *   to_morton/to_point kaolin/csrc/spc_math.h:93-121
 *   scan_octrees       kaolin/csrc/ops/spc/scan_octrees.cu:43-114
 *   generate_points    kaolin/csrc/ops/spc/generate_points.cu:28-81, spc_utils.cuh:140-160
 *   raytrace           kaolin/csrc/render/spc/raytrace_cuda.cu:63-304,485-607,
 *                      spc_render_utils.cuh:21-143
 *   voxelgrid          kaolin/ops/conversions/trianglemesh.py:29-110,
 *                      kaolin/ops/mesh/trianglemesh.py:339-457,
 *                      kaolin/ops/conversions/pointcloud.py:22-75
 * Pinned by the fixtures in tests/golden (reference KATs and reference-oracle outputs).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Pixel-row sampling for bench.py's cpu_baseline leg: the DIB-R loops process only
 * rows j with j % g_row_step == 0 (default 1 = every row). */
static int g_row_step = 1;
void or_set_row_step(int s) { g_row_step = s > 0 ? s : 1; }
/* Threads of the DIB-R loops (bench.py's all-threads cpu_baseline leg; default 1, the checker).
 * The forward loops write only their own pixels; the backward's double accumulators are then
 * added with OpenMP atomics, so only the order of exact double sums changes. */
static int g_threads = 1;
void or_set_threads(int n) { g_threads = n > 0 ? n : 1; }

#define T float
#define SUF f32
#include "oracle_typed.inc"
#undef T
#undef SUF
#define T double
#define SUF f64
#include "oracle_typed.inc"
#undef T
#undef SUF

/* ------------------------------------------------------------------ morton */
uint64_t or_to_morton(int x, int y, int z)
{
  uint64_t m = 0;
  for (unsigned i = 0; i < 15; i++) {
    unsigned i2 = i + i;
    uint64_t X = (uint64_t)(uint16_t)x, Y = (uint64_t)(uint16_t)y, Z = (uint64_t)(uint16_t)z;
    m |= (Z & (1ull << i)) << i2;
    m |= (Y & (1ull << i)) << (i2 + 1);
    m |= (X & (1ull << i)) << (i2 + 2);
  }
  return m;
}

void or_to_point(uint64_t m, int16_t *p)
{
  uint16_t x = 0, y = 0, z = 0;
  for (int i = 0; i < 15; i++) {
    x |= (uint16_t)((m & (1ull << (3 * i + 2))) >> (2 * i + 2));
    y |= (uint16_t)((m & (1ull << (3 * i + 1))) >> (2 * i + 1));
    z |= (uint16_t)((m & (1ull << (3 * i + 0))) >> (2 * i + 0));
  }
  p[0] = (int16_t)x; p[1] = (int16_t)y; p[2] = (int16_t)z;
}

/* ------------------------------------------------------------ mesh_to_spc */
typedef struct { double x, y, z; } d3;
static inline d3 d3mk(double x, double y, double z) { d3 r = {x, y, z}; return r; }
static inline d3 d3sub(d3 a, d3 b) { return d3mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline double d3dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline d3 d3cross(d3 a, d3 b) { return d3mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline d3 d3norm(d3 v) { double inv = 1.0 / sqrt(d3dot(v, v)); return d3mk(inv * v.x, inv * v.y, inv * v.z); }

static int sat_axis(d3 v0, d3 v1, d3 v2, float h, d3 axis)
{
  double d0 = d3dot(v0, axis), d1 = d3dot(v1, axis), d2 = d3dot(v2, axis);
  double maxd = fmax(d0, fmax(d1, d2));
  double mind = fmin(d0, fmin(d1, d2));
  double r = (double)h * (fabs(axis.x) + fabs(axis.y) + fabs(axis.z));
  float fd = (float)fmax(-maxd, mind);
  float fr = (float)r;
  return fd <= fr;
}

int or_tri_voxel_test(const float *fa, const float *fb, const float *fc, const float *c, float h)
{
  d3 va = d3mk((double)(fa[0] - c[0]), (double)(fa[1] - c[1]), (double)(fa[2] - c[2]));
  d3 vb = d3mk((double)(fb[0] - c[0]), (double)(fb[1] - c[1]), (double)(fb[2] - c[2]));
  d3 vc = d3mk((double)(fc[0] - c[0]), (double)(fc[1] - c[1]), (double)(fc[2] - c[2]));
  d3 ab = d3norm(d3sub(vb, va)), bc = d3norm(d3sub(vc, vb)), ca = d3norm(d3sub(va, vc));
  d3 axes[13] = {
    d3mk(0.0, -ab.z, ab.y), d3mk(0.0, -bc.z, bc.y), d3mk(0.0, -ca.z, ca.y),
    d3mk(ab.z, 0.0, -ab.x), d3mk(bc.z, 0.0, -bc.x), d3mk(ca.z, 0.0, -ca.x),
    d3mk(-ab.y, ab.x, 0.0), d3mk(-bc.y, bc.x, 0.0), d3mk(-ca.y, ca.x, 0.0),
    d3mk(1, 0, 0), d3mk(0, 1, 0), d3mk(0, 0, 1), d3cross(ab, bc)};
  for (int a = 0; a < 13; a++)
    if (!sat_axis(va, vb, vc, h, axes[a])) return 0;
  return 1;
}

static void voxel_center(uint64_t m, unsigned level, float *c, float *half)
{
  float two_level = (float)(1u << level);
  float vs = 2.0f / two_level;
  float h = (float)(0.5 * vs);
  int16_t p[3];
  or_to_point(m, p);
  c[0] = fmaf((float)p[0], vs, h - 1.0f);
  c[1] = fmaf((float)p[1], vs, h - 1.0f);
  c[2] = fmaf((float)p[2], vs, h - 1.0f);
  *half = h;
}

/* spc_math.h:229-258 (float closest point, used for barycentrics) */
typedef struct { float x, y, z; } f3;
static inline f3 f3mk(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 f3sub(f3 a, f3 b) { return f3mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 f3add(f3 a, f3 b) { return f3mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 f3mul(f3 a, float s) { return f3mk(a.x * s, a.y * s, a.z * s); }
static inline float f3dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline f3 f3cross(f3 a, f3 b) { return f3mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline float f3pe(f3 v, f3 e, f3 p) { f3 pv = f3sub(p, v); float len = f3dot(e, e); return f3dot(pv, e) / len; }
static inline int f3na(f3 v, f3 e, f3 n, f3 p) { return f3dot(f3cross(n, e), f3sub(p, v)) <= 0; }

static f3 tri_closest(f3 v1, f3 v2, f3 v3, f3 p)
{
  f3 e12 = f3sub(v2, v1), e23 = f3sub(v3, v2), e31 = f3sub(v1, v3);
  f3 n = f3cross(f3sub(v1, v2), e31);
  float uab = f3pe(v1, e12, p), uca = f3pe(v3, e31, p);
  if (uca > 1 && uab < 0) return v1;
  float ubc = f3pe(v2, e23, p);
  if (uab > 1 && ubc < 0) return v2;
  if (ubc > 1 && uca < 0) return v3;
  if (uab <= 1. && uab >= 0. && f3na(v1, e12, n, p)) return f3add(v1, f3mul(e12, uab));
  if (ubc <= 1. && ubc >= 0. && f3na(v2, e23, n, p)) return f3add(v2, f3mul(e23, ubc));
  if (uca <= 1. && uca >= 0. && f3na(v3, e31, n, p)) return f3add(v3, f3mul(e31, uca));
  float inv = 1.0f / sqrtf(f3dot(n, n));
  f3 un = f3mul(n, inv);
  float dist = (p.x - v1.x) * un.x + (p.y - v1.y) * un.y + (p.z - v1.z) * un.z;
  return f3sub(p, f3mul(un, dist));
}

void or_bary(const float *fv, uint64_t m, unsigned level, float *out2)
{
  float c[3], h;
  voxel_center(m, level, c, &h);
  f3 v1 = f3mk(fv[0], fv[1], fv[2]), v2 = f3mk(fv[3], fv[4], fv[5]), v3 = f3mk(fv[6], fv[7], fv[8]);
  f3 p = f3mk(c[0], c[1], c[2]);
  f3 cp = tri_closest(v1, v2, v3, p);
  f3 cr = f3cross(f3sub(v1, v2), f3sub(v1, v3));
  float delta = f3dot(cr, cr);
  f3 d1 = f3sub(cp, v1), d2 = f3sub(cp, v2), d3v = f3sub(cp, v3);
  f3 t;
  t = f3cross(d2, d3v); float da = sqrtf(f3dot(t, t));
  t = f3cross(d1, d3v); float db = sqrtf(f3dot(t, t));
  t = f3cross(d1, d2);  float dc = sqrtf(f3dot(t, t));
  float rs = 1.0f / sqrtf(delta);
  float bx = da * rs, by = db * rs, bz = dc * rs;
  if (bx < 0.0f) bx = 0.f;
  if (by < 0.0f) by = 0.f;
  if (bz < 0.0f) bz = 0.f;
  float s = (float)(1. / (double)(bx + by + bz));
  bx *= s; by *= s;
  out2[0] = bx; out2[1] = by;
}

/* or_bary over n leaves (face index per leaf into fv (F,3,3)); independent per leaf */
void or_bary_batch(const float *fv, const uint64_t *m, const int64_t *face, int64_t n, unsigned level, float *out)
{
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) or_bary(fv + face[i] * 9, m[i], level, out + 2 * i);
}

typedef struct { uint64_t m; int64_t t; } mt_pair;

static void stable_sort_pairs(mt_pair *a, size_t n)
{
  if (n < 2) return;
  mt_pair *tmp = (mt_pair *)malloc(n * sizeof(mt_pair));
  for (size_t w = 1; w < n; w *= 2) {
    for (size_t lo = 0; lo < n; lo += 2 * w) {
      size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      size_t i = lo, j = mid, k = lo;
      while (i < mid && j < hi) tmp[k++] = (a[j].m < a[i].m) ? a[j++] : a[i++];
      while (i < mid) tmp[k++] = a[i++];
      while (j < hi) tmp[k++] = a[j++];
    }
    memcpy(a, tmp, n * sizeof(mt_pair));
  }
  free(tmp);
}

/* Returns the number of unique leaves; fills *out_morton, *out_face (malloc'd,
 * caller frees with or_free).  Returns 0 for an empty result. */
int64_t or_mesh_to_spc_leaves(const float *fv, int64_t F, unsigned L,
                              uint64_t **out_morton, int64_t **out_face)
{
  size_t cnt = (size_t)F;
  mt_pair *cur = (mt_pair *)malloc((cnt ? cnt : 1) * sizeof(mt_pair));
  for (size_t i = 0; i < cnt; i++) { cur[i].m = 0; cur[i].t = (int64_t)i; }
  for (unsigned l = 0; l <= L; l++) {
    size_t nxt = 0;
    unsigned char *hit = (unsigned char *)malloc(cnt ? cnt : 1);
    for (size_t i = 0; i < cnt; i++) {
      float c[3], h;
      voxel_center(cur[i].m, l, c, &h);
      const float *v = fv + cur[i].t * 9;
      hit[i] = (unsigned char)or_tri_voxel_test(v, v + 3, v + 6, c, h);
      nxt += hit[i] ? (l < L ? 8 : 1) : 0;
    }
    if (nxt == 0) { free(hit); free(cur); *out_morton = NULL; *out_face = NULL; return 0; }
    mt_pair *n2 = (mt_pair *)malloc(nxt * sizeof(mt_pair));
    size_t o = 0;
    for (size_t i = 0; i < cnt; i++) {
      if (!hit[i]) continue;
      if (l < L) {
        int16_t p[3];
        or_to_point(cur[i].m, p);
        for (unsigned c = 0; c < 8; c++) {
          n2[o].m = or_to_morton(2 * p[0] + (c >> 2), 2 * p[1] + ((c >> 1) & 1), 2 * p[2] + (c & 1));
          n2[o].t = cur[i].t;
          o++;
        }
      } else {
        n2[o++] = cur[i];
      }
    }
    free(hit); free(cur);
    cur = n2; cnt = nxt;
  }
  stable_sort_pairs(cur, cnt);
  size_t u = 0;
  for (size_t i = 0; i < cnt; i++)
    if (i == 0 || cur[i].m != cur[i - 1].m) cur[u++] = cur[i];
  *out_morton = (uint64_t *)malloc(u * sizeof(uint64_t));
  *out_face = (int64_t *)malloc(u * sizeof(int64_t));
  for (size_t i = 0; i < u; i++) { (*out_morton)[i] = cur[i].m; (*out_face)[i] = cur[i].t; }
  free(cur);
  return (int64_t)u;
}

/* Sensitivity of mesh_to_spc's separating-axis decisions to the normalisation's rounding
 * (measurement, not a restatement).  The reference normalises the edges with CUDA's double
 * rsqrt (mesh_to_spc_cuda.cu:123-125 -> spc_math.h:240-243), which is not correctly rounded
 * (1 ulp); this restatement and the HIP kernel use 1.0 / sqrt.  For every proposal of the
 * level recursion (following the 1/sqrt decisions) this counts:
 *   counts[0] proposals tested, counts[1] proposals with some axis whose float-rounded
 *   |fd - fr| is at most one float ulp of fr (near the threshold), counts[2] proposals whose
 *   decision changes when every 1/sqrt is moved 1 ulp up, counts[3] ... 1 ulp down,
 *   counts[4] of those flips at the leaf level L. */
static d3 d3norm_ulp(d3 v, int dir)
{
  double inv = 1.0 / sqrt(d3dot(v, v));
  if (dir) inv = nextafter(inv, dir > 0 ? INFINITY : 0.0);
  return d3mk(inv * v.x, inv * v.y, inv * v.z);
}

static int tri_voxel_test_ulp(const float *fa, const float *fb, const float *fc, const float *c, float h, int dir,
                              int *near)
{
  d3 va = d3mk((double)(fa[0] - c[0]), (double)(fa[1] - c[1]), (double)(fa[2] - c[2]));
  d3 vb = d3mk((double)(fb[0] - c[0]), (double)(fb[1] - c[1]), (double)(fb[2] - c[2]));
  d3 vc = d3mk((double)(fc[0] - c[0]), (double)(fc[1] - c[1]), (double)(fc[2] - c[2]));
  d3 ab = d3norm_ulp(d3sub(vb, va), dir), bc = d3norm_ulp(d3sub(vc, vb), dir), ca = d3norm_ulp(d3sub(va, vc), dir);
  d3 axes[13] = {
    d3mk(0.0, -ab.z, ab.y), d3mk(0.0, -bc.z, bc.y), d3mk(0.0, -ca.z, ca.y),
    d3mk(ab.z, 0.0, -ab.x), d3mk(bc.z, 0.0, -bc.x), d3mk(ca.z, 0.0, -ca.x),
    d3mk(-ab.y, ab.x, 0.0), d3mk(-bc.y, bc.x, 0.0), d3mk(-ca.y, ca.x, 0.0),
    d3mk(1, 0, 0), d3mk(0, 1, 0), d3mk(0, 0, 1), d3cross(ab, bc)};
  int ok = 1;
  for (int a = 0; a < 13 && (ok || near); a++) {
    const d3 axis = axes[a];
    double d0 = d3dot(va, axis), d1 = d3dot(vb, axis), d2 = d3dot(vc, axis);
    double maxd = fmax(d0, fmax(d1, d2)), mind = fmin(d0, fmin(d1, d2));
    double r = (double)h * (fabs(axis.x) + fabs(axis.y) + fabs(axis.z));
    float fd = (float)fmax(-maxd, mind), fr = (float)r;
    if (near && fabsf(fd - fr) <= nextafterf(fabsf(fr), INFINITY) - fabsf(fr)) *near = 1;
    if (!(fd <= fr)) ok = 0;
    if (!ok && !near) break;
  }
  return ok;
}

void or_m2s_rsqrt_sensitivity(const float *fv, int64_t F, unsigned L, int64_t *counts)
{
  size_t cnt = (size_t)F;
  mt_pair *cur = (mt_pair *)malloc((cnt ? cnt : 1) * sizeof(mt_pair));
  for (size_t i = 0; i < cnt; i++) { cur[i].m = 0; cur[i].t = (int64_t)i; }
  for (int k = 0; k < 5; k++) counts[k] = 0;
  for (unsigned l = 0; l <= L && cnt; l++) {
    unsigned char *hit = (unsigned char *)malloc(cnt);
    int64_t c1 = 0, c2 = 0, c3 = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : c1, c2, c3)
    for (size_t i = 0; i < cnt; i++) {
      float c[3], h;
      voxel_center(cur[i].m, l, c, &h);
      const float *v = fv + cur[i].t * 9;
      int near = 0;
      const int base = tri_voxel_test_ulp(v, v + 3, v + 6, c, h, 0, &near);
      hit[i] = (unsigned char)base;
      c1 += near;
      if (near) {
        c2 += tri_voxel_test_ulp(v, v + 3, v + 6, c, h, 1, NULL) != base;
        c3 += tri_voxel_test_ulp(v, v + 3, v + 6, c, h, -1, NULL) != base;
      }
    }
    counts[0] += (int64_t)cnt; counts[1] += c1; counts[2] += c2; counts[3] += c3;
    if (l == L) counts[4] += c2 + c3;
    size_t nxt = 0;
    for (size_t i = 0; i < cnt; i++) nxt += hit[i] ? (l < L ? 8 : 0) : 0;
    mt_pair *n2 = (mt_pair *)malloc((nxt ? nxt : 1) * sizeof(mt_pair));
    size_t o = 0;
    for (size_t i = 0; i < cnt && l < L; i++) {
      if (!hit[i]) continue;
      int16_t p[3];
      or_to_point(cur[i].m, p);
      for (unsigned cc = 0; cc < 8; cc++) {
        n2[o].m = or_to_morton(2 * p[0] + (cc >> 2), 2 * p[1] + ((cc >> 1) & 1), 2 * p[2] + (cc & 1));
        n2[o].t = cur[i].t;
        o++;
      }
    }
    free(hit); free(cur);
    cur = n2; cnt = nxt;
  }
  free(cur);
}

/* morton_to_octree: level-major bytes, top-down.  Returns octree size; *out malloc'd. */
int64_t or_morton_to_octree(const uint64_t *mortons, int64_t n, unsigned L, uint8_t **out)
{
  uint64_t *cur = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
  memcpy(cur, mortons, n * sizeof(uint64_t));
  uint8_t **lv = (uint8_t **)calloc(L ? L : 1, sizeof(uint8_t *));
  int64_t *ln = (int64_t *)calloc(L ? L : 1, sizeof(int64_t));
  int64_t prev = n;
  for (unsigned i = L; i > 0; i--) {
    uint64_t *par = (uint64_t *)malloc((prev ? prev : 1) * sizeof(uint64_t));
    uint8_t *bytes = (uint8_t *)malloc(prev ? prev : 1);
    int64_t np = 0;
    for (int64_t t = 0; t < prev; t++) {
      if (t == 0 || (cur[t - 1] >> 3) != (cur[t] >> 3)) { par[np] = cur[t] >> 3; bytes[np] = 0; np++; }
      bytes[np - 1] |= (uint8_t)(1u << (cur[t] & 7));
    }
    lv[i - 1] = bytes; ln[i - 1] = np;
    free(cur); cur = par; prev = np;
  }
  free(cur);
  int64_t total = 0;
  for (unsigned l = 0; l < L; l++) total += ln[l];
  *out = (uint8_t *)malloc(total ? total : 1);
  int64_t o = 0;
  for (unsigned l = 0; l < L; l++) { memcpy(*out + o, lv[l], ln[l]); o += ln[l]; free(lv[l]); }
  free(lv); free(ln);
  return total;
}

/* -------------------------------------------------------- scan / generate */
/* pyramid_full: (B, 2, 17) zero-initialised by the caller (KAOLIN_SPC_MAX_LEVELS+2);
 * exsum: (sum(lengths) + B).  Returns level as scan_octrees.cu:43-114 does. */
int or_scan_octrees(const uint8_t *octrees, const int32_t *lengths, int B, int32_t *pyramid_full, int32_t *exsum)
{
  const int STR = 17;
  const uint8_t *O0 = octrees;
  int32_t *EX0 = exsum;
  int32_t *h0 = pyramid_full;
  int level = 0;
  for (int b = 0; b < B; b++) {
    uint32_t osize = (uint32_t)lengths[b];
    EX0[0] = 0;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < osize; i++) { acc += (uint32_t)__builtin_popcount(O0[i]); EX0[i + 1] = (int32_t)acc; }
    int32_t *Pmid = h0, *PmidSum = h0 + STR;
    uint32_t Lsize = 1, prevSum = 0, sum = 1;
    Pmid[0] = 1; PmidSum[0] = 0; PmidSum[1] = 1;
    level = 0;
    while (sum <= osize) {
      uint32_t currSum = (uint32_t)EX0[prevSum + 1];
      Lsize = currSum - prevSum;
      prevSum = currSum;
      Pmid[++level] = (int32_t)Lsize;
      sum += Lsize;
      PmidSum[level + 1] = (int32_t)sum;
    }
    O0 += osize; EX0 += osize + 1; h0 += 2 * STR;
  }
  return level;
}

/* pyramids: (B, 2, L+2) as returned by scan_octrees; points: (total, 3) int16. */
void or_generate_points(const uint8_t *octrees, const int32_t *pyramids, int B, int L,
                        const int32_t *exsum, int16_t *points)
{
  const uint8_t *oct = octrees;
  const int32_t *ex = exsum;
  int16_t *pts = points;
  for (int b = 0; b < B; b++) {
    const int32_t *pyr = pyramids + (size_t)b * 2 * (L + 2);
    const int32_t *pyrsum = pyr + L + 2;
    int32_t osize = pyrsum[L];
    int32_t total = pyrsum[L + 1];
    uint64_t *mort = (uint64_t *)calloc(total > 0 ? total : 1, sizeof(uint64_t));
    mort[0] = 0;
    const uint8_t *co = oct;
    const int32_t *cs = ex + 1;
    uint64_t *cm = mort;
    for (int l = 0; l < L; l++) {
      int n = pyr[l];
      for (int t = 0; t < n; t++) {
        uint8_t bits = co[t];
        uint64_t code = cm[t];
        int addr = cs[t];
        for (int i = 7; i >= 0; i--)
          if (bits & (1u << i)) mort[addr--] = 8 * code + (uint64_t)i;
      }
      co += n; cs += n; cm += n;
    }
    for (int32_t i = 0; i < total; i++) or_to_point(mort[i], pts + (size_t)i * 3);
    free(mort);
    pts += (size_t)total * 3;
    oct += osize;
    ex += osize + 1;
  }
}

/* -------------------------------------------------------------- raytrace */
static float ray_aabb(const float *q, const float *d, const float *inv, const float *sgn, const float *org, float r)
{
  float o[3] = {q[0] - org[0], q[1] - org[1], q[2] - org[2]};
  float cmax = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fabsf(o[2]));
  float winding = cmax < r ? -1.0f : 1.0f;
  winding *= r;
  if (winding < 0) return winding;
  float d0 = fmaf(winding, sgn[0], -o[0]) * inv[0];
  float d1 = fmaf(winding, sgn[1], -o[1]) * inv[1];
  float d2 = fmaf(winding, sgn[2], -o[2]) * inv[2];
  float ltxy = fmaf(d[1], d0, o[1]), ltxz = fmaf(d[2], d0, o[2]);
  float ltyx = fmaf(d[0], d1, o[0]), ltyz = fmaf(d[2], d1, o[2]);
  float ltzx = fmaf(d[0], d2, o[0]), ltzy = fmaf(d[1], d2, o[1]);
  int t0 = (d0 >= 0.0f) && (fabsf(ltxy) <= r) && (fabsf(ltxz) <= r);
  int t1 = (d1 >= 0.0f) && (fabsf(ltyx) <= r) && (fabsf(ltyz) <= r);
  int t2 = (d2 >= 0.0f) && (fabsf(ltzx) <= r) && (fabsf(ltzy) <= r);
  float s[3] = {0.0f, 0.0f, 0.0f};
  if (t0) s[0] = sgn[0]; else if (t1) s[1] = sgn[1]; else if (t2) s[2] = sgn[2];
  float dd = 0.0f;
  if (s[0] != 0.0f) dd = d0; else if (s[1] != 0.0f) dd = d1; else if (s[2] != 0.0f) dd = d2;
  if (dd != 0.0f) return dd;
  return 0.0f;
}

/* front-to-back child order: children sorted by (popcount(code ^ j), j);
 * equals VOXEL_ORDER of raytrace_cuda.cu:48-57. */
void or_voxel_order(uint8_t order[8][8])
{
  for (int c = 0; c < 8; c++) {
    int k = 0;
    for (int h = 0; h <= 3; h++)
      for (int j = 0; j < 8; j++)
        if (__builtin_popcount(c ^ j) == h) order[c][k++] = (uint8_t)j;
  }
}

/* Returns number of hits; *nuggets (N,2) int32 and *depth (N, 1|2) malloc'd. */
int64_t or_raytrace(const uint8_t *octree, const int16_t *points, const int32_t *exsum,
                    const float *ray_o, const float *ray_d, int64_t nrays, unsigned target_level,
                    int return_depth, int with_exit, int32_t **out_nug, float **out_depth)
{
  uint8_t order[8][8];
  or_voxel_order(order);
  int64_t num = nrays;
  int32_t *nug = (int32_t *)malloc((num ? num : 1) * 2 * sizeof(int32_t));
  for (int64_t i = 0; i < num; i++) { nug[2 * i] = (int32_t)i; nug[2 * i + 1] = 0; }
  int dd = with_exit ? 2 : 1;
  float *dep = NULL;
  *out_depth = NULL;
  for (unsigned l = 0; l <= target_level; l++) {
    uint32_t *info = (uint32_t *)calloc(num ? num : 1, sizeof(uint32_t));
    float *dl = NULL;
    const int last = (l == target_level);
    if (last && return_depth) dl = (float *)malloc((num ? num : 1) * dd * sizeof(float));
    float r = (float)(1.0 / (double)(float)(1u << l));
    int64_t total = 0;
    for (int64_t t = 0; t < num; t++) {
      int32_t ridx = nug[2 * t], pidx = nug[2 * t + 1];
      const int16_t *p = points + (size_t)pidx * 3;
      const float *o = ray_o + (size_t)ridx * 3, *d = ray_d + (size_t)ridx * 3;
      float vc[3] = {fmaf(r, fmaf(2.0f, (float)p[0], 1.0f), -1.0f),
                     fmaf(r, fmaf(2.0f, (float)p[1], 1.0f), -1.0f),
                     fmaf(r, fmaf(2.0f, (float)p[2], 1.0f), -1.0f)};
      float sgn[3] = {signbit(d[0]) ? 1.0f : -1.0f, signbit(d[1]) ? 1.0f : -1.0f, signbit(d[2]) ? 1.0f : -1.0f};
      float inv[3] = {(float)(1.0 / (double)d[0]), (float)(1.0 / (double)d[1]), (float)(1.0 / (double)d[2])};
      if (last && return_depth) {
        if (with_exit) {
          float nd[3] = {-d[0], -d[1], -d[2]};
          float xs[3] = {signbit(nd[0]) ? 1.0f : -1.0f, signbit(nd[1]) ? 1.0f : -1.0f, signbit(nd[2]) ? 1.0f : -1.0f};
          float en = ray_aabb(o, d, inv, sgn, vc, r);
          float ex = ray_aabb(o, d, inv, xs, vc, r);
          dl[2 * t] = en; dl[2 * t + 1] = ex;
          info[t] = (en > 0.0 && ex > 0.0) ? 1 : 0;
        } else {
          float dv = ray_aabb(o, d, inv, sgn, vc, r);
          dl[t] = dv;
          info[t] = dv > 0.0 ? 1 : 0;
        }
      } else {
        float dv = ray_aabb(o, d, inv, sgn, vc, r);
        if (!last) info[t] = dv != 0.0 ? (uint32_t)__builtin_popcount(octree[pidx]) : 0;
        else info[t] = dv > 0.0 ? 1 : 0;
      }
      total += info[t];
    }
    if (total == 0) {
      free(info); free(dl); free(nug);
      *out_nug = (int32_t *)malloc(2 * sizeof(int32_t));
      if (return_depth) *out_depth = (float *)malloc(dd * sizeof(float));
      return 0;
    }
    int32_t *n2 = (int32_t *)malloc(total * 2 * sizeof(int32_t));
    int64_t w = 0;
    if (!last) {
      for (int64_t t = 0; t < num; t++) {
        if (!info[t]) continue;
        int32_t ridx = nug[2 * t], pidx = nug[2 * t + 1];
        const int16_t *p = points + (size_t)pidx * 3;
        uint8_t ob = octree[pidx];
        uint32_t s = (uint32_t)exsum[pidx];
        float scale = (float)(1.0 / (double)(float)(1u << l));
        const float *org = ray_o + (size_t)ridx * 3;
        float x = (float)((double)(0.5f * org[0] + 0.5f) - (double)scale * ((double)(float)p[0] + 0.5));
        float y = (float)((double)(0.5f * org[1] + 0.5f) - (double)scale * ((double)(float)p[1] + 0.5));
        float z = (float)((double)(0.5f * org[2] + 0.5f) - (double)scale * ((double)(float)p[2] + 0.5));
        unsigned code = 0;
        if (x > 0) code = 4;
        if (y > 0) code += 2;
        if (z > 0) code += 1;
        for (int i = 0; i < 8; i++) {
          unsigned j = order[code][i];
          if (ob & (1u << j)) {
            unsigned c = (unsigned)__builtin_popcount(ob & ((2u << j) - 1));
            n2[2 * w] = ridx; n2[2 * w + 1] = (int32_t)(s + c); w++;
          }
        }
      }
    } else {
      if (return_depth) dep = (float *)malloc(total * dd * sizeof(float));
      for (int64_t t = 0; t < num; t++) {
        if (!info[t]) continue;
        n2[2 * w] = nug[2 * t]; n2[2 * w + 1] = nug[2 * t + 1];
        if (return_depth) for (int k = 0; k < dd; k++) dep[w * dd + k] = dl[t * dd + k];
        w++;
      }
    }
    free(info); free(dl); free(nug);
    nug = n2; num = total;
  }
  *out_nug = nug;
  *out_depth = dep;
  return num;
}

/* ------------------------------------------------------------- voxelgrid */
typedef struct { float a[3], b[3], c[3]; } tri_f;

static float edge2(const float *p, const float *q)
{
  float dx = p[0] - q[0], dy = p[1] - q[1], dz = p[2] - q[2];
  return dx * dx + dy * dy + dz * dz;
}

static void mark(const float *p, int R, uint8_t *grid)
{
  float mult = (float)(R - 1);
  float fx = nearbyintf(p[0] * mult), fy = nearbyintf(p[1] * mult), fz = nearbyintf(p[2] * mult);
  if (!(fx >= 0.f && fy >= 0.f && fz >= 0.f && fx <= (float)(R - 1) && fy <= (float)(R - 1) && fz <= (float)(R - 1))) return;
  int64_t x = (int64_t)fx, y = (int64_t)fy, z = (int64_t)fz;
  grid[(x * R + y) * R + z] = 1;
}

static void subdivide(tri_f t, float thr, int R, uint8_t *grid, int depth)
{
  float e1 = edge2(t.a, t.b), e2 = edge2(t.b, t.c), e3 = edge2(t.c, t.a);
  float mx = e1;
  if (e2 > mx) mx = e2;
  if (e3 > mx) mx = e3;
  if (!(mx > thr) || depth > 40) return;
  float v4[3], v5[3], v6[3];
  for (int k = 0; k < 3; k++) {
    v4[k] = (t.a[k] + t.c[k]) / 2; v5[k] = (t.a[k] + t.b[k]) / 2; v6[k] = (t.b[k] + t.c[k]) / 2;
  }
  mark(v4, R, grid); mark(v5, R, grid); mark(v6, R, grid);
  tri_f ch;
  memcpy(ch.a, t.a, 12); memcpy(ch.b, v4, 12); memcpy(ch.c, v5, 12); subdivide(ch, thr, R, grid, depth + 1);
  memcpy(ch.a, t.b, 12); memcpy(ch.b, v5, 12); memcpy(ch.c, v6, 12); subdivide(ch, thr, R, grid, depth + 1);
  memcpy(ch.a, v4, 12);  memcpy(ch.b, v5, 12); memcpy(ch.c, v6, 12); subdivide(ch, thr, R, grid, depth + 1);
  memcpy(ch.a, t.c, 12); memcpy(ch.b, v4, 12); memcpy(ch.c, v6, 12); subdivide(ch, thr, R, grid, depth + 1);
}

/* float32 path.  vertices (B,V,3); faces (F,3); origin (B,3) / scale (B) may be NULL
 * (then min / max-extent defaults).  grid: (B,R,R,R) uint8 zeroed by the caller. */
void or_voxelgrid_f32(const float *vertices, int B, int V, const int64_t *faces, int F, int R,
                      const float *origin, const float *scale, uint8_t *grid)
{
  double thr_d = ((double)(R - 1) / ((double)R * (double)R));
  float thr = (float)(thr_d * thr_d);
  float *pts = (float *)malloc((size_t)(V ? V : 1) * 3 * sizeof(float));
  for (int b = 0; b < B; b++) {
    const float *v = vertices + (size_t)b * V * 3;
    float o[3], s;
    if (origin) { o[0] = origin[b * 3]; o[1] = origin[b * 3 + 1]; o[2] = origin[b * 3 + 2]; }
    else {
      for (int k = 0; k < 3; k++) { o[k] = v[k]; for (int i = 1; i < V; i++) if (v[i * 3 + k] < o[k]) o[k] = v[i * 3 + k]; }
    }
    if (scale) s = scale[b];
    else {
      float mx[3];
      for (int k = 0; k < 3; k++) { mx[k] = v[k]; for (int i = 1; i < V; i++) if (v[i * 3 + k] > mx[k]) mx[k] = v[i * 3 + k]; }
      s = mx[0] - o[0];
      if (mx[1] - o[1] > s) s = mx[1] - o[1];
      if (mx[2] - o[2] > s) s = mx[2] - o[2];
    }
    for (int i = 0; i < V; i++)
      for (int k = 0; k < 3; k++) pts[i * 3 + k] = (v[i * 3 + k] - o[k]) / s;
    uint8_t *g = grid + (size_t)b * R * R * R;
    for (int i = 0; i < V; i++) mark(pts + i * 3, R, g);
    for (int f = 0; f < F; f++) {
      tri_f t;
      memcpy(t.a, pts + faces[f * 3] * 3, 12);
      memcpy(t.b, pts + faces[f * 3 + 1] * 3, 12);
      memcpy(t.c, pts + faces[f * 3 + 2] * 3, 12);
      subdivide(t, thr, R, g, 0);
    }
  }
  free(pts);
}

void or_free(void *p) { free(p); }
