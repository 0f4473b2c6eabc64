// prepare.hip -- DIB-R input preparation, fused.
//
// Reference (kaolin/render/mesh/utils.py:128-175 prepare_vertices):
//   vertices_camera = (vertices - trans.view(-1,1,3)) @ rot^T      (camera/legacy.py:22-37)
//                     or pad(vertices, 1) @ camera_transform        (utils.py:163-167)
//   vertices_image  = (vc * proj)[:, :, :2] / (vc * proj)[:, :, 2:3] (camera/legacy.py:120-139)
//   face_vertices_camera / _image = index_vertices_by_faces(...)    (ops/mesh/mesh.py:25-46)
//   face_normals = cross(c1 - c0, c2 - c0) / (norm + 1e-10)         (ops/mesh/trianglemesh.py:313-336)
// i.e. ~12 ATen launches (sub, bmm, mul, slice, div, two gathers, two subs, cross, norm, add,
// div) and their backward chain.  Here the forward is ONE launch, one thread per (view, face):
// the face's three corners are transformed and projected in registers and the three outputs
// written in the reference layouts.
//
// Backward (one fill + three launches):
//   1. per (view, face): the normal's backward (division, norm and cross, as autograd forms
//      them), added to the incoming grad of face_vertices_camera; the per-corner terms are
//      summed per vertex in double (global atomics, index_vertices_by_faces' scatter-add),
//      the face_vertices_image grads likewise;
//   2. per (view, vertex): the sums rounded once; the perspective backward; the transform's
//      backward gives grad_vertices; the camera terms (rot, trans, proj / transform) reduced
//      per view in double (workgroup sums, one atomic per workgroup);
//   3. the camera grads rounded once (summed over views broadcast to one camera).
// Broadcasting as in the reference: vertices, the camera and proj may each have batch 1
// or B (matmul / elementwise broadcasting); their grads are summed over the broadcast views.
// A face index outside [0, V) reads nothing and yields NaN outputs (torch's gather would
// raise a device assert).
#include "common.h"

namespace kl {

struct PrepSrc {
  int B, Bv, Bc, Bp;     // views; batch of vertices, camera (rot/trans or transform), proj (1 or B)
  int64_t V, F;
  int mode;              // 0: rot + trans, 1: transform (4,3)
};

template <typename T>
struct Cam {
  T m[12];  // mode 0: rot (3x3) row-major then trans (3); mode 1: transform (4x3) row-major
  T p[3];
};

template <typename T>
__device__ __forceinline__ void load_cam(const PrepSrc &s, int b, const T *rot, const T *trans, const T *xf,
                                         const T *proj, Cam<T> &c) {
  const int bc = s.Bc == 1 ? 0 : b;
  if (s.mode == 0) {
#pragma unroll
    for (int k = 0; k < 9; k++) c.m[k] = rot[bc * 9 + k];
#pragma unroll
    for (int k = 0; k < 3; k++) c.m[9 + k] = trans[bc * 3 + k];
  } else {
#pragma unroll
    for (int k = 0; k < 12; k++) c.m[k] = xf[bc * 12 + k];
  }
  const int bp = s.Bp == 1 ? 0 : b;
#pragma unroll
  for (int k = 0; k < 3; k++) c.p[k] = proj[bp * 3 + k];
}

// camera coordinates of one vertex (legacy.py:35-36 / utils.py:163-167)
template <typename T>
__device__ __forceinline__ void to_camera(int mode, const Cam<T> &c, const T *v, T *out, T *tr) {
  if (mode == 0) {
    tr[0] = v[0] - c.m[9];
    tr[1] = v[1] - c.m[10];
    tr[2] = v[2] - c.m[11];
#pragma unroll
    for (int i = 0; i < 3; i++) out[i] = tr[0] * c.m[i * 3 + 0] + tr[1] * c.m[i * 3 + 1] + tr[2] * c.m[i * 3 + 2];
  } else {
    tr[0] = v[0];
    tr[1] = v[1];
    tr[2] = v[2];
#pragma unroll
    for (int i = 0; i < 3; i++) out[i] = v[0] * c.m[0 * 3 + i] + v[1] * c.m[1 * 3 + i] + v[2] * c.m[2 * 3 + i] + c.m[9 + i];
  }
}

template <typename T>
__device__ __forceinline__ bool face_corners(const PrepSrc &s, const int64_t *faces, int64_t f, int64_t *vi) {
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    vi[c] = faces[f * 3 + c];
    ok = ok && vi[c] >= 0 && vi[c] < s.V;
  }
  return ok;
}

template <typename T>
__global__ void prep_fwd_kernel(PrepSrc s, const T *__restrict__ verts, const int64_t *__restrict__ faces,
                                const T *__restrict__ rot, const T *__restrict__ trans, const T *__restrict__ xf,
                                const T *__restrict__ proj, T *__restrict__ fvc, T *__restrict__ fvi,
                                T *__restrict__ fn) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (f >= s.F) return;
  Cam<T> cam;
  load_cam(s, b, rot, trans, xf, proj, cam);
  int64_t vi[3];
  const bool ok = face_corners<T>(s, faces, f, vi);
  const T *vb = verts + (s.Bv == 1 ? 0 : (int64_t)b * s.V * 3);
  T c[3][3], img[3][2];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    T v[3], tr[3];
#pragma unroll
    for (int d = 0; d < 3; d++) v[d] = ok ? vb[vi[k] * 3 + d] : (T)NAN;
    to_camera(s.mode, cam, v, c[k], tr);
    const T pz = c[k][2] * cam.p[2];
    img[k][0] = (c[k][0] * cam.p[0]) / pz;
    img[k][1] = (c[k][1] * cam.p[1]) / pz;
  }
  const int64_t o = (int64_t)b * s.F + f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
#pragma unroll
    for (int d = 0; d < 3; d++) fvc[o * 9 + k * 3 + d] = c[k][d];
    fvi[o * 6 + k * 2 + 0] = img[k][0];
    fvi[o * 6 + k * 2 + 1] = img[k][1];
  }
  T e0[3], e1[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    e0[d] = c[1][d] - c[0][d];
    e1[d] = c[2][d] - c[0][d];
  }
  const T n0 = e0[1] * e1[2] - e0[2] * e1[1];
  const T n1 = e0[2] * e1[0] - e0[0] * e1[2];
  const T n2 = e0[0] * e1[1] - e0[1] * e1[0];
  const T len = kl_sqrt<T>(n0 * n0 + n1 * n1 + n2 * n2);
  const T den = len + (T)1e-10;
  fn[o * 3 + 0] = n0 / den;
  fn[o * 3 + 1] = n1 / den;
  fn[o * 3 + 2] = n2 / den;
}

// Workspace (doubles): per (view, vertex) 5 sums -- the grads of vertices_camera (3) and of
// vertices_image (2); per view 15 camera sums; per vertex 3 sums of a broadcast (Bv == 1)
// vertex tensor's grad.
struct PrepWs {
  double *gv;    // (B, V, kGvStride): camera x, y, z, image x, y
  double *cam;   // (B, 15): rot/transform 12 (m order), proj 3
  double *gvb;   // (V, 3) when Bv == 1
};

// per-vertex backward accumulator stride in doubles (see prep_bwd_face_kernel)
constexpr int kGvStride = 8;
static size_t prep_ws_bytes(int B, int64_t V) {
  return al256((size_t)B * V * kGvStride * 8) + al256((size_t)B * 15 * 8) + al256((size_t)V * 3 * 8);
}

static PrepWs prep_ws(void *ws, int B, int64_t V) {
  char *p = (char *)ws;
  PrepWs w;
  w.gv = (double *)p;
  p += al256((size_t)B * V * kGvStride * 8);
  w.cam = (double *)p;
  p += al256((size_t)B * 15 * 8);
  w.gvb = (double *)p;
  return w;
}

// The per-vertex accumulators are 8 doubles (one 64-byte line: camera-space x, y, z, image x,
// y, pad), so that the five adds of one corner, issued by five adjacent lanes, leave as one
// memory-side atomic request.  Each face's 15 terms are staged in LDS and then added with
// (face, corner, term) spread over the lanes: one thread adding its face's 15 terms itself
// sent 15 scattered requests per face (114 us for 4 views x 50k faces, against ~20 requests
// per ns chip-wide).
template <typename T>
__global__ void __launch_bounds__(256) prep_bwd_face_kernel(PrepSrc s, const T *__restrict__ verts, const int64_t *__restrict__ faces,
                                     const T *__restrict__ rot, const T *__restrict__ trans,
                                     const T *__restrict__ xf, const T *__restrict__ proj,
                                     const T *__restrict__ g_fvc, const T *__restrict__ g_fvi,
                                     const T *__restrict__ g_fn, double *__restrict__ gv) {
  __shared__ double s_val[256][15];
  __shared__ int64_t s_vi[256][3];
  const int tid = threadIdx.x;
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + tid;
  const int b = blockIdx.y;
  int64_t vi[3] = {0, 0, 0};
  const bool ok = f < s.F && face_corners<T>(s, faces, f, vi);  // a bad index adds nothing
  T gc[3][3], gi[3][2];
#pragma unroll
  for (int k = 0; k < 3; k++) {
#pragma unroll
    for (int d = 0; d < 3; d++) gc[k][d] = (T)0;
    gi[k][0] = gi[k][1] = (T)0;
  }
  if (ok) {
    const int64_t o = (int64_t)b * s.F + f;
    if (g_fvc) {
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int d = 0; d < 3; d++) gc[k][d] = g_fvc[o * 9 + k * 3 + d];
    }
    if (g_fvi) {
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int d = 0; d < 2; d++) gi[k][d] = g_fvi[o * 6 + k * 2 + d];
    }
    if (g_fn) {
      Cam<T> cam;
      load_cam(s, b, rot, trans, xf, proj, cam);
      const T *vb = verts + (s.Bv == 1 ? 0 : (int64_t)b * s.V * 3);
      T c[3][3];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        T v[3], tr[3];
#pragma unroll
        for (int d = 0; d < 3; d++) v[d] = vb[vi[k] * 3 + d];
        to_camera(s.mode, cam, v, c[k], tr);
      }
      T e0[3], e1[3];
#pragma unroll
      for (int d = 0; d < 3; d++) {
        e0[d] = c[1][d] - c[0][d];
        e1[d] = c[2][d] - c[0][d];
      }
      T n[3];
      n[0] = e0[1] * e1[2] - e0[2] * e1[1];
      n[1] = e0[2] * e1[0] - e0[0] * e1[2];
      n[2] = e0[0] * e1[1] - e0[1] * e1[0];
      const T len = kl_sqrt<T>(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      const T den = len + (T)1e-10;
      const T g[3] = {g_fn[o * 3 + 0], g_fn[o * 3 + 1], g_fn[o * 3 + 2]};
      // out = n / den: grad_n = g / den; grad_den = sum(-g * n / (den * den)) (autograd's div)
      T gden = (T)0;
      T gn[3];
#pragma unroll
      for (int d = 0; d < 3; d++) {
        gn[d] = g[d] / den;
        gden += -g[d] * n[d] / (den * den);
      }
      // den = norm + 1e-10; norm backward: grad * n / norm (0 where norm == 0)
      if (len != (T)0) {
#pragma unroll
        for (int d = 0; d < 3; d++) gn[d] += n[d] * (gden / len);
      }
      // n = cross(e0, e1): grad_e0 = cross(e1, gn), grad_e1 = cross(gn, e0)
      const T ge0[3] = {e1[1] * gn[2] - e1[2] * gn[1], e1[2] * gn[0] - e1[0] * gn[2],
                        e1[0] * gn[1] - e1[1] * gn[0]};
      const T ge1[3] = {gn[1] * e0[2] - gn[2] * e0[1], gn[2] * e0[0] - gn[0] * e0[2],
                        gn[0] * e0[1] - gn[1] * e0[0]};
#pragma unroll
      for (int d = 0; d < 3; d++) {
        gc[1][d] += ge0[d];
        gc[2][d] += ge1[d];
        gc[0][d] += -ge0[d] - ge1[d];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
#pragma unroll
    for (int d = 0; d < 3; d++) s_val[tid][k * 5 + d] = (double)gc[k][d];
    s_val[tid][k * 5 + 3] = (double)gi[k][0];
    s_val[tid][k * 5 + 4] = (double)gi[k][1];
    s_vi[tid][k] = vi[k];
  }
  __syncthreads();
  double *gb = gv + (int64_t)b * s.V * kGvStride;
  const int64_t f0 = (int64_t)blockIdx.x * blockDim.x;
  const int nf = (int)(s.F - f0 < (int64_t)blockDim.x ? s.F - f0 : (int64_t)blockDim.x);
  for (int i = tid; i < nf * 15; i += blockDim.x) {
    const int fl = i / 15, j = i % 15;
    const double v = s_val[fl][j];
    if (v != 0.0) atomicAdd(gb + s_vi[fl][j / 5] * kGvStride + j % 5, v);
  }
}

// sum of v over the workgroup in double, then one atomic (every thread calls it)
__device__ __forceinline__ void block_add(double v, double *s_red, double *dst) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s_red[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += s_red[w];
    if (t != 0.0) atomicAdd(dst, t);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) prep_bwd_vertex_kernel(PrepSrc s, const T *__restrict__ verts,
                                                              const T *__restrict__ rot, const T *__restrict__ trans,
                                                              const T *__restrict__ xf, const T *__restrict__ proj,
                                                              const double *__restrict__ gv, T *__restrict__ g_verts,
                                                              double *__restrict__ cam_acc,
                                                              double *__restrict__ gvb) {
  __shared__ double s_red[4];
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  const bool live = v < s.V;
  Cam<T> cam;
  load_cam(s, b, rot, trans, xf, proj, cam);
  T gcam[15];
#pragma unroll
  for (int k = 0; k < 15; k++) gcam[k] = (T)0;
  if (live) {
    const T *vp = verts + (s.Bv == 1 ? 0 : (int64_t)b * s.V * 3) + v * 3;
    const T vv[3] = {vp[0], vp[1], vp[2]};
    T c[3], tr[3];
    to_camera(s.mode, cam, vv, c, tr);
    const double *g5 = gv + ((int64_t)b * s.V + v) * kGvStride;
    T gc[3] = {(T)g5[0], (T)g5[1], (T)g5[2]};  // scatter-add of face_vertices_camera's grads
    const T gi[2] = {(T)g5[3], (T)g5[4]};       // ... and of face_vertices_image's
    // perspective_camera backward: pp = c * p; img = pp[:2] / pp[2]
    const T pp[3] = {c[0] * cam.p[0], c[1] * cam.p[1], c[2] * cam.p[2]};
    T gpp[3];
    gpp[0] = gi[0] / pp[2];
    gpp[1] = gi[1] / pp[2];
    gpp[2] = -gi[0] * pp[0] / (pp[2] * pp[2]) + -gi[1] * pp[1] / (pp[2] * pp[2]);
#pragma unroll
    for (int d = 0; d < 3; d++) {
      gc[d] += gpp[d] * cam.p[d];
      gcam[12 + d] = gpp[d] * c[d];
    }
    T gvx[3];
    if (s.mode == 0) {
      // c = tr @ rot^T: grad_tr = gc @ rot; grad_rot[i][j] = gc_i * tr_j; grad_trans = -grad_tr
#pragma unroll
      for (int j = 0; j < 3; j++) gvx[j] = gc[0] * cam.m[0 * 3 + j] + gc[1] * cam.m[1 * 3 + j] + gc[2] * cam.m[2 * 3 + j];
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) gcam[i * 3 + j] = gc[i] * tr[j];
#pragma unroll
      for (int j = 0; j < 3; j++) gcam[9 + j] = -gvx[j];
    } else {
      // c = [v, 1] @ T: grad_v_j = sum_i gc_i T[j][i]; grad_T[j][i] = pad_j gc_i
#pragma unroll
      for (int j = 0; j < 3; j++) gvx[j] = gc[0] * cam.m[j * 3 + 0] + gc[1] * cam.m[j * 3 + 1] + gc[2] * cam.m[j * 3 + 2];
#pragma unroll
      for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++) gcam[j * 3 + i] = vv[j] * gc[i];
#pragma unroll
      for (int i = 0; i < 3; i++) gcam[9 + i] = gc[i];
    }
    if (s.Bv == 1 && gvb) {
#pragma unroll
      for (int j = 0; j < 3; j++)
        if (gvx[j] != (T)0) atomicAdd(gvb + v * 3 + j, (double)gvx[j]);
    } else if (g_verts) {
#pragma unroll
      for (int j = 0; j < 3; j++) g_verts[((int64_t)b * s.V + v) * 3 + j] = gvx[j];
    }
  }
  if (cam_acc) {
#pragma unroll 1
    for (int k = 0; k < 15; k++) block_add((double)gcam[k], s_red, cam_acc + b * 15 + k);
  }
}

// Camera grads (and a broadcast vertex tensor's) rounded once; cameras broadcast over views
// (Bc == 1 or Bp == 1) sum their views in double first.
template <typename T>
__global__ void prep_bwd_final_kernel(PrepSrc s, const double *__restrict__ cam_acc, T *__restrict__ g_m,
                                      T *__restrict__ g_proj, const double *__restrict__ gvb,
                                      T *__restrict__ g_verts) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s.Bv == 1 && g_verts && t < s.V * 3) g_verts[t] = (T)gvb[t];
  if (g_m && t < (int64_t)s.Bc * 12) {
    const int bc = (int)(t / 12), k = (int)(t % 12);
    double a = 0.0;
    if (s.Bc == 1)
      for (int b = 0; b < s.B; b++) a += cam_acc[b * 15 + k];
    else
      a = cam_acc[bc * 15 + k];
    g_m[t] = (T)a;
  }
  if (g_proj && t < (int64_t)s.Bp * 3) {
    const int bp = (int)(t / 3), k = (int)(t % 3);
    double a = 0.0;
    if (s.Bp == 1)
      for (int b = 0; b < s.B; b++) a += cam_acc[b * 15 + 12 + k];
    else
      a = cam_acc[bp * 15 + 12 + k];
    g_proj[t] = (T)a;
  }
}

static int prep_check(int B, int Bv, int Bc, int Bp, int64_t V, int64_t F, int mode) {
  KL_REQUIRE(B >= 0 && V >= 0 && F >= 0, "prepare_vertices: negative size");
  KL_REQUIRE((Bv == 1 || Bv == B) && (Bc == 1 || Bc == B) && (Bp == 1 || Bp == B),
             "prepare_vertices: vertices, camera and projection batches must be 1 or the view count");
  KL_REQUIRE(mode == 0 || mode == 1, "prepare_vertices: unknown camera mode");
  KL_REQUIRE(B <= 65535, "prepare_vertices: at most 65535 views per call");
  return KL_OK;
}

template <typename T>
static int prep_fwd(PrepSrc s, const void *verts, const int64_t *faces, const void *rot, const void *trans,
                    const void *xf, const void *proj, void *fvc, void *fvi, void *fn, hipStream_t st) {
  if (s.B == 0 || s.F == 0) return KL_OK;
  hipLaunchKernelGGL(prep_fwd_kernel<T>, dim3((unsigned)cdiv(s.F, 256), s.B), dim3(256), 0, st, s, (const T *)verts,
                     faces, (const T *)rot, (const T *)trans, (const T *)xf, (const T *)proj, (T *)fvc, (T *)fvi,
                     (T *)fn);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

template <typename T>
static int prep_bwd(PrepSrc s, const void *verts, const int64_t *faces, const void *rot, const void *trans,
                    const void *xf, const void *proj, const void *g_fvc, const void *g_fvi, const void *g_fn,
                    void *g_verts, void *g_m, void *g_proj, void *ws, hipStream_t st) {
  if (s.B == 0) return KL_OK;
  PrepWs w = prep_ws(ws, s.B, s.V);
  KL_CHECK_RC(fill_async(ws, 0, prep_ws_bytes(s.B, s.V), st));
  if (s.F > 0 && s.V > 0 && (g_fvc || g_fvi || g_fn)) {
    hipLaunchKernelGGL(prep_bwd_face_kernel<T>, dim3((unsigned)cdiv(s.F, 256), s.B), dim3(256), 0, st, s,
                       (const T *)verts, faces, (const T *)rot, (const T *)trans, (const T *)xf, (const T *)proj,
                       (const T *)g_fvc, (const T *)g_fvi, (const T *)g_fn, w.gv);
    KL_CHECK_LAUNCH();
  }
  const bool cam = g_m || g_proj;
  if (s.V > 0 && (g_verts || cam)) {
    // vertices of batch B: written directly; of batch 1: summed over the views in double
    T *gvo = s.Bv == 1 ? nullptr : (T *)g_verts;
    double *gvb = s.Bv == 1 && g_verts ? w.gvb : nullptr;
    hipLaunchKernelGGL(prep_bwd_vertex_kernel<T>, dim3((unsigned)cdiv(s.V, 256), s.B), dim3(256), 0, st, s,
                       (const T *)verts, (const T *)rot, (const T *)trans, (const T *)xf, (const T *)proj,
                       (const double *)w.gv, gvo, cam ? w.cam : nullptr, gvb);
    KL_CHECK_LAUNCH();
  }
  const int64_t nfin = s.V * 3 > (int64_t)s.B * 15 ? s.V * 3 : (int64_t)s.B * 15;
  if (nfin > 0 && (cam || (s.Bv == 1 && g_verts))) {
    hipLaunchKernelGGL(prep_bwd_final_kernel<T>, dim3((unsigned)cdiv(nfin, 256)), dim3(256), 0, st, s,
                       (const double *)w.cam, (T *)g_m, (T *)g_proj, (const double *)w.gvb,
                       s.Bv == 1 ? (T *)g_verts : nullptr);
    KL_CHECK_LAUNCH();
  }
  return KL_OK;
}

}  // namespace kl

using namespace kl;

extern "C" size_t kl_prepare_vertices_bwd_workspace_bytes(int B, int64_t V) { return prep_ws_bytes(B, V); }

extern "C" int kl_prepare_vertices_forward(kl_dtype dtype, int B, int Bv, int Bc, int Bp, int64_t V, int64_t F,
                                           const void *vertices, const int64_t *faces, const void *camera_rot,
                                           const void *camera_trans, const void *camera_transform,
                                           const void *camera_proj, void *face_vertices_camera,
                                           void *face_vertices_image, void *face_normals, kl_stream stream) {
  const int mode = camera_transform ? 1 : 0;
  KL_CHECK_RC(prep_check(B, Bv, Bc, Bp, V, F, mode));
  KL_REQUIRE(mode == 1 || (camera_rot && camera_trans), "prepare_vertices: camera_rot and camera_trans required");
  PrepSrc s{B, Bv, Bc, Bp, V, F, mode};
  switch (dtype) {
    case KL_F32:
      return prep_fwd<float>(s, vertices, faces, camera_rot, camera_trans, camera_transform, camera_proj,
                             face_vertices_camera, face_vertices_image, face_normals, S(stream));
    case KL_F64:
      return prep_fwd<double>(s, vertices, faces, camera_rot, camera_trans, camera_transform, camera_proj,
                              face_vertices_camera, face_vertices_image, face_normals, S(stream));
    default:
      break;
  }
  set_error("prepare_vertices: f32 / f64 only");
  return KL_E_INVALID;
}

extern "C" int kl_prepare_vertices_backward(kl_dtype dtype, int B, int Bv, int Bc, int Bp, int64_t V, int64_t F,
                                            const void *vertices, const int64_t *faces, const void *camera_rot,
                                            const void *camera_trans, const void *camera_transform,
                                            const void *camera_proj, const void *grad_face_vertices_camera,
                                            const void *grad_face_vertices_image, const void *grad_face_normals,
                                            void *grad_vertices, void *grad_camera, void *grad_camera_proj,
                                            void *ws, size_t ws_bytes, kl_stream stream) {
  const int mode = camera_transform ? 1 : 0;
  KL_CHECK_RC(prep_check(B, Bv, Bc, Bp, V, F, mode));
  KL_REQUIRE(mode == 1 || (camera_rot && camera_trans), "prepare_vertices: camera_rot and camera_trans required");
  KL_REQUIRE(ws && ws_bytes >= prep_ws_bytes(B, V), "prepare_vertices backward: workspace too small");
  PrepSrc s{B, Bv, Bc, Bp, V, F, mode};
  switch (dtype) {
    case KL_F32:
      return prep_bwd<float>(s, vertices, faces, camera_rot, camera_trans, camera_transform, camera_proj,
                             grad_face_vertices_camera, grad_face_vertices_image, grad_face_normals, grad_vertices,
                             grad_camera, grad_camera_proj, ws, S(stream));
    case KL_F64:
      return prep_bwd<double>(s, vertices, faces, camera_rot, camera_trans, camera_transform, camera_proj,
                              grad_face_vertices_camera, grad_face_vertices_image, grad_face_normals,
                              grad_vertices, grad_camera, grad_camera_proj, ws, S(stream));
    default:
      break;
  }
  set_error("prepare_vertices: f32 / f64 only");
  return KL_E_INVALID;
}
