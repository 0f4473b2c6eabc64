// rays.hip -- the deprecated ray generators of _C.render.spc (SURVEY.md §2.1 "next" ray-ops row):
// generate_primary_rays_cuda and generate_shadow_rays_cuda.
//
// Reference: raytrace.cpp:111-166 / 234-283 (bindings, host matrix set-up) over
// raytrace_cuda.cu:764-909 (kernels); bindings.cpp:86,88.  Neither has a Python caller or a
// test in the reference: results follow the restated arithmetic (host set-up in plain float,
// device rows as CUDA contracts them, fma chains) and the tests hold them to a few ulps of a
// float64 restatement (parity unpinned beyond that: no reference output exists).
//
// Kept behaviour of the reference, quirks included:
// * primary rays: pixel (tidx % width, tidx / height) -- the row uses the height, so for
//   width != height the rows repeat or skip; origin = row 2 of the matrix product applied to
//   (0, 0, 1, 0), direction = (px, py, 0, 1) applied (not normalised);
// * shadow rays: the hit count is the exclusive scan's entry at num - 1 (the last ray's own
//   hit is not counted); src / dst / map are the first `count` rows.
#include <hipcub/hipcub.hpp>

#include <cmath>

#include "common.h"

namespace kl {

struct M44 {
  float m[4][4];
};

// spc_math.h matmul4x4 / mul4x4 in plain float (the host set-up)
static M44 m44_mul(const M44 &a, const M44 &b) {
  M44 c;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      float s = a.m[i][0] * b.m[0][j];
      s = s + a.m[i][1] * b.m[1][j];
      s = s + a.m[i][2] * b.m[2][j];
      s = s + a.m[i][3] * b.m[3][j];
      c.m[i][j] = s;
    }
  return c;
}

// a * m, a row vector, with the fma chain CUDA's contraction gives mul4x4's sums
__device__ __forceinline__ float row_dot(float a0, float a1, float a2, float a3, const M44 &m, int j) {
  return fmaf(a3, m.m[3][j], fmaf(a2, m.m[2][j], fmaf(a1, m.m[1][j], a0 * m.m[0][j])));
}

__global__ void __launch_bounds__(256) primary_rays_kernel(uint32_t num, uint32_t width, uint32_t height, M44 tf,
                                                           float *__restrict__ org, float *__restrict__ dir) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= num) return;
  const float px = (float)(t % width), py = (float)(t / height);
  for (int j = 0; j < 3; j++) {
    org[(size_t)t * 3 + j] = row_dot(0.f, 0.f, 1.f, 0.f, tf, j);
    dir[(size_t)t * 3 + j] = row_dot(px, py, 0.f, 1.f, tf, j);
  }
}

// raytrace_cuda.cu plane_intersect: info = 1 and the hit point when the ray meets the plane ahead
__global__ void __launch_bounds__(256) shadow_hit_kernel(uint32_t num, const float *__restrict__ ro,
                                                         const float *__restrict__ rd, float4 plane,
                                                         float *__restrict__ hit, uint32_t *__restrict__ info) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= num) return;
  const float ox = ro[(size_t)t * 3], oy = ro[(size_t)t * 3 + 1], oz = ro[(size_t)t * 3 + 2];
  const float dx = rd[(size_t)t * 3], dy = rd[(size_t)t * 3 + 1], dz = rd[(size_t)t * 3 + 2];
  const float a = fmaf(oz, plane.z, fmaf(oy, plane.y, ox * plane.x)) + plane.w;
  const float b = fmaf(dz, plane.z, fmaf(dy, plane.y, dx * plane.x));
  uint32_t ok = 0;
  if ((double)fabsf(b) > 1e-3) {
    const float s = -a / b;
    if (s > 0.0f) {
      hit[(size_t)t * 3] = fmaf(s, dx, ox);
      hit[(size_t)t * 3 + 1] = fmaf(s, dy, oy);
      hit[(size_t)t * 3 + 2] = fmaf(s, dz, oz);
      ok = 1;
    }
  }
  info[t] = ok;
}

// compactify + set_shadow_rays in one pass: row psum[t] of the output takes ray t's hit; rows
// past the reference's count are not written
__global__ void __launch_bounds__(256) shadow_emit_kernel(uint32_t num, const float *__restrict__ hit,
                                                          const uint32_t *__restrict__ info,
                                                          const uint32_t *__restrict__ psum, float3 light,
                                                          float *__restrict__ src, float *__restrict__ dst,
                                                          int32_t *__restrict__ map) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= num || !info[t]) return;
  const uint32_t o = psum[t];
  if (o >= psum[num - 1]) return;
  const float vx = hit[(size_t)t * 3] - light.x, vy = hit[(size_t)t * 3 + 1] - light.y,
              vz = hit[(size_t)t * 3 + 2] - light.z;
  const float inv = rsqrtf(fmaf(vz, vz, fmaf(vy, vy, vx * vx)));
  dst[(size_t)o * 3] = vx * inv;
  dst[(size_t)o * 3 + 1] = vy * inv;
  dst[(size_t)o * 3 + 2] = vz * inv;
  src[(size_t)o * 3] = light.x;
  src[(size_t)o * 3 + 1] = light.y;
  src[(size_t)o * 3 + 2] = light.z;
  map[o] = (int32_t)t;
}

static float3 f3_norm(float x, float y, float z) {
  const float inv = 1.0f / sqrtf(x * x + y * y + z * z);
  return make_float3(x * inv, y * inv, z * inv);
}

}  // namespace kl

using namespace kl;

extern "C" int kl_generate_primary_rays(uint32_t height, uint32_t width, const float *eye, const float *at,
                                        const float *up, float fov, const float *world, float *ray_o, float *ray_d,
                                        kl_stream stream) {
  KL_REQUIRE(eye && at && up && world, "generate_primary_rays: null host argument");
  const uint64_t num64 = (uint64_t)width * height;
  KL_REQUIRE(num64 < ((uint64_t)1 << 32), "generate_primary_rays: width * height must be < 2^32");
  const uint32_t num = (uint32_t)num64;
  if (num == 0) return KL_OK;
  M44 winv;  // transpose(world)
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) winv.m[i][j] = world[j * 4 + i];
  const float ar = (float)width / (float)height;
  const float th = tanf(0.5f * fov);
  const float W = (float)width, H = (float)height;
  const M44 pvp{{{2.0f * ar * th / W, 0.f, 0.f, 0.f},
                 {0.f, 2.0f * th / H, 0.f, 0.f},
                 {0.f, 0.f, 0.f, 1.f},
                 {ar * th * (1.0f - W) / W, th * (1.0f - H) / H, -1.f, 0.f}}};
  const float3 z = f3_norm(at[0] - eye[0], at[1] - eye[1], at[2] - eye[2]);
  // crs3(z, up)
  const float3 x = f3_norm(z.y * up[2] - up[1] * z.z, z.z * up[0] - up[2] * z.x, z.x * up[1] - up[0] * z.y);
  const float3 y = make_float3(x.y * z.z - z.y * x.z, x.z * z.x - z.z * x.x, x.x * z.y - z.x * x.y);
  const M44 view{{{x.x, x.y, x.z, 0.f}, {y.x, y.y, y.z, 0.f}, {-z.x, -z.y, -z.z, 0.f}, {eye[0], eye[1], eye[2], 1.f}}};
  const M44 tf = m44_mul(m44_mul(pvp, view), winv);
  hipLaunchKernelGGL(primary_rays_kernel, dim3((unsigned)cdiv(num, 256)), dim3(256), 0, S(stream), num, width, height,
                     tf, ray_o, ray_d);
  KL_CHECK_LAUNCH();
  return KL_OK;
}

extern "C" size_t kl_generate_shadow_rays_workspace_bytes(int64_t num) {
  size_t tb = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                         (int)(num > 0 ? num : 1));
  const size_t n = (size_t)(num > 0 ? num : 1);
  return ((n * 12 + 255) & ~(size_t)255) + 2 * ((n * 4 + 255) & ~(size_t)255) + tb + 256;
}

extern "C" int kl_generate_shadow_rays(int64_t num, const float *ray_o, const float *ray_d, const float *light,
                                       const float *plane, float *src, float *dst, int32_t *map, int64_t *count,
                                       void *workspace, size_t workspace_bytes, kl_stream stream) {
  KL_REQUIRE(num >= 0 && num < ((int64_t)1 << 31), "generate_shadow_rays: num must be in [0, 2^31)");
  KL_REQUIRE(light && plane && count, "generate_shadow_rays: null host argument");
  *count = 0;
  if (num == 0) return KL_OK;
  KL_REQUIRE(workspace && workspace_bytes >= kl_generate_shadow_rays_workspace_bytes(num),
             "generate_shadow_rays: workspace too small");
  hipStream_t st = S(stream);
  const size_t n = (size_t)num;
  uint8_t *w = (uint8_t *)workspace;
  float *hit = (float *)w;
  w += (n * 12 + 255) & ~(size_t)255;
  uint32_t *info = (uint32_t *)w;
  w += (n * 4 + 255) & ~(size_t)255;
  uint32_t *psum = (uint32_t *)w;
  w += (n * 4 + 255) & ~(size_t)255;
  size_t tb = 0;
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, info, psum, (int)num, st));
  // raytrace.cpp:259-263: the light and the plane mapped from [-1, 1]^3 to [0, 1]^3
  const float3 lt = make_float3(0.5f * (light[0] + 1.0f), 0.5f * (light[1] + 1.0f), 0.5f * (light[2] + 1.0f));
  const float4 pl = make_float4(2.0f * plane[0], 2.0f * plane[1], 2.0f * plane[2],
                                plane[3] - plane[0] - plane[1] - plane[2]);
  const unsigned g = (unsigned)cdiv(num, 256);
  hipLaunchKernelGGL(shadow_hit_kernel, dim3(g), dim3(256), 0, st, (uint32_t)num, ray_o, ray_d, pl, hit, info);
  KL_CHECK_LAUNCH();
  KL_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(w, tb, info, psum, (int)num, st));
  hipLaunchKernelGGL(shadow_emit_kernel, dim3(g), dim3(256), 0, st, (uint32_t)num, (const float *)hit,
                     (const uint32_t *)info, (const uint32_t *)psum, lt, src, dst, map);
  KL_CHECK_LAUNCH();
  uint32_t c = 0;
  KL_CHECK_HIP(hipMemcpyAsync(&c, psum + num - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  KL_CHECK_HIP(hipStreamSynchronize(st));
  *count = c;
  return KL_OK;
}
