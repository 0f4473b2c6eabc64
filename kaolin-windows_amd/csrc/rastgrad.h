// rastgrad.h -- the rasterizer backward's per-pixel terms (rasterization_cuda.cu:262-399), shared
// by the per-face gather (raster.hip) and the pixel-major DIB-R backward (dibrbwd.hip).
#pragma once

#include "common.h"

namespace kl {

// d(interpolated feature)/d(face vertices) of one pixel (rasterization_cuda.cu:287-399).
template <typename T>
struct BaryGrad {
  T dw1dax, dw1day, dw1dbx, dw1dby, dw1dcx, dw1dcy;
  T dw2dax, dw2day, dw2dbx, dw2dby, dw2dcx, dw2dcy;
  T k3sq;
  __device__ __forceinline__ void init(const T v[6], T w_a, T w_b, T w_c, float eps) {
    const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
    const T x0 = w_a * ax + w_b * bx + w_c * cx;
    const T y0 = w_a * ay + w_b * by + w_c * cy;
    const T m = bx - ax, p = by - ay, n = cx - ax, q = cy - ay, s = x0 - ax, t = y0 - ay;
    const T k1 = s * q - n * t;
    const T k2 = m * t - s * p;
    T k3 = m * q - n * p;
    k3 = (T)((double)k3 + copysign((double)eps, (double)k3));
    const T zero = (T)0;
    const T dk1dm = zero, dk1dn = -t, dk1dp = zero, dk1dq = s, dk1ds = q, dk1dt = -n;
    const T dk2dm = t, dk2dn = zero, dk2dp = -s, dk2dq = zero, dk2ds = -p, dk2dt = m;
    const T dk3dm = q, dk3dn = -p, dk3dp = -n, dk3dq = m, dk3ds = zero, dk3dt = zero;
    const T dw1dm = dk1dm * k3 - dk3dm * k1, dw1dn = dk1dn * k3 - dk3dn * k1;
    const T dw1dp = dk1dp * k3 - dk3dp * k1, dw1dq = dk1dq * k3 - dk3dq * k1;
    const T dw1ds = dk1ds * k3 - dk3ds * k1, dw1dt = dk1dt * k3 - dk3dt * k1;
    const T dw2dm = dk2dm * k3 - dk3dm * k2, dw2dn = dk2dn * k3 - dk3dn * k2;
    const T dw2dp = dk2dp * k3 - dk3dp * k2, dw2dq = dk2dq * k3 - dk3dq * k2;
    const T dw2ds = dk2ds * k3 - dk3ds * k2, dw2dt = dk2dt * k3 - dk3dt * k2;
    dw1dax = -(dw1dm + dw1dn + dw1ds);
    dw1day = -(dw1dp + dw1dq + dw1dt);
    dw1dbx = dw1dm; dw1dby = dw1dp; dw1dcx = dw1dn; dw1dcy = dw1dq;
    dw2dax = -(dw2dm + dw2dn + dw2ds);
    dw2day = -(dw2dp + dw2dq + dw2dt);
    dw2dbx = dw2dm; dw2dby = dw2dp; dw2dcx = dw2dn; dw2dcy = dw2dq;
    k3sq = k3 * k3;
  }
  // the six dL/d(vertex coordinate) terms of feature channel with grad gd and values c0..c2
  __device__ __forceinline__ void terms(T gd, T c0, T c1, T c2, T out[6]) const {
    const T dIdax = (c1 - c0) * dw1dax + (c2 - c0) * dw2dax;
    const T dIday = (c1 - c0) * dw1day + (c2 - c0) * dw2day;
    const T dIdbx = (c1 - c0) * dw1dbx + (c2 - c0) * dw2dbx;
    const T dIdby = (c1 - c0) * dw1dby + (c2 - c0) * dw2dby;
    const T dIdcx = (c1 - c0) * dw1dcx + (c2 - c0) * dw2dcx;
    const T dIdcy = (c1 - c0) * dw1dcy + (c2 - c0) * dw2dcy;
    const T dldI = gd / k3sq;
    out[0] = dldI * dIdax;
    out[1] = dldI * dIday;
    out[2] = dldI * dIdbx;
    out[3] = dldI * dIdby;
    out[4] = dldI * dIdcx;
    out[5] = dldI * dIdcy;
  }
};

}  // namespace kl
