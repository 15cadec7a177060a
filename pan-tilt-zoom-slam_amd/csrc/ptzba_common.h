// Shared device helpers for libptzba (gfx950 / CDNA4, wave64).
//
// Camera model.  The reference's BA projection
// TransFunction.from_ray_to_image (transformation.py:99-135) is a closed form in atan/sqrt; it is
// algebraically  q = R_x(tilt) R_y(pan) p,  p = [tan th, -tan ph * sqrt(tan^2 th + 1), 1],
//   x = u + f q0/q2,   y = v + f q1/|q2|          (|q2| in y only: the closed form's semantics)
// with R_x, R_y as in ptz_camera.py:73-79.  We evaluate the q form: per-frame trig (cos/sin of pan
// and tilt) and per-landmark trig (tan th, tan ph, ...) are hoisted into small tables so the
// per-observation work is a 3x3 rotation, one divide and the 2x5 analytic Jacobian.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PTZ_D2R 0.017453292519943295
#define WAVE 64

// Per-frame table: 8 reals (32 B fp32 / 64 B fp64) -> two 16-B loads.
template <typename real>
struct alignas(8 * sizeof(real)) FrameTab {
  real ca, sa, cb, sb, f, pad0, pad1, pad2;
};

// Per-landmark table: ray direction p = [p0, p1, 1] and its derivatives.
//   dp/dth = [d0t, d1t, 0]      dp/dph = [0, d1p, 0]
template <typename real>
struct alignas(8 * sizeof(real)) RayTab {
  real p0, p1, d0t, d1t, d1p, pad0, pad1, pad2;
};

// Build the frame table entry from a pose (degrees) in fp64 and round once.
template <typename real>
__device__ __forceinline__ FrameTab<real> make_frame_tab(double pan, double tilt, double f) {
  double a = pan * PTZ_D2R, b = tilt * PTZ_D2R;
  double sa, ca, sb, cb;
  sincos(a, &sa, &ca);
  sincos(b, &sb, &cb);
  FrameTab<real> t;
  t.ca = (real)ca; t.sa = (real)sa; t.cb = (real)cb; t.sb = (real)sb; t.f = (real)f;
  t.pad0 = t.pad1 = t.pad2 = (real)0;
  return t;
}

template <typename real>
__device__ __forceinline__ RayTab<real> make_ray_tab(double theta, double phi) {
  double th = theta * PTZ_D2R, ph = phi * PTZ_D2R;
  double tt = tan(th), tp = tan(ph);
  double sec_abs = sqrt(tt * tt + 1.0);                       // sqrt(tan^2+1) as ptz_camera.py:205
  double cth = cos(th), cph = cos(ph);
  double sec2t = 1.0 / (cth * cth), sec2p = 1.0 / (cph * cph);
  RayTab<real> r;
  r.p0 = (real)tt;
  r.p1 = (real)(-tp * sec_abs);
  r.d0t = (real)sec2t;                                       // d tan(th)/d th
  r.d1t = (real)(-tp * tt * sec2t / sec_abs);                // d(-tan ph sqrt(1+tan^2 th))/d th
  r.d1p = (real)(-sec2p * sec_abs);                          // d(-tan ph sqrt(1+tan^2 th))/d ph
  r.pad0 = r.pad1 = r.pad2 = (real)0;
  return r;
}

// Projection only.  Returns image x, y.
template <typename real>
__device__ __forceinline__ void ptz_project(const FrameTab<real>& F, const RayTab<real>& R, real u, real v,
                                            real& x, real& y) {
  real w0 = F.ca * R.p0 - F.sa;
  real w2 = F.sa * R.p0 + F.ca;
  real q1 = F.cb * R.p1 + F.sb * w2;
  real q2 = -F.sb * R.p1 + F.cb * w2;
  real iq = (real)1 / q2;
  x = u + F.f * w0 * iq;
  y = v + F.f * q1 * fabs(iq);
}

// Projection + analytic Jacobian J[2][5] w.r.t. (pan, tilt, f, theta, phi), all angles in degrees
// (verified against central FD of from_ray_to_image).
template <typename real>
__device__ __forceinline__ void ptz_project_jac(const FrameTab<real>& F, const RayTab<real>& R, real u, real v,
                                                real& x, real& y, real J[2][5]) {
  const real D = (real)PTZ_D2R;
  real w0 = F.ca * R.p0 - F.sa;
  real w2 = F.sa * R.p0 + F.ca;
  real q0 = w0;
  real q1 = F.cb * R.p1 + F.sb * w2;
  real q2 = -F.sb * R.p1 + F.cb * w2;
  real iq = (real)1 / q2;
  real iaq = fabs(iq);
  real sg = q2 >= (real)0 ? (real)1 : (real)-1;
  x = u + F.f * q0 * iq;
  y = v + F.f * q1 * iaq;
  // d(x,y)/dq
  real fx = F.f * iq, fxz = -F.f * q0 * iq * iq;
  real fy = F.f * iaq, fyz = -F.f * q1 * sg * iq * iq;
  // dq/dpan = [-w2, sb w0, cb w0] D
  real a0 = -w2 * D, a1 = F.sb * w0 * D, a2 = F.cb * w0 * D;
  J[0][0] = fx * a0 + fxz * a2;
  J[1][0] = fy * a1 + fyz * a2;
  // dq/dtilt = [0, q2, -q1] D
  J[0][1] = fxz * (-q1 * D);
  J[1][1] = fy * (q2 * D) + fyz * (-q1 * D);
  // d/df
  J[0][2] = q0 * iq;
  J[1][2] = q1 * iaq;
  // dq/dth = [ca d0, cb d1 + sb sa d0, -sb d1 + cb sa d0] D
  real t0 = F.ca * R.d0t * D;
  real t1 = (F.cb * R.d1t + F.sb * F.sa * R.d0t) * D;
  real t2 = (-F.sb * R.d1t + F.cb * F.sa * R.d0t) * D;
  J[0][3] = fx * t0 + fxz * t2;
  J[1][3] = fy * t1 + fyz * t2;
  // dq/dph = [0, cb e1, -sb e1] D
  real e1 = F.cb * R.d1p * D, e2 = -F.sb * R.d1p * D;
  J[0][4] = fxz * e2;
  J[1][4] = fy * e1 + fyz * e2;
}

// ---------------------------------------------------------------- wave64 helpers
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

// Make this wave's LDS writes visible to its own later LDS reads by other lanes, and stop the
// compiler from moving LDS accesses across this point (LDS ops of one wave execute in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// an int carried in a real-typed slot (bit pattern; the low word for double)
template <typename real>
__device__ __forceinline__ real __int_as_real(int i);
template <>
__device__ __forceinline__ float __int_as_real<float>(int i) { return __int_as_float(i); }
template <>
__device__ __forceinline__ double __int_as_real<double>(int i) { return __longlong_as_double((long long)i); }
__device__ __forceinline__ int __real_as_int(float x) { return __float_as_int(x); }
__device__ __forceinline__ int __real_as_int(double x) { return (int)__double_as_longlong(x); }
