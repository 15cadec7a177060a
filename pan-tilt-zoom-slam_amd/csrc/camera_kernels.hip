// Batched camera-model kernels (fp64): the L1 geometry API of the reference, on the GPU.
//   k_ray_to_image   TransFunction.from_ray_to_image (transformation.py:99-135), q form, |q2| in y
//   k_image_to_ray   TransFunction.from_image_to_ray (transformation.py:137-175)
//   k_project_rays   PTZCamera.project_ray (ptz_camera.py:191-210): K (R p + d), SIGNED q2,
//                    displacement d = w[0:3] + w[3:6] f (ptz_camera.py:106-115)
//   k_back_project   PTZCamera.back_project_to_ray (ptz_camera.py:287-312)
//   k_h_jacobian     PtzSlam.compute_h_jacobian (ptz_slam.py:73-138): the same central differences
//                    (0.001 deg, 0.1 px) of project_ray, written into the dense [2n, 3+2n] H
#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

__device__ __forceinline__ void rot_tp(double pan, double tilt, double R[3][3]) {
  double sa, ca, sb, cb;
  sincos(pan * PTZ_D2R, &sa, &ca);
  sincos(tilt * PTZ_D2R, &sb, &cb);
  // R_tilt @ R_pan, ptz_camera.py:73-79
  R[0][0] = ca;       R[0][1] = 0;   R[0][2] = -sa;
  R[1][0] = sb * sa;  R[1][1] = cb;  R[1][2] = sb * ca;
  R[2][0] = cb * sa;  R[2][1] = -sb; R[2][2] = cb * ca;
}

__global__ void k_ray_to_image(int64_t n, double u, double v, const double* __restrict__ f,
                               const double* __restrict__ cp, const double* __restrict__ ct,
                               const double* __restrict__ th, const double* __restrict__ ph,
                               double* __restrict__ x, double* __restrict__ y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  FrameTab<double> F = make_frame_tab<double>(cp[i], ct[i], f[i]);
  RayTab<double> Rt = make_ray_tab<double>(th[i], ph[i]);
  double xx, yy;
  ptz_project<double>(F, Rt, u, v, xx, yy);
  x[i] = xx;
  y[i] = yy;
}

__device__ __forceinline__ void back_project(double u, double v, double f, double pan, double tilt,
                                             const double* d6, double x, double y, double& th, double& ph) {
  double R[3][3];
  rot_tp(pan, tilt, R);
  double c[3] = {(x - u) / f, (y - v) / f, 1.0};
  if (d6) {
    c[0] -= d6[0] + d6[3] * f;
    c[1] -= d6[1] + d6[4] * f;
    c[2] -= d6[2] + d6[5] * f;
  }
  // R^-1 = R^T
  double p0 = R[0][0] * c[0] + R[1][0] * c[1] + R[2][0] * c[2];
  double p1 = R[0][1] * c[0] + R[1][1] * c[1] + R[2][1] * c[2];
  double p2 = R[0][2] * c[0] + R[1][2] * c[1] + R[2][2] * c[2];
  th = atan(p0 / p2) / PTZ_D2R;
  ph = atan(-p1 / sqrt(p0 * p0 + p2 * p2)) / PTZ_D2R;
}

__global__ void k_image_to_ray(int64_t n, double u, double v, const double* __restrict__ f,
                               const double* __restrict__ cp, const double* __restrict__ ct,
                               const double* __restrict__ x, const double* __restrict__ y,
                               double* __restrict__ th, double* __restrict__ ph) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a, b;
  back_project(u, v, f[i], cp[i], ct[i], nullptr, x[i], y[i], a, b);
  th[i] = a;
  ph[i] = b;
}

struct Disp {
  double d[6];
};

__device__ __forceinline__ void project_ray_mat(double u, double v, double f, const double R[3][3], const Disp& D,
                                                bool has_d, double th, double ph, double& x, double& y) {
  double t = tan(th * PTZ_D2R);
  double p[3] = {t, -tan(ph * PTZ_D2R) * sqrt(t * t + 1.0), 1.0};
  double c[3];
  for (int r = 0; r < 3; ++r) c[r] = R[r][0] * p[0] + R[r][1] * p[1] + R[r][2] * p[2];
  if (has_d) {
    c[0] += D.d[0] + D.d[3] * f;
    c[1] += D.d[1] + D.d[4] * f;
    c[2] += D.d[2] + D.d[5] * f;
  }
  double w = c[2];
  x = (f * c[0] + u * w) / w;
  y = (f * c[1] + v * w) / w;
}

__global__ void k_project_rays(int64_t n, double u, double v, double f, double pan, double tilt, Disp D, int has_d,
                               const double* __restrict__ rays, double* __restrict__ xy) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double R[3][3];
  rot_tp(pan, tilt, R);
  double x, y;
  project_ray_mat(u, v, f, R, D, has_d, rays[2 * i], rays[2 * i + 1], x, y);
  xy[2 * i] = x;
  xy[2 * i + 1] = y;
}

__global__ void k_back_project(int64_t n, double u, double v, double f, double pan, double tilt, Disp D, int has_d,
                               const double* __restrict__ xy, double* __restrict__ rays) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a, b;
  back_project(u, v, f, pan, tilt, has_d ? D.d : nullptr, xy[2 * i], xy[2 * i + 1], a, b);
  rays[2 * i] = a;
  rays[2 * i + 1] = b;
}

__global__ void k_h_jacobian(int64_t n, double u, double v, double f, double pan, double tilt, Disp D, int has_d,
                             const double* __restrict__ rays, double* __restrict__ H) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double da = 0.001, dfl = 0.1;
  const double th = rays[2 * i], ph = rays[2 * i + 1];
  const int64_t ncol = 3 + 2 * n;
  double R[3][3], x1, y1, x2, y2;
  double* h0 = H + (2 * i) * ncol;
  double* h1 = H + (2 * i + 1) * ncol;
  rot_tp(pan - da, tilt, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x1, y1);
  rot_tp(pan + da, tilt, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x2, y2);
  h0[0] = (x2 - x1) / (2 * da);
  h1[0] = (y2 - y1) / (2 * da);
  rot_tp(pan, tilt - da, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x1, y1);
  rot_tp(pan, tilt + da, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x2, y2);
  h0[1] = (x2 - x1) / (2 * da);
  h1[1] = (y2 - y1) / (2 * da);
  rot_tp(pan, tilt, R);
  project_ray_mat(u, v, f - dfl, R, D, has_d, th, ph, x1, y1);
  project_ray_mat(u, v, f + dfl, R, D, has_d, th, ph, x2, y2);
  h0[2] = (x2 - x1) / (2 * dfl);
  h1[2] = (y2 - y1) / (2 * dfl);
  project_ray_mat(u, v, f, R, D, has_d, th - da, ph, x1, y1);
  project_ray_mat(u, v, f, R, D, has_d, th + da, ph, x2, y2);
  h0[3 + 2 * i] = (x2 - x1) / (2 * da);
  h1[3 + 2 * i] = (y2 - y1) / (2 * da);
  project_ray_mat(u, v, f, R, D, has_d, th, ph - da, x1, y1);
  project_ray_mat(u, v, f, R, D, has_d, th, ph + da, x2, y2);
  h0[4 + 2 * i] = (x2 - x1) / (2 * da);
  h1[4 + 2 * i] = (y2 - y1) / (2 * da);
}

static inline dim3 g1(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }
static inline Disp mkdisp(const double* d6, int& has) {
  Disp D{};
  has = d6 ? 1 : 0;
  if (d6)
    for (int k = 0; k < 6; ++k) D.d[k] = d6[k];
  return D;
}

void launch_ray_to_image(int64_t n, double u, double v, const double* f, const double* cp, const double* ct,
                         const double* th, const double* ph, double* x, double* y, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_ray_to_image, g1(n), dim3(256), 0, st, n, u, v, f, cp, ct, th, ph, x, y);
}
void launch_image_to_ray(int64_t n, double u, double v, const double* f, const double* cp, const double* ct,
                         const double* x, const double* y, double* th, double* ph, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_image_to_ray, g1(n), dim3(256), 0, st, n, u, v, f, cp, ct, x, y, th, ph);
}
void launch_project_rays(int64_t n, double u, double v, double f, double pan, double tilt, const double* d6,
                         const double* rays, double* xy, hipStream_t st) {
  int has;
  Disp D = mkdisp(d6, has);
  if (n > 0) hipLaunchKernelGGL(k_project_rays, g1(n), dim3(256), 0, st, n, u, v, f, pan, tilt, D, has, rays, xy);
}
void launch_back_project(int64_t n, double u, double v, double f, double pan, double tilt, const double* d6,
                         const double* xy, double* rays, hipStream_t st) {
  int has;
  Disp D = mkdisp(d6, has);
  if (n > 0) hipLaunchKernelGGL(k_back_project, g1(n), dim3(256), 0, st, n, u, v, f, pan, tilt, D, has, xy, rays);
}
void launch_h_jacobian(int64_t n, double u, double v, double f, double pan, double tilt, const double* d6,
                       const double* rays, double* H, hipStream_t st) {
  int has;
  Disp D = mkdisp(d6, has);
  if (n > 0) hipLaunchKernelGGL(k_h_jacobian, g1(n), dim3(256), 0, st, n, u, v, f, pan, tilt, D, has, rays, H);
}

}  // namespace ptzba
