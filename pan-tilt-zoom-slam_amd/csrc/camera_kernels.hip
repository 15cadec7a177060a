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
#include "camera_model.h"

namespace ptzba {

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
  double h[10];
  h_fd_block(u, v, f, pan, tilt, D, has_d, rays[2 * i], rays[2 * i + 1], h);
  const int64_t ncol = 3 + 2 * n;
  double* h0 = H + (2 * i) * ncol;
  double* h1 = H + (2 * i + 1) * ncol;
  for (int q = 0; q < 3; ++q) { h0[q] = h[q]; h1[q] = h[3 + q]; }
  h0[3 + 2 * i] = h[6]; h0[4 + 2 * i] = h[7];
  h1[3 + 2 * i] = h[8]; h1[4 + 2 * i] = h[9];
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
