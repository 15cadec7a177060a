// PTZCamera ray model shared by the camera and EKF kernels (fp64):
//   rot_tp          R_tilt R_pan (ptz_camera.py:73-79)
//   project_ray_mat PTZCamera.project_ray (ptz_camera.py:191-210): K (R p + d), signed q2
//   back_project    PTZCamera.back_project_to_ray (ptz_camera.py:287-312)
#pragma once
#include "ptzba_common.h"

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

// PtzSlam.compute_h_jacobian (ptz_slam.py:73-138) for one ray: the reference's central differences
// (0.001 deg for angles, 0.1 px for f) of project_ray.  h[0..2] = dx/d(pan, tilt, f),
// h[3..5] = dy/d(pan, tilt, f), h[6..7] = dx/d(theta, phi), h[8..9] = dy/d(theta, phi).
__device__ __forceinline__ void h_fd_block(double u, double v, double f, double pan, double tilt, const Disp& D,
                                           bool has_d, double th, double ph, double h[10]) {
  const double da = 0.001, dfl = 0.1;
  double R[3][3], x1, y1, x2, y2;
  rot_tp(pan - da, tilt, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x1, y1);
  rot_tp(pan + da, tilt, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x2, y2);
  h[0] = (x2 - x1) / (2 * da);
  h[3] = (y2 - y1) / (2 * da);
  rot_tp(pan, tilt - da, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x1, y1);
  rot_tp(pan, tilt + da, R);
  project_ray_mat(u, v, f, R, D, has_d, th, ph, x2, y2);
  h[1] = (x2 - x1) / (2 * da);
  h[4] = (y2 - y1) / (2 * da);
  rot_tp(pan, tilt, R);
  project_ray_mat(u, v, f - dfl, R, D, has_d, th, ph, x1, y1);
  project_ray_mat(u, v, f + dfl, R, D, has_d, th, ph, x2, y2);
  h[2] = (x2 - x1) / (2 * dfl);
  h[5] = (y2 - y1) / (2 * dfl);
  project_ray_mat(u, v, f, R, D, has_d, th - da, ph, x1, y1);
  project_ray_mat(u, v, f, R, D, has_d, th + da, ph, x2, y2);
  h[6] = (x2 - x1) / (2 * da);
  h[8] = (y2 - y1) / (2 * da);
  project_ray_mat(u, v, f, R, D, has_d, th, ph - da, x1, y1);
  project_ray_mat(u, v, f, R, D, has_d, th, ph + da, x2, y2);
  h[7] = (x2 - x1) / (2 * da);
  h[9] = (y2 - y1) / (2 * da);
}

}  // namespace ptzba
