// EKF tracking state and update on the GPU (gfx950, fp64).
//
//   ptzekf_update       PtzSlam.ekf_update        ptz_slam.py:210-289
//   ptzekf_remove_rays  PtzSlam.remove_rays       ptz_slam.py:291-315
//   ptzekf_add_rays     PtzSlam.add_rays (state)  ptz_slam.py:376-384
//   ptzekf_add_pose_cov tracking() predict step   ptz_slam.py:424-426
//
// The ray landmarks [R,2] and the dense state covariance [(3+2R)^2] stay resident in HBM between
// frames (the reference keeps them as numpy arrays and re-grows them with row_stack every frame).
//
// Update without an explicit inverse.  With P the covariance restricted to (pose, matched rays),
// H the [2r x (3+2r)] measurement Jacobian and y the innovation, the augmented symmetric matrix
//
//        [ S = H P H^T + sigma I    H P   ]          (S block padded to a multiple of 32 with I)
//   M =  [ (H P)^T                  P     ]
//        [ y^T                      0     ]
//
// is factored by the tiled (signed) Cholesky of chol_kernels.hip only through the S columns (plus one
// flush launch of the trailing update).  The trailing block is then the Schur complement
//   P - (HP)^T S^-1 HP = (I - K H) P          and in the y row   -y^T S^-1 H P = -(K y)^T,
// i.e. the reference's Kalman gain K = P H^T S^-1 (ptz_slam.py:256-262) and updated covariance
// (:280) in one factorisation.  H is block sparse (3 dense pose columns + one 2x2 block per ray), so
// H P and H P H^T are assembled directly from the gathered covariance.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../../include/ptzba.h"
#include "camera_model.h"
#include "host_util.h"
#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

static inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// project every ray with the predicted camera; vis = strictly inside the image (ptz_camera.py:223-227)
__global__ void k_ekf_project(int n, double u, double v, double f, double pan, double tilt, Disp D, int has_d,
                              const double* __restrict__ rays, double* __restrict__ xy, uint8_t* __restrict__ vis,
                              int height, int width) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double R[3][3], x, y;
  rot_tp(pan, tilt, R);
  project_ray_mat(u, v, f, R, D, has_d, rays[2 * i], rays[2 * i + 1], x, y);
  xy[2 * i] = x;
  xy[2 * i + 1] = y;
  vis[i] = (x > 0 && x < width && y > 0 && y < height) ? 1 : 0;
}

// per matched ray: 2x5 FD Jacobian block (ptz_slam.py:251-254 -> :73-138) and innovation
// y = observed - predicted (:228-230)
__global__ void k_ekf_hblocks(int nr, const int32_t* __restrict__ matched, const int32_t* __restrict__ o1,
                              const double* __restrict__ obs_xy, const double* __restrict__ pred_xy,
                              const double* __restrict__ rays, double u, double v, double f, double pan, double tilt,
                              Disp D, int has_d, double* __restrict__ Hc, double* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  const int r = matched[i];
  double h[10];
  h_fd_block(u, v, f, pan, tilt, D, has_d, rays[2 * r], rays[2 * r + 1], h);
  for (int k = 0; k < 10; ++k) Hc[(int64_t)i * 10 + k] = h[k];
  y[2 * i] = obs_xy[2 * (int64_t)o1[i]] - pred_xy[2 * r];
  y[2 * i + 1] = obs_xy[2 * (int64_t)o1[i] + 1] - pred_xy[2 * r + 1];
}

// state index of reduced column c (pose 0..2, then 2 per matched ray), ptz_slam.py:239-245
__device__ __forceinline__ int64_t pr_index(int c, const int32_t* __restrict__ matched) {
  return c < 3 ? c : 3 + 2 * (int64_t)matched[(c - 3) >> 1] + ((c - 3) & 1);
}

struct EkfDims {
  int nr, m, mp, n, yr;  // matched rays, 2nr, padded S size, 3+2nr, y row
  int64_t ld, ns;        // M leading dimension, covariance stride (3+2R)
};

// (HP)^T block: M[mp + c][2i + a] = sum_q H[2i+a][q] P[q][c] + sum_b H[2i+a][3+2i+b] P[3+2i+b][c]
// and the P block M[mp + c][mp + c'] = cov[pr(c)][pr(c')]; x = column c (coalesced over cov rows)
__global__ void k_ekf_assemble_hp(EkfDims d, const int32_t* __restrict__ matched, const double* __restrict__ cov,
                                  const double* __restrict__ Hc, double* __restrict__ M) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int rowi = blockIdx.y;  // 0..nr-1: H rows 2i, 2i+1 ; nr..nr+n-1: P row
  if (c >= d.n) return;
  const int64_t pc = pr_index(c, matched);
  if (rowi < d.nr) {
    const int i = rowi;
    const double* h = Hc + (int64_t)i * 10;
    const int64_t r0 = 3 + 2 * (int64_t)matched[i];
    const double p0 = cov[0 * d.ns + pc], p1 = cov[1 * d.ns + pc], p2 = cov[2 * d.ns + pc];
    const double pa = cov[r0 * d.ns + pc], pb = cov[(r0 + 1) * d.ns + pc];
    const double hp0 = h[0] * p0 + h[1] * p1 + h[2] * p2 + h[6] * pa + h[7] * pb;
    const double hp1 = h[3] * p0 + h[4] * p1 + h[5] * p2 + h[8] * pa + h[9] * pb;
    double* dst = M + (int64_t)(d.mp + c) * d.ld + 2 * i;
    dst[0] = hp0;
    dst[1] = hp1;
  } else {
    const int a = rowi - d.nr;  // P row a, write lower part (c <= a)
    if (c > a) return;
    M[(int64_t)(d.mp + a) * d.ld + d.mp + c] = cov[pr_index(a, matched) * d.ns + pc];
  }
}

// S = H P H^T + sigma I (lower, row r' >= column r) from the (HP)^T block, the padding identity and
// the y row.  x = column r (coalesced reads of (HP)^T rows), y = row r'.
__global__ void k_ekf_assemble_s(EkfDims d, const double* __restrict__ Hc, const double* __restrict__ y,
                                 double sigma, double* __restrict__ M) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int rp = blockIdx.y;
  if (rp < d.m) {
    if (r > rp) return;
    const int i2 = rp >> 1, a2 = rp & 1;
    const double* h = Hc + (int64_t)i2 * 10;
    const double* hpT = M + (int64_t)d.mp * d.ld + r;  // (HP)^T[c][r] = M[mp + c][r]
    double s = hpT[0] * h[3 * a2] + hpT[d.ld] * h[3 * a2 + 1] + hpT[2 * d.ld] * h[3 * a2 + 2] +
               hpT[(int64_t)(3 + 2 * i2) * d.ld] * h[6 + 2 * a2] + hpT[(int64_t)(4 + 2 * i2) * d.ld] * h[7 + 2 * a2];
    if (r == rp) s += sigma;
    M[(int64_t)rp * d.ld + r] = s;
    return;
  }
  // rp == m: padding diagonal, y row and trailing identity
  if (r < d.m) M[(int64_t)d.yr * d.ld + r] = y[r];
  for (int64_t k = d.m + r; k < d.mp; k += (int64_t)gridDim.x * blockDim.x) M[k * d.ld + k] = 1.0;
  for (int64_t k = d.yr + r; k < d.ld; k += (int64_t)gridDim.x * blockDim.x) M[k * d.ld + k] = 1.0;
}

__device__ __forceinline__ double pu(const EkfDims& d, const double* __restrict__ M, int a, int b) {
  const int hi = max(a, b), lo = min(a, b);
  return M[(int64_t)(d.mp + hi) * d.ld + d.mp + lo];
}

// K y = -(y row of the trailing block); rays[matched] += (K y)[3:], ky3 = (K y)[0:3]
// (ptz_slam.py:262-277); pose covariance block (:281)
__global__ void k_ekf_apply_vec(EkfDims d, const int32_t* __restrict__ matched, const double* __restrict__ M,
                                const int* __restrict__ info, double* __restrict__ rays, double* __restrict__ cov,
                                double* __restrict__ ky3) {
  if (info[0] != 0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const double* yrow = M + (int64_t)d.yr * d.ld + d.mp;
  if (t < 3) ky3[t] = -yrow[t];
  if (t < 9) {
    const int q = t / 3, q2 = t % 3;
    cov[q * d.ns + q2] = pu(d, M, q, q2);
  }
  if (t < d.nr) {
    const int64_t r = matched[t];
    rays[2 * r] += -yrow[3 + 2 * t];
    rays[2 * r + 1] += -yrow[4 + 2 * t];
  }
}

// the reference's write-back (ptz_slam.py:282-289): only the (theta,theta) and (phi,phi) entries of
// every matched ray pair are copied back; pose-ray and theta-phi cross terms keep their old values
__global__ void k_ekf_apply_cov(EkfDims d, const int32_t* __restrict__ matched, const double* __restrict__ M,
                                const int* __restrict__ info, double* __restrict__ cov) {
  if (info[0] != 0) return;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (k >= d.nr) return;
  const int64_t r1 = 3 + 2 * (int64_t)matched[j], c1 = 3 + 2 * (int64_t)matched[k];
  cov[r1 * d.ns + c1] = pu(d, M, 3 + 2 * j, 3 + 2 * k);
  cov[(r1 + 1) * d.ns + c1 + 1] = pu(d, M, 4 + 2 * j, 4 + 2 * k);
}

// remove_rays: out[a][b] = old[keep[a]][keep[b]] (np.delete on both axes, ptz_slam.py:314-315)
__global__ void k_ekf_gather_cov(const double* __restrict__ old, int64_t ns_old, const int32_t* __restrict__ keep,
                                 int64_t ns_new, double* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int a = blockIdx.y;
  if (b >= ns_new) return;
  out[(int64_t)a * ns_new + b] = old[(int64_t)keep[a] * ns_old + keep[b]];
}

__global__ void k_ekf_gather_rays(const double* __restrict__ old, const int32_t* __restrict__ keep_ray, int n,
                                  double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[2 * i] = old[2 * (int64_t)keep_ray[i]];
  out[2 * i + 1] = old[2 * (int64_t)keep_ray[i] + 1];
}

// add_rays: new rows/columns are zero with angle_var on the diagonal (ptz_slam.py:380-383)
__global__ void k_ekf_grow_cov(const double* __restrict__ old, int64_t ns_old, int64_t ns_new, double var,
                               double* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int a = blockIdx.y;
  if (b >= ns_new) return;
  double x;
  if (a < ns_old && b < ns_old) x = old[(int64_t)a * ns_old + b];
  else x = (a == b) ? var : 0.0;
  out[(int64_t)a * ns_new + b] = x;
}

struct Q9 {
  double q[9];
};
__global__ void k_ekf_add_pose(double* __restrict__ cov, int64_t ns, Q9 q) {
  const int t = threadIdx.x;
  if (t < 9) cov[(t / 3) * ns + (t % 3)] += q.q[t];
}

}  // namespace ptzba

using namespace ptzba;

struct ptzekf_ctx {
  int device = 0;
  hipStream_t st = nullptr;
  int n_ray = 0;
  DBuf rays[2], cov[2];
  int cur = 0;
  DBuf pred_xy, vis, obs_xy, idx, Hc, yv, M, tasks, Ldiag, info, ky3, sgn;
  std::vector<uint8_t> vis_h;
  std::vector<int> task_off;
  std::vector<int4> tasks_host;
  int64_t plan_ld = -1;
  int plan_mp = -1, n_launch = 0;
  int64_t ns() const { return 3 + 2 * (int64_t)n_ray; }
};

static Disp make_disp(const double* d6, int& has) {
  Disp D{};
  has = d6 ? 1 : 0;
  if (d6)
    for (int k = 0; k < 6; ++k) D.d[k] = d6[k];
  return D;
}

// task list of the partial factorisation: tile columns 0..Tm-1 (panel + trailing, each updated by
// the previous column), then one flush launch applying panel Tm-1 to the trailing block (i >= j >= Tm)
static int build_partial_plan(ptzekf_ctx* h, int64_t ld, int mp) {
  if (h->plan_ld == ld && h->plan_mp == mp) return 0;
  const int T = (int)(ld / CHOL_NB), Tm = mp / CHOL_NB;
  std::vector<int4> tasks;
  h->task_off.assign(Tm + 2, 0);
  for (int k = 0; k <= Tm; ++k) {
    h->task_off[k] = (int)tasks.size();
    const int w = chol_pack_updates(k - 1, -1, 1);  // k == 0: no update panel
    if (k < Tm)
      for (int i = k; i < T; ++i) tasks.push_back(make_int4(0, i, k, w));
    if (k >= 1)
      for (int j = (k < Tm ? k + 1 : Tm); j < T; ++j)
        for (int i = j; i < T; ++i) tasks.push_back(make_int4(1, i, j, w));
  }
  h->task_off[Tm + 1] = (int)tasks.size();
  h->n_launch = Tm + 1;
  if (h->tasks.reserve(tasks.size() * sizeof(int4) + 16)) return -1;
  HIPCHK(hipMemcpyAsync(h->tasks.p, tasks.data(), tasks.size() * sizeof(int4), hipMemcpyHostToDevice, h->st));
  HIPCHK(hipStreamSynchronize(h->st));  // ordered before the factorisation launches on h->st
  h->tasks_host = tasks;
  h->plan_ld = ld;
  h->plan_mp = mp;
  return 0;
}

ptzekf_handle ptzekf_new(int device) {
  if (select_device(device)) return nullptr;
  auto* h = new ptzekf_ctx();
  h->device = device;
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    fail("hipStreamCreate failed");
    return nullptr;
  }
  if (h->info.alloc(16) || h->ky3.alloc(64)) {
    (void)hipStreamDestroy(h->st);
    delete h;
    return nullptr;
  }
  return h;
}

void ptzekf_delete(ptzekf_handle h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->st);
  (void)hipStreamDestroy(h->st);
  delete h;
}

int ptzekf_num_rays(ptzekf_handle h) { return h ? h->n_ray : fail("null handle"); }

int ptzekf_set_state(ptzekf_handle h, int32_t n_ray, const double* rays, const double* cov) {
  if (!h) return fail("null handle");
  if (n_ray < 0) return fail("n_ray < 0");
  if ((n_ray > 0 && !rays) || !cov) return fail("rays/cov must not be NULL");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  const int64_t ns = 3 + 2 * (int64_t)n_ray;
  h->cur = 0;
  if (h->rays[0].reserve((size_t)n_ray * 16 + 16) || h->cov[0].reserve((size_t)(ns * ns) * 8)) return -1;
  if (n_ray) HIPCHK(hipMemcpyAsync(h->rays[0].p, rays, (size_t)n_ray * 16, hipMemcpyHostToDevice, h->st));
  HIPCHK(hipMemcpyAsync(h->cov[0].p, cov, (size_t)(ns * ns) * 8, hipMemcpyHostToDevice, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  h->n_ray = n_ray;
  return 0;
}

int ptzekf_get_state(ptzekf_handle h, double* rays, double* cov) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  const int64_t ns = h->ns();
  if (rays && h->n_ray) HIPCHK(hipMemcpy(rays, h->rays[h->cur].p, (size_t)h->n_ray * 16, hipMemcpyDeviceToHost));
  if (cov) HIPCHK(hipMemcpy(cov, h->cov[h->cur].p, (size_t)(ns * ns) * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ptzekf_add_pose_cov(ptzekf_handle h, const double* q9) {
  if (!h || !q9) return fail("null argument");
  if (!h->cov[h->cur].p) return fail("no state: call ptzekf_set_state first");
  HIPCHK(hipSetDevice(h->device));
  Q9 q;
  for (int k = 0; k < 9; ++k) q.q[k] = q9[k];
  hipLaunchKernelGGL(k_ekf_add_pose, dim3(1), dim3(64), 0, h->st, h->cov[h->cur].as<double>(), h->ns(), q);
  HIPCHK(hipGetLastError());
  return 0;
}

int ptzekf_remove_rays(ptzekf_handle h, int64_t n, const int64_t* index) {
  if (!h) return fail("null handle");
  if (n < 0 || (n > 0 && !index)) return fail("bad index list");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->device));
  const int R = h->n_ray;
  std::vector<uint8_t> drop(R, 0);
  for (int64_t k = 0; k < n; ++k) {
    int64_t i = index[k];
    if (i < 0) i += R;  // numpy negative indexing (np.delete)
    if (i < 0 || i >= R) return fail("ray index %lld out of range (%d rays)", (long long)index[k], R);
    drop[i] = 1;
  }
  std::vector<int32_t> keep_ray, keep_state = {0, 1, 2};
  for (int i = 0; i < R; ++i)
    if (!drop[i]) {
      keep_ray.push_back(i);
      keep_state.push_back(3 + 2 * i);
      keep_state.push_back(4 + 2 * i);
    }
  const int Rn = (int)keep_ray.size();
  const int64_t ns_old = h->ns(), ns_new = 3 + 2 * (int64_t)Rn;
  const int nx = 1 - h->cur;
  if (h->rays[nx].reserve((size_t)Rn * 16 + 16) || h->cov[nx].reserve((size_t)(ns_new * ns_new) * 8) ||
      h->idx.reserve((keep_ray.size() + keep_state.size()) * 4))
    return -1;
  int32_t* dk = h->idx.as<int32_t>();
  HIPCHK(hipMemcpyAsync(dk, keep_state.data(), keep_state.size() * 4, hipMemcpyHostToDevice, h->st));
  HIPCHK(hipMemcpyAsync(dk + keep_state.size(), keep_ray.data(), keep_ray.size() * 4, hipMemcpyHostToDevice, h->st));
  hipLaunchKernelGGL(k_ekf_gather_cov, dim3(nblk(ns_new), (unsigned)ns_new), dim3(256), 0, h->st,
                     h->cov[h->cur].as<double>(), ns_old, dk, ns_new, h->cov[nx].as<double>());
  if (Rn)
    hipLaunchKernelGGL(k_ekf_gather_rays, dim3(nblk(Rn)), dim3(256), 0, h->st, h->rays[h->cur].as<double>(),
                       dk + keep_state.size(), Rn, h->rays[nx].as<double>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->st));  // host index vectors go out of scope
  h->cur = nx;
  h->n_ray = Rn;
  return 0;
}

int ptzekf_add_rays(ptzekf_handle h, int64_t n, const double* rays, double var) {
  if (!h) return fail("null handle");
  if (n < 0 || (n > 0 && !rays)) return fail("bad ray list");
  if (n == 0) return 0;
  if (!h->cov[h->cur].p) return fail("no state: call ptzekf_set_state first");
  HIPCHK(hipSetDevice(h->device));
  const int R = h->n_ray, Rn = R + (int)n;
  const int64_t ns_old = h->ns(), ns_new = 3 + 2 * (int64_t)Rn;
  const int nx = 1 - h->cur;
  if (h->rays[nx].reserve((size_t)Rn * 16 + 16) || h->cov[nx].reserve((size_t)(ns_new * ns_new) * 8)) return -1;
  if (R) HIPCHK(hipMemcpyAsync(h->rays[nx].p, h->rays[h->cur].p, (size_t)R * 16, hipMemcpyDeviceToDevice, h->st));
  HIPCHK(hipMemcpyAsync(h->rays[nx].as<double>() + 2 * (int64_t)R, rays, (size_t)n * 16, hipMemcpyHostToDevice, h->st));
  hipLaunchKernelGGL(k_ekf_grow_cov, dim3(nblk(ns_new), (unsigned)ns_new), dim3(256), 0, h->st,
                     h->cov[h->cur].as<double>(), ns_old, ns_new, var, h->cov[nx].as<double>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->st));
  h->cur = nx;
  h->n_ray = Rn;
  return 0;
}

int ptzekf_project_visible(ptzekf_handle h, double u, double v, const double* disp6, const double* ptz,
                           int32_t height, int32_t width, double* xy_out, double* index_out, int32_t* count_out) {
  if (!h || !ptz || !count_out) return fail("null argument");
  HIPCHK(hipSetDevice(h->device));
  const int R = h->n_ray;
  *count_out = 0;
  if (R == 0) return 0;
  if (h->pred_xy.reserve((size_t)R * 16) || h->vis.reserve((size_t)R)) return -1;
  int has;
  Disp D = make_disp(disp6, has);
  hipLaunchKernelGGL(k_ekf_project, dim3(nblk(R)), dim3(256), 0, h->st, R, u, v, ptz[2], ptz[0], ptz[1], D, has,
                     h->rays[h->cur].as<double>(), h->pred_xy.as<double>(), h->vis.as<uint8_t>(), height, width);
  HIPCHK(hipGetLastError());
  std::vector<double> xy((size_t)R * 2);
  h->vis_h.resize(R);
  HIPCHK(hipMemcpyAsync(xy.data(), h->pred_xy.p, (size_t)R * 16, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipMemcpyAsync(h->vis_h.data(), h->vis.p, (size_t)R, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  int c = 0;
  for (int i = 0; i < R; ++i)
    if (h->vis_h[i]) {
      if (xy_out) { xy_out[2 * c] = xy[2 * i]; xy_out[2 * c + 1] = xy[2 * i + 1]; }
      if (index_out) index_out[c] = (double)i;
      ++c;
    }
  *count_out = c;
  return 0;
}

int ptzekf_update(ptzekf_handle h, double u, double v, const double* disp6, double* ptz_inout, int64_t n_obs,
                  const double* obs_xy, const int64_t* obs_index, int32_t height, int32_t width, double observe_var,
                  double* velocity_out, int32_t* n_matched_out) {
  if (!h || !ptz_inout) return fail("null argument");
  if (n_obs < 0 || (n_obs > 0 && (!obs_xy || !obs_index))) return fail("bad observation list");
  if (!h->cov[h->cur].p) return fail("no state: call ptzekf_set_state first");
  HIPCHK(hipSetDevice(h->device));
  const int R = h->n_ray;
  const double pan = ptz_inout[0], tilt = ptz_inout[1], f = ptz_inout[2];
  int has;
  Disp D = make_disp(disp6, has);
  // 1. predicted keypoints of every ray, in-image flags (ptz_slam.py:222-224)
  std::vector<int32_t> o1, matched;
  if (R > 0) {
    if (h->pred_xy.reserve((size_t)R * 16) || h->vis.reserve((size_t)R)) return -1;
    hipLaunchKernelGGL(k_ekf_project, dim3(nblk(R)), dim3(256), 0, h->st, R, u, v, f, pan, tilt, D, has,
                       h->rays[h->cur].as<double>(), h->pred_xy.as<double>(), h->vis.as<uint8_t>(), height, width);
    HIPCHK(hipGetLastError());
    h->vis_h.resize(R);
    HIPCHK(hipMemcpyAsync(h->vis_h.data(), h->vis.p, (size_t)R, hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    // 2. get_overlap_index (util.py:75-97): the reference's two-pointer walk over the observed index
    //    list and the (ascending) predicted index list
    std::vector<int32_t> pred;
    pred.reserve(R);
    for (int i = 0; i < R; ++i)
      if (h->vis_h[i]) pred.push_back(i);
    size_t p1 = 0, p2 = 0;
    while (p1 < (size_t)n_obs && p2 < pred.size()) {
      if (obs_index[p1] == pred[p2]) {
        o1.push_back((int32_t)p1);
        matched.push_back(pred[p2]);
        ++p1;
        ++p2;
      } else if (obs_index[p1] < pred[p2]) {
        ++p1;
      } else {
        ++p2;
      }
    }
  }
  const int nr = (int)matched.size();
  if (n_matched_out) *n_matched_out = nr;
  if (nr == 0) {
    // S is 0x0: K y = 0, (I - K H) P = P (ptz_slam.py:256-289 with empty y)
    if (velocity_out) velocity_out[0] = velocity_out[1] = velocity_out[2] = 0.0;
    return 0;
  }
  EkfDims d;
  d.nr = nr;
  d.m = 2 * nr;
  d.mp = (d.m + CHOL_NB - 1) / CHOL_NB * CHOL_NB;
  d.n = 3 + 2 * nr;
  d.yr = d.mp + d.n;
  d.ld = ((int64_t)d.yr + 1 + CHOL_NB - 1) / CHOL_NB * CHOL_NB;
  d.ns = h->ns();
  const int Tm = d.mp / CHOL_NB;
  if (build_partial_plan(h, d.ld, d.mp)) return -1;
  if (h->idx.reserve((size_t)nr * 8) || h->obs_xy.reserve((size_t)n_obs * 16) || h->Hc.reserve((size_t)nr * 80) ||
      h->yv.reserve((size_t)nr * 16) || h->M.reserve((size_t)(d.ld * d.ld) * 8) ||
      h->Ldiag.reserve((size_t)Tm * CHOL_NB * CHOL_NB * 8) || h->sgn.reserve((size_t)d.ld * 8))
    return -1;
  int32_t* d_matched = h->idx.as<int32_t>();
  int32_t* d_o1 = d_matched + nr;
  HIPCHK(hipMemcpyAsync(d_matched, matched.data(), (size_t)nr * 4, hipMemcpyHostToDevice, h->st));
  HIPCHK(hipMemcpyAsync(d_o1, o1.data(), (size_t)nr * 4, hipMemcpyHostToDevice, h->st));
  HIPCHK(hipMemcpyAsync(h->obs_xy.p, obs_xy, (size_t)n_obs * 16, hipMemcpyHostToDevice, h->st));
  double* M = h->M.as<double>();
  double* cov = h->cov[h->cur].as<double>();
  HIPCHK(hipMemsetAsync(M, 0, (size_t)(d.ld * d.ld) * 8, h->st));
  HIPCHK(hipMemsetAsync(h->info.p, 0, 16, h->st));
  // 3. H blocks and innovation, then the augmented matrix
  hipLaunchKernelGGL(k_ekf_hblocks, dim3(nblk(nr)), dim3(256), 0, h->st, nr, d_matched, d_o1,
                     h->obs_xy.as<double>(), h->pred_xy.as<double>(), h->rays[h->cur].as<double>(), u, v, f, pan, tilt,
                     D, has, h->Hc.as<double>(), h->yv.as<double>());
  hipLaunchKernelGGL(k_ekf_assemble_hp, dim3(nblk(d.n), (unsigned)(nr + d.n)), dim3(256), 0, h->st, d, d_matched,
                     cov, h->Hc.as<double>(), M);
  hipLaunchKernelGGL(k_ekf_assemble_s, dim3(nblk(d.m), (unsigned)(d.m + 1)), dim3(256), 0, h->st, d,
                     h->Hc.as<double>(), h->yv.as<double>(), observe_var, M);
  HIPCHK(hipGetLastError());
  // 4. partial factorisation through the S columns (+ flush of the trailing update).  Signed form
  //    S = L Sigma L^T: the reference inverts S with np.linalg.inv (ptz_slam.py:258), and its covariance
  //    write-back (ptz_slam.py:282-289) leaves P indefinite after some frames, so S can have negative
  //    eigenvalues; for an SPD S the signed factor is the Cholesky factor, bit for bit.
  launch_cholesky(M, d.ld, h->tasks.as<int4>(), h->task_off.data(), h->n_launch, h->Ldiag.as<double>(),
                  h->info.as<int>(), h->st, h->sgn.as<double>(), h->tasks_host.data());
  HIPCHK(hipGetLastError());
  // 5. state update and covariance write-back (skipped on the device when S was not SPD)
  hipLaunchKernelGGL(k_ekf_apply_vec, dim3(nblk(std::max(nr, 9))), dim3(256), 0, h->st, d, d_matched, M,
                     h->info.as<int>(), h->rays[h->cur].as<double>(), cov, h->ky3.as<double>());
  hipLaunchKernelGGL(k_ekf_apply_cov, dim3(nblk(nr), (unsigned)nr), dim3(256), 0, h->st, d, d_matched, M,
                     h->info.as<int>(), cov);
  HIPCHK(hipGetLastError());
  double ky[3];
  int info = 0;
  HIPCHK(hipMemcpyAsync(ky, h->ky3.p, 24, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipMemcpyAsync(&info, h->info.p, 4, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  if (info != 0) return fail("innovation covariance H P H^T + R is singular (zero pivot, flag %d)", info);
  ptz_inout[0] = pan + ky[0];
  ptz_inout[1] = tilt + ky[1];
  ptz_inout[2] = f + ky[2];
  if (velocity_out)
    for (int k = 0; k < 3; ++k) velocity_out[k] = ky[k];
  return 0;
}
