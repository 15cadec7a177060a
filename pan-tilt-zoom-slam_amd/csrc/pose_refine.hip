// Pose-only refinement with the rays fixed (gfx950, fp64).
//
// relocalization.py:186 refines a lost camera's (pan, tilt, f) with
//   least_squares(_compute_residual, pose, x_scale='jac', ftol=1e-4, method='trf', args=(rays, points, u, v))
// over the from_ray_to_image residual (relocalization.py:22-40).  Here one 256-thread workgroup per
// hypothesis runs the whole Levenberg-Marquardt loop on the device: residual + 2x3 analytic pose
// Jacobian per correspondence (the BA projection of ptzba_common.h, |q2| in y), block reduction of
// J^T W J (6) / J^T W r (3) / cost, a 3x3 damped solve, trial evaluation, gain-ratio acceptance and
// scipy-style termination — with the same Marquardt scaling and lambda rule as ptzba.LMSolver.
// Hypotheses share the correspondence set or take CSR subsets of it (preemptive-RANSAC style batches,
// SURVEY §8f-3).
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/ptzba.h"
#include "host_util.h"
#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

constexpr int RF_THREADS = 256;

struct RefineArgs {
  int n_hyp;
  double* ptz;             // [n_hyp][3] in/out
  const int64_t* sub_off;  // [n_hyp+1] or nullptr
  const int32_t* sub_idx;
  int64_t n_corr;
  const double* rays;  // [n_corr][2]
  const double* pts;   // [n_corr][2]
  double u, v;
  int max_iter, loss;
  double ftol, xtol, fs2, inv_fs2;
  double* cost_out;
  int* iters_out;
  int* status_out;
};

// sum over the workgroup of nv values (wave reduce, then LDS)
template <int NV>
__device__ __forceinline__ void block_sum(double (&x)[NV], double (*red)[NV]) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) x[k] = wave_sum(x[k]);
  if (lane_id() == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) red[w][k] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0;
    for (int q = 0; q < RF_THREADS / WAVE; ++q) s += red[q][k];
    x[k] = s;
  }
  __syncthreads();
}

// cost (0.5 sum rho) and, with JAC, J^T W J (upper 6) and J^T W r (3) at pose p
template <bool JAC>
__device__ void rf_eval(const RefineArgs& a, int h, const double p[3], double (&out)[10], double (*red)[10]) {
  const FrameTab<double> F = make_frame_tab<double>(p[0], p[1], p[2]);
  double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t b0 = a.sub_off ? a.sub_off[h] : 0, b1 = a.sub_off ? a.sub_off[h + 1] : a.n_corr;
  for (int64_t k = b0 + threadIdx.x; k < b1; k += RF_THREADS) {
    const int64_t c = a.sub_off ? (int64_t)a.sub_idx[k] : k;
    const RayTab<double> R = make_ray_tab<double>(a.rays[2 * c], a.rays[2 * c + 1]);
    double x, y, J[2][5];
    if (JAC) ptz_project_jac<double>(F, R, a.u, a.v, x, y, J);
    else ptz_project<double>(F, R, a.u, a.v, x, y);
    const double rx = x - a.pts[2 * c], ry = y - a.pts[2 * c + 1];
    double wx = 1, wy = 1, c2;
    if (a.loss == PTZBA_LOSS_LINEAR) {
      c2 = rx * rx + ry * ry;
    } else {  // scipy 'huber' as in K1: rho(z) = z | 2 sqrt(z) - 1, IRLS weight rho'(z)
      const double zx = rx * rx * a.inv_fs2, zy = ry * ry * a.inv_fs2;
      const double sx = sqrt(zx), sy = sqrt(zy);
      const bool ix = zx <= 1.0, iy = zy <= 1.0;
      wx = ix ? 1.0 : 1.0 / sx;
      wy = iy ? 1.0 : 1.0 / sy;
      c2 = a.fs2 * ((ix ? zx : 2 * sx - 1) + (iy ? zy : 2 * sy - 1));
    }
    acc[9] += c2;
    if (JAC) {
      int t = 0;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i; j < 3; ++j) acc[t++] += wx * J[0][i] * J[0][j] + wy * J[1][i] * J[1][j];
#pragma unroll
      for (int i = 0; i < 3; ++i) acc[6 + i] += wx * J[0][i] * rx + wy * J[1][i] * ry;
    }
  }
  block_sum<10>(acc, red);
#pragma unroll
  for (int k = 0; k < 10; ++k) out[k] = acc[k];
  out[9] *= 0.5;
}

__global__ __launch_bounds__(RF_THREADS) void k_refine_poses(RefineArgs a) {
  __shared__ double red[RF_THREADS / WAVE][10];
  __shared__ double sh_trial[3];
  __shared__ int sh_ctl[2];  // [0]: 1 = stop, [1]: 1 = accepted
  const int h = blockIdx.x;
  double p[3] = {a.ptz[3 * h], a.ptz[3 * h + 1], a.ptz[3 * h + 2]};
  double lin[10];
  rf_eval<true>(a, h, p, lin, red);
  double cost = lin[9];
  double lam = 1e-4, nu = 2.0, D[3] = {0, 0, 0};
  int it = 0, status = 0;
  for (; it < a.max_iter;) {
    // damped 3x3 solve (H + lam diag(D)) d = -g with Marquardt scaling D = max over history of diag(H)
    double d[3] = {0, 0, 0}, pred = 0;
    bool ok = true;
    if (threadIdx.x == 0) {
      const double Hd[3] = {lin[0], lin[3], lin[5]};
      for (int i = 0; i < 3; ++i) D[i] = fmax(D[i], fmax(Hd[i], 1e-12));
      double A[3][3] = {{lin[0] + lam * D[0], lin[1], lin[2]},
                        {lin[1], lin[3] + lam * D[1], lin[4]},
                        {lin[2], lin[4], lin[5] + lam * D[2]}};
      double g[3] = {lin[6], lin[7], lin[8]};
      // Cholesky
      double L00 = A[0][0];
      ok = L00 > 0;
      L00 = sqrt(fmax(L00, 1e-300));
      const double L10 = A[1][0] / L00, L20 = A[2][0] / L00;
      double L11 = A[1][1] - L10 * L10;
      ok = ok && L11 > 0;
      L11 = sqrt(fmax(L11, 1e-300));
      const double L21 = (A[2][1] - L20 * L10) / L11;
      double L22 = A[2][2] - L20 * L20 - L21 * L21;
      ok = ok && L22 > 0;
      L22 = sqrt(fmax(L22, 1e-300));
      const double y0 = -g[0] / L00, y1 = (-g[1] - L10 * y0) / L11, y2 = (-g[2] - L20 * y0 - L21 * y1) / L22;
      d[2] = y2 / L22;
      d[1] = (y1 - L21 * d[2]) / L11;
      d[0] = (y0 - L10 * d[1] - L20 * d[2]) / L00;
      for (int i = 0; i < 3; ++i) pred += -0.5 * g[i] * d[i] + 0.5 * lam * D[i] * d[i] * d[i];
      for (int i = 0; i < 3; ++i) sh_trial[i] = p[i] + d[i];
    }
    __syncthreads();
    const double t[3] = {sh_trial[0], sh_trial[1], sh_trial[2]};
    double tr[10];
    rf_eval<false>(a, h, t, tr, red);
    if (threadIdx.x == 0) {
      const double new_cost = tr[9];
      const double actual = cost - new_cost;
      const bool num_ok = ok && isfinite(new_cost) && pred > 0;
      const double rho = num_ok ? actual / pred : -1.0;
      int stop = 0, acc = 0;
      if (rho > 0) {
        acc = 1;
        lam = fmax(1e-12, lam * fmax(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) * (2.0 * rho - 1.0) * (2.0 * rho - 1.0)));
        nu = 2.0;
        const double dx2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double x2 = t[0] * t[0] + t[1] * t[1] + t[2] * t[2];
        if (actual < a.ftol * cost && rho > 0.25) { stop = 1; status = 2; }       // scipy ftol
        else if (sqrt(dx2) < a.xtol * (a.xtol + sqrt(x2))) { stop = 1; status = 3; }  // scipy xtol
        cost = new_cost;
      } else {
        lam = lam > 0 ? lam * nu : 1e-9;
        nu *= 2.0;
        if (lam > 1e16) { stop = 1; status = -1; }
      }
      sh_ctl[0] = stop;
      sh_ctl[1] = acc;
    }
    __syncthreads();
    const int stop = sh_ctl[0], acc = sh_ctl[1];
    if (acc) {
      ++it;
      p[0] = t[0]; p[1] = t[1]; p[2] = t[2];
      if (!stop) rf_eval<true>(a, h, p, lin, red);
    }
    __syncthreads();
    if (stop) break;
  }
  if (threadIdx.x == 0) {
    a.ptz[3 * h] = p[0];
    a.ptz[3 * h + 1] = p[1];
    a.ptz[3 * h + 2] = p[2];
    if (a.cost_out) a.cost_out[h] = cost;
    if (a.iters_out) a.iters_out[h] = it;
    if (a.status_out) a.status_out[h] = status;
  }
}

}  // namespace ptzba

using namespace ptzba;

int ptz_refine_poses(int device, int32_t n_hyp, double* ptz_inout, int64_t n_corr, const double* rays,
                     const double* points, double u, double v, const int64_t* subset_offsets,
                     const int32_t* subset_index, const ptz_refine_opts* opts, double* cost_out, int32_t* iters_out,
                     int32_t* status_out) {
  if (n_hyp < 0 || n_corr < 0) return fail("bad sizes");
  if (n_hyp == 0) return 0;
  if (!ptz_inout || (n_corr > 0 && (!rays || !points))) return fail("null argument");
  ptz_refine_opts o{100, PTZBA_LOSS_LINEAR, 1e-4, 1e-8, 1.0};
  if (opts) o = *opts;
  if (o.max_iter < 0 || !(o.ftol >= 0) || !(o.xtol >= 0)) return fail("bad options");
  if (o.loss == PTZBA_LOSS_HUBER && !(o.f_scale > 0)) return fail("huber needs f_scale > 0");
  int64_t n_sub = 0;
  if (subset_offsets) {
    if (subset_offsets[0] != 0) return fail("subset_offsets[0] must be 0");
    for (int h = 0; h < n_hyp; ++h)
      if (subset_offsets[h + 1] < subset_offsets[h]) return fail("subset_offsets not ascending");
    n_sub = subset_offsets[n_hyp];
    for (int64_t k = 0; k < n_sub; ++k)
      if (subset_index[k] < 0 || subset_index[k] >= n_corr) return fail("subset index %lld out of range", (long long)k);
  }
  if (select_device(device)) return -1;
  DBuf dptz, drays, dpts, doff, didx, dcost, dit, dst;
  if (dptz.alloc((size_t)n_hyp * 24) || drays.alloc((size_t)n_corr * 16) || dpts.alloc((size_t)n_corr * 16) ||
      dcost.alloc((size_t)n_hyp * 8) || dit.alloc((size_t)n_hyp * 4) || dst.alloc((size_t)n_hyp * 4))
    return -1;
  HIPCHK(hipMemcpy(dptz.p, ptz_inout, (size_t)n_hyp * 24, hipMemcpyHostToDevice));
  if (n_corr) {
    HIPCHK(hipMemcpy(drays.p, rays, (size_t)n_corr * 16, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dpts.p, points, (size_t)n_corr * 16, hipMemcpyHostToDevice));
  }
  if (subset_offsets) {
    if (doff.alloc((size_t)(n_hyp + 1) * 8) || didx.alloc((size_t)n_sub * 4 + 4)) return -1;
    HIPCHK(hipMemcpy(doff.p, subset_offsets, (size_t)(n_hyp + 1) * 8, hipMemcpyHostToDevice));
    if (n_sub) HIPCHK(hipMemcpy(didx.p, subset_index, (size_t)n_sub * 4, hipMemcpyHostToDevice));
  }
  RefineArgs a;
  a.n_hyp = n_hyp;
  a.ptz = dptz.as<double>();
  a.sub_off = subset_offsets ? doff.as<int64_t>() : nullptr;
  a.sub_idx = subset_offsets ? didx.as<int32_t>() : nullptr;
  a.n_corr = n_corr;
  a.rays = drays.as<double>();
  a.pts = dpts.as<double>();
  a.u = u;
  a.v = v;
  a.max_iter = o.max_iter;
  a.loss = o.loss;
  a.ftol = o.ftol;
  a.xtol = o.xtol;
  a.fs2 = o.f_scale * o.f_scale;
  a.inv_fs2 = 1.0 / a.fs2;
  a.cost_out = dcost.as<double>();
  a.iters_out = dit.as<int>();
  a.status_out = dst.as<int>();
  hipLaunchKernelGGL(k_refine_poses, dim3(n_hyp), dim3(RF_THREADS), 0, nullptr, a);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(ptz_inout, dptz.p, (size_t)n_hyp * 24, hipMemcpyDeviceToHost));
  if (cost_out) HIPCHK(hipMemcpy(cost_out, dcost.p, (size_t)n_hyp * 8, hipMemcpyDeviceToHost));
  if (iters_out) HIPCHK(hipMemcpy(iters_out, dit.p, (size_t)n_hyp * 4, hipMemcpyDeviceToHost));
  if (status_out) HIPCHK(hipMemcpy(status_out, dst.p, (size_t)n_hyp * 4, hipMemcpyDeviceToHost));
  return 0;
}
