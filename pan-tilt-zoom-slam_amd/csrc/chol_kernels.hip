// Dense fp64 Cholesky solve of the reduced camera system (gfx950).
//
// The reduced camera system S (3(N-1) x 3(N-1), SPD, block-banded: keyframes couple only to pan
// neighbours) replaces scipy's dense SVD of the full Jacobian (trf.py:467 via bundle_adjustment.py:200).
//
// Storage: row-major [ld][ld] lower triangle, ld = roundup(n + 1, 32).  Row n holds b^T (augmented
// right-hand side) with a huge diagonal, so row n of the factor is y = L^-1 b: the forward
// substitution comes out of the factorisation for free.  Rows > n are identity padding.
//
// Factorisation: 32x32 tiles, ONE launch per tile column k ("delayed update"):
//   panel task (i, k):  T_ik <- A_ik - L_{i,k-1} L_{k,k-1}^T,  D <- A_kk - L_{k,k-1} L_{k,k-1}^T,
//                       factor D in one wave (rows in registers, pivot column broadcast via LDS),
//                       L_ik = T_ik L_kk^-T (lane per row, forward substitution)   [i == k: write L_kk]
//   trailing task (i, j), i >= j > k:  A_ij <- A_ij - L_{i,k-1} L_{j,k-1}^T
// Panel k-1's update reaches every tile exactly once (column k through the panel tasks, columns > k
// through the trailing tasks of the same launch), so one launch per column suffices.  Only tiles
// inside the profile (envelope) of S are visited; the envelope of L equals that of S.
// Back substitution L^T x = y: one 1024-thread workgroup, 32-column steps, envelope-limited.
#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

constexpr int NB = CHOL_NB;
constexpr double AUG_DIAG = 1e300;

__device__ __forceinline__ double bcast(double v, int j) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}

// augmented row / padding: A[n][j] = b[j], A[n][n] = huge, A[i][i] = 1 for i > n
__global__ void k_chol_prepare(double* __restrict__ A, int64_t ld, int n, const double* __restrict__ b, int* info) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) info[0] = 0;
  if (i < n) A[(int64_t)n * ld + i] = b[i];
  if (i == n) A[i * ld + i] = AUG_DIAG;
  if (i > n && i < ld) A[i * ld + i] = 1.0;
}

void launch_chol_prepare(double* A, int64_t ld, int n, double* b, int* info, hipStream_t st) {
  hipLaunchKernelGGL(k_chol_prepare, dim3((unsigned)((ld + 255) / 256)), dim3(256), 0, st, A, ld, n, b, info);
}

// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void load_tile(double (*dst)[NB + 1], const double* __restrict__ src, int64_t ld) {
  for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) dst[e >> 5][e & 31] = src[(int64_t)(e >> 5) * ld + (e & 31)];
}

// C -= A B^T for 32x32 tiles in LDS (256 threads: 32 rows x 8 groups of 4 columns)
__device__ __forceinline__ void tile_gemm_nt_sub(double (*C)[NB + 1], double (*A)[NB + 1], double (*B)[NB + 1]) {
  const int rr = threadIdx.x >> 3;
  const int cc = (threadIdx.x & 7) * 4;
  double acc[4] = {0, 0, 0, 0};
#pragma unroll 8
  for (int m = 0; m < NB; ++m) {
    const double x = A[rr][m];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += x * B[cc + q][m];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) C[rr][cc + q] -= acc[q];
}

// One wave factors the 32x32 SPD tile D (LDS) in place into its lower Cholesky factor; rdg[j] = 1/L_jj.
// Lane i keeps row i in registers; the pivot column is broadcast with v_readlane (no LDS round trips,
// no spills): right-looking on the unscaled pivot column, row_i[m] -= (A_ij / A_jj) A_mj, and at the
// end L_ij = A_ij / sqrt(A_jj).
__device__ __forceinline__ void wave_potrf32(double (*D)[NB + 1], double* rdg, int* info) {
  const int lane = lane_id();
  const int i = lane & (NB - 1);
  double row[NB], dg[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = D[i][m];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double d = bcast(row[j], j);
    if (!(d > 0.0)) {
      bad = true;
      d = 1e-300;
    }
    const double li = row[j] * (1.0 / d);
#pragma unroll
    for (int m = j + 1; m < NB; ++m) row[m] -= li * bcast(row[j], m);
    dg[j] = d;
  }
  if (bad && lane == 0) atomicOr(info, 1);
  if (lane < NB) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const double r = 1.0 / sqrt(dg[j]);
      D[i][j] = (j <= i) ? row[j] * r : 0.0;
      if (lane == j) rdg[j] = r;
    }
  }
  wave_lds_fence();
}

__global__ __launch_bounds__(256) void k_chol_step(double* __restrict__ A, int64_t ld, int k,
                                                   const int* __restrict__ tasks, const int* __restrict__ colfirst,
                                                   double* __restrict__ Ldiag, int* info) {
  __shared__ double sC[NB][NB + 1];  // target tile (panel T_ik / trailing A_ij)
  __shared__ double sD[NB][NB + 1];  // diagonal tile -> L_kk
  __shared__ double sA[NB][NB + 1];  // L_{i,k-1}
  __shared__ double sB[NB][NB + 1];  // L_{k,k-1} or L_{j,k-1}
  __shared__ double rdg[NB];
  const int task = tasks[blockIdx.x];
  const int type = task >> 30;
  const int i = (task >> 15) & 0x7fff;
  const int j = task & 0x7fff;
  const int64_t NBl = NB;
#ifndef CHOL_VARIANT
#define CHOL_VARIANT 0
#endif
  if (type == 1) {
#if CHOL_VARIANT == 3
    return;
#endif
    // trailing: A_ij -= L_{i,k-1} L_{j,k-1}^T
    double* C = A + i * NBl * ld + j * NBl;
    load_tile(sC, C, ld);
    load_tile(sA, A + i * NBl * ld + (k - 1) * NBl, ld);
    load_tile(sB, A + j * NBl * ld + (k - 1) * NBl, ld);
    __syncthreads();
    tile_gemm_nt_sub(sC, sA, sB);
    __syncthreads();
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) C[(int64_t)(e >> 5) * ld + (e & 31)] = sC[e >> 5][e & 31];
    return;
  }
  // panel task (i, k)
  const bool diag_only = (i == k);
  const bool upd_k = (k > 0) && colfirst[k] <= k - 1;
  const bool upd_i = (k > 0) && colfirst[i] <= k - 1;
  load_tile(sD, A + (int64_t)k * NBl * ld + k * NBl, ld);
  if (!diag_only) load_tile(sC, A + i * NBl * ld + k * NBl, ld);
  if (upd_k) load_tile(sB, A + (int64_t)k * NBl * ld + (k - 1) * NBl, ld);
  if (upd_i && !diag_only) load_tile(sA, A + i * NBl * ld + (k - 1) * NBl, ld);
  __syncthreads();
  if (upd_k) tile_gemm_nt_sub(sD, sB, sB);
  if (upd_k && upd_i && !diag_only) tile_gemm_nt_sub(sC, sA, sB);
  __syncthreads();
#if CHOL_VARIANT != 1
  if (threadIdx.x < WAVE) wave_potrf32(sD, rdg, info);
#else
  if (threadIdx.x < NB) rdg[threadIdx.x] = 1.0;
#endif
  __syncthreads();
  if (diag_only) {
    // A_kk itself stays untouched: other panel workgroups of this launch are still reading it
    double* C = Ldiag + (int64_t)k * NB * NB;
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) C[e] = sD[e >> 5][e & 31];
    return;
  }
  // L_ik = T_ik L_kk^-T : lane r solves row r
  if (threadIdx.x < NB && CHOL_VARIANT != 2) {
    const int r = threadIdx.x;
    double x[NB];
#pragma unroll
    for (int m = 0; m < NB; ++m) x[m] = sC[r][m];
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      x[jj] *= rdg[jj];
#pragma unroll
      for (int m = jj + 1; m < NB; ++m) x[m] -= x[jj] * sD[m][jj];
      __builtin_amdgcn_sched_barrier(0);  // keep each step's LDS reads in the step (no hoisting -> no spills)
    }
#pragma unroll
    for (int m = 0; m < NB; ++m) sC[r][m] = x[m];
  }
  __syncthreads();
  double* C = A + i * NBl * ld + k * NBl;
  for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) C[(int64_t)(e >> 5) * ld + (e & 31)] = sC[e >> 5][e & 31];
}

void launch_cholesky(double* A, int64_t ld, const int* tasks, const int* task_off_host, const int* colfirst,
                     double* Ldiag, int* info, hipStream_t st) {
  const int T = (int)(ld / NB);
  for (int k = 0; k < T; ++k) {
    const int n = task_off_host[k + 1] - task_off_host[k];
    if (n > 0)
      hipLaunchKernelGGL(k_chol_step, dim3(n), dim3(256), 0, st, A, ld, k, tasks + task_off_host[k], colfirst, Ldiag,
                         info);
  }
}

// ---------------------------------------------------------------------------------------------
// back substitution L^T x = y with y = row n of the factor; x written to xout[0..n)
__global__ __launch_bounds__(1024) void k_chol_backsolve(const double* __restrict__ L, int64_t ld, int n,
                                                         const int* __restrict__ rowend,
                                                         const double* __restrict__ Ldiag, double* __restrict__ xout) {
  extern __shared__ __attribute__((aligned(16))) double xv[];  // [ld]
  __shared__ double part[32][NB + 1];
  __shared__ double Lkk[NB][NB + 1];
  const int t = threadIdx.x;
  const int c = t & 31, sub = t >> 5;
  const int Tn = (n + NB - 1) / NB;
  // y = row n of the factor: off-diagonal tiles in place, the last partial tile in Ldiag
  const int tn = n / NB, rn = n - tn * NB;
  for (int i = t; i < ld; i += blockDim.x)
    xv[i] = (i >= n) ? 0.0 : (i < tn * NB ? L[(int64_t)n * ld + i] : Ldiag[((int64_t)tn * NB + rn) * NB + (i - tn * NB)]);
  __syncthreads();
  for (int kt = Tn - 1; kt >= 0; --kt) {
    const int64_t c0 = (int64_t)kt * NB;
    // stage L_kk and the envelope-limited column-block dot products
    Lkk[t >> 5][t & 31] = Ldiag[(int64_t)kt * NB * NB + t];
    double s = 0;
    const int r1 = min(rowend[kt], n);
#pragma unroll 4
    for (int i = (int)c0 + NB + sub; i < r1; i += 32) s += L[(int64_t)i * ld + c0 + c] * xv[i];
    part[sub][c] = s;
    __syncthreads();
    if (t < WAVE) {
      const int lane = t;
      double tr = 0;
      if (lane < NB) {
        for (int q = 0; q < 32; ++q) tr += part[q][lane];
        tr = xv[c0 + lane] - tr;
      }
      // upper-triangular solve L_kk^T x = tr, lane r holds tr_r
      const double rd = lane < NB ? 1.0 / Lkk[lane][lane] : 0.0;
#pragma unroll
      for (int jj = NB - 1; jj >= 0; --jj) {
        const double tj = bcast(tr, jj) * bcast(rd, jj);
        if (lane == jj) tr = tj;
        if (lane < jj) tr -= Lkk[jj][lane] * tj;
      }
      if (lane < NB && c0 + lane < n) xv[c0 + lane] = tr;
    }
    __syncthreads();
  }
  for (int i = t; i < n; i += blockDim.x) xout[i] = xv[i];
}

void launch_chol_backsolve(const double* L, int64_t ld, int n, const int* rowend, const double* Ldiag, double* xout,
                           hipStream_t st) {
  hipLaunchKernelGGL(k_chol_backsolve, dim3(1), dim3(1024), (size_t)ld * sizeof(double), st, L, ld, n, rowend, Ldiag,
                     xout);
}

}  // namespace ptzba
