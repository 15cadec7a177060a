// Dense fp64 Cholesky + triangular solves for the reduced camera system (gfx950).
//
// The reduced camera system S (3(N-1) x 3(N-1), SPD) replaces scipy's dense SVD of the full
// Jacobian (trf.py:467 via bundle_adjustment.py:200).  Right-looking blocked factorisation with
// 32x32 tiles, in place, lower triangle, row-major:
//   k_chol_diag   one wave factors the diagonal tile in LDS (no block barriers)
//   k_chol_panel  one wave per 64 panel rows: row-wise forward substitution against L_kk
//                 (L_kk broadcast from LDS), records which 32-row tiles are non-zero
//   k_chol_update 32x32 tile SYRK/GEMM trailing update; tiles whose panel rows are zero are skipped
//                 (S is block-banded: keyframes only couple to pan neighbours)
// followed by one-workgroup forward and backward substitution.
#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

constexpr int NB = CHOL_NB;

__global__ void k_chol_prepare(double* __restrict__ A, int64_t ld, int n, double* __restrict__ b, int* info) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) info[0] = 0;
  if (i >= n && i < ld) {
    A[i * ld + i] = 1.0;
    b[i] = 0.0;
  }
}

void launch_chol_prepare(double* A, int64_t ld, int n, double* b, int* info, hipStream_t st) {
  hipLaunchKernelGGL(k_chol_prepare, dim3((unsigned)((ld + 255) / 256)), dim3(256), 0, st, A, ld, n, b, info);
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_chol_diag(double* __restrict__ A, int64_t ld, int k, int* info) {
  __shared__ double T[NB][NB + 1];
  const int lane = threadIdx.x;
  double* base = A + (int64_t)k * NB * ld + (int64_t)k * NB;
  for (int e = lane; e < NB * NB; e += WAVE) T[e / NB][e % NB] = base[(int64_t)(e / NB) * ld + (e % NB)];
  wave_lds_fence();
  const int i = lane & (NB - 1);
  const int h = lane >> 5;
  for (int j = 0; j < NB; ++j) {
    double d = T[j][j];
    if (!(d > 0.0)) {
      if (lane == 0) atomicOr(info, 1);
      d = 1e-300;
    }
    const double rs = 1.0 / sqrt(d);
    wave_lds_fence();
    if (h == 0 && i >= j) T[i][j] *= rs;
    wave_lds_fence();
    const double li = T[i][j];
    if (i > j)
      for (int m = j + 1 + h; m <= i; m += 2) T[i][m] -= li * T[m][j];
    wave_lds_fence();
  }
  for (int e = lane; e < NB * NB; e += WAVE) {
    const int r = e / NB, c = e % NB;
    if (c <= r) base[(int64_t)r * ld + c] = T[r][c];
  }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_chol_panel(double* __restrict__ A, int64_t ld, int k, int* tile_nz) {
  __shared__ double Lk[NB][NB + 1];
  __shared__ double idg[NB];
  const int lane = threadIdx.x;
  const double* dbase = A + (int64_t)k * NB * ld + (int64_t)k * NB;
  for (int e = lane; e < NB * NB; e += WAVE) {
    const int r = e / NB, c = e % NB;
    Lk[r][c] = c <= r ? dbase[(int64_t)r * ld + c] : 0.0;
  }
  wave_lds_fence();
  if (lane < NB) idg[lane] = 1.0 / Lk[lane][lane];
  wave_lds_fence();
  const int64_t row = (int64_t)(k + 1) * NB + (int64_t)blockIdx.x * WAVE + lane;
  const bool valid = row < ld;
  double x[NB];
  double* rp = A + row * ld + (int64_t)k * NB;
#pragma unroll
  for (int j = 0; j < NB; ++j) x[j] = valid ? rp[j] : 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    x[j] *= idg[j];
#pragma unroll
    for (int m = j + 1; m < NB; ++m) x[m] -= x[j] * Lk[m][j];
  }
  bool nz = false;
  if (valid) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      rp[j] = x[j];
      nz |= (x[j] != 0.0);
    }
  }
  const unsigned long long bal = __ballot(nz);
  const int tile0 = (int)(((int64_t)(k + 1) * NB + (int64_t)blockIdx.x * WAVE) / NB);
  const int ntiles = (int)(ld / NB);
  if (lane == 0 && tile0 < ntiles) tile_nz[tile0] = (bal & 0xffffffffull) != 0;
  if (lane == 32 && tile0 + 1 < ntiles) tile_nz[tile0 + 1] = (bal >> 32) != 0;
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chol_update(double* __restrict__ A, int64_t ld, int k,
                                                     const int* __restrict__ tile_nz) {
  const int i = k + 1 + blockIdx.x;
  const int j = k + 1 + blockIdx.y;
  if (j > i) return;
  if (!tile_nz[i] || !tile_nz[j]) return;
  __shared__ double Li[NB][NB + 1];
  __shared__ double Lj[NB][NB + 1];
  const double* pi = A + (int64_t)i * NB * ld + (int64_t)k * NB;
  const double* pj = A + (int64_t)j * NB * ld + (int64_t)k * NB;
  for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, c = e % NB;
    Li[r][c] = pi[(int64_t)r * ld + c];
    Lj[r][c] = pj[(int64_t)r * ld + c];
  }
  __syncthreads();
  const int rr = threadIdx.x >> 3;
  const int cc = (threadIdx.x & 7) * 4;
  double acc[4] = {0, 0, 0, 0};
#pragma unroll 8
  for (int m = 0; m < NB; ++m) {
    const double a = Li[rr][m];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += a * Lj[cc + q][m];
  }
  double* C = A + ((int64_t)i * NB + rr) * ld + (int64_t)j * NB + cc;
#pragma unroll
  for (int q = 0; q < 4; ++q) C[q] -= acc[q];
}

void launch_cholesky(double* A, int64_t ld, int* info, int* tile_nz, hipStream_t st) {
  const int T = (int)(ld / NB);
  for (int k = 0; k < T; ++k) {
    hipLaunchKernelGGL(k_chol_diag, dim3(1), dim3(64), 0, st, A, ld, k, info);
    if (k + 1 < T) {
      const int rows = (T - k - 1) * NB;
      hipLaunchKernelGGL(k_chol_panel, dim3((rows + WAVE - 1) / WAVE), dim3(64), 0, st, A, ld, k, tile_nz);
      hipLaunchKernelGGL(k_chol_update, dim3(T - k - 1, T - k - 1), dim3(256), 0, st, A, ld, k, tile_nz);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// one workgroup: forward L y = b, then backward L^T x = y (b overwritten); y lives in LDS
__global__ __launch_bounds__(1024) void k_chol_solve(const double* __restrict__ L, int64_t ld, double* __restrict__ b) {
  extern __shared__ __attribute__((aligned(16))) double yv[];
  const int t = threadIdx.x;
  const int T = (int)(ld / NB);
  for (int i = t; i < ld; i += blockDim.x) yv[i] = b[i];
  __syncthreads();
  const int r = t >> 5, sub = t & 31;  // 32 rows x 32 partial lanes
  // forward
  for (int kt = 0; kt < T; ++kt) {
    const int64_t row = (int64_t)kt * NB + r;
    double s = 0;
    const double* lp = L + row * ld;
    for (int c = sub; c < kt * NB; c += 32) s += lp[c] * yv[c];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    if (sub == 0) yv[row] -= s;
    __syncthreads();
    if (t < WAVE) {
      const int rl = t & (NB - 1);
      const double* dl = L + (int64_t)kt * NB * ld + (int64_t)kt * NB;
      for (int j = 0; j < NB; ++j) {
        if (t == j) yv[kt * NB + j] /= dl[(int64_t)j * ld + j];
        wave_lds_fence();
        if (t < NB && rl > j) yv[kt * NB + rl] -= dl[(int64_t)rl * ld + j] * yv[kt * NB + j];
        wave_lds_fence();
      }
    }
    __syncthreads();
  }
  // backward: x_kt = L_kk^-T (y_kt - sum_{i>kt} L_{i,kt}^T x_i)
  for (int kt = T - 1; kt >= 0; --kt) {
    const int c = r;
    double s = 0;
    for (int64_t i = (int64_t)(kt + 1) * NB + sub; i < ld; i += 32) s += L[i * ld + (int64_t)kt * NB + c] * yv[i];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    if (sub == 0) yv[kt * NB + c] -= s;
    __syncthreads();
    if (t < WAVE) {
      const double* dl = L + (int64_t)kt * NB * ld + (int64_t)kt * NB;
      for (int j = NB - 1; j >= 0; --j) {
        if (t == j) yv[kt * NB + j] /= dl[(int64_t)j * ld + j];
        wave_lds_fence();
        if (t < j) yv[kt * NB + t] -= dl[(int64_t)j * ld + t] * yv[kt * NB + j];
        wave_lds_fence();
      }
    }
    __syncthreads();
  }
  for (int i = t; i < ld; i += blockDim.x) b[i] = yv[i];
}

void launch_chol_solve(const double* L, int64_t ld, double* b, hipStream_t st) {
  hipLaunchKernelGGL(k_chol_solve, dim3(1), dim3(1024), (size_t)ld * sizeof(double), st, L, ld, b);
}

}  // namespace ptzba
