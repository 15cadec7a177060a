// Microbenchmark (tool, not product code): the fused 32x32 fp64 potrf + TRSM of a Cholesky panel task
// (D = L L^T, X = T L^-T) -- the library's lookahead sweep (wg_potrf_trsm32_df, chol_kernels.hip) against
// a blocked right-looking form whose trailing updates run on the fp64 matrix cores:
//   per diagonal block of BK columns: every wave factors the BKxBK block and inverts it in registers
//   (redundantly: no hand-off), each thread forms one L entry of the panel (rows below the block, T rows
//   included) as a row of A times L_kk^-T, then the MFMA tiles update the trailing columns.
// Each workgroup (256 threads) repeats the task REPS times on its own tile; all workgroups run at once, so
// the time is the per-task latency.  Checks L and X against the library sweep.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/potrf_mfma_bench.hip -o tools/potrf_mfma_bench
#include "../pan-tilt-zoom-slam_amd/csrc/chol_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ptzba;
constexpr int REPS = 16;

// rows 0..31 of the combined panel are D, rows 32..63 are T
__device__ __forceinline__ double* prow(double (*D)[NB + 1], double (*T)[NB + 1], int r) {
  return r < NB ? D[r] : T[r - NB];
}

template <int BK>
__device__ __forceinline__ void wg_potrf_trsm32_mb(double (*D)[NB + 1], double (*T)[NB + 1], int* info) {
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int nrow = T ? 2 * NB : NB;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < NB / BK; ++k) {
    const int kb = k * BK;
    // ---- A: factor the BK x BK diagonal block and invert its factor, in registers (every thread)
    double G[BK][BK], Li[BK][BK], y[BK];
#pragma unroll
    for (int i = 0; i < BK; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) G[i][j] = D[kb + i][kb + j];
#pragma unroll
    for (int j = 0; j < BK; ++j) {
      double d = G[j][j];
      if (!(d > 0.0)) {
        bad = true;
        d = 1e-300;
      }
      y[j] = rsq_fast(d);
      G[j][j] = d * y[j];
#pragma unroll
      for (int i = j + 1; i < BK; ++i) G[i][j] *= y[j];
#pragma unroll
      for (int i = j + 1; i < BK; ++i)
#pragma unroll
        for (int m = j + 1; m <= i; ++m) G[i][m] = fma(-G[i][j], G[m][j], G[i][m]);
    }
    // Li = L_kk^-1 (lower): Li[i][i] = y_i, Li[i][j] = -y_i sum_{m=j}^{i-1} L[i][m] Li[m][j]
#pragma unroll
    for (int j = 0; j < BK; ++j) {
      Li[j][j] = y[j];
#pragma unroll
      for (int i = j + 1; i < BK; ++i) {
        double s = 0.0;
#pragma unroll
        for (int m = j; m < i; ++m) s = fma(G[i][m], Li[m][j], s);
        Li[i][j] = -y[i] * s;
      }
    }
    // ---- B: panel rows r >= kb + BK: L_r,kb+c = sum_{m <= c} A_r,kb+m Li[c][m]; the block itself = G
    const int r0 = kb + BK, nr = nrow - r0;
    double av[2][BK];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int e = t + 256 * p, r = r0 + e / BK;
      if (e < nr * BK) {
        const double* src = prow(D, T, r) + kb;
#pragma unroll
        for (int m = 0; m < BK; ++m) av[p][m] = src[m];
      }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int e = t + 256 * p, r = r0 + e / BK, c = e % BK;
      if (e < nr * BK) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < BK; ++m)
          if (m <= c) s = fma(av[p][m], Li[c][m], s);
        prow(D, T, r)[kb + c] = s;
      }
    }
    if (t < BK * BK) {
      const int i = t / BK, j = t % BK;
      if (j <= i) D[kb + i][kb + j] = G[i][j];
    }
    __syncthreads();
    // ---- C: trailing columns j >= kb + BK (D columns), rows r >= kb + BK:  A_rj -= sum_c L_rc L_jc
    if (kb + BK < NB) {
      const int rb0 = (r0 / 16) * 16, cb0 = (r0 / 16) * 16;
      const int nrb = (nrow - rb0 + 15) / 16, ncb = (NB - cb0) / 16;
      const int li = l & 15, lk = l >> 4;
      for (int ob = w; ob < nrb * ncb; ob += 4) {
        const int R0 = rb0 + 16 * (ob / ncb), J0 = cb0 + 16 * (ob % ncb);
        v4f64 acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = prow(D, T, R0 + lk + 4 * q)[J0 + li];
#pragma unroll
        for (int s = 0; s < BK / 4; ++s) {
          const double a = -prow(D, T, R0 + li)[kb + 4 * s + lk];
          const double b = D[J0 + li][kb + 4 * s + lk];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = R0 + lk + 4 * q, j = J0 + li;
          if (r >= r0 && j >= r0) prow(D, T, r)[j] = acc[q];
        }
      }
      __syncthreads();
    }
  }
  if (bad && t == 0) atomicOr(info, 1);
  for (int e = t; e < NB * NB; e += 256) {
    const int i = e >> 5, j = e & 31;
    if (j > i) D[i][j] = 0.0;
  }
  __syncthreads();
}

template <int V>
__global__ __launch_bounds__(256) void k_bench(const double* __restrict__ A, const double* __restrict__ Tg,
                                               double* __restrict__ L, double* __restrict__ X, int* info) {
  __shared__ double sD[NB][NB + 1];
  __shared__ double sC[NB][NB + 1];
  __shared__ __attribute__((aligned(16))) double s_lb[NB / LA_BW][2 * NB][LA_BW];
  __shared__ __attribute__((aligned(16))) double s_pb[LA_BW][LA_BW];
  __shared__ int s_flags[NB / LA_BW + 1];
  const double* a = A + (size_t)blockIdx.x * NB * NB;
  const double* tt = Tg + (size_t)blockIdx.x * NB * NB;
  for (int rep = 0; rep < REPS; ++rep) {
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
      sD[e >> 5][e & 31] = a[e];
      sC[e >> 5][e & 31] = tt[e];
    }
    __syncthreads();
    if (V == 0) wg_potrf_trsm32_df<LA_BW>(sD, sC, s_lb, s_pb, s_flags, info);
    if (V == 4) wg_potrf_trsm32_mb<4>(sD, sC, info);
    if (V == 8) wg_potrf_trsm32_mb<8>(sD, sC, info);
    __syncthreads();
  }
  for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
    L[(size_t)blockIdx.x * NB * NB + e] = sD[e >> 5][e & 31];
    X[(size_t)blockIdx.x * NB * NB + e] = sC[e >> 5][e & 31];
  }
}

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

template <int V>
double run(int nb, double* dA, double* dT, double* dL, double* dX, int* dinfo, std::vector<double>& L,
           std::vector<double>& X) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_bench<V>, dim3(nb), dim3(256), 0, 0, dA, dT, dL, dX, dinfo);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k_bench<V>, dim3(nb), dim3(256), 0, 0, dA, dT, dL, dX, dinfo);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  L.resize((size_t)nb * NB * NB);
  X.resize((size_t)nb * NB * NB);
  CK(hipMemcpy(L.data(), dL, L.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(X.data(), dX, X.size() * 8, hipMemcpyDeviceToHost));
  return ms * 1e3 / 5 / REPS;
}

int main() {
  const int nb = 64;
  std::vector<double> A((size_t)nb * NB * NB), T((size_t)nb * NB * NB);
  srand(1);
  for (int b = 0; b < nb; ++b) {
    std::vector<double> B(NB * NB);
    for (auto& x : B) x = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < NB; ++i)
      for (int j = 0; j < NB; ++j) {
        double s = (i == j) ? NB : 0.0;
        for (int k = 0; k < NB; ++k) s += B[i * NB + k] * B[j * NB + k];
        A[(size_t)b * NB * NB + i * NB + j] = s;
        T[(size_t)b * NB * NB + i * NB + j] = (double)rand() / RAND_MAX - 0.5;
      }
  }
  double *dA, *dT, *dL, *dX;
  int* dinfo;
  CK(hipMalloc(&dA, A.size() * 8));
  CK(hipMalloc(&dT, T.size() * 8));
  CK(hipMalloc(&dL, A.size() * 8));
  CK(hipMalloc(&dX, A.size() * 8));
  CK(hipMalloc(&dinfo, 4));
  CK(hipMemset(dinfo, 0, 4));
  CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dT, T.data(), T.size() * 8, hipMemcpyHostToDevice));
  std::vector<double> L0, X0, L, X;
  const double us0 = run<0>(nb, dA, dT, dL, dX, dinfo, L0, X0);
  printf("%-34s %8.3f us\n", "library lookahead sweep (df)", us0);
  auto cmp = [&](const char* name, double us) {
    double el = 0, ex = 0;
    for (size_t i = 0; i < L.size(); ++i) el = fmax(el, fabs(L[i] - L0[i]));
    for (size_t i = 0; i < X.size(); ++i) ex = fmax(ex, fabs(X[i] - X0[i]));
    printf("%-34s %8.3f us   max|dL| %.2e  max|dX| %.2e\n", name, us, el, ex);
  };
  cmp("blocked MFMA BK=4", run<4>(nb, dA, dT, dL, dX, dinfo, L, X));
  cmp("blocked MFMA BK=8", run<8>(nb, dA, dT, dL, dX, dinfo, L, X));
  int info = 0;
  CK(hipMemcpy(&info, dinfo, 4, hipMemcpyDeviceToHost));
  printf("info %d\n", info);
  return 0;
}
