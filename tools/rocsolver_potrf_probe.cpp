// Calibration probe (not product code): rocSOLVER dpotrf time at the headline reduced-system size.
#include <hip/hip_runtime.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>
#include <vector>
#include <random>
int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1504;
  std::vector<double> A((size_t)n * n);
  std::mt19937 g(1); std::uniform_real_distribution<double> U(-1, 1);
  for (int i = 0; i < n; ++i) for (int j = 0; j <= i; ++j) { double v = U(g) * (abs(i - j) < 420 ? 1 : 0); A[(size_t)i*n+j] = v; A[(size_t)j*n+i] = v; }
  for (int i = 0; i < n; ++i) A[(size_t)i*n+i] = 1000.0;
  double *dA, *dB; int* info;
  hipMalloc(&dA, A.size() * 8); hipMalloc(&dB, A.size() * 8); hipMalloc(&info, 4);
  hipMemcpy(dB, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  rocblas_handle h; rocblas_create_handle(&h);
  hipStream_t st; hipStreamCreate(&st); rocblas_set_stream(h, st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 3; ++it) { hipMemcpyAsync(dA, dB, A.size()*8, hipMemcpyDeviceToDevice, st); rocsolver_dpotrf(h, rocblas_fill_lower, n, dA, n, info); }
  hipStreamSynchronize(st);
  float tot = 0; int reps = 20;
  for (int it = 0; it < reps; ++it) {
    hipMemcpyAsync(dA, dB, A.size()*8, hipMemcpyDeviceToDevice, st);
    hipEventRecord(e0, st); rocsolver_dpotrf(h, rocblas_fill_lower, n, dA, n, info); hipEventRecord(e1, st);
    hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); tot += ms;
  }
  int hinfo; hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost);
  printf("rocsolver_dpotrf n=%d avg %.3f ms info=%d\n", n, tot / reps, hinfo);
  return 0;
}
