// Accuracy of the gfx950 fp64 reciprocal / reciprocal-sqrt estimates (v_rcp_f64, v_rsq_f64) and of
// one / two Newton steps on them, against long-double host references.  Decides how many Newton
// steps the Cholesky pivot chain needs.
//   hipcc -O3 --offload-arch=gfx950 tools/rcp_probe.hip -o /tmp/rcp_probe && /tmp/rcp_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void k_probe(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  double r = __builtin_amdgcn_rcp(d);
  out[7 * i + 0] = r;
  r = fma(r, fma(-d, r, 1.0), r);
  out[7 * i + 1] = r;
  out[7 * i + 2] = fma(r, fma(-d, r, 1.0), r);
  double y = __builtin_amdgcn_rsq(d);
  out[7 * i + 3] = y;
  y = y * fma(-0.5 * d * y, y, 1.5);
  out[7 * i + 4] = y;
  out[7 * i + 5] = y * fma(-0.5 * d * y, y, 1.5);
  const double y0 = __builtin_amdgcn_rsq(d);
  const double e = fma(-d * y0, y0, 1.0);
  out[7 * i + 6] = fma(y0 * e, fma(e, 0.375, 0.5), y0);  // series step (chol rsq_fast)
}

int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), out(7 * (size_t)n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> e(-300.0, 300.0), m(1.0, 2.0);
  for (int i = 0; i < n; ++i) x[i] = (i < n / 2) ? m(g) : std::ldexp(m(g), (int)e(g) * 3);
  double *dx, *dout;
  if (hipMalloc(&dx, n * sizeof(double)) || hipMalloc(&dout, out.size() * sizeof(double))) return 1;
  hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice);
  k_probe<<<n / 256, 256>>>(dx, dout, n);
  hipMemcpy(out.data(), dout, out.size() * sizeof(double), hipMemcpyDeviceToHost);
  double worst[7] = {0};
  for (int i = 0; i < n; ++i) {
    const long double rr = 1.0L / (long double)x[i], rs = 1.0L / sqrtl((long double)x[i]);
    for (int k = 0; k < 7; ++k) {
      const long double ref = k < 3 ? rr : rs;
      const double err = (double)fabsl(((long double)out[7 * (size_t)i + k] - ref) / ref);
      if (err > worst[k]) worst[k] = err;
    }
  }
  const char* nm[7] = {"rcp", "rcp+1NR", "rcp+2NR", "rsq", "rsq+1NR", "rsq+2NR", "rsq+ser"};
  for (int k = 0; k < 7; ++k) printf("%-8s max rel err %.3e (%.2f ulp)\n", nm[k], worst[k], worst[k] / 2.220446e-16);
  hipFree(dx);
  hipFree(dout);
  return 0;
}
