// Dependent-chain latencies of the fp64 operations on the pivot sweep's critical path (one wave, gfx950):
// v_fma_f64, v_mul_f64, v_rsq_f64, rsq + series step, v_readlane (VGPR -> SGPR -> fp64 operand), ds_read_b64
// round trip.  Cycles per dependent op from s_memtime around 256-op chains (tools/chol_timing.py's clock).
//   hipcc -O3 --offload-arch=gfx950 tools/lat_probe.hip -o tools/lat_probe && tools/lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 256;
// the cycle counter read after its inputs are ready: the asm consumes v, so the chain must have issued first
__device__ __forceinline__ long long stamp(double v) {
  long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(v) : "memory");
  return t;
}

__device__ __forceinline__ double bcast(double v, int j) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}

__global__ void probe(double* out, long long* cyc, double seed) {
  __shared__ double lds[64 * 4];
  const int lane = threadIdx.x;
  double x = seed + lane * 1e-3;
  lds[lane] = x;
  __syncthreads();
  long long t0, t1;
  // 0: fma chain
  t0 = stamp(x);
#pragma unroll
  for (int i = 0; i < N; ++i) x = fma(x, 0.9999999, 1e-7);
  t1 = stamp(x);
  if (lane == 0) cyc[0] = t1 - t0;
  // 1: mul chain
  t0 = stamp(x);
#pragma unroll
  for (int i = 0; i < N; ++i) x = x * 1.0000001;
  t1 = stamp(x);
  if (lane == 0) cyc[1] = t1 - t0;
  // 2: rsq chain (hardware estimate only)
  double y = x;
  t0 = stamp(y);
#pragma unroll
  for (int i = 0; i < N; ++i) y = __builtin_amdgcn_rsq(y);
  t1 = stamp(y);
  if (lane == 0) cyc[2] = t1 - t0;
  // 3: readlane -> fma chain (the pivot gather pattern: a VALU result broadcast and consumed)
  double z = x;
  t0 = stamp(z);
#pragma unroll
  for (int i = 0; i < N; ++i) z = fma(bcast(z, i & 63), 0.999, 1e-3);
  t1 = stamp(z);
  if (lane == 0) cyc[3] = t1 - t0;
  // 4: LDS round trip chain (store then dependent load of another lane's value)
  double u = x;
  t0 = stamp(u);
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    lds[(lane + 1) & 63] = u;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    u = lds[lane] + 1e-9;
  }
  t1 = stamp(u);
  if (lane == 0) cyc[4] = (t1 - t0) * 4;  // per 64 -> scale to N = 256
  // 5: independent fma throughput (8 chains)
  double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  t0 = stamp(a0 + a7);
#pragma unroll
  for (int i = 0; i < N / 8; ++i) {
    a0 = fma(a0, 0.99, 1e-3); a1 = fma(a1, 0.99, 1e-3); a2 = fma(a2, 0.99, 1e-3); a3 = fma(a3, 0.99, 1e-3);
    a4 = fma(a4, 0.99, 1e-3); a5 = fma(a5, 0.99, 1e-3); a6 = fma(a6, 0.99, 1e-3); a7 = fma(a7, 0.99, 1e-3);
  }
  t1 = stamp(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
  if (lane == 0) cyc[5] = t1 - t0;
  // 6: independent readlane throughput (16 readlanes of one source, consumed by one add chain afterwards)
  double s = 0;
  t0 = stamp(a0);
#pragma unroll
  for (int i = 0; i < N / 2; ++i) s += bcast(a0, i & 63);
  t1 = stamp(s);
  if (lane == 0) cyc[6] = (t1 - t0) * 2;
  // 7: 8 independent rsq chains (transcendental issue rate)
  double r0 = a0, r1 = a1, r2 = a2, r3 = a3, r4 = a4, r5 = a5, r6 = a6, r7 = a7;
  t0 = stamp(r0 + r7);
#pragma unroll
  for (int i = 0; i < N / 8; ++i) {
    r0 = __builtin_amdgcn_rsq(r0); r1 = __builtin_amdgcn_rsq(r1); r2 = __builtin_amdgcn_rsq(r2); r3 = __builtin_amdgcn_rsq(r3);
    r4 = __builtin_amdgcn_rsq(r4); r5 = __builtin_amdgcn_rsq(r5); r6 = __builtin_amdgcn_rsq(r6); r7 = __builtin_amdgcn_rsq(r7);
  }
  t1 = stamp(r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7);
  if (lane == 0) cyc[7] = t1 - t0;
  s += r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
  out[lane] = x + y + z + u + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 16 * 8);
  const char* names[] = {"v_fma_f64 dependent", "v_mul_f64 dependent", "v_rsq_f64 dependent",
                         "readlane x2 + v_fma_f64 dependent", "ds_write + ds_read round trip (dependent)",
                         "v_fma_f64 independent (8 chains, issue)", "readlane pair + v_add_f64 (accumulate)",
                         "v_rsq_f64 independent (8 chains, issue)"};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, 1.5 + rep);
    hipDeviceSynchronize();
  }
  long long h[16];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  for (int k = 0; k < 8; ++k) printf("%-45s %6.1f cycles/op\n", names[k], (double)h[k] / N);
  return 0;
}
