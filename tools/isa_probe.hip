// Cycle costs on gfx950 of the building blocks of a one-wave 32x32 fp64 Cholesky step (tools only).
//   hipcc -O3 --offload-arch=gfx950 tools/isa_probe.hip -o tools/isa_probe && tools/isa_probe
// One wave per workgroup, s_memtime around N repetitions; prints cycles per element operation.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 496;

__device__ __forceinline__ double bcast(double v, int j) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}

// mode 0: x[m] -= li * bcast(x[j], m) over 31 m per j (the library's inner loop), 16 j
// mode 1: same FMAs with a lane-local operand (no broadcast)
// mode 2: readlane pairs only (accumulated so they are not dead)
// mode 3: FMAs with operands from uniform-address LDS reads (ds_read_b128), pipelined by the compiler
// mode 4: bpermute broadcast (ds_bpermute_b32 x2) instead of readlane
template <int MODE>
__global__ __launch_bounds__(64) void k_probe(const double* in, double* out, long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[64];
  const int lane = threadIdx.x;
  double x[32];
#pragma unroll
  for (int m = 0; m < 32; ++m) x[m] = in[lane * 32 + m];
  col[lane] = in[lane];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_sched_barrier(0);
  const long long t0 = clock64();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double li = x[j] * 1e-3;
    if (MODE == 0) {
#pragma unroll
      for (int m = j + 1; m < 32; ++m) x[m] -= li * bcast(x[j], m);
    } else if (MODE == 1) {
#pragma unroll
      for (int m = j + 1; m < 32; ++m) x[m] -= li * x[(m + j) & 31];
    } else if (MODE == 2) {
      double a = 0;
#pragma unroll
      for (int m = j + 1; m < 32; ++m) a += bcast(x[j], m);
      x[j + 1] += a;
    } else if (MODE == 3) {
#pragma unroll
      for (int m = j + 1; m < 32; ++m) x[m] -= li * col[(m + j) & 63];
    } else if (MODE == 4) {
#pragma unroll
      for (int m = j + 1; m < 32; ++m) {
        int lo = __builtin_amdgcn_ds_bpermute(m * 4, __double2loint(x[j]));
        int hi = __builtin_amdgcn_ds_bpermute(m * 4, __double2hiint(x[j]));
        x[m] -= li * __hiloint2double(hi, lo);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  const long long t1 = clock64();
  __builtin_amdgcn_sched_barrier(0);
  double s = 0;
#pragma unroll
  for (int m = 0; m < 32; ++m) s += x[m];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, const double* in, double* out, long long* cyc) {
  hipLaunchKernelGGL(k_probe<MODE>, dim3(1), dim3(64), 0, 0, in, out, cyc);
  hipLaunchKernelGGL(k_probe<MODE>, dim3(1), dim3(64), 0, 0, in, out, cyc);
  long long c = 0;
  hipDeviceSynchronize();
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  int elems = 0;
  for (int j = 0; j < 16; ++j) elems += 31 - j;
  printf("%-34s %7lld cycles  %6.2f cycles/element (%d elements)\n", name, c, (double)c / elems, elems);
}

int main() {
  double *in, *out;
  long long* cyc;
  hipMalloc(&in, 64 * 32 * 8);
  hipMalloc(&out, 64 * 64 * 8);
  hipMalloc(&cyc, 64 * 8);
  hipMemset(in, 0, 64 * 32 * 8);
  run<0>("readlane bcast + fma (library)", in, out, cyc);
  run<1>("fma, lane-local operand", in, out, cyc);
  run<2>("readlane pairs only", in, out, cyc);
  run<3>("fma, LDS uniform-address operand", in, out, cyc);
  run<4>("bpermute bcast + fma", in, out, cyc);
  return 0;
}
