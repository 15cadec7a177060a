// Fixed cost of a factorisation level's launch on gfx950: chains of back-to-back launches on one stream, each
// kernel's work trivial, timed by events over many chains (what the 26 level launches of config 3 pay besides
// their tasks).  Variants: (a) an empty kernel, 128 workgroups of 256 threads; (b) the same with 34 KB of LDS
// touched per workgroup; (c) a hand-off chain: workgroup 0 of launch L reads an 8-KB tile written by launch L - 1
// (agent-scope loads / stores as the level launches' COH tiles), i.e. launch + one tile round trip.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o tools/launch_probe && tools/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 100000) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_lds(int* out) {
  __shared__ double s[4 * 32 * 33];
  for (int e = threadIdx.x; e < 4 * 32 * 33; e += 256) s[e] = e;
  __syncthreads();
  if (threadIdx.x == 0 && s[blockIdx.x & 1023] < 0) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_handoff(double* tile, int lvl) {
  if (blockIdx.x != 0) return;
  double v[4];
  for (int q = 0; q < 4; ++q)
    v[q] = __hip_atomic_load(tile + threadIdx.x + 256 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int q = 0; q < 4; ++q)
    __hip_atomic_store(tile + threadIdx.x + 256 * q, v[q] + lvl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  int* out;
  double* tile;
  hipMalloc(&out, 64);
  hipMalloc(&tile, 1024 * sizeof(double));
  hipMemset(tile, 0, 1024 * sizeof(double));
  hipStream_t st;
  hipStreamCreate(&st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int L = 26, REP = 400;
  const char* names[] = {"empty kernel, 128 x 256", "34 KB LDS written, 128 x 256", "tile hand-off, 128 x 256"};
  for (int v = 0; v < 3; ++v) {
    for (int pass = 0; pass < 2; ++pass) {  // pass 0: warm-up
      hipEventRecord(e0, st);
      for (int r = 0; r < REP; ++r)
        for (int l = 0; l < L; ++l) {
          if (v == 0) hipLaunchKernelGGL(k_empty, dim3(128), dim3(256), 0, st, out);
          if (v == 1) hipLaunchKernelGGL(k_lds, dim3(128), dim3(256), 0, st, out);
          if (v == 2) hipLaunchKernelGGL(k_handoff, dim3(128), dim3(256), 0, st, tile, l);
        }
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-32s %6.2f us per launch (chains of %d launches, %d chains)\n", names[v], 1e3 * ms / (REP * L), L, REP);
  }
  return 0;
}
