// Byte calibration of the rocprofv3 FETCH_SIZE / WRITE_SIZE counters for the access widths K1 uses
// (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel streams a 1 GiB buffer (4x the Infinity Cache) once,
// coalesced (consecutive lanes, consecutive elements), with 1-, 4-, 8- or 16-byte loads per lane, or
// writes it with 16-byte stores; every kernel runs twice.  Run under two separate PMC passes:
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib.bin
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d DIR -o run --output-format csv -- ./tools/pmc_calib.bin
//   (same with WRITE_SIZE), then tools/pmc_calib_summary.py DIR_FETCH DIR_WRITE
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ p, size_t n, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = p[i];
    acc += reinterpret_cast<const unsigned char*>(&v)[sizeof(T) - 1];
  }
  if (acc == 0x12345u) out[0] = acc;  // keeps the loads; never true for the fill pattern
}

__global__ __launch_bounds__(256) void k_write16(uint4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

int main() {
  const size_t bytes = size_t(1) << 30;
  void* buf = nullptr;
  unsigned* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
  const dim3 grid(4096), block(256);
  for (int rep = 0; rep < 2; ++rep) {
    k_read<uint8_t><<<grid, block>>>((const uint8_t*)buf, bytes, out);
    k_read<uint32_t><<<grid, block>>>((const uint32_t*)buf, bytes / 4, out);
    k_read<uint2><<<grid, block>>>((const uint2*)buf, bytes / 8, out);
    k_read<uint4><<<grid, block>>>((const uint4*)buf, bytes / 16, out);
    k_write16<<<grid, block>>>((uint4*)buf, bytes / 16);
  }
  // a 128 MiB table read three times back to back: resident in the 256 MiB Infinity Cache after the first
  // pass -- shows whether cache hits reach the counters
  for (int rep = 0; rep < 3; ++rep) k_read<uint2><<<grid, block>>>((const uint2*)buf, (bytes / 8) / 8, out);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("streamed %zu bytes per kernel\n", bytes);
  hipFree(buf);
  hipFree(out);
  return 0;
}
