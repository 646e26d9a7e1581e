// FETCH_SIZE calibration on gfx950 (MI355X_MICROARCH.md §HBM: "Other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").  Streams a
// 1 GiB buffer (far beyond the 256 MiB Infinity Cache) with 8-byte-per-lane loads (the consume
// kernel's column streams) and with 16-byte-per-lane loads, one launch each; rocprofv3
// --pmc FETCH_SIZE over this binary gives KiB per launch against exactly 1 GiB read.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void Read8(const uint64_t* __restrict__ p, uint64_t n, uint64_t* __restrict__ out) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) acc ^= p[i];
  if (acc == 0x123456789ull) out[blockIdx.x] = acc;  // never true for the zeroed buffer: no store traffic
}

__global__ void Read16(const ulonglong2* __restrict__ p, uint64_t n, uint64_t* __restrict__ out) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) { ulonglong2 v = p[i]; acc ^= v.x ^ v.y; }
  if (acc == 0x123456789ull) out[blockIdx.x] = acc;
}

int main() {
  const uint64_t bytes = 1ull << 30;
  void* buf = nullptr;
  uint64_t* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, bytes);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(Read8, dim3(4096), dim3(256), 0, 0, static_cast<const uint64_t*>(buf), bytes / 8, out);
    hipLaunchKernelGGL(Read16, dim3(4096), dim3(256), 0, 0, static_cast<const ulonglong2*>(buf), bytes / 16, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("read %llu bytes per launch\n", static_cast<unsigned long long>(bytes));
  return 0;
}
