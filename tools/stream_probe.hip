// Microbenchmarks for the consume kernel's building blocks on gfx950 (tools/, not product):
// how fast can one stream an 8-byte column, filter it with ballots, and gather a second column
// for the selected rows, at the C2 shape (100M rows, ~12% selected)?  Prints ms and GB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint32_t XcdRemap(uint32_t orig, uint32_t nwg) {
  uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// (a) grid-stride 8 B/lane stream, K loads in flight per thread.
template <int K>
__global__ void __launch_bounds__(256) Stream8(const int64_t* __restrict__ a, int64_t n, unsigned long long* out) {
  int64_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * K;
  for (int64_t base = static_cast<int64_t>(XcdRemap(blockIdx.x, gridDim.x)) * 256 * K; base < n; base += stride) {
    int64_t v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t r = base + k * 256 + threadIdx.x;
      v[k] = r < n ? a[r] : 0;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) acc += v[k] >= 400;
  }
  if (acc == 0x7fffffff) atomicAdd(out, 1ull);
}

// (b) 16 B/lane stream.
template <int K>
__global__ void __launch_bounds__(256) Stream16(const int64_t* __restrict__ a, int64_t n, unsigned long long* out) {
  int64_t acc = 0;
  const int64_t n2 = n / 2;
  const longlong2* p = reinterpret_cast<const longlong2*>(a);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * K;
  for (int64_t base = static_cast<int64_t>(XcdRemap(blockIdx.x, gridDim.x)) * 256 * K; base < n2; base += stride) {
    longlong2 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t r = base + k * 256 + threadIdx.x;
      v[k] = r < n2 ? p[r] : make_longlong2(0, 0);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) acc += (v[k].x >= 400) + (v[k].y >= 400);
  }
  if (acc == 0x7fffffff) atomicAdd(out, 1ull);
}

// (c) filter status >= 400 and gather lat[r] of passing rows in the same thread (masked
// coalesced loads), sum them (no staging write).
template <int K>
__global__ void __launch_bounds__(256) FilterGatherSame(const int64_t* __restrict__ st, const int64_t* __restrict__ lat, int64_t n,
                                                        unsigned long long* out) {
  int64_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * K;
  for (int64_t base = static_cast<int64_t>(XcdRemap(blockIdx.x, gridDim.x)) * 256 * K; base < n; base += stride) {
    bool p[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t r = base + k * 256 + threadIdx.x;
      p[k] = r < n && st[r] >= 400;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t r = base + k * 256 + threadIdx.x;
      if (p[k]) acc += lat[r];
    }
  }
  if (acc == 0x7fffffff) atomicAdd(out, 1ull);
}

// (d) filter, ballot-compact the passing rows of each 8192-row tile into LDS, then gather lat
// of the compacted rows (dense lanes, the current consume kernel's phase 2 shape) and write
// (u32 slot, u64 value) staging records at a per-tile cursor.
__global__ void __launch_bounds__(256) FilterCompactGather(const int64_t* __restrict__ st, const int64_t* __restrict__ lat, int64_t n,
                                                           unsigned long long* cursor, uint32_t* sslot, uint64_t* sval) {
  constexpr int K = 32;
  __shared__ uint16_t s_sel[8192];
  __shared__ uint32_t s_w[4];
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ntiles = (n + 8191) / 8192;
  for (int64_t t = XcdRemap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const int64_t row0 = t * 8192;
    bool p[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t r = row0 + k * 256 + threadIdx.x;
      p[k] = r < n && st[r] >= 400;
    }
    unsigned long long m[K];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m[k] = __ballot(p[k]);
      tot += __popcll(m[k]);
    }
    if (lane == 0) s_w[wid] = tot;
    __syncthreads();
    uint32_t wb = 0, all = 0;
    for (int w = 0; w < 4; ++w) {
      wb += w < wid ? s_w[w] : 0;
      all += s_w[w];
    }
    if (threadIdx.x == 0) s_base = atomicAdd(cursor, static_cast<unsigned long long>(all));
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (p[k]) s_sel[wb + __popcll(m[k] & ((1ull << lane) - 1))] = static_cast<uint16_t>(k * 256 + threadIdx.x);
      wb += __popcll(m[k]);
    }
    __syncthreads();
    const uint64_t b = s_base;
    for (uint32_t i = threadIdx.x; i < all; i += 256) {
      const int64_t r = row0 + s_sel[i];
      sval[b + i] = static_cast<uint64_t>(lat[r]);
      sslot[b + i] = static_cast<uint32_t>(r);
    }
    __syncthreads();
  }
}

// (e) gather of 16-byte payload words at random-ish offsets of the selected rows (the key
// gather shape): for each selected row, 2 x 16 B loads at pay[off[r]].
__global__ void __launch_bounds__(256) FilterGatherPayload(const int64_t* __restrict__ st, const int32_t* __restrict__ off,
                                                           const uint8_t* __restrict__ pay, int64_t n, unsigned long long* out) {
  constexpr int K = 32;
  __shared__ uint16_t s_sel[8192];
  __shared__ uint32_t s_w[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ntiles = (n + 8191) / 8192;
  uint64_t acc = 0;
  for (int64_t t = XcdRemap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const int64_t row0 = t * 8192;
    bool p[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t r = row0 + k * 256 + threadIdx.x;
      p[k] = r < n && st[r] >= 400;
    }
    unsigned long long m[K];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m[k] = __ballot(p[k]);
      tot += __popcll(m[k]);
    }
    if (lane == 0) s_w[wid] = tot;
    __syncthreads();
    uint32_t wb = 0, all = 0;
    for (int w = 0; w < 4; ++w) {
      wb += w < wid ? s_w[w] : 0;
      all += s_w[w];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (p[k]) s_sel[wb + __popcll(m[k] & ((1ull << lane) - 1))] = static_cast<uint16_t>(k * 256 + threadIdx.x);
      wb += __popcll(m[k]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < all; i += 256) {
      const int64_t r = row0 + s_sel[i];
      const int32_t o = off[r];
      ulonglong2 a, b;
      __builtin_memcpy(&a, pay + o, 16);
      __builtin_memcpy(&b, pay + o + 16, 16);
      acc += a.x ^ a.y ^ b.x ^ b.y;
    }
    __syncthreads();
  }
  if (acc == 0x7fffffff) atomicAdd(out, 1ull);
}

template <typename F>
static float TimeIt(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

__global__ void Fill(int64_t* st, int64_t* lat, int32_t* off, int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += gridDim.x * 256ll) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ULL;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ULL;
    x ^= x >> 29;
    st[i] = (x % 100) < 12 ? 404 : 200;
    lat[i] = static_cast<int64_t>(x >> 20);
    off[i] = static_cast<int32_t>((i & ((1 << 26) - 1)) * 24);  // < 2^31, inside pay
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 100000000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int64_t *st, *lat;
  int32_t* off;
  uint8_t* pay;
  unsigned long long* out;
  uint32_t* sslot;
  uint64_t* sval;
  CK(hipMalloc(&st, n * 8));
  CK(hipMalloc(&lat, n * 8));
  CK(hipMalloc(&off, n * 4 + 64));
  CK(hipMalloc(&pay, n * 24 + 64));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&sslot, n * 4));
  CK(hipMalloc(&sval, n * 8));
  CK(hipMemset(pay, 1, n * 24 + 64));
  Fill<<<cus * 8, 256>>>(st, lat, off, n);
  CK(hipDeviceSynchronize());
  const double gb8 = n * 8 / 1e9;
  auto report = [&](const char* name, float ms, double gb) { std::printf("%-40s %8.4f ms  %7.1f GB/s\n", name, ms, gb / (ms / 1e3)); };
  for (int bpc : {4, 8, 16}) {
    const int grid = cus * bpc;
    char nm[96];
    std::snprintf(nm, sizeof nm, "stream8 K=8 bpc=%d", bpc);
    report(nm, TimeIt([&] { Stream8<8><<<grid, 256>>>(st, n, out); }, 20), gb8);
    std::snprintf(nm, sizeof nm, "stream8 K=32 bpc=%d", bpc);
    report(nm, TimeIt([&] { Stream8<32><<<grid, 256>>>(st, n, out); }, 20), gb8);
    std::snprintf(nm, sizeof nm, "stream16 K=8 bpc=%d", bpc);
    report(nm, TimeIt([&] { Stream16<8><<<grid, 256>>>(st, n, out); }, 20), gb8);
    std::snprintf(nm, sizeof nm, "filter+gather same-thread K=16 bpc=%d", bpc);
    report(nm, TimeIt([&] { FilterGatherSame<16><<<grid, 256>>>(st, lat, n, out); }, 20), 2 * gb8);
    std::snprintf(nm, sizeof nm, "filter+compact+gather+stage bpc=%d", bpc);
    report(nm, TimeIt([&] { (void)hipMemsetAsync(out, 0, 8); FilterCompactGather<<<grid, 256>>>(st, lat, n, out, sslot, sval); }, 20), 2 * gb8);
    std::snprintf(nm, sizeof nm, "filter+compact+payload2x16 bpc=%d", bpc);
    report(nm, TimeIt([&] { FilterGatherPayload<<<grid, 256>>>(st, off, pay, n, out); }, 20), gb8 + n * 24 / 1e9);
  }
  return 0;
}
