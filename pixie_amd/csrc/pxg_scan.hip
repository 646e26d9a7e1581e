// Device-wide exclusive scan: reduce -> scan block sums (recursive) -> downsweep.
#include "pxg_scan.h"

namespace pxg {

template <typename T>
__device__ __forceinline__ T WaveInclusiveScan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// Block exclusive scan of per-thread values; returns the exclusive prefix, *block_total set.
template <typename T>
__device__ __forceinline__ T BlockExclusiveScan(T v, T* lds /*[kScanBlock/64]*/, T* block_total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T inc = WaveInclusiveScan(v);
  if (lane == 63) lds[wid] = inc;
  __syncthreads();
  T wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kScanBlock / 64; ++w) {
    T x = lds[w];
    if (w < wid) wbase += x;
    tot += x;
  }
  __syncthreads();
  *block_total = tot;
  return wbase + inc - v;
}

template <typename T>
__global__ void __launch_bounds__(kScanBlock) ScanReduceKernel(const T* __restrict__ in, int64_t n, T* __restrict__ sums) {
  __shared__ T lds[kScanBlock / 64];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
  T acc = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + static_cast<int64_t>(k) * kScanBlock + threadIdx.x;
    if (i < n) acc += in[i];
  }
  T tot;
  (void)BlockExclusiveScan(acc, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// Scan a tile: each thread owns kScanItems consecutive items. The tile goes through LDS so that
// the global loads and stores stay coalesced (a wave touches 64 consecutive elements per
// instruction, not 64 elements kScanItems apart); row j of the tile sits at j + j / kScanItems,
// which keeps a thread's consecutive items off each other's banks. In-place (in == out) is fine:
// a block reads its whole tile before it writes any of it.
template <typename T>
__global__ void __launch_bounds__(kScanBlock) ScanDownsweepKernel(const T* __restrict__ in, T* __restrict__ out, int64_t n,
                                                                  const T* __restrict__ block_base, T* __restrict__ total) {
  constexpr int kPad = kScanItems + 1;
  __shared__ T lds[kScanBlock / 64];
  __shared__ T tile[kScanBlock * kPad];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int j = k * kScanBlock + t;
    const int64_t i = base + j;
    tile[j + j / kScanItems] = i < n ? in[i] : T(0);
  }
  __syncthreads();
  T vals[kScanItems];
  T acc = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    vals[k] = tile[t * kPad + k];
    acc += vals[k];
  }
  T tot;
  T prefix = BlockExclusiveScan(acc, lds, &tot);  // its barriers also order the tile reads above
  T run = prefix + (block_base ? block_base[blockIdx.x] : T(0));
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    tile[t * kPad + k] = run;
    run += vals[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int j = k * kScanBlock + t;
    const int64_t i = base + j;
    if (i < n) out[i] = tile[j + j / kScanItems];
  }
  if (total && blockIdx.x == gridDim.x - 1 && t == kScanBlock - 1) *total = run;
}

size_t ScanScratchBytes(int64_t n) {
  size_t bytes = 0;
  int64_t m = n;
  while (m > kScanTile) {
    m = (m + kScanTile - 1) / kScanTile;
    bytes += (static_cast<size_t>(m) + 16) * sizeof(uint64_t);
  }
  return bytes + 64;
}

template <typename T>
static int32_t ScanImpl(Ctx* ctx, hipStream_t stream, const T* in, T* out, int64_t n, T* total, uint8_t* scratch) {
  if (n <= 0) {
    if (total) PXG_HIP(hipMemsetAsync(total, 0, sizeof(T), stream));
    return PXG_OK;
  }
  int64_t nblocks = (n + kScanTile - 1) / kScanTile;
  if (nblocks == 1) {
    return LaunchOn(ctx, stream, "scan_downsweep", ScanDownsweepKernel<T>, dim3(1), dim3(kScanBlock), 0, in, out, n,
                    static_cast<const T*>(nullptr), total);
  }
  T* sums = reinterpret_cast<T*>(scratch);
  uint8_t* rest = scratch + (static_cast<size_t>(nblocks) + 16) * sizeof(uint64_t);
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, stream, "scan_reduce", ScanReduceKernel<T>, dim3(static_cast<unsigned>(nblocks)), dim3(kScanBlock),
                               0, in, n, sums));
  PXG_RETURN_IF_ERROR(ScanImpl<T>(ctx, stream, sums, sums, nblocks, static_cast<T*>(nullptr), rest));
  return LaunchOn(ctx, stream, "scan_downsweep", ScanDownsweepKernel<T>, dim3(static_cast<unsigned>(nblocks)), dim3(kScanBlock), 0,
                  in, out, n, static_cast<const T*>(sums), total);
}

int32_t ScanExclusiveU64(Ctx* ctx, const uint64_t* in, uint64_t* out, int64_t n, uint64_t* total, void* scratch) {
  return ScanImpl<uint64_t>(ctx, ctx->stream, in, out, n, total, static_cast<uint8_t*>(scratch));
}
int32_t ScanExclusiveU32(Ctx* ctx, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total, void* scratch) {
  return ScanImpl<uint32_t>(ctx, ctx->stream, in, out, n, total, static_cast<uint8_t*>(scratch));
}

int32_t ScanExclusiveU32On(Ctx* ctx, hipStream_t stream, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total,
                           void* scratch) {
  return ScanImpl<uint32_t>(ctx, stream, in, out, n, total, static_cast<uint8_t*>(scratch));
}

}  // namespace pxg
