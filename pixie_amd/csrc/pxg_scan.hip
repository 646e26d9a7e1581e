// Device-wide exclusive scan: reduce -> scan block sums (recursive) -> downsweep.
#include "pxg_scan.h"

#include <atomic>

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
  T x[kScanItems];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {  // every load issued before the first use (clamped index)
    const int64_t i = base + static_cast<int64_t>(k) * kScanBlock + threadIdx.x;
    x[k] = in[i < n ? i : n - 1];
  }
  T acc = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) acc += base + static_cast<int64_t>(k) * kScanBlock + threadIdx.x < n ? x[k] : T(0);
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
  {
    // All loads in flight before the LDS writes: a guarded load per item compiled to a branch
    // and a wait per item (16 serialised round trips per thread).
    T x[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      const int64_t i = base + k * kScanBlock + t;
      x[k] = in[i < n ? i : n - 1];
    }
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      const int j = k * kScanBlock + t;
      tile[j + j / kScanItems] = base + j < n ? x[k] : T(0);
    }
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

// Single-pass exclusive scan of u32 values (decoupled look-back): one launch instead of the
// reduce / spine / downsweep chain, whose ~5 us per launch dominated the small scans of a
// finalize (dense ids, chunk counts, key lengths: 3 launches each).  Tile b publishes its sum
// right after its block scan, then wave 0 walks back over the 64 preceding status words at a
// time until it meets an inclusive prefix.  A status word is epoch(31) | inclusive(1) |
// value(32); a word of another epoch reads as "not published yet".  Values are summed mod 2^32,
// exactly as the multi-kernel scan does.  Tiles wait only on lower block ids, which are
// dispatched first, so the spin always ends.  Status words are relaxed agent-scope atomics (the
// value travels in the status word itself, so no other data needs ordering).
constexpr uint64_t kLbInclBit = uint64_t(1) << 32;
__global__ void __launch_bounds__(kScanBlock) ScanLookbackU32Kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int64_t n,
                                                                    uint32_t* __restrict__ total, uint64_t* __restrict__ status,
                                                                    uint64_t epoch_tag) {
  constexpr int kPad = kScanItems + 1;
  __shared__ uint32_t lds[kScanBlock / 64];
  __shared__ uint32_t tile[kScanBlock * kPad];
  __shared__ uint32_t s_excl;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
  const int t = threadIdx.x, lane = t & 63;
  {
    uint32_t x[kScanItems];  // all loads in flight first (as in ScanDownsweepKernel)
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      const int64_t i = base + k * kScanBlock + t;
      x[k] = in[i < n ? i : n - 1];
    }
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      const int j = k * kScanBlock + t;
      tile[j + j / kScanItems] = base + j < n ? x[k] : 0u;
    }
  }
  __syncthreads();
  uint32_t vals[kScanItems];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    vals[k] = tile[t * kPad + k];
    acc += vals[k];
  }
  uint32_t tot;
  const uint32_t prefix = BlockExclusiveScan(acc, lds, &tot);
  const uint32_t b = blockIdx.x;
  if (t == 0) {
    __hip_atomic_store(&status[b], epoch_tag | (b == 0 ? kLbInclBit : 0) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (b == 0) s_excl = 0;
  }
  if (b > 0 && t < 64) {
    uint32_t excl = 0;
    int64_t j = static_cast<int64_t>(b) - 1;
    while (true) {
      const int64_t idx = j - lane;
      const uint64_t w = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (epoch_tag | kLbInclBit);
      const bool ready = (w & ~((kLbInclBit << 1) - 1)) == epoch_tag;
      const unsigned long long incl = __ballot(ready && (w & kLbInclBit));
      const unsigned long long notready = __ballot(!ready);
      const int fi = incl ? __ffsll(static_cast<long long>(incl)) - 1 : 64;
      const unsigned long long need = fi == 64 ? ~0ULL : ((2ULL << fi) - 1);
      if (notready & need) continue;  // a predecessor has not published: read the window again
      uint32_t v = lane <= fi ? static_cast<uint32_t>(w) : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      excl += v;
      if (fi < 64) break;
      j -= 64;
    }
    if (lane == 0) {
      __hip_atomic_store(&status[b], epoch_tag | kLbInclBit | static_cast<uint32_t>(excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_excl = excl;
    }
  }
  __syncthreads();
  uint32_t run = prefix + s_excl;
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
  if (total && b == gridDim.x - 1 && t == kScanBlock - 1) *total = run;
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
// u32 scans of more than one tile take the single-pass look-back kernel.  Its status words live
// in the context's per-stream array (Ctx::scan_status), zeroed once when it is allocated, and
// carry a process-wide epoch that every scan advances.  So a word the kernel reads is either
// this scan's, an older scan's of this process (an older epoch: "not published"), or zero.
// Status words in the caller's scratch were not safe: device memory freed by another process
// (the GPU tests' rank processes) comes back with that process's words, whose epochs count from
// 1 as ours do, and a tile that read one as its predecessor's prefix got a wrong offset
// (a datagen append with non-monotone string offsets, 12 groups lost by a sharded C2 run).
constexpr int64_t kLbMaxTiles = 65536;  // 256M elements; larger scans keep the three-kernel path
static uint64_t* LbStatus(Ctx* ctx, hipStream_t stream) {
  const int i = stream == ctx->stream ? 0 : stream == ctx->side ? 1 : stream == ctx->side2 ? 2 : -1;
  if (i < 0) return nullptr;
  DevBuf& b = ctx->scan_status[i];
  if (!b.p) {
    if (b.Alloc(static_cast<size_t>(kLbMaxTiles) * 8) != PXG_OK) return nullptr;
    if (hipMemsetAsync(b.p, 0, b.bytes, stream) != hipSuccess) {  // ordered before every scan of this stream
      b.Free();
      return nullptr;
    }
  }
  return b.as<uint64_t>();
}

static int32_t ScanU32(Ctx* ctx, hipStream_t stream, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total, void* scratch) {
  const int64_t nblocks = (n + kScanTile - 1) / kScanTile;
  uint64_t* status = n > 0 && nblocks > 1 && nblocks <= kLbMaxTiles && !EnvFlag("PXG_SCAN_3PASS") ? LbStatus(ctx, stream) : nullptr;
  if (!status) return ScanImpl<uint32_t>(ctx, stream, in, out, n, total, static_cast<uint8_t*>(scratch));
  static std::atomic<uint32_t> g_epoch{0};
  uint32_t ep = (g_epoch.fetch_add(1, std::memory_order_relaxed) + 1) & 0x7FFFFFFFu;
  if (ep == 0) ep = (g_epoch.fetch_add(1, std::memory_order_relaxed) + 1) & 0x7FFFFFFFu;
  const uint64_t tag = static_cast<uint64_t>(ep) << 33;
  return LaunchOn(ctx, stream, "scan_lookback", ScanLookbackU32Kernel, dim3(static_cast<unsigned>(nblocks)), dim3(kScanBlock), 0, in, out,
                  n, total, status, tag);
}

int32_t ScanExclusiveU32(Ctx* ctx, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total, void* scratch) {
  return ScanU32(ctx, ctx->stream, in, out, n, total, scratch);
}

int32_t ScanExclusiveU32On(Ctx* ctx, hipStream_t stream, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total,
                           void* scratch) {
  return ScanU32(ctx, stream, in, out, n, total, scratch);
}

}  // namespace pxg
