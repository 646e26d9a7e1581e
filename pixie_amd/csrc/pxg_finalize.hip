// Agg finalize: group the staging records by slot (stable LSD radix sort), reduce each group
// (ConvertAggHashMapToRowBatch + UDA Finalize, agg_node.cc:303-349), build quantile digests and
// extract the group keys from the arena.
#include <cstdlib>
#include <algorithm>

#include "pxg_agg_host.h"
#include "pxg_keys.h"
#include "pxg_scan.h"
#include "pxg_sort.h"
#include "pxg_tdigest.h"

namespace pxg {

constexpr int kRadixBlock = 256;
constexpr int kRadixItems = 12;
constexpr int kRadixTile = kRadixBlock * kRadixItems;
constexpr int kRadixBits = 8;
constexpr int kRadixBuckets = 1 << kRadixBits;

struct ValPtrs {
  uint64_t* p[kMaxVals];
};
struct ConstValPtrs {
  const uint64_t* p[kMaxVals];
};

// Sort key of a staged record.  Pass 0 reads table slots and maps them through `rank` (slot ->
// dense group id; kDeferredSlot / empty -> G, which sorts last); later passes read dense ids.
__device__ __forceinline__ uint32_t DenseKey(uint32_t k, const uint32_t* __restrict__ rank, uint32_t cap, uint32_t G) {
  if (!rank) return k;
  return k < cap ? rank[k] : G;
}

__global__ void __launch_bounds__(kRadixBlock) RadixHistKernel(const uint32_t* __restrict__ keys, uint64_t n,
                                                               const uint32_t* __restrict__ rank, uint32_t cap, uint32_t G,
                                                               int shift, uint32_t* __restrict__ hist, uint32_t nblocks) {
  __shared__ uint32_t h[4][kRadixBuckets];
  uint32_t* hf = &h[0][0];
  for (int i = threadIdx.x; i < 4 * kRadixBuckets; i += kRadixBlock) hf[i] = 0;
  __syncthreads();
  const int wid = threadIdx.x >> 6;
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kRadixTile;
  // Every key load first, then every rank gather, then the counts: the tile's loads are all
  // in flight together.
  uint32_t kk[kRadixItems];
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = base + static_cast<uint64_t>(k) * kRadixBlock + threadIdx.x;
    kk[k] = i < n ? keys[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = base + static_cast<uint64_t>(k) * kRadixBlock + threadIdx.x;
    kk[k] = i < n ? DenseKey(kk[k], rank, cap, G) : 0u;
  }
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = base + static_cast<uint64_t>(k) * kRadixBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[wid][(kk[k] >> shift) & (kRadixBuckets - 1)], 1u);
  }
  __syncthreads();
  const int d = threadIdx.x;
  hist[static_cast<uint64_t>(d) * nblocks + blockIdx.x] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

// Wave-local LDS ordering for lanes of one wave exchanging data through LDS.
__device__ __forceinline__ void WaveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stable scatter.  Wave w of a block owns the contiguous quarter [w * 1024, (w + 1) * 1024) of
// the block's 4096-item tile, in (k, lane) order, so a wave's running per-digit counts live in
// its own LDS slice and need no block barrier inside the item loop: ranks within a wave come
// from an 8-ballot match of the digit bits.  The tile is then reordered by digit in LDS and
// written out in digit runs (consecutive threads -> consecutive addresses), instead of one
// scattered 4- or 8-byte store per item.
__global__ void __launch_bounds__(kRadixBlock) RadixScatterKernel(const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout,
                                                                  ConstValPtrs vin, ValPtrs vout, int nvals, uint64_t n,
                                                                  const uint32_t* __restrict__ rank, uint32_t cap, uint32_t G,
                                                                  int shift, const uint32_t* __restrict__ offs, uint32_t nblocks) {
  constexpr int kWaves = kRadixBlock / 64;
  constexpr int kPerWave = kRadixTile / kWaves;
  // 42 KB of LDS (3 blocks per CU): per-wave digit counts, turned in place into the tile-local
  // start of each (wave, digit); one 8-byte-per-item staging buffer that carries the keys,
  // then each value stream; the digit of every tile position.
  __shared__ uint32_t whist[kWaves][kRadixBuckets];
  __shared__ uint32_t dstart[kRadixBuckets];         // tile-local start of each digit
  __shared__ uint32_t gofs[kRadixBuckets];           // global start of this tile's digit run
  __shared__ uint64_t s_buf[kRadixTile];
  __shared__ uint8_t s_dig[kRadixTile];
  uint32_t* s_key = reinterpret_cast<uint32_t*>(s_buf);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  for (int d = lane; d < kRadixBuckets; d += 64) whist[wid][d] = 0;
  WaveSync();
  const uint64_t tile0 = static_cast<uint64_t>(blockIdx.x) * kRadixTile;
  const uint64_t wbase = tile0 + static_cast<uint64_t>(wid) * kPerWave;
  const int tn = static_cast<int>(min(static_cast<uint64_t>(kRadixTile), n - tile0));
  uint32_t part[kRadixItems], keys[kRadixItems], dig[kRadixItems];
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
    const bool valid = i < n;
    const uint32_t key = valid ? DenseKey(kin[i], rank, cap, G) : 0u;
    const uint32_t d = (key >> shift) & (kRadixBuckets - 1);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kRadixBits; ++b) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long m = __ballot(valid && bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t r = static_cast<uint32_t>(__popcll(peers & lanemask_lt));
    const uint32_t pre = valid ? whist[wid][d] : 0u;
    WaveSync();
    if (valid && r == 0) whist[wid][d] = pre + static_cast<uint32_t>(__popcll(peers));
    WaveSync();
    part[k] = pre + r;
    keys[k] = key;
    dig[k] = d;
  }
  __syncthreads();
  {
    const int d = threadIdx.x;  // kRadixBlock == kRadixBuckets
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += whist[w][d];
    // exclusive scan of the tile's digit totals (one digit per thread) through LDS
    dstart[d] = tot;
    __syncthreads();
    for (int o = 1; o < kRadixBuckets; o <<= 1) {
      const uint32_t x = d >= o ? dstart[d - o] : 0u;
      __syncthreads();
      dstart[d] += x;
      __syncthreads();
    }
    const uint32_t start = dstart[d] - tot;
    __syncthreads();
    dstart[d] = start;
    gofs[d] = offs[static_cast<uint64_t>(d) * nblocks + blockIdx.x];
    uint32_t acc = start;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {  // in place: whist[w][d] becomes the start of (w, d)
      const uint32_t c = whist[w][d];
      whist[w][d] = acc;
      acc += c;
    }
  }
  __syncthreads();
  uint32_t lpos[kRadixItems];
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    lpos[k] = whist[wid][dig[k]] + part[k];
    if (wbase + static_cast<uint64_t>(k) * 64 + lane < n) {
      s_key[lpos[k]] = keys[k];
      s_dig[lpos[k]] = static_cast<uint8_t>(dig[k]);
    }
  }
  __syncthreads();
  // Keys out in digit runs.
  for (int j = threadIdx.x; j < tn; j += kRadixBlock) {
    const uint32_t d = s_dig[j];
    kout[gofs[d] + (j - dstart[d])] = s_key[j];
  }
  // Each value stream through the same LDS reordering (the staging buffer is reused).
  for (int v = 0; v < nvals; ++v) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRadixItems; ++k) {
      const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
      if (i < n) s_buf[lpos[k]] = vin.p[v][i];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < tn; j += kRadixBlock) {
      const uint32_t d = s_dig[j];
      vout.p[v][gofs[d] + (j - dstart[d])] = s_buf[j];
    }
  }
}

// Dense group ids of the table's occupied slots, in slot order (rank = exclusive scan of the
// occupancy flags); gslot[rank] = slot.
__global__ void SlotFlagsKernel(const unsigned long long* __restrict__ slots, uint32_t cap, uint32_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) flags[i] = slots[i] != 0 ? 1u : 0u;
}
__global__ void SlotGslotKernel(const unsigned long long* __restrict__ slots, uint32_t cap, const uint32_t* __restrict__ rank,
                                uint32_t* __restrict__ gslot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap && slots[i] != 0) gslot[rank[i]] = i;
}

// Group starts straight from the sorted dense ids: the first index of every id (ids are dense,
// so no scan is needed); gstart[G] = the number of records with a valid group.
__global__ void GroupHeadsKernel(const uint32_t* __restrict__ keys, uint64_t n, uint32_t G, uint32_t* __restrict__ gstart) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  if (i == 0 || keys[i - 1] != k) gstart[k < G ? k : G] = static_cast<uint32_t>(i);
  if (i == n - 1 && k < G) gstart[G] = static_cast<uint32_t>(n);
}

// ---------------------------------------------------------------------------------------
// Per-group UDA reductions, two levels: one wave per chunk of <= kRedChunk rows of a group
// writes a partial state; one thread per group combines its chunks in order.  Balanced for
// any group-size skew (the largest C2 group holds ~6% of all rows).
// ---------------------------------------------------------------------------------------
constexpr uint32_t kRedChunk = 2048;

__device__ __forceinline__ uint64_t WaveSumU64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double WaveSumF64(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int64_t WaveMinI64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    int64_t x = __shfl_xor(v, o, 64);
    v = x < v ? x : v;
  }
  return v;
}
__device__ __forceinline__ int64_t WaveMaxI64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    int64_t x = __shfl_xor(v, o, 64);
    v = x > v ? x : v;
  }
  return v;
}

struct UdaOut {
  uint64_t* p[kMaxUdas];
};

__global__ void GroupChunkCountKernel(const uint32_t* __restrict__ gstart, uint32_t ngroups, uint32_t* __restrict__ cbase) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  cbase[g] = (gstart[g + 1] - gstart[g] + kRedChunk - 1) / kRedChunk;
}

// chunk -> group map (one thread per group writes its chunks), so a chunk's wave finds its
// group with one load instead of a binary search over cbase.
__global__ void ChunkGroupKernel(const uint32_t* __restrict__ cbase, uint32_t ngroups, uint32_t* __restrict__ cgroup) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  for (uint32_t c = cbase[g]; c < cbase[g + 1]; ++c) cgroup[c] = g;
}

// Partial state per (uda, chunk): SUM/MINSUM/MEAN = sum (int64 bits or double bits),
// MIN/MAX = order-preserving int64 of the extreme (NaN skipped), COUNT unused.
__global__ void __launch_bounds__(256) ChunkReduceKernel(const AggPlanDev* __restrict__ plan, const uint32_t* __restrict__ gstart,
                                                         const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ cgroup,
                                                         uint32_t ngroups, ConstValPtrs vals, uint64_t* __restrict__ partial,
                                                         uint64_t pstride) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nchunks = cbase[ngroups];
  if (w >= nchunks) return;
  const uint32_t g = cgroup[w];
  const uint32_t s = gstart[g] + (w - cbase[g]) * kRedChunk;
  const uint32_t e = min(gstart[g + 1], s + kRedChunk);
  for (int u = 0; u < plan->n_udas; ++u) {
    const int kind = plan->uda_kind[u];
    const int at = plan->uda_arg_type[u];
    const int vi = plan->uda_val[u];
    if (kind == PXG_UDA_COUNT || kind == PXG_UDA_QUANTILES) continue;
    const uint64_t* v = vals.p[vi];
    uint64_t r = 0;
    if (kind == PXG_UDA_MEAN_MERGE) {  // MeanUDA::Merge: sizes into the second partial row
      const uint64_t* sz = vals.p[plan->uda_val2[u]];
      double acc = 0;
      uint64_t n = 0;
      for (uint32_t i = s + lane; i < e; i += 64) {
        acc += AsF(v[i]);
        n += sz[i];
      }
      r = FBits(WaveSumF64(acc));
      n = WaveSumU64(n);
      if (lane == 0) partial[static_cast<uint64_t>(plan->n_udas + u) * pstride + w] = n;
    } else if (kind == PXG_UDA_SUM || kind == PXG_UDA_MINSUM || kind == PXG_UDA_MEAN) {
      if (at == PXG_FLOAT64) {
        double acc = 0;
        for (uint32_t i = s + lane; i < e; i += 64) acc += AsF(v[i]);
        r = FBits(WaveSumF64(acc));
      } else if (kind == PXG_UDA_MEAN) {
        double acc = 0;
        for (uint32_t i = s + lane; i < e; i += 64) acc += static_cast<double>(static_cast<int64_t>(v[i]));
        r = FBits(WaveSumF64(acc));
      } else {
        uint64_t acc = 0;
        for (uint32_t i = s + lane; i < e; i += 64) acc += v[i];
        r = WaveSumU64(acc);
      }
    } else if (kind == PXG_UDA_MAX) {
      int64_t m = INT64_MIN;
      if (at == PXG_FLOAT64) {
        for (uint32_t i = s + lane; i < e; i += 64) {
          const uint64_t x = v[i];
          if (!isnan(AsF(x))) { const int64_t o = OrderedFromDouble(x); m = o > m ? o : m; }
        }
      } else {
        for (uint32_t i = s + lane; i < e; i += 64) { const int64_t x = static_cast<int64_t>(v[i]); m = x > m ? x : m; }
      }
      r = static_cast<uint64_t>(WaveMaxI64(m));
    } else if (kind == PXG_UDA_MIN) {
      int64_t m = INT64_MAX;
      if (at == PXG_FLOAT64) {
        for (uint32_t i = s + lane; i < e; i += 64) {
          const uint64_t x = v[i];
          if (!isnan(AsF(x))) { const int64_t o = OrderedFromDouble(x); m = o < m ? o : m; }
        }
      } else {
        for (uint32_t i = s + lane; i < e; i += 64) { const int64_t x = static_cast<int64_t>(v[i]); m = x < m ? x : m; }
      }
      r = static_cast<uint64_t>(WaveMinI64(m));
    }
    if (lane == 0) partial[static_cast<uint64_t>(u) * pstride + w] = r;
  }
}

// UDA Finalize per group (math_ops.h: CountUDA/SumUDA/MeanUDA/MinUDA/MaxUDA).  With
// plan->emit_states every group's states are also written in Serialize() layout (partial agg).
__global__ void GroupCombineKernel(const AggPlanDev* __restrict__ plan, const uint32_t* __restrict__ gstart,
                                   const uint32_t* __restrict__ cbase, uint32_t ngroups, const uint64_t* __restrict__ partial,
                                   uint64_t pstride, UdaOut out, uint8_t* __restrict__ states) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const uint64_t cnt = gstart[g + 1] - gstart[g];
  const uint32_t c0 = cbase[g], c1 = cbase[g + 1];
  for (int u = 0; u < plan->n_udas; ++u) {
    const int kind = plan->uda_kind[u];
    const int at = plan->uda_arg_type[u];
    const uint64_t* p = partial + static_cast<uint64_t>(u) * pstride;
    uint64_t r = 0;
    switch (kind) {
      case PXG_UDA_COUNT: r = cnt; break;
      case PXG_UDA_SUM:
      case PXG_UDA_MINSUM:
        if (at == PXG_FLOAT64) {
          double acc = 0;
          for (uint32_t c = c0; c < c1; ++c) acc += AsF(p[c]);
          r = FBits(acc);
        } else {
          uint64_t acc = 0;
          for (uint32_t c = c0; c < c1; ++c) acc += p[c];
          r = acc + static_cast<uint64_t>(plan->uda_init[u]);
        }
        break;
      case PXG_UDA_MEAN: {
        double acc = 0;
        for (uint32_t c = c0; c < c1; ++c) acc += AsF(p[c]);
        r = FBits(acc / static_cast<double>(cnt));
        if (states) {  // MeanInfo {uint64 size; double count} (math_ops.h:621-624)
          uint64_t* st = reinterpret_cast<uint64_t*>(states + static_cast<uint64_t>(g) * plan->state_rec + plan->state_off[u]);
          st[0] = cnt;
          st[1] = FBits(acc);
        }
        break;
      }
      case PXG_UDA_MEAN_MERGE: {
        const uint64_t* pn = partial + static_cast<uint64_t>(plan->n_udas + u) * pstride;
        double acc = 0;
        uint64_t n = 0;
        for (uint32_t c = c0; c < c1; ++c) {
          acc += AsF(p[c]);
          n += pn[c];
        }
        r = FBits(acc / static_cast<double>(n));
        break;
      }
      case PXG_UDA_MAX: {
        int64_t m = at == PXG_FLOAT64 ? OrderedFromDouble(FBits(kDblMin)) : INT64_MIN;  // MaxUDA init numeric_limits<T>::min()
        for (uint32_t c = c0; c < c1; ++c) { const int64_t x = static_cast<int64_t>(p[c]); m = x > m ? x : m; }
        r = at == PXG_FLOAT64 ? DoubleFromOrdered(m) : static_cast<uint64_t>(m);
        break;
      }
      case PXG_UDA_MIN: {
        int64_t m = at == PXG_FLOAT64 ? OrderedFromDouble(FBits(kDblMax)) : INT64_MAX;
        for (uint32_t c = c0; c < c1; ++c) { const int64_t x = static_cast<int64_t>(p[c]); m = x < m ? x : m; }
        r = at == PXG_FLOAT64 ? DoubleFromOrdered(m) : static_cast<uint64_t>(m);
        break;
      }
      default: continue;  // QUANTILES: digest kernels
    }
    out.p[u][g] = r;
    // count, sum, min, max: the state is the finalized 8-byte value (math_ops.h:602-757).
    if (states && kind != PXG_UDA_MEAN)
      *reinterpret_cast<uint64_t*>(states + static_cast<uint64_t>(g) * plan->state_rec + plan->state_off[u]) = r;
  }
}

// ---------------------------------------------------------------------------------------
// Quantiles.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t QKey(uint64_t raw, int arg_type) {
  const uint64_t bits = arg_type == PXG_FLOAT64 ? raw : FBits(static_cast<double>(static_cast<int64_t>(raw)));
  return SortKeyF(bits);
}
__device__ __forceinline__ double QVal(uint64_t key) { return AsF(FromSortKeyF(key)); }

constexpr uint64_t kNegInfKey = 0x000FFFFFFFFFFFFFULL;  // SortKeyF(-inf) = ~0xFFF0... = 0x000F...F
constexpr uint64_t kPosInfKey = 0xFFF0000000000000ULL;  // SortKeyF(+inf) = 0x7FF0... ^ 0x8000...

// Size classes: 0 tiny (<= 64, one wave, registers), 1 small (<= 1024, one wave, LDS),
// 2 mid (<= 4096, one workgroup, LDS), 3 big (chunk sort + merge in HBM).
constexpr uint32_t kTinyMax = 64;
constexpr uint32_t kSmallMax = 1024;
constexpr int kNumClasses = 4;

__global__ void __launch_bounds__(256) ClassifyGroupsKernel(const uint32_t* __restrict__ gstart, uint32_t ngroups,
                                                            uint32_t* __restrict__ lists, uint32_t* __restrict__ counts,
                                                            uint32_t mid_max) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  int cls = -1;
  if (g < ngroups) {
    const uint32_t n = gstart[g + 1] - gstart[g];
    cls = n <= kTinyMax ? 0 : (n <= kSmallMax ? 1 : (n <= mid_max ? 2 : 3));
  }
  // Block-aggregated list appends: wave leaders reserve within the block in LDS, then one
  // global atomic per class per block (the four class counters are hot addresses).
  __shared__ uint32_t s_cnt[kNumClasses], s_base[kNumClasses];
  if (threadIdx.x < kNumClasses) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t wofs[kNumClasses];
  unsigned long long wm[kNumClasses];
#pragma unroll
  for (int c = 0; c < kNumClasses; ++c) {
    wm[c] = __ballot(cls == c);
    const int leader = wm[c] ? __ffsll(static_cast<long long>(wm[c])) - 1 : 0;
    uint32_t o = 0;
    if (wm[c] && lane == leader) o = atomicAdd(&s_cnt[c], static_cast<uint32_t>(__popcll(wm[c])));
    wofs[c] = __shfl(o, leader, 64);
  }
  __syncthreads();
  if (threadIdx.x < kNumClasses) s_base[threadIdx.x] = s_cnt[threadIdx.x] ? atomicAdd(&counts[threadIdx.x], s_cnt[threadIdx.x]) : 0u;
  __syncthreads();
#pragma unroll
  for (int c = 0; c < kNumClasses; ++c)
    if (cls == c) lists[static_cast<uint64_t>(c) * ngroups + s_base[c] + wofs[c] + __popcll(wm[c] & lanemask_lt)] = g;
}

__device__ __forceinline__ uint64_t BitonicStepWave(uint64_t x, int lane, int k, int j) {
  const uint64_t y = __shfl_xor(x, j, 64);
  const bool up = (lane & k) == 0;
  const bool lower = (lane & j) == 0;
  const uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
  return (lower == up) ? mn : mx;
}

// One wave per group with n <= 64: register bitonic sort, singleton digest.
__global__ void __launch_bounds__(256) QuantTinyKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nlist_p,
                                                       const uint32_t* __restrict__ gstart, const uint64_t* __restrict__ vals,
                                                       int arg_type, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint32_t li = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (li >= *nlist_p) return;
  const uint32_t g = list[li];
  const uint32_t s = gstart[g], n = gstart[g + 1] - s;
  uint64_t key = lane < static_cast<int>(n) ? QKey(vals[s + lane], arg_type) : ~0ULL;
  for (int k = 2; k <= 64; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) key = BitonicStepWave(key, lane, k, j);
  const bool valid = lane < static_cast<int>(n) && key >= kNegInfKey && key <= kPosInfKey;
  const bool neg_nan = lane < static_cast<int>(n) && key < kNegInfKey;
  const uint32_t lead = static_cast<uint32_t>(__popcll(__ballot(neg_nan)));
  const int64_t W = __popcll(__ballot(valid));
  double q = lane < 7 ? kQuantileQ[lane] : 0.0;
  // Every lane participates in the shuffles the value accessor performs.
  double res = 0;
  if (W == 0) {
    res = __longlong_as_double(0x7FF8000000000000LL);
  } else {
    auto val = [&](int64_t j) -> double { return QVal(__shfl(key, static_cast<int>(lead + j), 64)); };
    // Uniform-control version of SingletonQuantile: every lane evaluates with its own q.
    const double Wd = static_cast<double>(W);
    const double index = q * Wd;
    const double v0 = val(0);
    const double vlast = val(W - 1);
    const double mn = StdMin(kDblMax, v0);
    const double mx = StdMax(kDblMin, vlast);
    // lower_bound over cum(j) = j + 0.5 (j < W), cum(W) = W
    int64_t j = 0;
    if (index > W - 0.5) j = W;
    else { j = static_cast<int64_t>(ceil(index - 0.5)); if (j < 0) j = 0; }
    const int64_t jm1 = j > 0 ? j - 1 : 0;
    const int64_t jj = j < W ? j : W - 1;
    const double vjm1 = val(jm1);
    const double vj = val(jj);
    if (W == 1) {
      res = v0;
    } else if (index <= 0.5) {
      res = mn + 2.0 * index / 1.0 * (v0 - mn);
    } else if (j < W) {
      const double z1 = index - (static_cast<double>(j - 1) + 0.5);
      const double z2 = (static_cast<double>(j) + 0.5) - index;
      res = WeightedAverage(vjm1, z2, vj, z1);
    } else {
      const double z1 = index - Wd - 1.0 / 2.0;
      const double z2 = 1.0 / 2 - z1;
      res = WeightedAverage(vlast, z1, mx, z2);
    }
  }
  if (lane < 7) out[static_cast<uint64_t>(g) * 7 + lane] = res;
}


// One wave per group with 64 < n <= 1024: bitonic sort in the wave's LDS slice, singleton
// digest (W <= 1024 <= kSingletonMaxW).  Waves of a workgroup work on different groups and
// never meet at a barrier.
constexpr int kSmallWaves = 4;
__global__ void __launch_bounds__(256) QuantSmallKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nlist_p,
                                                        const uint32_t* __restrict__ gstart, const uint64_t* __restrict__ vals,
                                                        int arg_type, double* __restrict__ out) {
  __shared__ uint64_t keys[kSmallWaves][kSmallMax];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t li = blockIdx.x * kSmallWaves + wid;
  if (li >= *nlist_p) return;
  uint64_t* a = keys[wid];
  const uint32_t g = list[li];
  const uint32_t s = gstart[g];
  const int n = static_cast<int>(gstart[g + 1] - s);
  int P = 128;
  while (P < n) P <<= 1;
  uint64_t cv = 0, cneg = 0;
  for (int i = lane; i < P; i += 64) {
    uint64_t k = ~0ULL;
    if (i < n) {
      k = QKey(vals[s + i], arg_type);
      cv += (k >= kNegInfKey && k <= kPosInfKey) ? 1 : 0;
      cneg += k < kNegInfKey ? 1 : 0;
    }
    a[i] = k;
  }
  const int64_t W = static_cast<int64_t>(WaveSumU64(cv));
  const int64_t lead = static_cast<int64_t>(WaveSumU64(cneg));
  WaveSync();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = lane; t < (P >> 1); t += 64) {
        const int lo = 2 * t - (t & (j - 1));
        const int hi = lo + j;
        const uint64_t x = a[lo], y = a[hi];
        if ((x > y) == ((lo & k) == 0)) {
          a[lo] = y;
          a[hi] = x;
        }
      }
      WaveSync();
    }
  }
  if (lane < 7) {
    out[static_cast<uint64_t>(g) * 7 + lane] =
        W == 0 ? __longlong_as_double(0x7FF8000000000000LL)
               : SingletonQuantile(kQuantileQ[lane], W, [&](int64_t j) -> double { return QVal(a[lead + j]); });
  }
}

constexpr int kMidMax = 4096;
constexpr int kMidCentroids = 2048;

// ---------------------------------------------------------------------------------------
// Block merge sort of up to 16 * blockDim.x u64 keys in LDS (replaces the LDS bitonic sort:
// ~5x fewer LDS operations and 16 barriers instead of 78 for 4096 keys).  Each thread sorts
// 16 keys in registers with a bitonic network, then log2(P/16) rounds merge pairs of sorted
// runs: every thread finds its 16 outputs' start on the merge path (binary search) and merges
// them serially (ties from the left run first: stable).  The LDS array is padded by one key
// per 16 (PadIdx) so the thread-contiguous accesses spread over the banks.
// ---------------------------------------------------------------------------------------
constexpr int kMsIpt = 16;
__device__ __forceinline__ int PadIdx(int j) { return j + (j >> 4); }
constexpr int PaddedLen(int n) { return n + (n >> 4); }

__device__ __forceinline__ void CmpSwap(uint64_t& x, uint64_t& y) {
  const uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
  x = lo;
  y = hi;
}

__device__ __forceinline__ void SortNetwork16(uint64_t (&r)[kMsIpt]) {
#pragma unroll
  for (int k = 2; k <= kMsIpt; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < kMsIpt; ++i) {
        const int l = i ^ j;
        if (l > i) {
          if ((i & k) == 0) CmpSwap(r[i], r[l]);
          else CmpSwap(r[l], r[i]);
        }
      }
    }
  }
}

// Sorts a[0, P) (logical indices, PadIdx layout), P a power of two in [16, 16 * blockDim.x].
__device__ void BlockMergeSortLds(uint64_t* a, int P) {
  const int t = threadIdx.x;
  const bool act = t * kMsIpt < P;
  uint64_t r[kMsIpt];
  if (act) {
#pragma unroll
    for (int i = 0; i < kMsIpt; ++i) r[i] = a[PadIdx(t * kMsIpt + i)];
    SortNetwork16(r);
#pragma unroll
    for (int i = 0; i < kMsIpt; ++i) a[PadIdx(t * kMsIpt + i)] = r[i];
  }
  __syncthreads();
  for (int w = kMsIpt; w < P; w <<= 1) {
    if (act) {
      const int base = (t * kMsIpt) & ~(2 * w - 1);
      const int d = t * kMsIpt - base;
      const int A0 = base, B0 = base + w;
      int lo = d > w ? d - w : 0, hi = d < w ? d : w;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (!(a[PadIdx(B0 + d - 1 - mid)] < a[PadIdx(A0 + mid)])) lo = mid + 1;
        else hi = mid;
      }
      int ia = lo, ib = d - lo;
      uint64_t ka = ia < w ? a[PadIdx(A0 + ia)] : ~0ULL;
      uint64_t kb = ib < w ? a[PadIdx(B0 + ib)] : ~0ULL;
#pragma unroll
      for (int k = 0; k < kMsIpt; ++k) {
        const bool takeA = ib >= w || (ia < w && !(kb < ka));
        if (takeA) {
          r[k] = ka;
          ++ia;
          ka = ia < w ? a[PadIdx(A0 + ia)] : ~0ULL;
        } else {
          r[k] = kb;
          ++ib;
          kb = ib < w ? a[PadIdx(B0 + ib)] : ~0ULL;
        }
      }
    }
    __syncthreads();
    if (act) {
#pragma unroll
      for (int k = 0; k < kMsIpt; ++k) a[PadIdx(t * kMsIpt + k)] = r[k];
    }
    __syncthreads();
  }
}


// Lower bound of `key` in sorted a[0, n).
template <typename Acc>
__device__ __forceinline__ int64_t LowerBoundKey(Acc a, int64_t n, uint64_t key) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a(mid) < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Digest of a sorted key array accessible through `keyat` (block-cooperative).  Only the
// centroid means tdigest::quantile() reads are computed (<= 4 per quantile): a recording pass
// of DigestQuantile lists them (its control flow depends on positions only, never on means),
// then each is computed — the reference's incremental mean for centroids of <= kSeqMean
// values (every centroid while W <= ~10000), sum/count cooperatively for larger ones.
// Timing-only diagnosis (PXG_DIAG_QUANT): 1 skips the centroid-boundary chain, 2 skips the
// mid-group LDS sort.  Results are garbage when set; never set outside tools/.
__device__ int g_diag_quant = 0;

constexpr int kNeed = 7 * 4;
constexpr int64_t kSeqMean = 16;

struct DigestShared {
  int64_t meta[4];
  int32_t need[kNeed];
  double mean[kNeed];
  double red[4];
};

// Centroid boundaries precomputed by DigestChainKernel for a group assumed NaN-free (W = n);
// `starts` == nullptr: none.
struct PreChain {
  const uint32_t* starts;
  int64_t nc;
  int64_t W;
};

// Centroid-boundary chains (DigestBoundaries) of many groups at once, one thread per group:
// the chain is sequential per group (~1100 steps for any W > kSingletonMaxW), so running it
// inside each group's digest workgroup serialised the whole workgroup behind one lane.
constexpr int kChainCap = 2048;
// Chain slots: list a (mid groups) at [0, a_cap), list b (big groups) at [a_cap, ...).
__global__ void __launch_bounds__(64) DigestChainKernel(const uint32_t* __restrict__ list_a, const uint32_t* __restrict__ na_p,
                                                        uint32_t a_cap, const uint32_t* __restrict__ list_b,
                                                        const uint32_t* __restrict__ nb_p, const uint32_t* __restrict__ gstart,
                                                        uint32_t* __restrict__ starts_out, int32_t* __restrict__ nc_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t na = *na_p, nb = *nb_p;
  if (i < a_cap ? i >= na : i - a_cap >= nb) return;
  const uint32_t g = i < a_cap ? list_a[i] : list_b[i - a_cap];
  const int64_t W = gstart[g + 1] - gstart[g];
  nc_out[i] = W <= kSingletonMaxW ? -2 : static_cast<int32_t>(DigestBoundaries(W, starts_out + static_cast<uint64_t>(i) * kChainCap, kChainCap));
}

__device__ __forceinline__ PreChain PreChainAt(const uint32_t* starts_all, const int32_t* nc_all, uint32_t i, int64_t n) {
  PreChain p;
  p.starts = starts_all ? starts_all + static_cast<uint64_t>(i) * kChainCap : nullptr;
  p.nc = starts_all ? nc_all[i] : -1;
  p.W = n;
  return p;
}

template <typename KeyAt>
__device__ void BlockDigest(KeyAt keyat, int64_t n, uint32_t* starts_buf, int64_t max_c, PreChain pre, double* out7,
                            unsigned int* err, DigestShared& sh) {
  const int t = threadIdx.x;
  // trim NaNs: keys < kNegInfKey (negative NaN) at the front, > kPosInfKey at the back
  if (t == 0) {
    const int64_t lead = LowerBoundKey(keyat, n, kNegInfKey);
    const int64_t tail = LowerBoundKey(keyat, n, kPosInfKey + 1);
    sh.meta[0] = lead;
    sh.meta[1] = tail - lead;
  }
  __syncthreads();
  const int64_t lead = sh.meta[0], W = sh.meta[1];
  auto val = [&](int64_t j) -> double { return QVal(keyat(lead + j)); };
  if (W <= kSingletonMaxW) {
    if (t < 7) out7[t] = W == 0 ? __longlong_as_double(0x7FF8000000000000LL) : SingletonQuantile(kQuantileQ[t], W, val);
    __syncthreads();
    return;
  }
  const bool use_pre = pre.starts != nullptr && pre.W == W && pre.nc >= 0;
  const uint32_t* starts = use_pre ? pre.starts : starts_buf;
  if (t == 0) {
    int64_t nc;
    if (use_pre) nc = pre.nc;
    else nc = g_diag_quant == 1 ? (starts_buf[0] = 0, 1) : DigestBoundaries(W, starts_buf, max_c);
    if (nc < 0) atomicExch(err, 1u);
    sh.meta[2] = nc < 0 ? 0 : nc;
  }
  if (t < kNeed) sh.need[t] = -1;
  __syncthreads();
  const int64_t nc = sh.meta[2];
  auto start = [&](int64_t j) -> int64_t { return starts[j]; };
  auto cend = [&](int64_t j) -> int64_t { return j + 1 < nc ? starts[j + 1] : W; };
  if (t < 7) {
    int k = 0;
    (void)DigestQuantile(kQuantileQ[t], nc, W, start, [&](int64_t j) -> double {
      if (k < 4) sh.need[t * 4 + k] = static_cast<int32_t>(j);
      ++k;
      return 0.0;
    });
  }
  __syncthreads();
  if (t < kNeed && sh.need[t] >= 0) {
    const int64_t j = sh.need[t], s = start(j), e = cend(j);
    if (e - s <= kSeqMean) sh.mean[t] = CentroidMean(val, s, e);
  }
  for (int i = 0; i < kNeed; ++i) {  // uniform loop: large centroids, block sum
    const int64_t j = sh.need[i];
    if (j < 0) continue;
    const int64_t s = start(j), e = cend(j);
    if (e - s <= kSeqMean) continue;
    double acc = 0;
    for (int64_t x = s + t; x < e; x += blockDim.x) acc += val(x);
    acc = WaveSumF64(acc);
    if ((t & 63) == 0) sh.red[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
      double tot = 0;
      for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) tot += sh.red[w];
      sh.mean[i] = tot / static_cast<double>(e - s);
    }
    __syncthreads();
  }
  __syncthreads();
  if (t < 7) {
    int k = 0;
    out7[t] = DigestQuantile(kQuantileQ[t], nc, W, start, [&](int64_t) -> double {
      const double m = sh.mean[t * 4 + (k < 4 ? k : 3)];
      ++k;
      return m;
    });
  }
  __syncthreads();
}

// One workgroup per group with 1024 < n <= 4096: LDS bitonic sort + digest.
__global__ void __launch_bounds__(256) QuantMidKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ gstart,
                                                      const uint32_t* __restrict__ chain_starts, const int32_t* __restrict__ chain_nc,
                                                      const uint32_t* __restrict__ nlist_p, const uint64_t* __restrict__ vals,
                                                      int arg_type, double* __restrict__ out, unsigned int* __restrict__ err) {
  __shared__ uint64_t keys[PaddedLen(kMidMax)];
  __shared__ uint32_t starts[kMidCentroids];
  __shared__ DigestShared sh;
  if (blockIdx.x >= *nlist_p) return;
  const uint32_t g = list[blockIdx.x];
  const uint32_t s = gstart[g], n = gstart[g + 1] - s;
  int P = 64;
  while (P < static_cast<int>(n)) P <<= 1;
  for (int i = threadIdx.x; i < P; i += blockDim.x) keys[PadIdx(i)] = i < static_cast<int>(n) ? QKey(vals[s + i], arg_type) : ~0ULL;
  __syncthreads();
  if (g_diag_quant != 2) BlockMergeSortLds(keys, P);
  BlockDigest([&](int64_t i) -> uint64_t { return keys[PadIdx(static_cast<int>(i))]; }, n, starts, kMidCentroids,
              PreChainAt(chain_starts, chain_nc, blockIdx.x, n), out + static_cast<uint64_t>(g) * 7, err, sh);
}

// Big groups: chunk sort (one workgroup per 4096-element chunk) into sort keys.
struct BigChunk {
  uint64_t off;    // absolute staging offset of the chunk
  uint64_t g_off;  // absolute staging offset of its group
  uint32_t len;    // <= kMidMax
  uint32_t g_n;    // group size
  uint32_t passes; // merge passes the group needs (ceil(log2(g_n / kMidMax)))
  uint32_t pad;
};

__global__ void __launch_bounds__(256) BigChunkSortKernel(const BigChunk* __restrict__ chunks, const uint32_t* __restrict__ nchunks_p,
                                                          const uint64_t* __restrict__ vals, int arg_type, uint64_t* __restrict__ outk) {
  if (blockIdx.x >= *nchunks_p) return;
  __shared__ uint64_t keys[PaddedLen(kMidMax)];
  const BigChunk c = chunks[blockIdx.x];
  for (int i = threadIdx.x; i < kMidMax; i += blockDim.x) keys[PadIdx(i)] = i < static_cast<int>(c.len) ? QKey(vals[c.off + i], arg_type) : ~0ULL;
  __syncthreads();
  BlockMergeSortLds(keys, kMidMax);
  for (int i = threadIdx.x; i < static_cast<int>(c.len); i += blockDim.x) outk[c.off + i] = keys[PadIdx(i)];
}

struct BigGroup {
  uint64_t off;     // absolute staging offset of the group
  uint64_t n;
  uint64_t eoff;    // prefix of element counts (for the flattened launch)
  uint32_t g;
  uint32_t passes;  // merge passes it needs: its sorted keys end in keysA (even) / keysB (odd)
};

// Big-group metadata on the device (one block): per big group its offset, size and merge-pass
// count, and its 4096-key chunks; meta gets the chunk total and the largest group.
constexpr int kSetupBlock = 1024;
__global__ void __launch_bounds__(kSetupBlock) BigSetupKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                              const uint32_t* __restrict__ gstart, BigGroup* __restrict__ groups,
                                                              BigChunk* __restrict__ chunks, uint32_t* __restrict__ meta_out) {
  __shared__ uint32_t scan[kSetupBlock];
  __shared__ uint32_t s_max;
  const uint32_t nbig = *count;
  const int t = threadIdx.x;
  if (t == 0) s_max = 0;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nbig; b0 += kSetupBlock) {
    const uint32_t i = b0 + t;
    uint32_t g = 0, off = 0, n = 0, nch = 0;
    if (i < nbig) {
      g = list[i];
      off = gstart[g];
      n = gstart[g + 1] - off;
      nch = (n + kMidMax - 1) / kMidMax;
      atomicMax(&s_max, n);
    }
    scan[t] = nch;
    __syncthreads();
    for (int o = 1; o < kSetupBlock; o <<= 1) {
      const uint32_t x = t >= o ? scan[t - o] : 0u;
      __syncthreads();
      scan[t] += x;
      __syncthreads();
    }
    const uint32_t cbase = carry + scan[t] - nch;
    const uint32_t tot = scan[kSetupBlock - 1];
    __syncthreads();
    if (i < nbig) {
      uint32_t passes = 0;
      for (uint64_t r = kMidMax; r < n; r *= 2) ++passes;
      BigGroup B;
      B.off = off;
      B.n = n;
      B.eoff = 0;
      B.g = g;
      B.passes = passes;
      groups[i] = B;
      for (uint32_t c = 0; c < nch; ++c) {
        BigChunk C;
        C.off = static_cast<uint64_t>(off) + static_cast<uint64_t>(c) * kMidMax;
        C.g_off = off;
        C.len = min(static_cast<uint32_t>(kMidMax), n - c * kMidMax);
        C.g_n = n;
        C.passes = passes;
        C.pad = 0;
        chunks[cbase + c] = C;
      }
    }
    carry += tot;
  }
  __syncthreads();
  if (t == 0) {
    meta_out[0] = carry;  // total chunks
    meta_out[1] = s_max;  // largest big group
  }
}

// Merge-path split of diagonal d between sorted runs A[0,na) and B[0,nb) (ties: A first), by
// one wave: 64 probes per round, so ~log64(n) dependent global round trips instead of log2.
__device__ __forceinline__ int64_t WaveMergePath(const uint64_t* __restrict__ A, int64_t na, const uint64_t* __restrict__ B,
                                                 int64_t nb, int64_t d) {
  const int lane = threadIdx.x & 63;
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t i = lo + lane * step;
    // pred(i): the split lies above i  <=>  !(B[d-1-i] < A[i])
    const bool pr = i < hi && !(B[d - 1 - i] < A[i]);
    const int c = __popcll(__ballot(pr));
    const int64_t nlo = c > 0 ? lo + (c - 1) * step + 1 : lo;
    const int64_t nhi = lo + c * step < hi ? lo + c * step : hi;
    lo = nlo;
    hi = nhi;
  }
  return lo;
}

// One merge pass over big groups: runs of width w are merged pairwise; one workgroup makes
// one 4096-key output tile: its merge-path splits (wave searches), the two input slices
// staged into LDS with coalesced loads, then 16 outputs per thread by a serial LDS merge.
// Groups that are already sorted (passes <= pass) are skipped: their keys stay put.
__global__ void __launch_bounds__(256) BigMergeTileKernel(const BigChunk* __restrict__ chunks, const uint32_t* __restrict__ nchunks_p,
                                                          const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t w,
                                                          uint32_t pass) {
  if (blockIdx.x >= *nchunks_p) return;
  __shared__ uint64_t s[kMidMax];
  __shared__ int64_t s_split[2];
  const BigChunk c = chunks[blockIdx.x];
  if (c.passes <= pass) return;
  const int64_t n = c.g_n, j0 = static_cast<int64_t>(c.off - c.g_off), len = c.len;
  const int64_t pb = j0 & ~static_cast<int64_t>(2 * w - 1);
  const int64_t na = min(static_cast<int64_t>(w), n - pb);
  const int64_t nb = max(int64_t(0), min(static_cast<int64_t>(w), n - pb - static_cast<int64_t>(w)));
  const uint64_t* A = in + c.g_off + pb;
  const uint64_t* B = A + w;
  uint64_t* o = out + c.off;
  const int t = threadIdx.x;
  if (nb == 0) {
    for (int i = t; i < len; i += blockDim.x) o[i] = A[j0 - pb + i];
    return;
  }
  const int64_t d0 = j0 - pb, d1 = d0 + len;
  const int wid = t >> 6;
  if (wid < 2) {
    const int64_t sp = WaveMergePath(A, na, B, nb, wid == 0 ? d0 : d1);
    if ((t & 63) == 0) s_split[wid] = sp;
  }
  __syncthreads();
  const int64_t a0 = s_split[0], a1 = s_split[1];
  const int64_t b0 = d0 - a0, b1 = d1 - a1;
  const int la = static_cast<int>(a1 - a0), lb = static_cast<int>(b1 - b0);
  for (int i = t; i < la; i += blockDim.x) s[i] = A[a0 + i];
  for (int i = t; i < lb; i += blockDim.x) s[la + i] = B[b0 + i];
  __syncthreads();
  const int d = t * kMsIpt;
  if (d >= len) return;
  const uint64_t* SA = s;
  const uint64_t* SB = s + la;
  int lo = d > lb ? d - lb : 0, hi = d < la ? d : la;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (!(SB[d - 1 - mid] < SA[mid])) lo = mid + 1;
    else hi = mid;
  }
  int ia = lo, ib = d - lo;
  uint64_t ka = ia < la ? SA[ia] : ~0ULL;
  uint64_t kb = ib < lb ? SB[ib] : ~0ULL;
  const int cnt = len - d < kMsIpt ? static_cast<int>(len - d) : kMsIpt;
  for (int k = 0; k < cnt; ++k) {
    const bool takeA = ib >= lb || (ia < la && !(kb < ka));
    if (takeA) {
      o[d + k] = ka;
      ++ia;
      ka = ia < la ? SA[ia] : ~0ULL;
    } else {
      o[d + k] = kb;
      ++ib;
      kb = ib < lb ? SB[ib] : ~0ULL;
    }
  }
}


constexpr int kBigCentroids = 8192;

__global__ void __launch_bounds__(256) BigDigestKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ ngroups_p,
                                                       const uint64_t* __restrict__ keysA,
                                                       const uint64_t* __restrict__ keysB,
                                                       uint32_t* __restrict__ starts_all, const uint32_t* __restrict__ chain_starts,
                                                       const int32_t* __restrict__ chain_nc, double* __restrict__ out,
                                                       unsigned int* __restrict__ err) {
  __shared__ DigestShared sh;
  if (blockIdx.x >= *ngroups_p) return;
  const BigGroup G = groups[blockIdx.x];
  uint32_t* starts = starts_all + static_cast<uint64_t>(blockIdx.x) * kBigCentroids;
  const uint64_t* k = ((G.passes & 1) ? keysB : keysA) + G.off;
  BlockDigest([&](int64_t i) -> uint64_t { return k[i]; }, static_cast<int64_t>(G.n), starts, kBigCentroids,
              PreChainAt(chain_starts, chain_nc, blockIdx.x, static_cast<int64_t>(G.n)), out + static_cast<uint64_t>(G.g) * 7, err, sh);
}

// ---------------------------------------------------------------------------------------
// Keys out of the arena.
// ---------------------------------------------------------------------------------------
struct KeyOutDev {
  uint64_t* fixed[kMaxKeys];  // 8 B (16 B for UINT128) per group
  uint32_t* len[kMaxKeys];    // STRING lengths
};

__global__ void KeyExtractKernel(const AggPlanDev* __restrict__ plan, const uint32_t* __restrict__ gslot, uint32_t ngroups,
                                 const unsigned long long* __restrict__ slots, const uint64_t* __restrict__ arena, KeyOutDev ko) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const unsigned long long w = slots[gslot[g]];
  KeySet k;
  LoadKeysArena(plan, arena + static_cast<uint32_t>(w), k);
  for (int i = 0; i < plan->n_keys; ++i) {
    const int t = plan->key_types[i];
    if (t == PXG_STRING) {
      ko.len[i][g] = static_cast<uint32_t>(k.v[i].b);
    } else if (t == PXG_UINT128) {
      ko.fixed[i][2 * g] = k.v[i].a;
      ko.fixed[i][2 * g + 1] = k.v[i].b;
    } else if (t == PXG_BOOLEAN) {
      reinterpret_cast<uint8_t*>(ko.fixed[i])[g] = static_cast<uint8_t>(k.v[i].a);
    } else {
      ko.fixed[i][g] = k.v[i].a;
    }
  }
}

__global__ void KeyStringCopyKernel(const AggPlanDev* __restrict__ plan, int key, const uint32_t* __restrict__ gslot,
                                    uint32_t ngroups, const unsigned long long* __restrict__ slots,
                                    const uint64_t* __restrict__ arena, const uint32_t* __restrict__ offs,
                                    uint8_t* __restrict__ data) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const unsigned long long w = slots[gslot[g]];
  KeySet k;
  LoadKeysArena(plan, arena + static_cast<uint32_t>(w), k);
  const uint8_t* src = reinterpret_cast<const uint8_t*>(k.v[key].a);
  const uint32_t len = static_cast<uint32_t>(k.v[key].b);
  uint8_t* dst = data + offs[g];
  // 8-byte unaligned word copies (gfx950 serves unaligned global accesses), bytes for the tail.
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t x;
    __builtin_memcpy(&x, src + i, 8);
    __builtin_memcpy(dst + i, &x, 8);
  }
  for (; i < len; ++i) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------------
// Host orchestration.
// ---------------------------------------------------------------------------------------
static int Log2Ceil(uint64_t x) {
  int b = 0;
  while ((uint64_t(1) << b) < x) ++b;
  return b;
}

// meta: u64 [0] rows with a valid slot | u32 @8 groups | u32 @16 digest error | u32 @32.. class counts
__global__ void FinalizeInitKernel(uint8_t* meta, uint64_t n) {
  if (threadIdx.x == 0) {
    *reinterpret_cast<unsigned long long*>(meta) = n;
    *reinterpret_cast<uint32_t*>(meta + 8) = 0;
    *reinterpret_cast<uint32_t*>(meta + 16) = 0;
    for (int c = 0; c < kNumClasses; ++c) reinterpret_cast<uint32_t*>(meta + 32)[c] = 0;
  }
}

int32_t RadixSortPairs(Ctx* ctx, const uint32_t* keys, const uint32_t* rank, uint32_t cap, uint32_t G, const uint64_t* vals,
                       uint64_t n, RadixWs& ws, const uint32_t** skeys, const uint64_t** svals) {
  if (n == 0 || n >= (uint64_t(1) << 32)) return SetError(PXG_INVALID_ARGUMENT, "radix sort of %llu records", static_cast<unsigned long long>(n));
  const int nbits = std::max(1, Log2Ceil(static_cast<uint64_t>(G) + 1));
  const int passes = (nbits + kRadixBits - 1) / kRadixBits;
  const uint32_t nblocks = static_cast<uint32_t>((n + kRadixTile - 1) / kRadixTile);
  const uint64_t nh = static_cast<uint64_t>(kRadixBuckets) * nblocks;
  for (int b = 0; b < 2; ++b) {
    PXG_RETURN_IF_ERROR(ws.key[b].Ensure(n * 4 + 16));
    PXG_RETURN_IF_ERROR(ws.val[b].Ensure(n * 8 + 16));
  }
  PXG_RETURN_IF_ERROR(ws.hist.Ensure(nh * 4 + 64));
  PXG_RETURN_IF_ERROR(ws.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(nh + 1)) + 64));
  const uint32_t* kin = keys;
  ConstValPtrs vin;
  for (int v = 0; v < kMaxVals; ++v) vin.p[v] = nullptr;
  vin.p[0] = vals;
  int cur = 0;
  for (int p = 0; p < passes; ++p) {
    const int shift = p * kRadixBits;
    const uint32_t* rk = p == 0 ? rank : nullptr;
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_hist", RadixHistKernel, dim3(nblocks), dim3(kRadixBlock), 0, kin, n, rk, cap, G, shift,
                               ws.hist.as<uint32_t>(), nblocks));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, ws.hist.as<uint32_t>(), ws.hist.as<uint32_t>(), static_cast<int64_t>(nh), nullptr, ws.scan.p));
    ValPtrs vout;
    for (int v = 0; v < kMaxVals; ++v) vout.p[v] = nullptr;
    vout.p[0] = ws.val[cur].as<uint64_t>();
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scatter", RadixScatterKernel, dim3(nblocks), dim3(kRadixBlock), 0, kin, ws.key[cur].as<uint32_t>(),
                               vin, vout, 1, n, rk, cap, G, shift, ws.hist.as<const uint32_t>(), nblocks));
    kin = ws.key[cur].as<const uint32_t>();
    vin.p[0] = ws.val[cur].as<const uint64_t>();
    cur ^= 1;
  }
  *skeys = kin;
  *svals = vin.p[0];
  return PXG_OK;
}

int32_t GroupStarts(Ctx* ctx, const uint32_t* skeys, uint64_t n, uint32_t G, uint32_t* gstart) {
  return Launch(ctx, "group_heads", GroupHeadsKernel, dim3(GridFor(static_cast<int64_t>(n), 256, 1 << 30)), dim3(256), 0, skeys, n, G, gstart);
}

// Side streams forked by finalize are joined back into the main stream on every exit path, so
// an early error return never leaves side-stream kernels running on workspace buffers that a
// later reset / Ensure could free or reallocate.
struct SideJoinGuard {
  Ctx* ctx;
  bool side = false, side2 = false;
  ~SideJoinGuard() {
    if (side) (void)JoinSide(ctx);
    if (side2) (void)JoinSide2(ctx);
  }
};

int32_t AggFinalizeImpl(Agg* a) {
  Ctx* ctx = a->ctx;
  SideJoinGuard guard{ctx};
  HostClock clk;
  AggResult& R = a->res;
  Agg::FinalizeWs& ws = a->ws;
  R.Clear();
  const uint64_t n = a->st_n;
  if (n == 0) {
    R.ready = true;
    return PXG_OK;
  }
  if (n >= (uint64_t(1) << 32)) return SetError(PXG_UNIMPLEMENTED, "more than 2^32 staged rows in one aggregation");
  PXG_RETURN_IF_ERROR(ws.meta.Ensure(64));
  uint8_t* meta = ws.meta.as<uint8_t>();
  uint32_t* d_ngroups = reinterpret_cast<uint32_t*>(meta + 8);
  unsigned int* d_err = reinterpret_cast<unsigned int*>(meta + 16);
  uint32_t* d_cls = reinterpret_cast<uint32_t*>(meta + 32);
  {
    static const int diag = [] {
      const char* e = std::getenv("PXG_DIAG_QUANT");
      return e ? std::atoi(e) : 0;
    }();
    if (diag) PXG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_diag_quant), &diag, sizeof(int)));
  }
  PXG_RETURN_IF_ERROR(Launch(ctx, "finalize_init", FinalizeInitKernel, dim3(1), dim3(64), 0, meta, n));

  // 1. Dense group ids: rank of every occupied table slot (slot order).
  const uint32_t ngroups = static_cast<uint32_t>(a->inserted);
  R.n_groups = ngroups;
  if (ngroups == 0) {
    R.ready = true;
    return PXG_OK;
  }
  bool keys_on_side2 = false;
  PXG_RETURN_IF_ERROR(ws.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(std::max<uint64_t>(n, a->cap) + 1)) + 64));
  void* scan_tmp = ws.scan.p;
  PXG_RETURN_IF_ERROR(ws.rank.Ensure(static_cast<size_t>(a->cap) * 4 + 16));
  PXG_RETURN_IF_ERROR(ws.gslot.Ensure(static_cast<size_t>(ngroups) * 4));
  PXG_RETURN_IF_ERROR(Launch(ctx, "slot_flags", SlotFlagsKernel, dim3(GridFor(a->cap, 256, 1 << 30)), dim3(256), 0,
                             a->slots.as<const unsigned long long>(), a->cap, ws.rank.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, ws.rank.as<const uint32_t>(), ws.rank.as<uint32_t>(), a->cap, d_ngroups, scan_tmp));
  PXG_RETURN_IF_ERROR(Launch(ctx, "slot_gslot", SlotGslotKernel, dim3(GridFor(a->cap, 256, 1 << 30)), dim3(256), 0,
                             a->slots.as<const unsigned long long>(), a->cap, ws.rank.as<const uint32_t>(), ws.gslot.as<uint32_t>()));

  // Group keys out of the arena, on side stream 2 while the radix sort runs on the main
  // stream (ConvertAggHashMapToRowBatch group columns, agg_node.cc:303-349).  String payloads
  // are sized by the arena (an upper bound), so no count comes back to the host first.
  {
    KeyOutDev ko;
    for (int k = 0; k < kMaxKeys; ++k) {
      ko.fixed[k] = nullptr;
      ko.len[k] = nullptr;
    }
    for (int k = 0; k < a->n_keys; ++k) {
      const int t = a->key_types[k];
      if (t == PXG_STRING) {
        PXG_RETURN_IF_ERROR(R.key_offsets[k].Ensure((static_cast<size_t>(ngroups) + 1) * 4));
        PXG_RETURN_IF_ERROR(R.key_data[k].Ensure(static_cast<size_t>(a->arena_words) * 8 + 16));
        ko.len[k] = R.key_offsets[k].as<uint32_t>();
      } else {
        PXG_RETURN_IF_ERROR(R.key_fixed[k].Ensure(static_cast<size_t>(ngroups) * (t == PXG_UINT128 ? 16 : 8)));
        ko.fixed[k] = R.key_fixed[k].as<uint64_t>();
      }
    }
    if (a->n_keys > 0) {
      PXG_RETURN_IF_ERROR(ws.scan2.Ensure(ScanScratchBytes(static_cast<int64_t>(ngroups) + 1) + 64));
      PXG_RETURN_IF_ERROR(ForkSide2(ctx));
      guard.side2 = true;
      PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "key_extract", KeyExtractKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0,
                                   a->d_plan.as<const AggPlanDev>(), static_cast<const uint32_t*>(ws.gslot.as<uint32_t>()), ngroups,
                                   a->slots.as<const unsigned long long>(), a->arena.as<const uint64_t>(), ko));
      for (int k = 0; k < a->n_keys; ++k) {
        if (a->key_types[k] != PXG_STRING) continue;
        uint32_t* off = R.key_offsets[k].as<uint32_t>();
        PXG_RETURN_IF_ERROR(ScanExclusiveU32On(ctx, ctx->side2, off, off, ngroups, off + ngroups, ws.scan2.p));
        PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "key_string_copy", KeyStringCopyKernel, dim3(GridFor(ngroups, 256, 1 << 30)),
                                     dim3(256), 0, a->d_plan.as<const AggPlanDev>(), k,
                                     static_cast<const uint32_t*>(ws.gslot.as<uint32_t>()), ngroups,
                                     a->slots.as<const unsigned long long>(), a->arena.as<const uint64_t>(),
                                     static_cast<const uint32_t*>(R.key_offsets[k].as<uint32_t>()), R.key_data[k].as<uint8_t>()));
      }
      keys_on_side2 = true;
    }
  }

  // 2. Stable LSD radix sort of (dense id, vals...) by dense id (ceil(log2(G + 1) / 8) passes);
  //    records without a group (deferred slots) get id G and sort last.  The staging itself is
  //    left as it is (slots), so finalize can run again and export still works.
  const int nbits = std::max(1, Log2Ceil(static_cast<uint64_t>(ngroups) + 1));
  const int passes = (nbits + kRadixBits - 1) / kRadixBits;
  const uint32_t nblocks = static_cast<uint32_t>((n + kRadixTile - 1) / kRadixTile);
  for (int b = 0; b < 2; ++b) {
    PXG_RETURN_IF_ERROR(ws.skey[b].Ensure(n * 4 + 16));
    for (int v = 0; v < a->n_vals; ++v) PXG_RETURN_IF_ERROR(ws.sval[b][v].Ensure(n * 8 + 16));
  }
  const uint64_t nh = static_cast<uint64_t>(kRadixBuckets) * nblocks;
  PXG_RETURN_IF_ERROR(ws.hist.Ensure(nh * 4 + 64));
  PXG_RETURN_IF_ERROR(ws.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(std::max<uint64_t>(std::max<uint64_t>(nh, n), a->cap) + 1)) + 64));
  scan_tmp = ws.scan.p;
  const uint32_t* kin = a->st_slot.as<const uint32_t>();
  ConstValPtrs vin;
  for (int v = 0; v < kMaxVals; ++v) vin.p[v] = v < a->n_vals ? a->st_val[v].as<const uint64_t>() : nullptr;
  int cur = 0;
  for (int p = 0; p < passes; ++p) {
    const int shift = p * kRadixBits;
    const uint32_t* rank = p == 0 ? ws.rank.as<const uint32_t>() : nullptr;
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_hist", RadixHistKernel, dim3(nblocks), dim3(kRadixBlock), 0, kin, n, rank, a->cap, ngroups,
                               shift, ws.hist.as<uint32_t>(), nblocks));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, ws.hist.as<uint32_t>(), ws.hist.as<uint32_t>(), static_cast<int64_t>(nh), nullptr, scan_tmp));
    ValPtrs vout;
    for (int v = 0; v < kMaxVals; ++v) vout.p[v] = v < a->n_vals ? ws.sval[cur][v].as<uint64_t>() : nullptr;
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scatter", RadixScatterKernel, dim3(nblocks), dim3(kRadixBlock), 0, kin,
                               ws.skey[cur].as<uint32_t>(), vin, vout, a->n_vals, n, rank, a->cap, ngroups, shift,
                               ws.hist.as<const uint32_t>(), nblocks));
    kin = ws.skey[cur].as<const uint32_t>();
    for (int v = 0; v < kMaxVals; ++v) vin.p[v] = v < a->n_vals ? ws.sval[cur][v].as<const uint64_t>() : nullptr;
    cur ^= 1;
  }
  const uint32_t* skeys = kin;  // sorted dense ids; vin = the values in the same order
  // 3. Group starts (first index of every id).
  PXG_RETURN_IF_ERROR(ws.gstart.Ensure((static_cast<size_t>(ngroups) + 1) * 4));
  const uint32_t* gstart = ws.gstart.as<const uint32_t>();
  PXG_RETURN_IF_ERROR(Launch(ctx, "group_heads", GroupHeadsKernel, dim3(GridFor(static_cast<int64_t>(n), 256, 1 << 30)), dim3(256), 0,
                             skeys, n, ngroups, ws.gstart.as<uint32_t>()));
  // 3. UDA reductions (chunk partials, then per-group combine).
  const ConstValPtrs cv = vin;
  UdaOut uo;
  for (int u = 0; u < kMaxUdas; ++u) uo.p[u] = nullptr;
  bool any_q = false, any_red = false;
  for (int u = 0; u < a->n_udas; ++u) {
    const bool q = a->uda_kind[u] == PXG_UDA_QUANTILES;
    any_q |= q;
    any_red |= !q && a->uda_kind[u] != PXG_UDA_COUNT;
    PXG_RETURN_IF_ERROR(R.uda_out[u].Ensure(static_cast<size_t>(ngroups) * (q ? 7 * 8 : 8)));
    uo.p[u] = R.uda_out[u].as<uint64_t>();
  }
  PXG_RETURN_IF_ERROR(ws.cbase.Ensure((static_cast<size_t>(ngroups) + 1) * 4));
  uint32_t* cbase = ws.cbase.as<uint32_t>();
  const uint64_t max_chunks = static_cast<uint64_t>(ngroups) + n / kRedChunk + 1;
  // With quantiles, issued after the boundary chains are forked (they run in their shadow).
  auto RunReductions = [&]() -> int32_t {
  if (any_red) {
    PXG_RETURN_IF_ERROR(Launch(ctx, "group_chunk_count", GroupChunkCountKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0, gstart,
                               ngroups, cbase));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, cbase, cbase, ngroups, cbase + ngroups, scan_tmp));
    PXG_RETURN_IF_ERROR(ws.partial.Ensure(max_chunks * a->n_udas * 2 * 8));
    PXG_RETURN_IF_ERROR(ws.cgroup.Ensure(max_chunks * 4 + 16));
    PXG_RETURN_IF_ERROR(Launch(ctx, "chunk_group", ChunkGroupKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0,
                               static_cast<const uint32_t*>(cbase), ngroups, ws.cgroup.as<uint32_t>()));
    PXG_RETURN_IF_ERROR(Launch(ctx, "chunk_reduce", ChunkReduceKernel, dim3(static_cast<unsigned>((max_chunks * 64 + 255) / 256)), dim3(256), 0,
                               a->d_plan.as<const AggPlanDev>(), gstart, static_cast<const uint32_t*>(cbase),
                               ws.cgroup.as<const uint32_t>(), ngroups, cv, ws.partial.as<uint64_t>(), max_chunks));
  }
  uint8_t* states = nullptr;
  if (a->emit_states && a->state_rec > 0) {
    PXG_RETURN_IF_ERROR(R.states.Ensure(static_cast<size_t>(ngroups) * a->state_rec + 16));
    states = R.states.as<uint8_t>();
  }
  PXG_RETURN_IF_ERROR(Launch(ctx, "group_combine", GroupCombineKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0,
                             a->d_plan.as<const AggPlanDev>(), gstart, static_cast<const uint32_t*>(cbase), ngroups,
                             ws.partial.as<const uint64_t>(), max_chunks, uo, states));
  return PXG_OK;
  };
  if (!any_q) PXG_RETURN_IF_ERROR(RunReductions());
  // Big-group digests, after side stream 2's merges (see below).
  std::vector<int> big_pending;
  uint32_t n_big_groups = 0;
  const uint32_t* chain_starts_big = nullptr;
  const int32_t* chain_nc_big = nullptr;
  // On side stream 2, behind its merges; the boundary chains come from the side stream (its
  // join event was recorded before the mid digests were issued).
  auto RunBigDigests = [&]() -> int32_t {
    if (big_pending.empty()) return PXG_OK;
    PXG_HIP(hipStreamWaitEvent(ctx->side2, ctx->ev_join, 0));
    for (int u : big_pending) {
      PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "quant_big_digest", BigDigestKernel, dim3(n_big_groups), dim3(256), 0,
                                 ws.big.as<const BigGroup>(), static_cast<const uint32_t*>(d_cls + 3), ws.keysA.as<const uint64_t>(),
                                 ws.keysB.as<const uint64_t>(), ws.bstarts.as<uint32_t>(), chain_starts_big, chain_nc_big,
                                 R.uda_out[u].as<double>(), d_err));
    }
    big_pending.clear();
    return PXG_OK;
  };
  // 4. Quantile digests.
  if (any_q) {
    PXG_RETURN_IF_ERROR(ws.lists.Ensure(static_cast<size_t>(ngroups) * kNumClasses * 4));
    PXG_RETURN_IF_ERROR(Launch(ctx, "classify_groups", ClassifyGroupsKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0, gstart,
                               ngroups, ws.lists.as<uint32_t>(), d_cls, static_cast<uint32_t>(kMidMax)));
    const uint32_t* lists = ws.lists.as<const uint32_t>();
    // Big-group metadata on the device; one readback of the class counts, the big-group chunk
    // total and the largest group (grid sizes and the merge-pass count).
    const uint64_t big_cap = n / (kMidMax + 1) + 1;  // groups of > kMidMax rows
    const uint64_t chunk_cap = n / kMidMax + big_cap + 1;
    PXG_RETURN_IF_ERROR(ws.big.Ensure(big_cap * sizeof(BigGroup)));
    PXG_RETURN_IF_ERROR(ws.bchunks.Ensure(chunk_cap * sizeof(BigChunk)));
    uint32_t* d_bigmeta = reinterpret_cast<uint32_t*>(meta + 48);
    PXG_RETURN_IF_ERROR(Launch(ctx, "big_setup", BigSetupKernel, dim3(1), dim3(kSetupBlock), 0, lists + 3 * static_cast<uint64_t>(ngroups),
                               static_cast<const uint32_t*>(d_cls + 3), gstart, ws.big.as<BigGroup>(), ws.bchunks.as<BigChunk>(),
                               d_bigmeta));
    // Class counts + big-group metadata to pinned memory right away; the host waits on this
    // event only, while the digests below keep the GPU busy.
    uint8_t* pin = static_cast<uint8_t*>(ctx->pinned);
    PXG_HIP(hipMemcpyAsync(pin + 64, d_cls, 24, hipMemcpyDeviceToHost, ctx->stream));  // cls[4] @32, bigmeta[2] @48
    PXG_HIP(hipEventRecord(ctx->ev_meta, ctx->stream));
    // Kernels whose work lists are counted on the device launch right away with upper-bound
    // grids (blocks past the device count exit); the host reads the counts back only after
    // them, so the tiny / small digests and the boundary chains run while it waits.
    const uint32_t mid_cap = static_cast<uint32_t>(std::min<uint64_t>(ngroups, n / (kSmallMax + 1) + 1));
    const uint32_t big_cap32 = static_cast<uint32_t>(std::min<uint64_t>(ngroups, big_cap));
    const uint32_t n_chain_cap = mid_cap + big_cap32;
    PXG_RETURN_IF_ERROR(ws.chain_nc.Ensure(static_cast<size_t>(n_chain_cap) * 4));
    PXG_RETURN_IF_ERROR(ws.chain_starts.Ensure(static_cast<size_t>(n_chain_cap) * kChainCap * 4));
    const uint32_t* chain_starts = ws.chain_starts.as<const uint32_t>();
    const int32_t* chain_nc = ws.chain_nc.as<const int32_t>();
    // Chains: latency-bound (a few waves, ~1100 dependent steps each), on the side stream.
    PXG_RETURN_IF_ERROR(ForkSide(ctx));
    guard.side = true;
    PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side, "digest_chain", DigestChainKernel, dim3((n_chain_cap + 63) / 64), dim3(64), 0,
                                 lists + 2 * static_cast<uint64_t>(ngroups), static_cast<const uint32_t*>(d_cls + 2), mid_cap,
                                 lists + 3 * static_cast<uint64_t>(ngroups), static_cast<const uint32_t*>(d_cls + 3), gstart,
                                 ws.chain_starts.as<uint32_t>(), ws.chain_nc.as<int32_t>()));
    PXG_RETURN_IF_ERROR(RunReductions());
    const uint32_t small_cap = static_cast<uint32_t>(std::min<uint64_t>(ngroups, n / (kTinyMax + 1) + 1));
    for (int u = 0; u < a->n_udas; ++u) {
      if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
      const uint64_t* vals = cv.p[a->uda_val[u]];
      const int at = a->uda_arg_type[u];
      double* qo = R.uda_out[u].as<double>();
      PXG_RETURN_IF_ERROR(Launch(ctx, "quant_tiny", QuantTinyKernel, dim3((ngroups + 3) / 4), dim3(256), 0, lists,
                                 static_cast<const uint32_t*>(d_cls), gstart, vals, at, qo));
      PXG_RETURN_IF_ERROR(Launch(ctx, "quant_small", QuantSmallKernel, dim3((small_cap + kSmallWaves - 1) / kSmallWaves), dim3(256), 0,
                                 lists + static_cast<uint64_t>(ngroups), static_cast<const uint32_t*>(d_cls + 1), gstart, vals, at, qo));
    }
    uint32_t hm[6];
    clk.Mark("finalize: issue to meta");
    PXG_HIP(hipEventSynchronize(ctx->ev_meta));
    clk.Mark("finalize: meta wait");
    std::memcpy(hm, pin + 64, 24);
    uint32_t cls[kNumClasses] = {hm[0], hm[1], hm[2], hm[3]};
    const uint32_t n_big = cls[3], n_bchunks = hm[4];
    n_big_groups = n_big;
    chain_starts_big = chain_starts + static_cast<uint64_t>(mid_cap) * kChainCap;
    chain_nc_big = chain_nc + mid_cap;
    const uint64_t big_max = hm[5];
    if (n_big > 0) {
      PXG_RETURN_IF_ERROR(ws.keysA.Ensure(n * 8));
      PXG_RETURN_IF_ERROR(ws.keysB.Ensure(n * 8));
      PXG_RETURN_IF_ERROR(ws.bstarts.Ensure(static_cast<size_t>(n_big) * kBigCentroids * 4));
    }
    // Big groups: chunk sort + merge passes on side stream 2 (their late passes hold few
    // workgroups), overlapping the mid digests and the key output on the main stream; the big
    // digests join it at the end of finalize.  Each quantile UDA forks again, so its sorts
    // start after the previous UDA's big digest has read the shared key buffers.
    bool first_big = true;
    for (int u = 0; u < a->n_udas; ++u) {
      if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
      const uint64_t* vals = cv.p[a->uda_val[u]];
      const int at = a->uda_arg_type[u];
      if (n_big > 0) {
        // The first big path needs only what precedes the metadata readback (sorted values,
        // chunk list), so it starts alongside the tiny / small digests.
        if (first_big) PXG_HIP(hipStreamWaitEvent(ctx->side2, ctx->ev_meta, 0));
        else PXG_RETURN_IF_ERROR(ForkSide2(ctx));
        guard.side2 = true;
        first_big = false;
        PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "quant_big_chunk_sort", BigChunkSortKernel, dim3(n_bchunks), dim3(256), 0,
                                     ws.bchunks.as<const BigChunk>(), static_cast<const uint32_t*>(d_bigmeta), vals, at,
                                     ws.keysA.as<uint64_t>()));
        DevBuf* src = &ws.keysA;
        DevBuf* dst = &ws.keysB;
        uint32_t pass = 0;
        for (uint64_t w = kMidMax; w < big_max; w *= 2, ++pass) {
          PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "quant_big_merge", BigMergeTileKernel, dim3(n_bchunks), dim3(256), 0,
                                       ws.bchunks.as<const BigChunk>(), static_cast<const uint32_t*>(d_bigmeta),
                                       src->as<const uint64_t>(), dst->as<uint64_t>(), w, pass));
          std::swap(src, dst);
        }
      }
      PXG_RETURN_IF_ERROR(JoinSide(ctx));
      guard.side = false;
      double* qo = R.uda_out[u].as<double>();
      if (cls[2] > 0)
        PXG_RETURN_IF_ERROR(Launch(ctx, "quant_mid", QuantMidKernel, dim3(cls[2]), dim3(256), 0, lists + 2 * static_cast<uint64_t>(ngroups),
                                   gstart, chain_starts, chain_nc, static_cast<const uint32_t*>(d_cls + 2), vals, at, qo, d_err));
      if (n_big > 0) {
        big_pending.push_back(u);
        // A later quantile UDA reuses the key buffers: its digest must run before that UDA's sorts.
        bool more = false;
        for (int v = u + 1; v < a->n_udas; ++v) more = more || a->uda_kind[v] == PXG_UDA_QUANTILES;
        if (more) PXG_RETURN_IF_ERROR(RunBigDigests());
      }
    }
  }
  PXG_RETURN_IF_ERROR(RunBigDigests());
  if (keys_on_side2 || n_big_groups > 0) PXG_RETURN_IF_ERROR(JoinSide2(ctx));
  guard.side2 = false;
  // One sync for the digest error flag and every string-key total.
  std::vector<uint32_t> totals(kMaxKeys, 0);
  unsigned int err = 0;
  uint32_t* pin32 = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + 128);
  for (int k = 0; k < a->n_keys; ++k)
    if (a->key_types[k] == PXG_STRING)
      PXG_HIP(hipMemcpyAsync(pin32 + k, R.key_offsets[k].as<uint32_t>() + ngroups, 4, hipMemcpyDeviceToHost, ctx->stream));
  uint32_t g_dev = 0;
  PXG_HIP(hipMemcpyAsync(pin32 + kMaxKeys, d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipMemcpyAsync(pin32 + kMaxKeys + 1, d_ngroups, 4, hipMemcpyDeviceToHost, ctx->stream));
  clk.Mark("finalize: issue rest");
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  clk.Mark("finalize: final wait");
  for (int k = 0; k < a->n_keys; ++k)
    if (a->key_types[k] == PXG_STRING) totals[k] = pin32[k];
  err = pin32[kMaxKeys];
  g_dev = pin32[kMaxKeys + 1];
  if (err) return SetError(PXG_INTERNAL, "t-digest centroid capacity exceeded");
  if (g_dev != ngroups) return SetError(PXG_INTERNAL, "group table holds %u groups, host mirror says %u", g_dev, ngroups);
  for (int k = 0; k < a->n_keys; ++k)
    if (a->key_types[k] == PXG_STRING) R.key_data_len[k] = totals[k];
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  R.ready = true;
  return PXG_OK;
}

}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_agg_finalize(pxg_agg* agg, int64_t* n_groups) {
  if (!agg) return SetError(PXG_INVALID_ARGUMENT, "agg is null");
  PXG_RETURN_IF_ERROR(AggFinalizeImpl(&agg->impl));
  int64_t g = agg->impl.res.n_groups;
  if (agg->impl.n_keys == 0 && g == 0) g = 1;  // no-groups agg always emits one row
  if (n_groups) *n_groups = g;
  return PXG_OK;
}

// Finalize() of a freshly initialised UDA (math_ops.h:583-772): count 0, sum 0, mean 0/0 = NaN,
// min numeric_limits<T>::max(), max numeric_limits<T>::min(), minsum its init arg.
static uint64_t InitialFinalValue(int kind, int at, int64_t init) {
  double d = 0;
  uint64_t bits = 0;
  switch (kind) {
    case PXG_UDA_MINSUM: return static_cast<uint64_t>(init);
    case PXG_UDA_MEAN:
    case PXG_UDA_MEAN_MERGE: d = std::nan(""); std::memcpy(&bits, &d, 8); return bits;
    case PXG_UDA_MAX:
      if (at != PXG_FLOAT64) return static_cast<uint64_t>(INT64_MIN);
      d = 2.2250738585072014e-308;
      std::memcpy(&bits, &d, 8);
      return bits;
    case PXG_UDA_MIN:
      if (at != PXG_FLOAT64) return static_cast<uint64_t>(INT64_MAX);
      d = 1.7976931348623157e+308;
      std::memcpy(&bits, &d, 8);
      return bits;
    default: return 0;  // COUNT, SUM (0 and +0.0 share their bits)
  }
}

extern "C" int32_t pxg_agg_result(pxg_agg* agg, pxg_column_out* cols, int32_t n_cols) {
  if (!agg || !cols) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Agg& a = agg->impl;
  if (!a.res.ready) return SetError(PXG_FAILED_PRECONDITION, "pxg_agg_finalize has not run since the last consume");
  const int32_t n_val_cols = a.emit_states ? 1 : a.n_udas;
  if (n_cols != a.n_keys + n_val_cols) return SetError(PXG_INVALID_ARGUMENT, "expected %d result columns", a.n_keys + n_val_cols);
  const int64_t G = a.res.n_groups;
  const bool synth = a.n_keys == 0 && G == 0;  // AggregateGroupByNone over no rows
  const int64_t rows = synth ? 1 : G;
  for (int c = 0; c < n_cols; ++c) std::memset(&cols[c], 0, sizeof(cols[c]));
  for (int k = 0; k < a.n_keys; ++k) {
    pxg_column_out& o = cols[k];
    o.type = a.key_types[k];
    o.length = rows;
    if (o.type == PXG_STRING) {
      o.offsets = static_cast<int32_t*>(std::malloc((rows + 1) * 4));
      o.data = static_cast<uint8_t*>(std::malloc(a.res.key_data_len[k] + 16));
      o.data_len = a.res.key_data_len[k];
      if (G > 0) {
        PXG_HIP(hipMemcpy(o.offsets, a.res.key_offsets[k].p, (G + 1) * 4, hipMemcpyDeviceToHost));
        PXG_HIP(hipMemcpy(o.data, a.res.key_data[k].p, o.data_len, hipMemcpyDeviceToHost));
      } else {
        o.offsets[0] = 0;
      }
    } else {
      const size_t w = TypeWidth(o.type);
      o.values = std::malloc(std::max<size_t>(rows * w, 1));
      if (G > 0) {
        if (o.type == PXG_BOOLEAN) {
          PXG_HIP(hipMemcpy(o.values, a.res.key_fixed[k].p, G, hipMemcpyDeviceToHost));
        } else {
          PXG_HIP(hipMemcpy(o.values, a.res.key_fixed[k].p, G * w, hipMemcpyDeviceToHost));
        }
      }
    }
  }
  if (a.emit_states) {  // serialized_expressions: fixed-size records (operators.cc:251-257)
    pxg_column_out& o = cols[a.n_keys];
    o.type = PXG_STRING;
    o.length = rows;
    const int64_t rec = a.state_rec;
    o.offsets = static_cast<int32_t*>(std::malloc((rows + 1) * 4));
    o.data = static_cast<uint8_t*>(std::malloc(rows * rec + 16));
    o.data_len = rows * rec;
    for (int64_t g = 0; g <= rows; ++g) o.offsets[g] = static_cast<int32_t>(g * rec);
    if (!synth) {
      if (G > 0 && rec > 0) PXG_HIP(hipMemcpy(o.data, a.res.states.p, G * rec, hipMemcpyDeviceToHost));
    } else {
      // Initial states serialized (no-groups agg over zero rows): Mean {0, 0.0}, the rest as
      // their initial value.
      for (int u = 0; u < a.n_udas; ++u) {
        uint8_t* st = o.data + a.hplan.state_off[u];
        if (a.uda_kind[u] == PXG_UDA_MEAN) {
          std::memset(st, 0, 16);
        } else {
          const uint64_t v = InitialFinalValue(a.uda_kind[u], a.uda_arg_type[u], a.uda_init[u]);
          std::memcpy(st, &v, 8);
        }
      }
    }
    return PXG_OK;
  }
  for (int u = 0; u < a.n_udas; ++u) {
    pxg_column_out& o = cols[a.n_keys + u];
    o.type = a.uda_out_type[u];
    o.length = rows;
    const bool q = a.uda_kind[u] == PXG_UDA_QUANTILES;
    const size_t per = q ? 56 : 8;
    o.values = std::malloc(std::max<size_t>(rows * per, 8));
    if (!synth) {
      PXG_HIP(hipMemcpy(o.values, a.res.uda_out[u].p, G * per, hipMemcpyDeviceToHost));
      continue;
    }
    // Initial UDA states finalized (AggNode no-groups emit over zero rows, agg_node.cc:182-207).
    uint64_t* p = static_cast<uint64_t*>(o.values);
    if (q) {
      for (int j = 0; j < 7; ++j) { double nan = std::nan(""); std::memcpy(p + j, &nan, 8); }
    } else {
      p[0] = InitialFinalValue(a.uda_kind[u], a.uda_arg_type[u], a.uda_init[u]);
    }
  }
  return PXG_OK;
}
