// Agg finalize: group the staging records by slot (stable LSD radix sort), reduce each group
// (ConvertAggHashMapToRowBatch + UDA Finalize, agg_node.cc:303-349), build quantile digests and
// extract the group keys from the arena.
#include <cstdlib>
#include <algorithm>

#include "pxg_agg_host.h"
#include "pxg_keys.h"
#include "pxg_quant.h"
#include "pxg_scan.h"
#include "pxg_select.h"
#include "pxg_sort.h"
#include "pxg_tdigest.h"

namespace pxg {

// ---------------------------------------------------------------------------------------
// Per-group UDA reductions, two levels: one wave per chunk of <= kRedChunk rows of a group
// writes a partial state; one thread per group combines its chunks in order.  Balanced for
// any group-size skew (the largest C2 group holds ~6% of all rows).
// ---------------------------------------------------------------------------------------
constexpr uint32_t kRedChunk = 2048;

struct UdaOut {
  uint64_t* p[kMaxUdas];
};

__global__ void GroupChunkCountKernel(const uint32_t* __restrict__ gstart, uint32_t ngroups, uint32_t* __restrict__ cbase) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  cbase[g] = (gstart[g + 1] - gstart[g] + kRedChunk - 1) / kRedChunk;
}

// chunk -> group map: one thread per chunk finds its group by binary search over cbase (a thread
// per group writing its chunks left the largest group's thread ~3400 sequential stores at 1B rows).
__global__ void ChunkGroupKernel(const uint32_t* __restrict__ cbase, uint32_t ngroups, uint32_t* __restrict__ cgroup, uint32_t max_chunks) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= max_chunks || c >= cbase[ngroups]) return;
  uint32_t lo = 0, hi = ngroups;  // last g with cbase[g] <= c
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cbase[mid] <= c) lo = mid;
    else hi = mid;
  }
  cgroup[c] = lo;
}

// Partial rows per UDA: [u] the sum's high words (or the integer / extreme state), [n_udas + u]
// MEAN_MERGE sizes, [2 n_udas + u] the sum's low words.
constexpr int kPartialRows = 3;

// Partial state per (uda, chunk): SUM/MINSUM/MEAN = sum (int64 bits, or a double-double: high
// and low words), MIN/MAX = order-preserving int64 of the extreme (NaN skipped), COUNT unused.
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
      DD acc{0.0, 0.0};
      uint64_t n = 0;
      for (uint32_t i = s + lane; i < e; i += 64) {
        acc = DDAddD(acc, AsF(v[i]));
        n += sz[i];
      }
      acc = WaveSumDD(acc);
      r = FBits(acc.hi);
      n = WaveSumU64(n);
      if (lane == 0) {
        partial[static_cast<uint64_t>(plan->n_udas + u) * pstride + w] = n;
        partial[static_cast<uint64_t>(2 * plan->n_udas + u) * pstride + w] = FBits(acc.lo);
      }
    } else if (kind == PXG_UDA_SUM || kind == PXG_UDA_MINSUM || kind == PXG_UDA_MEAN) {
      if (at == PXG_FLOAT64 || kind == PXG_UDA_MEAN) {
        // Four loads in flight per lane (a dependent one-load loop left the pass latency-bound:
        // ~3 TB/s over the 1B-row staging), four partial sums added in a fixed order.
        const bool f64 = at == PXG_FLOAT64;
        auto dv = [f64](uint64_t x) { return f64 ? AsF(x) : static_cast<double>(static_cast<int64_t>(x)); };
        DD a0{0.0, 0.0}, a1{0.0, 0.0};
        uint32_t i = s + lane;
        for (; i + 192 < e; i += 256) {
          const uint64_t x0 = v[i], x1 = v[i + 64], x2 = v[i + 128], x3 = v[i + 192];
          a0 = DDAdd(a0, TwoSum(dv(x0), dv(x1)));
          a1 = DDAdd(a1, TwoSum(dv(x2), dv(x3)));
        }
        for (; i < e; i += 64) a0 = DDAddD(a0, dv(v[i]));
        const DD t = WaveSumDD(DDAdd(a0, a1));
        r = FBits(t.hi);
        if (lane == 0) partial[static_cast<uint64_t>(2 * plan->n_udas + u) * pstride + w] = FBits(t.lo);
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

// The same partial states with one thread per chunk and a sequential loop, for aggregations
// whose groups average a handful of rows (C3: ~2.4 rows per group over 5M groups), where a
// wave per chunk would leave 60 of its 64 lanes idle and pay six shuffle steps per UDA.
// Neighbouring threads take neighbouring groups, so their loads stay close to coalesced.
__global__ void __launch_bounds__(256) ChunkReduceThreadKernel(const AggPlanDev* __restrict__ plan, const uint32_t* __restrict__ gstart,
                                                               const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ cgroup,
                                                               uint32_t ngroups, ConstValPtrs vals, uint64_t* __restrict__ partial,
                                                               uint64_t pstride) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
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
    if (kind == PXG_UDA_MEAN_MERGE) {
      const uint64_t* sz = vals.p[plan->uda_val2[u]];
      DD acc{0.0, 0.0};
      uint64_t n = 0;
      for (uint32_t i = s; i < e; ++i) {
        acc = DDAddD(acc, AsF(v[i]));
        n += sz[i];
      }
      r = FBits(acc.hi);
      partial[static_cast<uint64_t>(plan->n_udas + u) * pstride + w] = n;
      partial[static_cast<uint64_t>(2 * plan->n_udas + u) * pstride + w] = FBits(acc.lo);
    } else if (kind == PXG_UDA_SUM || kind == PXG_UDA_MINSUM || kind == PXG_UDA_MEAN) {
      if (at == PXG_FLOAT64 || kind == PXG_UDA_MEAN) {
        const bool f64 = at == PXG_FLOAT64;
        DD acc{0.0, 0.0};
        for (uint32_t i = s; i < e; ++i) acc = DDAddD(acc, f64 ? AsF(v[i]) : static_cast<double>(static_cast<int64_t>(v[i])));
        r = FBits(acc.hi);
        partial[static_cast<uint64_t>(2 * plan->n_udas + u) * pstride + w] = FBits(acc.lo);
      } else {
        uint64_t acc = 0;
        for (uint32_t i = s; i < e; ++i) acc += v[i];
        r = acc;
      }
    } else if (kind == PXG_UDA_MAX) {
      int64_t m = INT64_MIN;
      for (uint32_t i = s; i < e; ++i) {
        const uint64_t x = v[i];
        if (at == PXG_FLOAT64) {
          if (!isnan(AsF(x))) { const int64_t o = OrderedFromDouble(x); m = o > m ? o : m; }
        } else {
          const int64_t y = static_cast<int64_t>(x);
          m = y > m ? y : m;
        }
      }
      r = static_cast<uint64_t>(m);
    } else if (kind == PXG_UDA_MIN) {
      int64_t m = INT64_MAX;
      for (uint32_t i = s; i < e; ++i) {
        const uint64_t x = v[i];
        if (at == PXG_FLOAT64) {
          if (!isnan(AsF(x))) { const int64_t o = OrderedFromDouble(x); m = o < m ? o : m; }
        } else {
          const int64_t y = static_cast<int64_t>(x);
          m = y < m ? y : m;
        }
      }
      r = static_cast<uint64_t>(m);
    }
    partial[static_cast<uint64_t>(u) * pstride + w] = r;
  }
}

// UDA Finalize per group (math_ops.h: CountUDA/SumUDA/MeanUDA/MinUDA/MaxUDA).  With
// plan->emit_states every group's states are also written in Serialize() layout (partial agg).
// One thread per group combines its chunk partials in order; a group of more than
// kCombineWaveChunks chunks is combined by its whole wave instead (lane i takes chunks i, i + 64,
// ..., then a fixed shuffle tree), so the largest groups (3400 chunks at 1B rows) are not one
// thread's chain of dependent loads (0.41 ms at 1B rows).  (Round 6: one wave for every group
// took group_combine 0.165 -> 0.078 ms at 1B rows, but the digests beside it slowed by more:
// N1 step 14.60 vs 14.56 ms, C2 2.123 -> 2.140 ms.)
constexpr uint32_t kCombineWaveChunks = 32;

// sum over c = cs, cs + step, ... < c1 of the double-doubles (p[c], plo[c]), added in c order (the
// same order as a plain loop, so bit-identical to it), with the loads of 8 chunks issued before
// their adds: a plain loop waited for each chunk's load before issuing the next.
__device__ __forceinline__ DD SumChunksDD(const uint64_t* __restrict__ p, const uint64_t* __restrict__ plo, uint32_t cs, uint32_t c1,
                                          uint32_t step) {
  constexpr int kB = 8;
  DD acc{0.0, 0.0};
  uint32_t c = cs;
  for (; c + (kB - 1) * step < c1; c += kB * step) {
    uint64_t hi[kB], lo[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      hi[j] = p[c + j * step];
      lo[j] = plo[c + j * step];
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) acc = DDAdd(acc, DD{AsF(hi[j]), AsF(lo[j])});
  }
  for (; c < c1; c += step) acc = DDAdd(acc, DD{AsF(p[c]), AsF(plo[c])});
  return acc;
}

template <bool WAVE>
__device__ __forceinline__ void CombineGroup(const AggPlanDev* __restrict__ plan, uint32_t g, uint64_t cnt, uint32_t c0, uint32_t c1,
                                             const uint64_t* __restrict__ partial, uint64_t pstride, UdaOut out,
                                             uint8_t* __restrict__ states) {
  const int lane = threadIdx.x & 63;
  const uint32_t cs = WAVE ? c0 + lane : c0, step = WAVE ? 64 : 1;
  const bool writer = !WAVE || lane == 0;
  for (int u = 0; u < plan->n_udas; ++u) {
    const int kind = plan->uda_kind[u];
    const int at = plan->uda_arg_type[u];
    const uint64_t* p = partial + static_cast<uint64_t>(u) * pstride;
    const uint64_t* plo = partial + static_cast<uint64_t>(2 * plan->n_udas + u) * pstride;  // sums' low words
    uint64_t r = 0;
    switch (kind) {
      case PXG_UDA_COUNT: r = cnt; break;
      case PXG_UDA_SUM:
      case PXG_UDA_MINSUM:
        if (at == PXG_FLOAT64) {
          DD acc = SumChunksDD(p, plo, cs, c1, step);
          if (WAVE) acc = WaveSumDD(acc);
          r = FBits(DDValue(acc));
        } else {
          uint64_t acc = 0;
          for (uint32_t c = cs; c < c1; c += step) acc += p[c];
          if (WAVE) acc = WaveSumU64(acc);
          r = acc + static_cast<uint64_t>(plan->uda_init[u]);
        }
        break;
      case PXG_UDA_MEAN: {
        DD dd = SumChunksDD(p, plo, cs, c1, step);
        if (WAVE) dd = WaveSumDD(dd);
        const double acc = DDValue(dd);
        r = FBits(acc / static_cast<double>(cnt));
        if (states && writer) {  // MeanInfo {uint64 size; double count} (math_ops.h:621-624)
          uint64_t* st = reinterpret_cast<uint64_t*>(states + static_cast<uint64_t>(g) * plan->state_rec + plan->state_off[u]);
          st[0] = cnt;
          st[1] = FBits(acc);
        }
        break;
      }
      case PXG_UDA_MEAN_MERGE: {
        const uint64_t* pn = partial + static_cast<uint64_t>(plan->n_udas + u) * pstride;
        DD dd{0.0, 0.0};
        uint64_t n = 0;
        for (uint32_t c = cs; c < c1; c += step) {
          dd = DDAdd(dd, DD{AsF(p[c]), AsF(plo[c])});
          n += pn[c];
        }
        if (WAVE) {
          dd = WaveSumDD(dd);
          n = WaveSumU64(n);
        }
        r = FBits(DDValue(dd) / static_cast<double>(n));
        break;
      }
      case PXG_UDA_MAX: {
        int64_t m = at == PXG_FLOAT64 ? OrderedFromDouble(FBits(kDblMin)) : INT64_MIN;  // MaxUDA init numeric_limits<T>::min()
        for (uint32_t c = cs; c < c1; c += step) { const int64_t x = static_cast<int64_t>(p[c]); m = x > m ? x : m; }
        if (WAVE) m = WaveMaxI64(m);
        r = at == PXG_FLOAT64 ? DoubleFromOrdered(m) : static_cast<uint64_t>(m);
        break;
      }
      case PXG_UDA_MIN: {
        int64_t m = at == PXG_FLOAT64 ? OrderedFromDouble(FBits(kDblMax)) : INT64_MAX;
        for (uint32_t c = cs; c < c1; c += step) { const int64_t x = static_cast<int64_t>(p[c]); m = x < m ? x : m; }
        if (WAVE) m = WaveMinI64(m);
        r = at == PXG_FLOAT64 ? DoubleFromOrdered(m) : static_cast<uint64_t>(m);
        break;
      }
      default: continue;  // QUANTILES: digest kernels
    }
    if (writer) {
      out.p[u][g] = r;
      // count, sum, min, max: the state is the finalized 8-byte value (math_ops.h:602-757).
      if (states && kind != PXG_UDA_MEAN)
        *reinterpret_cast<uint64_t*>(states + static_cast<uint64_t>(g) * plan->state_rec + plan->state_off[u]) = r;
    }
  }
}

__global__ void GroupCombineKernel(const AggPlanDev* __restrict__ plan, const uint32_t* __restrict__ gstart,
                                   const uint32_t* __restrict__ cbase, uint32_t ngroups, const uint64_t* __restrict__ partial,
                                   uint64_t pstride, UdaOut out, uint8_t* __restrict__ states) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = g < ngroups;
  const uint32_t c0 = valid ? cbase[g] : 0, c1 = valid ? cbase[g + 1] : 0;
  const uint64_t cnt = valid ? gstart[g + 1] - gstart[g] : 0;
  const bool wide = valid && c1 - c0 > kCombineWaveChunks;
  if (valid && !wide) CombineGroup<false>(plan, g, cnt, c0, c1, partial, pstride, out, states);
  unsigned long long wm = __ballot(wide);
  while (wm) {  // wave-uniform loop over the wave's wide groups
    const int src = __ffsll(static_cast<long long>(wm)) - 1;
    wm &= wm - 1;
    CombineGroup<true>(plan, __shfl(g, src, 64), __shfl(cnt, src, 64), __shfl(c0, src, 64), __shfl(c1, src, 64), partial, pstride, out,
                       states);
  }
}

// ---------------------------------------------------------------------------------------
// Quantiles.
// ---------------------------------------------------------------------------------------
// Size classes: 0 tiny (<= 64, one wave, registers), 1 small (<= 1024, one wave, LDS),
// 2 mid (<= 4096, one workgroup, LDS), 3 big (chunk sort + merge in HBM).
constexpr uint32_t kTinyMax = 64;
constexpr uint32_t kSmallMax = 1024;
// Size classes: 0 tiny (<= 64), 1 small (<= 1024), 2 mid (<= 2048), 3 big (> mid_max), and the
// larger mid classes 4 (<= 4096), 5 (<= 8192), 6 (<= 16384; empty while kMidClassMax is 8192):
// one LDS-sort workgroup per group, sized per class (QuantMidKernel<kMaxN>).  Counters of classes 0-3 at meta + 32, of 4-6 at
// meta + 64; lists[c * G ..] per class.
constexpr int kNumClasses = 4;
constexpr int kNumMidSub = 3;
constexpr int kAllClasses = kNumClasses + kNumMidSub;
// Groups above take the selection path (export: 4096).  8192: an LDS sort of a 4K-8K-value
// group costs half of its selection path (tools/quant_class_bench.py: 15M values in 6000-value
// groups 0.40 vs ~0.80 ms); at 8K-16K the two cost about the same and the 1024-thread sort ran
// on the critical stream (1B rows: 0.77 ms), so those groups stay on the selection path.
constexpr uint32_t kMidClassMax = 8192;
__device__ __forceinline__ int SizeClass(uint32_t n, uint32_t mid_max) {
  if (n > mid_max) return 3;
  return n <= kTinyMax ? 0 : n <= kSmallMax ? 1 : n <= 2048 ? 2 : n <= 4096 ? 4 : n <= 8192 ? 5 : 6;
}

// skip_flags (merged exchange): groups whose slot's flags word (macc, words per slot, last word)
// has the digest flag get no class; their quantiles come from the merged digest instead.
__global__ void __launch_bounds__(256) ClassifyGroupsKernel(const uint32_t* __restrict__ gstart, uint32_t ngroups,
                                                            uint32_t* __restrict__ lists, uint32_t* __restrict__ counts,
                                                            uint32_t* __restrict__ counts_mid, uint32_t mid_max,
                                                            const uint64_t* __restrict__ skip_flags, int flag_words,
                                                            const uint32_t* __restrict__ gslot, uint32_t early_from) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  int cls = -1;
  if (g < ngroups) {
    const uint32_t n = gstart[g + 1] - gstart[g];
    cls = SizeClass(n, mid_max);
    if (cls == 3 && g >= early_from) cls = -1;  // a designated big group: the early set serves it
    if (skip_flags && (skip_flags[static_cast<uint64_t>(gslot[g]) * flag_words + flag_words - 1] & 1ULL)) cls = -1;
  }
  // Block-aggregated list appends: wave leaders reserve within the block in LDS, then one
  // global atomic per class per block (the class counters are hot addresses).
  __shared__ uint32_t s_cnt[kAllClasses], s_base[kAllClasses];
  if (threadIdx.x < kAllClasses) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t wofs[kAllClasses];
  unsigned long long wm[kAllClasses];
#pragma unroll
  for (int c = 0; c < kAllClasses; ++c) {
    wm[c] = __ballot(cls == c);
    const int leader = wm[c] ? __ffsll(static_cast<long long>(wm[c])) - 1 : 0;
    uint32_t o = 0;
    if (wm[c] && lane == leader) o = atomicAdd(&s_cnt[c], static_cast<uint32_t>(__popcll(wm[c])));
    wofs[c] = __shfl(o, leader, 64);
  }
  __syncthreads();
  if (threadIdx.x < kAllClasses) {
    uint32_t* ctr = threadIdx.x < kNumClasses ? &counts[threadIdx.x] : &counts_mid[threadIdx.x - kNumClasses];
    s_base[threadIdx.x] = s_cnt[threadIdx.x] ? atomicAdd(ctr, s_cnt[threadIdx.x]) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < kAllClasses; ++c)
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


// One wave per group with 64 < n <= 1024: merge sort in the wave's LDS slice (WaveMergeSortLds),
// singleton digest (W <= 1024 <= kSingletonMaxW).  Waves of a workgroup work on
// different groups and never meet at a barrier.
constexpr int kSmallWaves = 4;
constexpr int kSmallPadded = kSmallMax + kSmallMax / 16;
__global__ void __launch_bounds__(256) QuantSmallKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nlist_p,
                                                        const uint32_t* __restrict__ gstart, const uint64_t* __restrict__ vals,
                                                        int arg_type, double* __restrict__ out) {
  __shared__ uint64_t keys[kSmallWaves][kSmallPadded];
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
  // The lane's loads (up to kSmallMax / 64) all issued before the first conversion: P / 64 is
  // uniform, so the guards are scalar branches and no load waits for the one before it.
  uint64_t raw[kSmallMax / 64];
#pragma unroll
  for (int k = 0; k < kSmallMax / 64; ++k)
    if (k * 64 < P) raw[k] = vals[s + min(lane + 64 * k, n - 1)];
#pragma unroll
  for (int k = 0; k < kSmallMax / 64; ++k) {
    if (k * 64 >= P) break;
    const int i = lane + 64 * k;
    uint64_t key = ~0ULL;
    if (i < n) {
      key = QKey(raw[k], arg_type);
      cv += (key >= kNegInfKey && key <= kPosInfKey) ? 1 : 0;
      cneg += key < kNegInfKey ? 1 : 0;
    }
    a[PadIdx(i)] = key;
  }
  const int64_t W = static_cast<int64_t>(WaveSumU64(cv));
  const int64_t lead = static_cast<int64_t>(WaveSumU64(cneg));
  WaveSync();
  WaveMergeSortLds(a, P);
  if (lane < 7) {
    out[static_cast<uint64_t>(g) * 7 + lane] =
        W == 0 ? __longlong_as_double(0x7FF8000000000000LL)
               : SingletonQuantile(kQuantileQ[lane], W, [&](int64_t j) -> double { return QVal(a[PadIdx(static_cast<int>(lead + j))]); });
  }
}

// Centroid-boundary chains of many groups at once, one wave per group (DigestBoundariesWave:
// ~10 chain steps per round); the chain is sequential per group (~1000-1200 steps for any
// W > kSingletonMaxW), so running it inside each group's digest workgroup serialised the
// whole workgroup behind it.
// Chain slots: list a (mid groups) at [0, a_cap), list b (big groups) at [a_cap, ...).
__global__ void __launch_bounds__(64 * kChainWaves) DigestChainKernel(const uint32_t* __restrict__ list_a, const uint32_t* __restrict__ na_p,
                                                                      uint32_t a_cap, const uint32_t* __restrict__ list_b,
                                                                      const uint32_t* __restrict__ nb_p, const uint32_t* __restrict__ gstart,
                                                                      uint32_t* __restrict__ starts_out, int32_t* __restrict__ nc_out) {
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t na = *na_p, nb = *nb_p;
  if (i < a_cap ? i >= na : i - a_cap >= nb) return;
  const uint32_t g = i < a_cap ? list_a[i] : list_b[i - a_cap];
  const int64_t W = gstart[g + 1] - gstart[g];
  const int32_t nc = W <= kSingletonMaxW ? -2 : static_cast<int32_t>(DigestBoundariesWave(W, starts_out + static_cast<uint64_t>(i) * kChainCap, kChainCap));
  if ((threadIdx.x & 63) == 0) nc_out[i] = nc;
}

// Boundary chains of every mid-class size W (kSingletonMaxW < W <= kMidMax).  A chain depends
// on W alone (DigestBoundaries never reads a value), so the table is built once per context
// (one wave per W, ~0.2 ms) and the mid digests index it by group size instead of waiting for
// the per-finalize chain kernel.  A group whose NaN-trimmed size differs from its row count
// builds its own chain in the digest (BlockDigest), as before.
constexpr int kMidChainW0 = kSingletonMaxW + 1;
constexpr int kMidChainN = static_cast<int>(kMidClassMax) - kSingletonMaxW;
__global__ void __launch_bounds__(256) MidChainTableKernel(uint32_t* __restrict__ starts, int32_t* __restrict__ nc) {
  const int i = static_cast<int>((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (i >= kMidChainN) return;
  const int64_t n = DigestBoundariesWave(static_cast<int64_t>(kMidChainW0 + i), starts + static_cast<uint64_t>(i) * kChainCap, kChainCap);
  if ((threadIdx.x & 63) == 0) nc[i] = static_cast<int32_t>(n);
}
__device__ __forceinline__ PreChain MidPreChain(const uint32_t* tab, const int32_t* tab_nc, int64_t n) {
  PreChain p;
  const bool in = n >= kMidChainW0 && n < kMidChainW0 + kMidChainN;
  p.starts = in ? tab + static_cast<uint64_t>(n - kMidChainW0) * kChainCap : nullptr;
  p.nc = in ? tab_nc[n - kMidChainW0] : -1;
  p.W = n;
  return p;
}

// One workgroup per group of a mid class (1024 < n <= 16384): LDS merge sort + digest, one
// launch per class, each workgroup sized to its class (kMaxN / 16 threads, kMaxN keys in LDS): a
// 256-thread workgroup left half its threads idle through the sort of a <= 2048-value group, and
// groups of 4K-16K values cost the selection path (sample, chain, plan, bin sorts per group)
// about twice what one LDS sort does (tools/quant_class_bench.py).
template <int kMaxN>
__global__ void __launch_bounds__(kMaxN / kMsIpt) QuantMidKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ gstart,
                                                                 const uint32_t* __restrict__ mid_starts, const int32_t* __restrict__ mid_nc,
                                                                 const uint32_t* __restrict__ nlist_p, const uint64_t* __restrict__ vals,
                                                                 int arg_type, double* __restrict__ out, unsigned int* __restrict__ err) {
  __shared__ uint64_t keys[PaddedLen(kMaxN)];
  __shared__ uint32_t starts[kMidCentroids];
  __shared__ DigestShared sh;
  if (blockIdx.x >= *nlist_p) return;
  const uint32_t g = list[blockIdx.x];
  const uint32_t s = gstart[g], n = gstart[g + 1] - s;
  int P = 64;
  while (P < static_cast<int>(n)) P <<= 1;
  {
    // All kMsIpt loads of a thread in flight before the first conversion (clamped rows: n >= 1);
    // a guarded load per loop step waited for each value before issuing the next.
    uint64_t raw[kMsIpt];
#pragma unroll
    for (int k = 0; k < kMsIpt; ++k) {
      const int i = threadIdx.x + k * (kMaxN / kMsIpt);
      raw[k] = vals[s + min(i, static_cast<int>(n) - 1)];
    }
#pragma unroll
    for (int k = 0; k < kMsIpt; ++k) {
      const int i = threadIdx.x + k * (kMaxN / kMsIpt);
      if (i < P) keys[PadIdx(i)] = i < static_cast<int>(n) ? QKey(raw[k], arg_type) : ~0ULL;
    }
  }
  __syncthreads();
  BlockMergeSortLds(keys, P);
  BlockDigest<true>([&](int64_t i) -> uint64_t { return keys[PadIdx(static_cast<int>(i))]; }, n, starts, kMidCentroids,
              MidPreChain(mid_starts, mid_nc, n), out + static_cast<uint64_t>(g) * 7, err, sh);
}

// The mid-class chain table of a context, built on the ctx stream on first use (every reader
// runs on that stream or after it).
static constexpr size_t kMidChainStartBytes = static_cast<size_t>(kMidChainN) * kChainCap * 4;
static int32_t EnsureMidChains(Ctx* ctx) {
  if (ctx->mid_chains.p) return PXG_OK;
  PXG_RETURN_IF_ERROR(ctx->mid_chains.Alloc(kMidChainStartBytes + static_cast<size_t>(kMidChainN) * 4));
  const int32_t rc = Launch(ctx, "mid_chain_table", MidChainTableKernel, dim3((kMidChainN + 3) / 4), dim3(256), 0,
                            ctx->mid_chains.as<uint32_t>(), reinterpret_cast<int32_t*>(ctx->mid_chains.as<uint8_t>() + kMidChainStartBytes));
  if (rc != PXG_OK) ctx->mid_chains.Free();
  return rc;
}
static const uint32_t* MidChainStarts(Ctx* ctx) { return ctx->mid_chains.as<const uint32_t>(); }
static const int32_t* MidChainNc(Ctx* ctx) {
  return reinterpret_cast<const int32_t*>(ctx->mid_chains.as<const uint8_t>() + kMidChainStartBytes);
}

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

// Big-group metadata on the device (one block): per big group its offset, size and merge-pass
// count, and its 4096-key chunks; meta gets the chunk total and the largest group.  large_list
// gets the indices of the groups above kSelLargeN values (any order) and large_cnt their count:
// the 512-thread / 70 KB splitter launch runs only those, instead of one block per big group
// that must find 70 KB of free LDS before it can exit.
constexpr int kSetupBlock = 1024;
__global__ void __launch_bounds__(kSetupBlock) BigSetupKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                              const uint32_t* __restrict__ gstart, BigGroup* __restrict__ groups,
                                                              BigChunk* __restrict__ chunks, uint32_t* __restrict__ meta_out,
                                                              uint32_t* __restrict__ large_list, uint32_t* __restrict__ large_cnt) {
  __shared__ uint32_t scan[kSetupBlock];
  __shared__ uint32_t s_off[kSetupBlock], s_n[kSetupBlock], s_pass[kSetupBlock];
  __shared__ uint32_t s_max, s_large;
  const uint32_t nbig = *count;
  const int t = threadIdx.x;
  if (t == 0) {
    s_max = 0;
    s_large = 0;
  }
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
    uint32_t passes = 0;
    for (uint64_t r = kMidMax; r < n; r *= 2) ++passes;
    if (i < nbig) {
      BigGroup B;
      B.off = off;
      B.n = n;
      B.c0 = cbase;
      B.nch = nch;
      B.g = g;
      B.passes = passes;
      groups[i] = B;
      if (n > kSelLargeN) large_list[atomicAdd(&s_large, 1u)] = i;
    }
    s_off[t] = off;
    s_n[t] = n;
    s_pass[t] = passes;
    __syncthreads();
    // The round's chunks, all threads together (one thread per group wrote up to ~1700 chunks of
    // the largest 1B-row group in a row): chunk c belongs to the group whose inclusive scan
    // first exceeds c.
    const uint32_t nvalid = min(static_cast<uint32_t>(kSetupBlock), nbig - b0);
    for (uint32_t c = t; c < tot; c += kSetupBlock) {
      uint32_t lo = 0, hi = nvalid - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (scan[mid] <= c) lo = mid + 1;
        else hi = mid;
      }
      const uint32_t j = lo, k = c - (scan[j] - (s_n[j] + kMidMax - 1) / kMidMax);
      BigChunk C;
      C.off = static_cast<uint64_t>(s_off[j]) + static_cast<uint64_t>(k) * kMidMax;
      C.g_off = s_off[j];
      C.len = min(static_cast<uint32_t>(kMidMax), s_n[j] - k * kMidMax);
      C.g_n = s_n[j];
      C.passes = s_pass[j];
      C.bidx = b0 + j;
      chunks[carry + c] = C;
    }
    __syncthreads();  // scan / s_* are rewritten by the next round
    carry += tot;
  }
  __syncthreads();
  if (t == 0) {
    meta_out[0] = carry;  // total chunks
    meta_out[1] = s_max;  // largest big group
    *large_cnt = s_large;
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

// Exchange export: the complete single-pass digest of a big group (what one rank ships for a
// group of more than 8 * delta values, oracle TDigest::FromValuesOnce): NaN trimmed, centroid
// boundaries from the precomputed chain (or the sequential one), every centroid's mean and
// weight -- the reference's incremental mean for centroids of <= kSeqMean values, sum / count
// above, as BlockDigest.  xcnt[b] = the centroid count, or -1 when the group ships its values.
constexpr int kXCentCap = kChainCap;
constexpr int64_t kXRawMax = 8000;  // 8 * delta
// 1024 threads per group: one group of several million values otherwise kept four waves
// streaming its large centroids alone (~1.2 ms of the export at 125M rows per rank).
constexpr int kCentListBlock = 1024;
__global__ void __launch_bounds__(kCentListBlock) CentroidListKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ ngroups_p,
                                                          const uint64_t* __restrict__ keysA, const uint64_t* __restrict__ keysB,
                                                          uint32_t* __restrict__ starts_all, const uint32_t* __restrict__ chain_starts,
                                                          const int32_t* __restrict__ chain_nc, uint64_t* __restrict__ xcent,
                                                          int32_t* __restrict__ xcnt) {
  __shared__ int64_t s_meta[3];
  if (blockIdx.x >= *ngroups_p) return;
  const BigGroup G = groups[blockIdx.x];
  const uint64_t* k = ((G.passes & 1) ? keysB : keysA) + G.off;
  const int64_t n = static_cast<int64_t>(G.n);
  const int t = threadIdx.x;
  auto keyat = [&](int64_t i) -> uint64_t { return k[i]; };
  if (t == 0) {
    const int64_t lead = LowerBoundKey(keyat, n, kNegInfKey);
    const int64_t tail = LowerBoundKey(keyat, n, kPosInfKey + 1);
    s_meta[0] = lead;
    s_meta[1] = tail - lead;
    s_meta[2] = -1;
  }
  __syncthreads();
  const int64_t lead = s_meta[0], W = s_meta[1];
  if (W <= kXRawMax) {
    if (t == 0) xcnt[blockIdx.x] = -1;
    return;
  }
  uint32_t* starts_buf = starts_all + static_cast<uint64_t>(blockIdx.x) * kBigCentroids;
  const PreChain pre = PreChainAt(chain_starts, chain_nc, blockIdx.x, n);
  const bool use_pre = pre.starts != nullptr && pre.W == W && pre.nc >= 0;
  const uint32_t* starts = use_pre ? pre.starts : starts_buf;
  if (t == 0) s_meta[2] = use_pre ? pre.nc : DigestBoundaries(W, starts_buf, kXCentCap);
  __syncthreads();
  const int64_t nc = s_meta[2];
  if (nc < 0 || nc > kXCentCap) {
    if (t == 0) xcnt[blockIdx.x] = -2;  // cannot happen for delta = 1000 (<= ~1600 centroids)
    return;
  }
  auto val = [&](int64_t j) -> double { return QVal(k[lead + j]); };
  uint64_t* out = xcent + static_cast<uint64_t>(blockIdx.x) * kXCentCap * 2;
  // Small centroids: one thread each, incremental means (Centroid::add order).
  for (int64_t j = t; j < nc; j += blockDim.x) {
    const int64_t s = starts[j], e = j + 1 < nc ? starts[j + 1] : W;
    if (e - s > kSeqMean) continue;
    out[2 * j] = FBits(CentroidMean(val, s, e));
    out[2 * j + 1] = static_cast<uint64_t>(e - s);
  }
  // Large centroids (thousands of values near the median of a multi-million-value group): one
  // wave each, coalesced loads and a fixed shuffle tree (a thread per centroid summed them
  // serially, ~2 ms per export at 125M rows per rank).
  const int lane = t & 63, wid = t >> 6, nw = static_cast<int>(blockDim.x >> 6);
  for (int64_t j = wid; j < nc; j += nw) {
    const int64_t s = starts[j], e = j + 1 < nc ? starts[j + 1] : W;
    if (e - s <= kSeqMean) continue;
    double acc = 0;
    for (int64_t x = s + lane; x < e; x += 64) acc += val(x);
    acc = WaveSumF64(acc);
    if (lane == 0) {
      out[2 * j] = FBits(acc / static_cast<double>(e - s));
      out[2 * j + 1] = static_cast<uint64_t>(e - s);
    }
  }
  if (t == 0) xcnt[blockIdx.x] = static_cast<int32_t>(nc);
}

// ---------------------------------------------------------------------------------------
// Merged digests (multi-GPU exchange).  An owner rank receives, per group, one
// contribution from every rank that holds rows of it: the raw values when that rank held at
// most 8 * delta of them (unprocessed), else the centroid list of its single-pass digest
// (processed).  The group's digest is tdigest's batch add (add(first, last), the multi-digest
// form of TDigest::merge, math_sketches.h:38): one k-way merge of the processed lists by mean,
// the raw values appended unprocessed, then -- since raw values are present or the merged list
// passes 2 * delta centroids -- one process(): sorted raw values merged in front of equal
// means, and the greedy pass with the q-scale limits over the total weight.  Restated against
// oracle/tdigest.h merge_batch (tests/test_digest_merge.py).
//
// Items of a group (contiguous after the finalize's grouping, in part order): value = the raw
// value (the UDA's argument type) or the centroid mean (double bits); wt = part << 48 | weight
// (weight 0 marks a raw value).  One 512-thread workgroup per merged group:
//   A. part segments;  B. raw runs sorted in LDS (NaN dropped, as add() drops it) and every run
//   copied to scratch as (sort key, weight);  C. pairwise stable merge rounds (left run first:
//   raw runs are listed first, so raw values precede equal centroid means, as inplace_merge
//   puts the unprocessed range first);  D/E. the greedy pass by one thread over LDS windows;
//   F/G. min / max as the merge tracks them, tdigest quantile() x7.
// ---------------------------------------------------------------------------------------
constexpr int kMergeThreads = 512;
constexpr int kMergeRawMax = kMergeThreads * kMsIpt;  // 8192: the largest raw run (8 * delta = 8000)
constexpr int kMergeOutCap = 4096;
constexpr int kMergeWin = 2048;
constexpr int kXParts = 64;
constexpr int kWtPartShift = 48;
constexpr uint64_t kWtMask = (uint64_t(1) << kWtPartShift) - 1;
constexpr int64_t kMaxProcessed = 2000;  // 2 * ceil(delta): a merged list above this is processed

__device__ __forceinline__ int64_t MergePathSplit(const uint64_t* __restrict__ A, int64_t na, const uint64_t* __restrict__ B, int64_t nb,
                                                  int64_t d) {
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (!(B[d - 1 - mid] < A[mid])) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(kMergeThreads) DigestMergeKernel(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nlist_p,
                                                                   const uint32_t* __restrict__ gstart, const uint64_t* __restrict__ vals,
                                                                   const uint64_t* __restrict__ wt, int arg_type, uint64_t* __restrict__ mk0,
                                                                   uint64_t* __restrict__ mw0, uint64_t* __restrict__ mk1,
                                                                   uint64_t* __restrict__ mw1, double* __restrict__ out,
                                                                   unsigned int* __restrict__ err) {
  __shared__ uint64_t s_keys[PaddedLen(kMergeRawMax)];  // raw-run sort; then the greedy windows
  __shared__ double s_mean[kMergeOutCap];
  __shared__ int64_t s_start[kMergeOutCap];
  __shared__ int64_t s_seg[kXParts];
  __shared__ int64_t s_run[kXParts + 1];
  __shared__ int64_t s_cnt[2];
  __shared__ uint64_t s_wred[kMergeThreads / 64];
  __shared__ int s_nruns, s_nc;
  __shared__ int64_t s_cursor, s_ncent, s_nraw;
  __shared__ double s_mn, s_mx;
  if (blockIdx.x >= *nlist_p) return;
  const uint32_t g = list[blockIdx.x];
  const int64_t s = gstart[g], e = gstart[g + 1];
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  // A. first item of every part present
  for (int p = t; p < kXParts; p += kMergeThreads) s_seg[p] = -1;
  __syncthreads();
  for (int64_t i = s + t; i < e; i += kMergeThreads) {
    const uint64_t p = wt[i] >> kWtPartShift;
    if (i == s || (wt[i - 1] >> kWtPartShift) != p) s_seg[p & (kXParts - 1)] = i;
  }
  if (t == 0) {
    s_cursor = s;
    s_nruns = 0;
    s_ncent = 0;
    s_nraw = 0;
    s_mn = kDblMax;
    s_mx = kDblMin;
  }
  __syncthreads();
  // B. raw parts first (each sorted in LDS, NaN dropped), then centroid parts, into (mk0, mw0).
  for (int pass = 0; pass < 2; ++pass) {
    for (int p = 0; p < kXParts; ++p) {
      const int64_t lo = s_seg[p];
      if (lo < 0) continue;
      int64_t hi = e;
      for (int q = p + 1; q < kXParts; ++q)
        if (s_seg[q] >= 0) {
          hi = s_seg[q];
          break;
        }
      const bool raw = (wt[lo] & kWtMask) == 0;
      if (raw != (pass == 0)) continue;
      const int64_t n = hi - lo;
      const int64_t at = s_cursor;
      if (raw) {
        if (n > kMergeRawMax) {
          if (t == 0) atomicOr(err, 4u);
          continue;
        }
        int P = 16;
        while (P < n) P <<= 1;
        for (int i = t; i < P; i += kMergeThreads) s_keys[PadIdx(i)] = i < n ? QKey(vals[lo + i], arg_type) : ~0ULL;
        if (t < 2) s_cnt[t] = 0;
        __syncthreads();
        MergeSortLds<false>(s_keys, P, t);
        // NaN keys sort below -inf (negative NaN) and above +inf: count them, keep the rest
        for (int i = t; i < n; i += kMergeThreads) {
          const uint64_t k = s_keys[PadIdx(i)];
          if (k < kNegInfKey) atomicAdd(reinterpret_cast<unsigned long long*>(&s_cnt[0]), 1ULL);
          else if (k > kPosInfKey) atomicAdd(reinterpret_cast<unsigned long long*>(&s_cnt[1]), 1ULL);
        }
        __syncthreads();
        const int64_t lead = s_cnt[0], keep = n - s_cnt[0] - s_cnt[1];
        for (int64_t i = t; i < keep; i += kMergeThreads) {
          mk0[at + i] = s_keys[PadIdx(static_cast<int>(lead + i))];
          mw0[at + i] = 1;
        }
        __syncthreads();
        if (t == 0 && keep > 0) {
          s_run[s_nruns++] = at;
          s_cursor = at + keep;
          s_nraw += keep;
        }
      } else {
        for (int64_t i = t; i < n; i += kMergeThreads) {
          mk0[at + i] = SortKeyF(vals[lo + i]);
          mw0[at + i] = wt[lo + i] & kWtMask;
        }
        if (t == 0) {
          s_run[s_nruns++] = at;
          s_cursor = at + n;
          s_ncent += n;
          s_mn = StdMin(s_mn, AsF(vals[lo]));
          s_mx = StdMax(s_mx, AsF(vals[hi - 1]));
        }
      }
      __syncthreads();
    }
  }
  if (t == 0) s_run[s_nruns] = s_cursor;
  __syncthreads();
  const int64_t end = s_cursor;
  // C. pairwise stable merge rounds
  uint64_t *ks = mk0, *ws = mw0, *kd = mk1, *wd = mw1;
  int R = s_nruns;
  while (R > 1) {
    for (int j = 0; 2 * j < R; ++j) {
      const int64_t a0 = s_run[2 * j], a1 = s_run[2 * j + 1];
      const int64_t b1 = 2 * j + 1 < R ? s_run[2 * j + 2] : a1;
      const int64_t na = a1 - a0, nb = b1 - a1, len = na + nb;
      for (int64_t d0 = 0; d0 < len; d0 += static_cast<int64_t>(kMergeThreads) * kMsIpt) {
        const int64_t d = d0 + static_cast<int64_t>(t) * kMsIpt;
        if (d >= len) continue;
        int64_t ia = MergePathSplit(ks + a0, na, ks + a1, nb, d), ib = d - ia;
        const int cnt = len - d < kMsIpt ? static_cast<int>(len - d) : kMsIpt;
        for (int k = 0; k < cnt; ++k) {
          const bool takeA = ib >= nb || (ia < na && !(ks[a1 + ib] < ks[a0 + ia]));
          const int64_t src = takeA ? a0 + ia : a1 + ib;
          kd[a0 + d + k] = ks[src];
          wd[a0 + d + k] = ws[src];
          if (takeA) ++ia;
          else ++ib;
        }
      }
    }
    __syncthreads();
    if (t == 0) {
      const int R2 = (R + 1) / 2;
      for (int j = 0; j < R2; ++j) s_run[j] = s_run[2 * j];
      s_run[R2] = end;
    }
    __syncthreads();
    R = (R + 1) / 2;
    uint64_t* x = ks;
    ks = kd;
    kd = x;
    x = ws;
    ws = wd;
    wd = x;
  }
  // D. total weight (integral)
  uint64_t wsum = 0;
  for (int64_t i = s + t; i < end; i += kMergeThreads) wsum += ws[i];
  wsum = WaveSumU64(wsum);
  if (lane == 0) s_wred[wid] = wsum;
  __syncthreads();
  uint64_t Wt = 0;
  for (int w = 0; w < kMergeThreads / 64; ++w) Wt += s_wred[w];
  const bool do_process = s_nraw > 0 || s_ncent > kMaxProcessed;
  // E. the greedy pass (or, unprocessed, the merged list itself), one thread, LDS windows
  const double W = static_cast<double>(Wt);
  double w_so_far = 0, w_limit = 0, cm = 0, cw = 0;
  int nc = 0;
  bool ovf = false;
  uint64_t* s_w = s_keys + kMergeWin;
  for (int64_t w0 = s; w0 < end; w0 += kMergeWin) {
    const int64_t wn = end - w0 < kMergeWin ? end - w0 : kMergeWin;
    for (int64_t i = t; i < wn; i += kMergeThreads) {
      s_keys[i] = ks[w0 + i];
      s_w[i] = ws[w0 + i];
    }
    __syncthreads();
    if (t == 0) {
      for (int64_t i = 0; i < wn; ++i) {
        const double x = QVal(s_keys[i]);
        const double xw = static_cast<double>(s_w[i]);
        if (!do_process || (w0 == s && i == 0)) {  // a new centroid per item / the first one
          if (nc > 0 && nc <= kMergeOutCap) s_mean[nc - 1] = cm;
          if (nc < kMergeOutCap) s_start[nc] = static_cast<int64_t>(w_so_far);
          else ovf = true;
          ++nc;
          cm = x;
          cw = xw;
          w_so_far += xw;
          if (do_process) w_limit = W * IntegratedQ(1.0);
          continue;
        }
        const double projected = w_so_far + xw;
        if (projected <= w_limit) {
          w_so_far = projected;
          cw += xw;  // Centroid::add
          cm += xw * (x - cm) / cw;
        } else {
          const double k1 = IntegratedLocation(w_so_far / W);
          w_limit = W * IntegratedQ(k1 + 1.0);
          if (nc <= kMergeOutCap) s_mean[nc - 1] = cm;
          if (nc < kMergeOutCap) s_start[nc] = static_cast<int64_t>(w_so_far);
          else ovf = true;
          ++nc;
          w_so_far += xw;
          cm = x;
          cw = xw;
        }
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    if (nc > 0 && nc <= kMergeOutCap) s_mean[nc - 1] = cm;
    if (ovf) atomicOr(err, 8u);
    s_nc = ovf ? 0 : nc;
    if (do_process && nc > 0 && !ovf) {
      s_mn = StdMin(s_mn, s_mean[0]);
      s_mx = StdMax(s_mx, s_mean[nc - 1]);
    }
  }
  __syncthreads();
  // G. quantile() x7
  if (t < 7) {
    const int64_t ncv = s_nc;
    out[static_cast<uint64_t>(g) * 7 + t] =
        DigestQuantileMM(kQuantileQ[t], ncv, static_cast<int64_t>(Wt), [&](int64_t j) -> int64_t { return s_start[j]; },
                         [&](int64_t j) -> double { return s_mean[j]; }, s_mn, s_mx);
  }
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
  CopyBytesOverlap(data + offs[g], src, len);
}

// ---------------------------------------------------------------------------------------
// Host orchestration.
// ---------------------------------------------------------------------------------------

// meta: u64 [0] rows with a valid slot | u32 @8 groups | u32 @16 digest error | u32 @20 big groups
// left to the sort path | u32 @32.. class counts | u32 @48 big chunks, largest big group
__global__ void FinalizeInitKernel(uint8_t* meta, uint64_t n) {
  if (threadIdx.x == 0) {
    *reinterpret_cast<unsigned long long*>(meta) = n;
    *reinterpret_cast<uint32_t*>(meta + 8) = 0;
    *reinterpret_cast<uint32_t*>(meta + 16) = 0;
    *reinterpret_cast<uint32_t*>(meta + 20) = 0;
    for (int c = 0; c < kNumClasses; ++c) reinterpret_cast<uint32_t*>(meta + 32)[c] = 0;
    for (int c = 0; c < kNumMidSub; ++c) reinterpret_cast<uint32_t*>(meta + 64)[c] = 0;
  }
}


// Side streams forked by finalize are joined back into the main stream on every exit path, so
// an early error return never leaves side-stream kernels running on workspace buffers that a
// later reset / Ensure could free or reallocate.
// The early set: the designated groups of a fused split (ids [Gr, G)) above mid_max values.
// dstarts = the designated groups' starts (FusedSplitDesignatedStarts, j <= nd); they are
// copied to egs[0, nd] so the early set reads its own group starts (the rest's group-start pass
// writes gstart[Gr] concurrently).  One workgroup: nd <= kFsMaxU < 256.
__global__ void __launch_bounds__(256) DesignatedBigListKernel(const uint32_t* __restrict__ dstarts, const uint64_t* __restrict__ ftotal,
                                                               uint32_t G, uint32_t mid_max, uint32_t* __restrict__ egs,
                                                               uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
  __shared__ uint32_t s[kFsMaxU + 1];
  __shared__ uint32_t s_w[4];
  const uint32_t nd = min(static_cast<uint32_t>(*ftotal >> 32), kFsMaxU);
  const uint32_t t = threadIdx.x;
  if (t <= nd) {
    s[t] = dstarts[t];
    egs[t] = s[t];
  }
  __syncthreads();
  // ascending id order: a ballot per wave, then the waves in order
  const bool big = t < nd && s[t + 1] - s[t] > mid_max;
  const unsigned long long m = __ballot(big);
  if ((t & 63) == 0) s_w[t >> 6] = __popcll(m);
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < (t >> 6); ++w) before += s_w[w];
  if (big) list[before + __popcll(m & ((1ULL << (t & 63)) - 1))] = G - nd + t;
  if (t == 0) *count = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// The early big set runs whenever a fused split designated groups (PXG_EARLY_BIG=0: tests turn
// it off to compare).
static bool EarlyBigOn() {
  const char* e = std::getenv("PXG_EARLY_BIG");
  return !(e && e[0] == '0');
}

struct SideJoinGuard {
  Ctx* ctx;
  bool side = false, side2 = false;
  ~SideJoinGuard() {
    if (side) (void)JoinSide(ctx);
    if (side2) (void)JoinSide2(ctx);
  }
};


// Selected quantile lanes, lane-major (lane j of group g at out[j * G + g]) with pluck_float64's
// rule applied: 0.0 for a group whose 7 quantiles are not all finite (a NaN / inf one makes the
// reference's JSON unparsable, so pluck yields 0.0 for every key); fin[g] = that flag.  Each lane
// is then a ready FLOAT64 column for the post-aggregate map.
__global__ void QuantLanesKernel(const double* __restrict__ q, uint64_t G, uint32_t mask, double* __restrict__ out,
                                 uint8_t* __restrict__ fin) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= G) return;
  double v[7];
  bool f = true;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    v[k] = q[g * 7 + k];
    f = f && !isnan(v[k]) && !isinf(v[k]);
  }
  int o = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k)
    if ((mask >> k) & 1u) out[static_cast<uint64_t>(o++) * G + g] = f ? v[k] : 0.0;
  fin[g] = f ? 1 : 0;
}

// A quantiles result column requested as its plucked lanes (skip[c] = kSkipLanes | lane mask,
// pxg_agg_result_skip / pxg_agg_finalize_result): values = the lanes (QuantLanesKernel layout),
// data = the G finiteness bytes.  Host blocks are taken once; a second call (the finalize's
// sort-path fallback changed quantiles) rewrites them.  Stream-ordered, no wait.
constexpr uint8_t kSkipLanes = 0x80;
int32_t IssueLanes(Agg& a, int u, uint32_t mask, pxg_column_out& o) {
  const uint64_t G = static_cast<uint64_t>(a.res.n_groups);
  mask &= 0x7Fu;
  const int nsel = __builtin_popcount(mask);
  o.type = a.uda_out_type[u];
  o.length = static_cast<int64_t>(G);
  if (G == 0) return PXG_OK;
  if (!o.data) {
    o.values = ResultAlloc(std::max<size_t>(G * nsel * 8, 8));
    o.data = static_cast<uint8_t*>(ResultAlloc(G + 16));
    o.data_len = static_cast<int64_t>(G);
    if (!o.values || !o.data) return SetError(PXG_RESOURCE_UNAVAILABLE, "host result allocation failed");
  }
  PXG_RETURN_IF_ERROR(a.res.lanes.Ensure(G * (8 * nsel + 1) + 16));
  double* d_out = a.res.lanes.as<double>();
  uint8_t* d_fin = reinterpret_cast<uint8_t*>(d_out + G * nsel);
  PXG_RETURN_IF_ERROR(Launch(a.ctx, "quant_lanes", QuantLanesKernel, dim3(GridFor(static_cast<int64_t>(G), 256, 1 << 30)), dim3(256), 0,
                             a.res.uda_out[u].as<const double>(), G, mask, d_out, d_fin));
  if (nsel) PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.values, d_out, G * nsel * 8));
  return CopyD2H(a.ctx, a.ctx->stream, o.data, d_fin, G);
}

int32_t AggFinalizeTable(Agg* a) {
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
  // Streams the grouping moves: the plan's value streams.  The owner of a merged exchange moves
  // only the quantile stream (the items; every other output comes from the merged accumulators,
  // FinalizeMerged) and the items' weights: cv.p[x_qval] and cv.p[n_vals] after the grouping.
  const bool mq = a->merged && a->x_qval >= 0;
  const int nvs = a->merged ? (mq ? 2 : 1) : a->n_vals;
  PXG_RETURN_IF_ERROR(ws.meta.Ensure(96));
  uint8_t* meta = ws.meta.as<uint8_t>();
  uint32_t* d_ngroups = reinterpret_cast<uint32_t*>(meta + 8);
  unsigned int* d_err = reinterpret_cast<unsigned int*>(meta + 16);
  uint32_t* d_cls = reinterpret_cast<uint32_t*>(meta + 32);
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
  // Fused split (pxg_group.hip): large aggregations whose radix sort needs more than one pass
  // (PXG_FSPLIT=0 / 1: tests force it off / on).
  int gbits = 1;
  while ((uint64_t(1) << gbits) < static_cast<uint64_t>(ngroups) + 1) ++gbits;
  const bool fsplit = gbits > kRadixBits && FusedSplitOn(n);
  uint64_t* d_ftotal = nullptr;
  if (!fsplit) {
    PXG_RETURN_IF_ERROR(DenseIdsBySlot(ctx, a->slots.as<const unsigned long long>(), a->cap, ws.rank.as<uint32_t>(), ws.gslot.as<uint32_t>(),
                                       d_ngroups, scan_tmp));
  } else {
    PXG_RETURN_IF_ERROR(DesignateLargeGroups(ctx, a->slots.as<const unsigned long long>(), a->cap, a->st_slot.as<const uint32_t>(), n,
                                             ngroups, ws.split_cnt, ws.split_flags, ws.rank.as<uint32_t>(), ws.gslot.as<uint32_t>(),
                                             d_ngroups, scan_tmp, &d_ftotal));
  }

  clk.Mark("finalize: dense ids");
  // Group keys out of the arena, on side stream 2 while the radix sort runs on the main
  // stream (ConvertAggHashMapToRowBatch group columns, agg_node.cc:303-349).  String payloads
  // are sized by the arena (an upper bound), so no count comes back to the host first.  Side
  // stream 2 forks here; its launches are issued after the sort's, so the host reaches the
  // sort (the critical path) sooner.
  if (a->n_keys > 0) {
    PXG_RETURN_IF_ERROR(ForkSide2(ctx));
    guard.side2 = true;
  }
  auto IssueKeys = [&]() -> int32_t {
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
      // Early result: the key columns go to pooled pinned host blocks right behind their
      // kernels (STRING payloads copied up to the arena bound; the exact length is set after
      // the final synchronisation).
      if (a->early.want && !a->export_x && !a->merged && !a->emit_states) {
        bool ok = true;
        for (int k = 0; k < a->n_keys && ok; ++k) {
          pxg_column_out& o = a->early.cols[k];
          std::memset(&o, 0, sizeof(o));
          o.type = a->key_types[k];
          o.length = ngroups;
          if (o.type == PXG_STRING) {
            o.offsets = static_cast<int32_t*>(ResultAlloc((static_cast<size_t>(ngroups) + 1) * 4));
            o.data = static_cast<uint8_t*>(ResultAlloc(static_cast<size_t>(a->arena_words) * 8 + 16));
            ok = o.offsets && o.data;
            if (ok) {
              PXG_RETURN_IF_ERROR(CopyD2H(ctx, ctx->side2, o.offsets, R.key_offsets[k].p, (static_cast<size_t>(ngroups) + 1) * 4));
              if (a->arena_words > 0)
                PXG_RETURN_IF_ERROR(CopyD2H(ctx, ctx->side2, o.data, R.key_data[k].p, static_cast<size_t>(a->arena_words) * 8));
            }
          } else {
            const size_t w = o.type == PXG_BOOLEAN ? 1 : TypeWidth(o.type);
            o.values = ResultAlloc(std::max<size_t>(static_cast<size_t>(ngroups) * w, 1));
            ok = o.values != nullptr;
            if (ok) PXG_RETURN_IF_ERROR(CopyD2H(ctx, ctx->side2, o.values, R.key_fixed[k].p, static_cast<size_t>(ngroups) * w));
          }
        }
        a->early.keys = ok;
      }
    }
  }
    return PXG_OK;
  };
  // 2. Stable LSD radix sort of (dense id, vals...) by dense id (ceil(log2(G + 1) / 8) passes);
  //    records without a group (deferred slots) get id G and sort last.  The staging itself is
  //    left as it is (slots), so finalize can run again and export still works.
  for (int b = 0; b < 2; ++b) {
    PXG_RETURN_IF_ERROR(ws.skey[b].Ensure(n * 4 + 16));
    for (int v = 0; v < nvs; ++v) PXG_RETURN_IF_ERROR(ws.sval[b][v].Ensure(n * 8 + 16));
  }
  PXG_RETURN_IF_ERROR(ws.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(std::max<uint64_t>(n, a->cap) + 1)) + 64));
  scan_tmp = ws.scan.p;
  ConstValPtrs vin;
  uint32_t* kbuf[2];
  ValPtrs vbuf[2];
  for (int b = 0; b < 2; ++b) {
    kbuf[b] = ws.skey[b].as<uint32_t>();
    for (int v = 0; v < kMaxVals; ++v) vbuf[b].p[v] = v < nvs ? ws.sval[b][v].as<uint64_t>() : nullptr;
  }
  for (int v = 0; v < kMaxVals; ++v) vin.p[v] = v < a->n_vals && !a->merged ? a->st_val[v].as<const uint64_t>() : nullptr;
  if (a->merged) {  // [quantile items,] weights
    if (mq) vin.p[0] = a->st_val[a->x_qval].as<const uint64_t>();
    vin.p[mq ? 1 : 0] = a->st_wt.as<const uint64_t>();
  }
  const uint32_t* kin = nullptr;
  PXG_RETURN_IF_ERROR(ws.gstart.Ensure((static_cast<size_t>(ngroups) + 1) * 4));
  const uint32_t* gstart = ws.gstart.as<const uint32_t>();
  // The early big set (fused split only): the designated groups are final as soon as the split's
  // scatter has run, so their big ones start the selection path on side stream 2 while the rest
  // sort runs on the main stream (issued after the rest sort's launches, below).
  bool early_on = false;
  uint32_t early_gr = 0xFFFFFFFFu, early_nd = 0;
  uint64_t early_rows = 0;
  const uint32_t* early_dstarts = nullptr;
  if (fsplit) {
    // 2''. The fused split: one 9-bit pass (designated groups final, rest records by their low
    //      digit), then the rest records' remaining pass(es) by the higher digits.  The pass
    //      count of the rest comes from G (an upper bound of the rest ids), so the buffer the
    //      rest sort ends in is known before the rest count comes back.
    const int p2 = (gbits - kRadixBits + kRadixBits - 1) / kRadixBits;
    const int fin = p2 == 0 ? 1 : (p2 - 1) & 1;
    const uint32_t* base = nullptr;
    PXG_RETURN_IF_ERROR(FusedSplitPass(ctx, a->st_slot.as<const uint32_t>(), n, ws.rank.as<const uint32_t>(), a->cap, ngroups,
                                       static_cast<const uint64_t*>(d_ftotal), vin, nvs, ws.split_hist, ws.split_tot, ws.fs_keys, ws.rs,
                                       kbuf[1], vbuf[1], vbuf[fin], &base));
    uint8_t* pin = static_cast<uint8_t*>(ctx->pinned);
    PXG_RETURN_IF_ERROR(IssueKeys());
    PXG_HIP(hipEventSynchronize(ctx->ev_split));
    uint32_t n_rest = 0;
    uint64_t ft = 0;
    std::memcpy(&n_rest, pin + 104, 4);
    std::memcpy(&ft, pin + 112, 8);
    const uint32_t nd = std::min<uint32_t>(static_cast<uint32_t>(ft >> 32), kFsMaxU);
    const uint32_t Gr = ngroups - nd;
    for (int v = 0; v < kMaxVals; ++v) vin.p[v] = vbuf[fin].p[v];
    bool plan_q = false;
    for (int u = 0; u < a->n_udas; ++u) plan_q |= a->uda_kind[u] == PXG_UDA_QUANTILES;
    if (plan_q && nd > 0 && !a->export_x && !a->merged && !EnvFlag("PXG_BIG_SORT") && EarlyBigOn()) {
      early_on = true;
      early_gr = Gr;
      early_nd = nd;
      early_rows = n - n_rest;
      early_dstarts = FusedSplitDesignatedStarts(base);
      PXG_HIP(hipEventRecord(ctx->ev_early, ctx->stream));  // right behind the split's scatter
    }
    if (n_rest > 0) {
      const uint32_t* rkeys = kbuf[1];
      if (p2 > 0) {
        ConstValPtrs rin, rout;
        for (int v = 0; v < kMaxVals; ++v) rin.p[v] = vbuf[1].p[v];
        PXG_RETURN_IF_ERROR(RadixSortStreams(ctx, kbuf[1], nullptr, 0, Gr, rin, nvs, n_rest, kbuf, vbuf, ws.rs, &rkeys, &rout, kRadixBits,
                                             p2 * kRadixBits));
      }
      PXG_RETURN_IF_ERROR(GroupStarts(ctx, rkeys, static_cast<uint64_t>(n_rest), Gr, ws.gstart.as<uint32_t>()));
    }
    PXG_RETURN_IF_ERROR(FusedSplitGstart(ctx, base, static_cast<const uint64_t*>(d_ftotal), ngroups, ws.gstart.as<uint32_t>()));
  } else {
    PXG_RETURN_IF_ERROR(RadixSortStreams(ctx, a->st_slot.as<const uint32_t>(), ws.rank.as<const uint32_t>(), a->cap, ngroups, vin, nvs,
                                         n, kbuf, vbuf, ws.rs, &kin, &vin));
    PXG_RETURN_IF_ERROR(IssueKeys());
    const uint32_t* skeys = kin;  // sorted dense ids; vin = the values in the same order
    // 3. Group starts (first index of every id).
    PXG_RETURN_IF_ERROR(GroupStarts(ctx, skeys, n, ngroups, ws.gstart.as<uint32_t>()));
  }
  clk.Mark("finalize: grouping issued");
  if (a->merged) {  // back to stream numbering: the quantile stream at x_qval, the weights at n_vals
    const ConstValPtrs sorted = vin;
    for (int v = 0; v < kMaxVals; ++v) vin.p[v] = nullptr;
    if (mq) vin.p[a->x_qval] = sorted.p[0];
    vin.p[a->n_vals] = sorted.p[mq ? 1 : 0];
  }
  // 3. UDA reductions (chunk partials, then per-group combine).
  const ConstValPtrs cv = vin;
  UdaOut uo;
  for (int u = 0; u < kMaxUdas; ++u) uo.p[u] = nullptr;
  bool any_q = false, any_red = false;
  for (int u = 0; u < a->n_udas; ++u) {
    const bool q = a->uda_kind[u] == PXG_UDA_QUANTILES;
    any_q |= q;
    any_red |= !q && a->uda_kind[u] != PXG_UDA_COUNT && !a->merged;  // (merged: from the accumulators)
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
    clk.Mark("finalize: red chunk scan");
    PXG_RETURN_IF_ERROR(ws.partial.Ensure(max_chunks * a->n_udas * kPartialRows * 8));
    PXG_RETURN_IF_ERROR(ws.cgroup.Ensure(max_chunks * 4 + 16));
    clk.Mark("finalize: red ensure");
    PXG_RETURN_IF_ERROR(Launch(ctx, "chunk_group", ChunkGroupKernel, dim3(static_cast<unsigned>((max_chunks + 255) / 256)), dim3(256), 0,
                               static_cast<const uint32_t*>(cbase), ngroups, ws.cgroup.as<uint32_t>(), static_cast<uint32_t>(max_chunks)));
    if (n < 32 * static_cast<uint64_t>(ngroups)) {  // groups average < 32 rows: a thread per chunk
      PXG_RETURN_IF_ERROR(Launch(ctx, "chunk_reduce", ChunkReduceThreadKernel, dim3(static_cast<unsigned>((max_chunks + 255) / 256)),
                                 dim3(256), 0, a->d_plan.as<const AggPlanDev>(), gstart, static_cast<const uint32_t*>(cbase),
                                 ws.cgroup.as<const uint32_t>(), ngroups, cv, ws.partial.as<uint64_t>(), max_chunks));
    } else {
      PXG_RETURN_IF_ERROR(Launch(ctx, "chunk_reduce", ChunkReduceKernel, dim3(static_cast<unsigned>((max_chunks * 64 + 255) / 256)),
                                 dim3(256), 0, a->d_plan.as<const AggPlanDev>(), gstart, static_cast<const uint32_t*>(cbase),
                                 ws.cgroup.as<const uint32_t>(), ngroups, cv, ws.partial.as<uint64_t>(), max_chunks));
    }
  }
  uint8_t* states = nullptr;
  const AggPlanDev* cplan = a->d_plan.as<const AggPlanDev>();
  if (a->emit_states && a->state_rec > 0) {
    PXG_RETURN_IF_ERROR(R.states.Ensure(static_cast<size_t>(ngroups) * a->state_rec + 16));
    states = R.states.as<uint8_t>();
  } else if (a->export_x && a->hplan_x.state_rec > 0) {  // exchange export: every group's Serialize() states
    PXG_RETURN_IF_ERROR(ws.xstates.Ensure(static_cast<size_t>(ngroups) * a->hplan_x.state_rec + 16));
    states = ws.xstates.as<uint8_t>();
    cplan = a->d_plan_x.as<const AggPlanDev>();
  }
  if (!a->merged)  // (a merged run's outputs come from its accumulators: XFinalizeStatesKernel)
    PXG_RETURN_IF_ERROR(Launch(ctx, "group_combine", GroupCombineKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0,
                               cplan, gstart, static_cast<const uint32_t*>(cbase), ngroups,
                               ws.partial.as<const uint64_t>(), max_chunks, uo, states));
  clk.Mark("finalize: red kernels");
  if (a->early.want && !states && !a->merged && !a->export_x) {  // early result: the combined values
    bool ok = true;
    for (int u = 0; u < a->n_udas && ok; ++u) {
      if (a->uda_kind[u] == PXG_UDA_QUANTILES) continue;  // after the quantile kernels
      pxg_column_out& o = a->early.cols[a->n_keys + u];
      std::memset(&o, 0, sizeof(o));
      o.type = a->uda_out_type[u];
      o.length = ngroups;
      if (a->early.skip && a->early.skip[a->n_keys + u]) continue;
      o.values = ResultAlloc(std::max<size_t>(static_cast<size_t>(ngroups) * 8, 8));
      ok = o.values != nullptr;
      if (ok) PXG_RETURN_IF_ERROR(CopyD2H(ctx, ctx->stream, o.values, R.uda_out[u].p, static_cast<size_t>(ngroups) * 8));
    }
    a->early.vals = ok;
  }
  return PXG_OK;
  };
  if (!any_q) PXG_RETURN_IF_ERROR(RunReductions());
  uint32_t n_big_groups = 0;  // the late set's groups (host, after the meta readback)
  unsigned int* d_fallback = reinterpret_cast<unsigned int*>(meta + 20);
  // Full sort path of a set's big groups for quantile UDA u on stream st: chunk sort, merge
  // passes, digests.  Runs after the set's boundary chains (st must be ordered after them).
  auto BigSortPath = [&](const BigSet& S, hipStream_t st, int u) -> int32_t {
    const uint64_t* vals = cv.p[a->uda_val[u]];
    const int at = a->uda_arg_type[u];
    PXG_RETURN_IF_ERROR(ws.keysA.Ensure(n * 8));
    PXG_RETURN_IF_ERROR(ws.keysB.Ensure(n * 8));
    PXG_RETURN_IF_ERROR(ws.bstarts.Ensure(static_cast<size_t>(S.n_big) * kBigCentroids * 4));
    PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_big_chunk_sort", BigChunkSortKernel, dim3(S.n_chunks), dim3(256), 0,
                                 static_cast<const BigChunk*>(S.chunks), S.d_meta, vals, at, ws.keysA.as<uint64_t>()));
    DevBuf* src = &ws.keysA;
    DevBuf* dst = &ws.keysB;
    uint32_t pass = 0;
    for (uint64_t w = kMidMax; w < S.big_max; w *= 2, ++pass) {
      PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_big_merge", BigMergeTileKernel, dim3(S.n_chunks), dim3(256), 0,
                                   static_cast<const BigChunk*>(S.chunks), S.d_meta, src->as<const uint64_t>(), dst->as<uint64_t>(), w, pass));
      std::swap(src, dst);
    }
    // An exchange export ships values / centroid lists, not quantiles: no digests there.
    if (!a->export_x) {
      return LaunchOn(ctx, st, "quant_big_digest", BigDigestKernel, dim3(S.n_big), dim3(256), 0, static_cast<const BigGroup*>(S.big),
                      S.d_count, ws.keysA.as<const uint64_t>(), ws.keysB.as<const uint64_t>(), ws.bstarts.as<uint32_t>(), S.chain_starts,
                      S.chain_nc, R.uda_out[u].as<double>(), d_err);
    }
    // Exchange export: each big group's whole single-pass centroid list (those of > 8 * delta
    // values ship it instead of their values).
    PXG_RETURN_IF_ERROR(ws.xcent.Ensure(static_cast<size_t>(S.n_big) * kXCentCap * 16 + 16));
    PXG_RETURN_IF_ERROR(ws.xcnt.Ensure(static_cast<size_t>(S.n_big) * 4 + 16));
    return LaunchOn(ctx, st, "export_centroids", CentroidListKernel, dim3(S.n_big), dim3(kCentListBlock), 0, static_cast<const BigGroup*>(S.big),
                    S.d_count, ws.keysA.as<const uint64_t>(), ws.keysB.as<const uint64_t>(), ws.bstarts.as<uint32_t>(), S.chain_starts,
                    S.chain_nc, ws.xcent.as<uint64_t>(), ws.xcnt.as<int32_t>());
  };
  // The selection path of a set (pxg_select.hip) for quantile UDA u.
  auto SelInOf = [&](int u) -> SelIn {
    SelIn in;
    in.vals = cv.p[a->uda_val[u]];
    in.arg_type = a->uda_arg_type[u];
    in.n = n;
    in.keysA = &ws.keysA;
    in.sel_bin = &ws.sel_bin;
    in.d_fallback = d_fallback;
    in.out = R.uda_out[u].as<double>();
    return in;
  };
  auto EnsureSel = [&](const BigSet& S) -> int32_t { return SelEnsure(S, n, ws.keysA, ws.sel_bin); };
  auto BigSelectFront = [&](const BigSet& S, hipStream_t st, int u) -> int32_t { return SelFront(ctx, st, S, SelInOf(u)); };
  auto BigSelectBack = [&](const BigSet& S, hipStream_t st, int u) -> int32_t { return SelBack(ctx, st, S, SelInOf(u)); };
  BigSet SE;  // the early set
  if (early_on) {
    Agg::FinalizeWs::EarlyBig& E = ws.early;
    const uint32_t nd = early_nd;
    const uint64_t chunk_cap = early_rows / kMidMax + nd + 1;
    PXG_RETURN_IF_ERROR(E.meta.Ensure(16));
    PXG_RETURN_IF_ERROR(E.ids.Ensure(static_cast<size_t>(nd) * 4 + 16));
    PXG_RETURN_IF_ERROR(E.egs.Ensure(static_cast<size_t>(nd) * 4 + 16));
    PXG_RETURN_IF_ERROR(E.big.Ensure(static_cast<size_t>(nd) * (sizeof(BigGroup) + 4) + 32));
    PXG_RETURN_IF_ERROR(E.chunks.Ensure(chunk_cap * sizeof(BigChunk)));
    PXG_RETURN_IF_ERROR(E.chain_starts.Ensure(static_cast<size_t>(nd) * kChainCap * 4));
    PXG_RETURN_IF_ERROR(E.chain_nc.Ensure(static_cast<size_t>(nd) * 4));
    uint32_t* em = E.meta.as<uint32_t>();  // [0] groups, [1] chunks, [2] largest group, [3] large groups
    uint32_t* large_list = reinterpret_cast<uint32_t*>(E.big.as<uint8_t>() + static_cast<size_t>(nd) * sizeof(BigGroup));
    SE.big = E.big.as<BigGroup>();
    SE.chunks = E.chunks.as<BigChunk>();
    SE.d_count = em;
    SE.d_meta = em + 1;
    SE.n_big = nd;
    SE.n_chunks = static_cast<uint32_t>(chunk_cap);
    SE.chain_starts = E.chain_starts.as<const uint32_t>();
    SE.chain_nc = E.chain_nc.as<const int32_t>();
    SE.spl = &E.spl;
    SE.cnt = &E.cnt;
    SE.list = &E.list;
    SE.bstart = &E.bstart;
    SE.tag = &E.tag;
    SE.cbase = &E.cbase;
    SE.plan = &E.plan;
    SE.partial = &E.partial;
    SE.large_list = large_list;
    SE.large_cnt = em + 3;
    PXG_RETURN_IF_ERROR(EnsureSel(SE));
    PXG_HIP(hipStreamWaitEvent(ctx->side2, ctx->ev_early, 0));
    guard.side2 = true;
    PXG_HIP(hipMemsetAsync(em, 0, 16, ctx->side2));
    PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "quant_early_list", DesignatedBigListKernel, dim3(1), dim3(256), 0, early_dstarts,
                                 static_cast<const uint64_t*>(d_ftotal), ngroups, kMidClassMax, E.egs.as<uint32_t>(), E.ids.as<uint32_t>(), em));
    const uint32_t* egs_by_id = E.egs.as<const uint32_t>() - early_gr;  // group starts indexed by group id (ids [Gr, G) only)
    PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "big_setup", BigSetupKernel, dim3(1), dim3(kSetupBlock), 0, E.ids.as<const uint32_t>(),
                                 static_cast<const uint32_t*>(em), egs_by_id, SE.big, SE.chunks, em + 1, large_list, em + 3));
    PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side2, "digest_chain", DigestChainKernel, dim3((nd + kChainWaves - 1) / kChainWaves),
                                 dim3(64 * kChainWaves), 0, E.ids.as<const uint32_t>(), static_cast<const uint32_t*>(em), 0u,
                                 E.ids.as<const uint32_t>(), static_cast<const uint32_t*>(em), egs_by_id, E.chain_starts.as<uint32_t>(),
                                 E.chain_nc.as<int32_t>()));
    for (int u = 0; u < a->n_udas; ++u) {
      if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
      PXG_RETURN_IF_ERROR(BigSelectFront(SE, ctx->side2, u));
      PXG_RETURN_IF_ERROR(BigSelectBack(SE, ctx->side2, u));
    }
    clk.Mark("finalize: early big set issued");
  }
  bool big_select = false;
  BigSet SL;  // the late set: class 3 of the classification
  // 4. Quantile digests.
  if (any_q) {
    PXG_RETURN_IF_ERROR(ws.lists.Ensure(static_cast<size_t>(ngroups) * kAllClasses * 4));
    // A merged exchange's groups that received centroid lists get their quantiles from the
    // merged digest (FinalizeMerged): no class here, so the selection path never sees their
    // centroid means as values (which made it fall back to the full sort).
    const bool skip_merged = a->merged && a->macc_cap == a->cap;
    PXG_RETURN_IF_ERROR(Launch(ctx, "classify_groups", ClassifyGroupsKernel, dim3(GridFor(ngroups, 256, 1 << 30)), dim3(256), 0, gstart,
                               ngroups, ws.lists.as<uint32_t>(), d_cls, reinterpret_cast<uint32_t*>(meta + 64),
                               a->export_x ? static_cast<uint32_t>(kMidMax) : kMidClassMax,
                               skip_merged ? a->macc.as<const uint64_t>() : nullptr, a->macc_words,
                               ws.gslot.as<const uint32_t>(), early_gr));
    const uint32_t* lists = ws.lists.as<const uint32_t>();
    // Big-group metadata on the device; one readback of the class counts, the big-group chunk
    // total and the largest group (grid sizes and the merge-pass count).
    const uint64_t big_cap = n / (kMidMax + 1) + 1;  // groups of > kMidMax rows
    const uint64_t chunk_cap = n / kMidMax + big_cap + 1;
    PXG_RETURN_IF_ERROR(ws.big.Ensure(big_cap * sizeof(BigGroup) + 16 + big_cap * 4));
    uint32_t* large_cnt = reinterpret_cast<uint32_t*>(ws.big.as<uint8_t>() + big_cap * sizeof(BigGroup));
    uint32_t* large_list = large_cnt + 4;
    PXG_RETURN_IF_ERROR(ws.bchunks.Ensure(chunk_cap * sizeof(BigChunk)));
    uint32_t* d_bigmeta = reinterpret_cast<uint32_t*>(meta + 48);
    PXG_RETURN_IF_ERROR(Launch(ctx, "big_setup", BigSetupKernel, dim3(1), dim3(kSetupBlock), 0, lists + 3 * static_cast<uint64_t>(ngroups),
                               static_cast<const uint32_t*>(d_cls + 3), gstart, ws.big.as<BigGroup>(), ws.bchunks.as<BigChunk>(),
                               d_bigmeta, large_list, large_cnt));
    // Class counts + big-group metadata to pinned memory right away; the host waits on this
    // event only, while the digests below keep the GPU busy.
    clk.Mark("finalize: classes issued");
    uint8_t* pin = static_cast<uint8_t*>(ctx->pinned);
    {  // cls[4] @32, bigmeta[2] @48; mid classes 4-6
      const SmallCopy rb[2] = {{d_cls, 64, 24}, {meta + 64, 88, 4 * kNumMidSub}};
      PXG_RETURN_IF_ERROR(ReadbackSmall(ctx, ctx->stream, rb, 2));
    }
    PXG_HIP(hipEventRecord(ctx->ev_meta, ctx->stream));
    // Kernels whose work lists are counted on the device launch right away with upper-bound
    // grids (blocks past the device count exit); the host reads the counts back only after
    // them, so the tiny / small digests and the boundary chains run while it waits.
    const uint32_t big_cap32 = static_cast<uint32_t>(std::min<uint64_t>(ngroups, big_cap));
    const uint32_t n_chain_cap = big_cap32;  // mid groups read the per-context table
    PXG_RETURN_IF_ERROR(EnsureMidChains(ctx));
    clk.Mark("finalize: mid chains ready");
    PXG_RETURN_IF_ERROR(ws.chain_nc.Ensure(static_cast<size_t>(n_chain_cap) * 4));
    PXG_RETURN_IF_ERROR(ws.chain_starts.Ensure(static_cast<size_t>(n_chain_cap) * kChainCap * 4));
    const uint32_t* chain_starts = ws.chain_starts.as<const uint32_t>();
    const int32_t* chain_nc = ws.chain_nc.as<const int32_t>();
    // Chains: latency-bound (one wave per mid / big group, ~110 rounds each), on the side stream.
    PXG_RETURN_IF_ERROR(ForkSide(ctx));
    guard.side = true;
    PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side, "digest_chain", DigestChainKernel, dim3((n_chain_cap + kChainWaves - 1) / kChainWaves),
                                 dim3(64 * kChainWaves), 0,
                                 lists + 2 * static_cast<uint64_t>(ngroups), static_cast<const uint32_t*>(d_cls + 2), 0u,
                                 lists + 3 * static_cast<uint64_t>(ngroups), static_cast<const uint32_t*>(d_cls + 3), gstart,
                                 ws.chain_starts.as<uint32_t>(), ws.chain_nc.as<int32_t>()));
    PXG_HIP(hipEventRecord(ctx->ev_chain, ctx->side));
    // The small digests follow the chains on the side stream (neither needs the other); the
    // reductions and the tiny digests run on the main stream meanwhile.
    const uint32_t small_cap = static_cast<uint32_t>(std::min<uint64_t>(ngroups, n / (kTinyMax + 1) + 1));
    for (int u = 0; u < a->n_udas && !a->export_x; ++u) {  // (an export needs no quantiles)
      if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
      PXG_RETURN_IF_ERROR(LaunchOn(ctx, ctx->side, "quant_small", QuantSmallKernel, dim3((small_cap + kSmallWaves - 1) / kSmallWaves),
                                   dim3(256), 0, lists + static_cast<uint64_t>(ngroups), static_cast<const uint32_t*>(d_cls + 1), gstart,
                                   cv.p[a->uda_val[u]], a->uda_arg_type[u], R.uda_out[u].as<double>()));
    }
    clk.Mark("finalize: chains + small issued");
    PXG_RETURN_IF_ERROR(RunReductions());
    clk.Mark("finalize: reductions issued");
    // The tiny digests follow the small ones on the side stream when no early big set runs (C2
    // shape: the main stream then carries the reductions and the mid classes, the longest
    // chain; round 6, tools/step_ab.py at 100M rows: step 2.210 -> 2.173 ms).  With an early set
    // (1B rows) every placement measured the same (14.51-14.58 ms), so they stay on the main
    // stream there, as do the mid classes (on either side stream: 14.56-14.59 ms).
    const hipStream_t tiny_st = !early_on && guard.side ? ctx->side : ctx->stream;
    for (int u = 0; u < a->n_udas && !a->export_x; ++u) {
      if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
      PXG_RETURN_IF_ERROR(LaunchOn(ctx, tiny_st, "quant_tiny", QuantTinyKernel, dim3((ngroups + 3) / 4), dim3(256), 0, lists,
                                   static_cast<const uint32_t*>(d_cls), gstart, cv.p[a->uda_val[u]], a->uda_arg_type[u],
                                   R.uda_out[u].as<double>()));
    }
    uint32_t hm[6], hmid[kNumMidSub];
    clk.Mark("finalize: issue to meta");
    PXG_HIP(hipEventSynchronize(ctx->ev_meta));
    clk.Mark("finalize: meta wait");
    std::memcpy(hm, pin + 64, 24);
    std::memcpy(hmid, pin + 88, 4 * kNumMidSub);
    uint32_t cls[kNumClasses] = {hm[0], hm[1], hm[2], hm[3]};
    const uint32_t n_big = cls[3];
    n_big_groups = n_big;
    SL.big = ws.big.as<BigGroup>();
    SL.chunks = ws.bchunks.as<BigChunk>();
    SL.d_count = d_cls + 3;
    SL.d_meta = d_bigmeta;
    SL.n_big = n_big;
    SL.n_chunks = hm[4];
    SL.big_max = hm[5];
    SL.chain_starts = chain_starts;
    SL.chain_nc = chain_nc;
    SL.spl = &ws.sel_spl;
    SL.cnt = &ws.sel_cnt;
    SL.list = &ws.sel_list;
    SL.bstart = &ws.sel_bstart;
    SL.tag = &ws.sel_tag;
    SL.cbase = &ws.sel_cbase;
    SL.plan = &ws.sel_plan;
    SL.partial = &ws.sel_partial;
    SL.large_list = large_list;
    SL.large_cnt = large_cnt;
    // PXG_BIG_SORT=1 forces the full sort path for every big group (tests compare the two).
    big_select = n_big > 0 && !EnvFlag("PXG_BIG_SORT") && !a->export_x;
    if (big_select) PXG_RETURN_IF_ERROR(EnsureSel(SL));
    // Big groups on side stream 2, overlapping the mid digests and the key output on the main
    // stream: the selection path's sample + bin counts start right after the metadata readback,
    // the rest waits for the boundary chains.  Every quantile UDA's big work runs in order on
    // side stream 2, so later UDAs reuse the workspace safely.
    // With an early set on side stream 2, the late set takes the side stream (behind the small
    // digests), so the two sets' latency-bound chains of launches run side by side.
    hipStream_t lst = early_on ? ctx->side : ctx->side2;
    if (n_big > 0) {
      PXG_HIP(hipStreamWaitEvent(lst, ctx->ev_meta, 0));
      if (!early_on) guard.side2 = true;
    }
    // (Issuing the late set after the mid classes when an early set runs started QuantMid<8192>
    // 0.12 ms sooner at 1B rows but only moved the LDS contention: span 3.96 -> 4.02 ms.)
    auto IssueLate = [&](int u) -> int32_t {
      if (big_select) PXG_RETURN_IF_ERROR(BigSelectFront(SL, lst, u));
      if (n_big > 0) {
        PXG_HIP(hipStreamWaitEvent(lst, ctx->ev_chain, 0));
        PXG_RETURN_IF_ERROR(big_select ? BigSelectBack(SL, lst, u) : BigSortPath(SL, lst, u));
      }
      return PXG_OK;
    };
    for (int u = 0; u < a->n_udas; ++u) {
      if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
      const uint64_t* vals = cv.p[a->uda_val[u]];
      const int at = a->uda_arg_type[u];
      PXG_RETURN_IF_ERROR(IssueLate(u));
      double* qo = R.uda_out[u].as<double>();
      if (!a->export_x) {  // the mid classes, one launch each (largest first: the longest workgroups)
        const uint32_t* cnt_mid = reinterpret_cast<const uint32_t*>(meta + 64);
        if (hmid[1] > 0)
          PXG_RETURN_IF_ERROR(Launch(ctx, "quant_mid", QuantMidKernel<8192>, dim3(hmid[1]), dim3(8192 / kMsIpt), 0,
                                     lists + 5 * static_cast<uint64_t>(ngroups), gstart, MidChainStarts(ctx), MidChainNc(ctx),
                                     cnt_mid + 1, vals, at, qo, d_err));
        if (hmid[0] > 0)
          PXG_RETURN_IF_ERROR(Launch(ctx, "quant_mid", QuantMidKernel<4096>, dim3(hmid[0]), dim3(4096 / kMsIpt), 0,
                                     lists + 4 * static_cast<uint64_t>(ngroups), gstart, MidChainStarts(ctx), MidChainNc(ctx),
                                     cnt_mid, vals, at, qo, d_err));
        if (cls[2] > 0)
          PXG_RETURN_IF_ERROR(Launch(ctx, "quant_mid", QuantMidKernel<2048>, dim3(cls[2]), dim3(2048 / kMsIpt), 0,
                                     lists + 2 * static_cast<uint64_t>(ngroups), gstart, MidChainStarts(ctx), MidChainNc(ctx),
                                     static_cast<const uint32_t*>(d_cls + 2), vals, at, qo, d_err));
      }
    }
  }
  if (guard.side) PXG_RETURN_IF_ERROR(JoinSide(ctx));  // the small digests
  guard.side = false;
  if (keys_on_side2 || n_big_groups > 0 || early_on) PXG_RETURN_IF_ERROR(JoinSide2(ctx));
  guard.side2 = false;
  if (a->export_x) {
    // An export reads neither the string-key totals nor the result columns: its caller checks
    // the error flag and the device group count (ws.meta) with the readback it waits for anyway
    // (Agg::CheckExportFinalize), so the export finalize ends without a host wait of its own.
    a->x_vals = a->x_qval >= 0 ? cv.p[a->x_qval] : nullptr;
    a->x_wts = nullptr;
    a->x_nbig = n_big_groups;
    a->last_big_sort_groups = n_big_groups;
    a->x_check_pending = true;
    a->x_check_groups = ngroups;
    R.ready = true;
    return PXG_OK;
  }
  // Early result: quantile columns asked for as plucked lanes, behind the digests, so their
  // copies land within the synchronisation below.
  auto IssueEarlyLanes = [&]() -> int32_t {
    if (!a->early.want || !a->early.skip || a->merged) return PXG_OK;
    for (int u = 0; u < a->n_udas; ++u) {
      const uint8_t sk = a->early.skip[a->n_keys + u];
      if (a->uda_kind[u] == PXG_UDA_QUANTILES && (sk & kSkipLanes)) PXG_RETURN_IF_ERROR(IssueLanes(*a, u, sk, a->early.cols[a->n_keys + u]));
    }
    return PXG_OK;
  };
  PXG_RETURN_IF_ERROR(IssueEarlyLanes());
  // One sync for the digest error flag and every string-key total.
  std::vector<uint32_t> totals(kMaxKeys, 0);
  unsigned int err = 0;
  uint32_t* pin32 = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + 128);
  uint32_t g_dev = 0;
  {  // one launch for the string-key totals, the error / group count / fallback words, early meta
    SmallCopy rb[kMaxSmallCopies];
    int nrb = 0;
    const uint32_t b = 128;  // pin32's byte offset in the pinned scratch
    for (int k = 0; k < a->n_keys; ++k)
      if (a->key_types[k] == PXG_STRING) rb[nrb++] = {R.key_offsets[k].as<uint32_t>() + ngroups, b + 4 * k, 4};
    rb[nrb++] = {d_err, b + 4 * kMaxKeys, 4};
    rb[nrb++] = {d_ngroups, b + 4 * (kMaxKeys + 1), 4};
    rb[nrb++] = {d_fallback, b + 4 * (kMaxKeys + 2), 4};
    if (early_on) rb[nrb++] = {ws.early.meta.p, b + 4 * (kMaxKeys + 3), 12};
    PXG_RETURN_IF_ERROR(ReadbackSmall(ctx, ctx->stream, rb, nrb));
  }
  clk.Mark("finalize: issue rest");
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  clk.Mark("finalize: final wait");
  for (int k = 0; k < a->n_keys; ++k)
    if (a->key_types[k] == PXG_STRING) totals[k] = pin32[k];
  err = pin32[kMaxKeys];
  g_dev = pin32[kMaxKeys + 1];
  const bool any_select = big_select || early_on;
  const uint32_t n_fallback = any_select ? pin32[kMaxKeys + 2] : 0;
  a->last_big_sort_groups = any_select ? n_fallback : n_big_groups;
  if (any_select && n_fallback > 0) {
    // Some big group could not be served by selection (NaN values, a gathered bin past its
    // capacity: heavy ties).  With one quantile UDA the full sort path recomputes just those
    // groups (both sets' flagged groups as one set: their list, BigSetup and chains, then the
    // chunk sort / merges / digests); with several, every big group of both sets (the plans hold
    // the last UDA's flags only).  The chains and the sets' work are long done.
    if (early_on) {
      SE.n_big = pin32[kMaxKeys + 3];
      SE.n_chunks = pin32[kMaxKeys + 4];
      SE.big_max = pin32[kMaxKeys + 5];
    }
    int nq = 0;
    for (int u = 0; u < a->n_udas; ++u) nq += a->uda_kind[u] == PXG_UDA_QUANTILES ? 1 : 0;
    if (nq == 1) {
      const uint32_t cap_fb = (big_select ? SL.n_big : 0) + (early_on ? SE.n_big : 0);
      PXG_RETURN_IF_ERROR(ws.fb_list.Ensure(static_cast<size_t>(cap_fb) * 4 + 16));
      PXG_RETURN_IF_ERROR(ws.fb_meta.Ensure(16));
      uint32_t* fm = ws.fb_meta.as<uint32_t>();  // [0] groups, [1] chunks, [2] largest, [3] large groups
      uint32_t* fl = ws.fb_list.as<uint32_t>();
      PXG_HIP(hipMemsetAsync(fm, 0, 16, ctx->stream));
      for (const BigSet* S : {&SL, &SE}) {
        if (S->n_big == 0 || (S == &SL && !big_select)) continue;
        PXG_RETURN_IF_ERROR(SelFallbackList(ctx, *S, fl, fm));
      }
      // The subset in the late set's buffers (sized for every group above kMidMax values).
      BigSet SF;
      SF.big = ws.big.as<BigGroup>();
      SF.chunks = ws.bchunks.as<BigChunk>();
      SF.d_count = fm;
      SF.d_meta = fm + 1;
      SF.chain_starts = ws.chain_starts.as<const uint32_t>();
      SF.chain_nc = ws.chain_nc.as<const int32_t>();
      uint32_t* large_list = reinterpret_cast<uint32_t*>(ws.big.as<uint8_t>() + (n / (kMidMax + 1) + 1) * sizeof(BigGroup)) + 4;
      PXG_RETURN_IF_ERROR(Launch(ctx, "big_setup", BigSetupKernel, dim3(1), dim3(kSetupBlock), 0, static_cast<const uint32_t*>(fl),
                                 static_cast<const uint32_t*>(fm), gstart, SF.big, SF.chunks, fm + 1, large_list, fm + 3));
      PXG_RETURN_IF_ERROR(Launch(ctx, "digest_chain", DigestChainKernel, dim3((cap_fb + kChainWaves - 1) / kChainWaves), dim3(64 * kChainWaves), 0,
                                 static_cast<const uint32_t*>(fl), static_cast<const uint32_t*>(fm), 0u, static_cast<const uint32_t*>(fl),
                                 static_cast<const uint32_t*>(fm), gstart, ws.chain_starts.as<uint32_t>(), ws.chain_nc.as<int32_t>()));
      PXG_HIP(hipMemcpyAsync(pin32 + kMaxKeys + 6, fm, 12, hipMemcpyDeviceToHost, ctx->stream));
      PXG_HIP(hipStreamSynchronize(ctx->stream));
      SF.n_big = pin32[kMaxKeys + 6];
      SF.n_chunks = pin32[kMaxKeys + 7];
      SF.big_max = pin32[kMaxKeys + 8];
      for (int u = 0; u < a->n_udas; ++u)
        if (a->uda_kind[u] == PXG_UDA_QUANTILES && SF.n_big > 0) PXG_RETURN_IF_ERROR(BigSortPath(SF, ctx->stream, u));
    } else {
      PXG_RETURN_IF_ERROR(ws.bstarts.Ensure(static_cast<size_t>(std::max(SE.n_big, SL.n_big)) * kBigCentroids * 4 + 16));
      for (int u = 0; u < a->n_udas; ++u) {
        if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
        if (SL.n_big > 0) PXG_RETURN_IF_ERROR(BigSortPath(SL, ctx->stream, u));
        if (SE.n_big > 0) PXG_RETURN_IF_ERROR(BigSortPath(SE, ctx->stream, u));
      }
    }
    PXG_RETURN_IF_ERROR(IssueEarlyLanes());  // the recomputed groups' lanes
    PXG_HIP(hipMemcpyAsync(pin32 + kMaxKeys, d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    err = pin32[kMaxKeys];
  }
  if (err) return SetError(PXG_INTERNAL, "t-digest centroid capacity exceeded");
  a->x_vals = a->x_qval >= 0 ? cv.p[a->x_qval] : nullptr;
  a->x_wts = a->merged ? cv.p[a->n_vals] : nullptr;
  a->x_nbig = n_big_groups;
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
  return pxg_agg_result_skip(agg, cols, n_cols, nullptr);
}

extern "C" int32_t pxg_agg_quantile_lanes(pxg_agg* agg, int32_t uda, uint32_t lane_mask, double* host_out, uint8_t* host_finite) {
  if (!agg || !host_finite || (lane_mask && !host_out)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Agg& a = agg->impl;
  if (!a.res.ready) return SetError(PXG_FAILED_PRECONDITION, "pxg_agg_finalize has not run since the last consume");
  if (uda < 0 || uda >= a.n_udas || a.uda_kind[uda] != PXG_UDA_QUANTILES)
    return SetError(PXG_INVALID_ARGUMENT, "aggregate %d is not a quantiles UDA", uda);
  lane_mask &= 0x7Fu;
  const int nsel = __builtin_popcount(lane_mask);
  const uint64_t G = static_cast<uint64_t>(a.res.n_groups);
  if (G == 0) return PXG_OK;
  PXG_RETURN_IF_ERROR(a.res.lanes.Ensure(G * (8 * nsel + 1) + 16));
  double* d_out = a.res.lanes.as<double>();
  uint8_t* d_fin = reinterpret_cast<uint8_t*>(d_out + G * nsel);
  PXG_RETURN_IF_ERROR(Launch(a.ctx, "quant_lanes", QuantLanesKernel, dim3(GridFor(static_cast<int64_t>(G), 256, 1 << 30)), dim3(256), 0,
                             a.res.uda_out[uda].as<const double>(), G, lane_mask, d_out, d_fin));
  if (nsel) PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, host_out, d_out, G * nsel * 8));
  PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, host_finite, d_fin, G));
  PXG_HIP(hipStreamSynchronize(a.ctx->stream));
  return PXG_OK;
}

extern "C" int32_t pxg_agg_finalize_result(pxg_agg* agg, int64_t* n_groups, pxg_column_out* cols, int32_t n_cols, const uint8_t* skip) {
  if (!agg || !cols) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Agg& a = agg->impl;
  const int32_t n_val_cols = a.emit_states ? 1 : a.n_udas;
  if (n_cols != a.n_keys + n_val_cols) return SetError(PXG_INVALID_ARGUMENT, "expected %d result columns", a.n_keys + n_val_cols);
  for (int c = 0; c < n_cols; ++c) std::memset(&cols[c], 0, sizeof(cols[c]));
  const bool early = !a.emit_states && !a.merged && !a.hc_active && a.n_keys > 0;
  a.early.want = early;
  a.early.keys = a.early.vals = false;
  a.early.cols = cols;
  a.early.skip = skip;
  const int32_t rc = AggFinalizeImpl(&a);
  const bool got = a.early.keys && a.early.vals;
  a.early = Agg::EarlyResult();
  // A run that switched to partitioned groups (or failed, or stopped before issuing every copy)
  // drops what was copied early and takes the ordinary result path.
  const bool usable = rc == PXG_OK && got && !a.hc_active && a.res.n_groups > 0;
  if (!usable) {
    (void)hipStreamSynchronize(a.ctx->stream);
    pxg_result_free(cols, n_cols);
    for (int c = 0; c < n_cols; ++c) std::memset(&cols[c], 0, sizeof(cols[c]));
    if (rc != PXG_OK) return rc;
    int64_t g = a.res.n_groups;
    if (a.n_keys == 0 && g == 0) g = 1;
    if (n_groups) *n_groups = g;
    return pxg_agg_result_skip(agg, cols, n_cols, skip);
  }
  const int64_t G = a.res.n_groups;
  for (int k = 0; k < a.n_keys; ++k)
    if (a.key_types[k] == PXG_STRING) cols[k].data_len = a.res.key_data_len[k];
  // Quantile columns not skipped: 7 doubles per group, after the quantile kernels.
  bool q = false;
  for (int u = 0; u < a.n_udas; ++u) {
    pxg_column_out& o = cols[a.n_keys + u];
    if (a.uda_kind[u] != PXG_UDA_QUANTILES) continue;
    o.type = a.uda_out_type[u];
    o.length = G;
    if (skip && skip[a.n_keys + u]) continue;
    o.values = ResultAlloc(static_cast<size_t>(G) * 56);
    if (!o.values) {
      pxg_result_free(cols, n_cols);
      return SetError(PXG_RESOURCE_UNAVAILABLE, "host result allocation failed");
    }
    PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.values, a.res.uda_out[u].p, static_cast<size_t>(G) * 56));
    q = true;
  }
  if (q) PXG_HIP(hipStreamSynchronize(a.ctx->stream));
  if (n_groups) *n_groups = G;
  return PXG_OK;
}

extern "C" int32_t pxg_agg_result_device(pxg_agg* agg, pxg_column_view* cols, int32_t n_cols, int64_t* bytes) {
  if (!agg || !cols || !bytes) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Agg& a = agg->impl;
  if (!a.res.ready) return SetError(PXG_FAILED_PRECONDITION, "pxg_agg_finalize has not run since the last consume");
  if (n_cols != a.n_keys + a.n_udas) return SetError(PXG_INVALID_ARGUMENT, "expected %d result columns", a.n_keys + a.n_udas);
  if (a.emit_states) return SetError(PXG_UNIMPLEMENTED, "serialized states are assembled on the host");
  for (int u = 0; u < a.n_udas; ++u) {
    if (a.uda_kind[u] == PXG_UDA_QUANTILES) return SetError(PXG_UNIMPLEMENTED, "quantiles are rendered on the host");
    if (TypeWidth(a.uda_out_type[u]) != 8) return SetError(PXG_UNIMPLEMENTED, "UDA %d has no 8-byte device column", u);
  }
  const int64_t G = a.res.n_groups;
  if (a.n_keys == 0 && G == 0) return SetError(PXG_UNIMPLEMENTED, "the synthetic row of an empty group-less agg is built on the host");
  int64_t b = 0;
  for (int k = 0; k < a.n_keys; ++k) {
    pxg_column_view& v = cols[k];
    std::memset(&v, 0, sizeof(v));
    v.type = a.key_types[k];
    v.length = G;
    if (v.type == PXG_STRING) {
      v.offsets = a.res.key_offsets[k].as<const int32_t>();
      v.data = a.res.key_data[k].as<const uint8_t>();
      b += a.res.key_data_len[k];
    } else {
      v.values = a.res.key_fixed[k].p;
      b += static_cast<int64_t>(TypeWidth(v.type)) * G;
    }
  }
  for (int u = 0; u < a.n_udas; ++u) {
    pxg_column_view& v = cols[a.n_keys + u];
    std::memset(&v, 0, sizeof(v));
    v.type = a.uda_out_type[u];
    v.length = G;
    v.values = a.res.uda_out[u].p;
    b += 8 * G;
  }
  *bytes = b;
  return PXG_OK;
}

extern "C" int32_t pxg_agg_result_skip(pxg_agg* agg, pxg_column_out* cols, int32_t n_cols, const uint8_t* skip) {
  if (!agg || !cols) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Agg& a = agg->impl;
  if (!a.res.ready) return SetError(PXG_FAILED_PRECONDITION, "pxg_agg_finalize has not run since the last consume");
  const int32_t n_val_cols = a.emit_states ? 1 : a.n_udas;
  if (n_cols != a.n_keys + n_val_cols) return SetError(PXG_INVALID_ARGUMENT, "expected %d result columns", a.n_keys + n_val_cols);
  const int64_t G = a.res.n_groups;
  const bool synth = a.n_keys == 0 && G == 0;  // AggregateGroupByNone over no rows
  const int64_t rows = synth ? 1 : G;
  // The copies below are queued into pooled pinned blocks: an early error return must not leave
  // one in flight, or the caller's pxg_result_free could hand a block to the next query while a
  // DMA still writes into it.
  struct DrainOnExit {
    hipStream_t s;
    ~DrainOnExit() { (void)hipStreamSynchronize(s); }
  } drain{a.ctx->stream};
  for (int c = 0; c < n_cols; ++c) std::memset(&cols[c], 0, sizeof(cols[c]));
  for (int k = 0; k < a.n_keys; ++k) {
    pxg_column_out& o = cols[k];
    o.type = a.key_types[k];
    o.length = rows;
    if (o.type == PXG_STRING) {
      o.offsets = static_cast<int32_t*>(ResultAlloc((rows + 1) * 4));
      o.data = static_cast<uint8_t*>(ResultAlloc(a.res.key_data_len[k] + 16));
      o.data_len = a.res.key_data_len[k];
      if (G > 0) {
        PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.offsets, a.res.key_offsets[k].p, (G + 1) * 4));
        PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.data, a.res.key_data[k].p, o.data_len));
      } else {
        o.offsets[0] = 0;
      }
    } else {
      const size_t w = TypeWidth(o.type);
      o.values = ResultAlloc(std::max<size_t>(rows * w, 1));
      if (G > 0) {
        if (o.type == PXG_BOOLEAN) {
          PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.values, a.res.key_fixed[k].p, G));
        } else {
          PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.values, a.res.key_fixed[k].p, G * w));
        }
      }
    }
  }
  if (a.emit_states) {  // serialized_expressions: fixed-size records (operators.cc:251-257)
    pxg_column_out& o = cols[a.n_keys];
    o.type = PXG_STRING;
    o.length = rows;
    const int64_t rec = a.state_rec;
    o.offsets = static_cast<int32_t*>(ResultAlloc((rows + 1) * 4));
    o.data = static_cast<uint8_t*>(ResultAlloc(rows * rec + 16));
    o.data_len = rows * rec;
    for (int64_t g = 0; g <= rows; ++g) o.offsets[g] = static_cast<int32_t>(g * rec);
    if (!synth) {
      if (G > 0 && rec > 0) PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.data, a.res.states.p, G * rec));
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
    PXG_HIP(hipStreamSynchronize(a.ctx->stream));
    return PXG_OK;
  }
  for (int u = 0; u < a.n_udas; ++u) {
    pxg_column_out& o = cols[a.n_keys + u];
    o.type = a.uda_out_type[u];
    o.length = rows;
    if (skip && (skip[a.n_keys + u] & kSkipLanes) && a.uda_kind[u] == PXG_UDA_QUANTILES && !synth) {
      PXG_RETURN_IF_ERROR(IssueLanes(a, u, skip[a.n_keys + u], o));
      continue;
    }
    if (skip && skip[a.n_keys + u] && !synth) continue;  // left without buffers (the caller fetches it otherwise)
    const bool q = a.uda_kind[u] == PXG_UDA_QUANTILES;
    const size_t per = q ? 56 : 8;
    o.values = ResultAlloc(std::max<size_t>(rows * per, 8));
    if (!synth) {
      PXG_RETURN_IF_ERROR(CopyD2H(a.ctx, a.ctx->stream, o.values, a.res.uda_out[u].p, G * per));
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
  PXG_HIP(hipStreamSynchronize(a.ctx->stream));
  return PXG_OK;
}

int32_t pxg::LaunchDigestMerge(Agg* a, const uint32_t* dlist, const uint32_t* dcount, uint32_t cap_list) {
  Ctx* ctx = a->ctx;
  if (!a->x_vals || !a->x_wts || cap_list == 0) return PXG_OK;
  const uint64_t n = a->st_n;
  Agg::FinalizeWs& ws = a->ws;
  PXG_RETURN_IF_ERROR(ws.mrg.Ensure(n * 32 + 64));
  uint64_t* k0 = ws.mrg.as<uint64_t>();
  uint32_t* d_err = reinterpret_cast<uint32_t*>(ws.meta.as<uint8_t>() + 16);
  PXG_HIP(hipMemsetAsync(d_err, 0, 4, ctx->stream));
  for (int u = 0; u < a->n_udas; ++u) {
    if (a->uda_kind[u] != PXG_UDA_QUANTILES) continue;
    PXG_RETURN_IF_ERROR(Launch(ctx, "digest_merge", DigestMergeKernel, dim3(cap_list), dim3(kMergeThreads), 0, dlist, dcount,
                               ws.gstart.as<const uint32_t>(), a->x_vals, a->x_wts, a->uda_arg_type[u], k0, k0 + n, k0 + 2 * n, k0 + 3 * n,
                               a->res.uda_out[u].as<double>(), d_err));
  }
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + 120);
  PXG_HIP(hipMemcpyAsync(pin, d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  if (*pin) return SetError(PXG_INTERNAL, "merged digest overflow (flags %u)", *pin);
  return PXG_OK;
}

// Diagnostics: one merged digest (DigestMergeKernel) over n items already in part order
// (tests/test_digest_merge.py compares it with oracle/tdigest.h merge_batch).
extern "C" int32_t pxg_digest_merge(pxg_ctx* ctx, const uint64_t* d_vals, const uint64_t* d_wt, int64_t n, int32_t arg_type, double* d_out7) {
  if (!ctx || !d_vals || !d_wt || !d_out7 || n <= 0 || n >= (int64_t(1) << 31)) return SetError(PXG_INVALID_ARGUMENT, "bad pxg_digest_merge arguments");
  Ctx* c = &ctx->impl;
  DevBuf scratch;
  PXG_RETURN_IF_ERROR(scratch.Alloc(static_cast<size_t>(n) * 32 + 64));
  uint64_t* k0 = scratch.as<uint64_t>();
  uint32_t* meta = reinterpret_cast<uint32_t*>(k0 + 4 * n);
  const uint32_t hmeta[4] = {0u, 1u, 0u, static_cast<uint32_t>(n)};  // list {0}, count 1, gstart {0, n}
  PXG_HIP(hipMemcpyAsync(meta, hmeta, sizeof(hmeta), hipMemcpyHostToDevice, c->stream));
  PXG_HIP(hipMemsetAsync(meta + 4, 0, 4, c->stream));
  PXG_RETURN_IF_ERROR(Launch(c, "digest_merge", DigestMergeKernel, dim3(1), dim3(kMergeThreads), 0, static_cast<const uint32_t*>(meta),
                             static_cast<const uint32_t*>(meta + 1), static_cast<const uint32_t*>(meta + 2), d_vals, d_wt, arg_type, k0, k0 + n,
                             k0 + 2 * n, k0 + 3 * n, d_out7, meta + 4));
  uint32_t errv = 0;
  PXG_HIP(hipMemcpyAsync(&errv, meta + 4, 4, hipMemcpyDeviceToHost, c->stream));
  PXG_HIP(hipStreamSynchronize(c->stream));
  if (errv) return SetError(PXG_INTERNAL, "merged digest overflow (flags %u)", errv);
  return PXG_OK;
}

// Diagnostics: chains for given W by either chain builder (tests compare them).
__global__ void DiagChainKernel(const int64_t* __restrict__ w, int32_t n, int32_t wave, uint32_t* __restrict__ starts, int32_t cap,
                                int32_t* __restrict__ nc) {
  const int32_t i = static_cast<int32_t>((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (i >= n) return;
  uint32_t* s = starts + static_cast<uint64_t>(i) * cap;
  int64_t r;
  if (wave == 2) {  // instrumented: cycles in evaluation / resolution, rounds, rounds with an exact-path lane
    r = DigestBoundariesWave<true>(w[i], s, cap - 8, reinterpret_cast<uint64_t*>(s + cap - 8));
  } else if (wave) {
    r = DigestBoundariesWave(w[i], s, cap);
  } else {
    if ((threadIdx.x & 63) != 0) return;
    r = DigestBoundaries(w[i], s, cap);
  }
  if ((threadIdx.x & 63) == 0) nc[i] = static_cast<int32_t>(r);
}

extern "C" int32_t pxg_digest_chains(pxg_ctx* ctx, const int64_t* d_w, int32_t n, int32_t wave, uint32_t* d_starts, int32_t cap,
                                     int32_t* d_nc) {
  if (!ctx || !d_w || !d_starts || !d_nc || n < 0 || cap <= 0) return SetError(PXG_INVALID_ARGUMENT, "bad pxg_digest_chains arguments");
  if (n == 0) return PXG_OK;
  Ctx* c = &ctx->impl;
  PXG_RETURN_IF_ERROR(Launch(c, "diag_chain", DiagChainKernel, dim3((n + 3) / 4), dim3(256), 0, d_w, n, wave, d_starts, cap, d_nc));
  PXG_HIP(hipStreamSynchronize(c->stream));
  return PXG_OK;
}
