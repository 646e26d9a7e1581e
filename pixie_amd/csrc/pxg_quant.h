// Device pieces shared by the quantile digests of pxg_finalize.hip (tiny / small / mid classes,
// the big groups' sort path) and the selection path (pxg_select.hip): sort keys of the values,
// LDS merge sorts, the block digest, chain and big-group records.
#pragma once

#include <cstdint>

#include "pxg_device.h"
#include "pxg_keys.h"
#include "pxg_tdigest.h"

namespace pxg {

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


__device__ __forceinline__ uint64_t QKey(uint64_t raw, int arg_type) {
  const uint64_t bits = arg_type == PXG_FLOAT64 ? raw : FBits(static_cast<double>(static_cast<int64_t>(raw)));
  return SortKeyF(bits);
}
__device__ __forceinline__ double QVal(uint64_t key) { return AsF(FromSortKeyF(key)); }
// QKey with the argument type fixed at compile time (the selection passes: no int64 conversion
// computed and discarded per value).
template <bool kF64>
__device__ __forceinline__ uint64_t QKeyT(uint64_t raw) {
  return SortKeyF(kF64 ? raw : FBits(static_cast<double>(static_cast<int64_t>(raw))));
}

constexpr uint64_t kNegInfKey = 0x000FFFFFFFFFFFFFULL;  // SortKeyF(-inf) = ~0xFFF0... = 0x000F...F
constexpr uint64_t kPosInfKey = 0xFFF0000000000000ULL;  // SortKeyF(+inf) = 0x7FF0... ^ 0x8000...


// ---------------------------------------------------------------------------------------
// Merge sort of up to 16 * (threads) u64 keys in LDS (replaces the LDS bitonic sort:
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

// (Round 6: sorting each wave's runs of up to 1024 keys in registers first -- a bitonic network
// with the lane-crossing steps as shuffles, replacing the first six merge rounds -- passed the
// digest parity tests but measured no faster: C2 step 2.055 / 2.093 vs 2.047 / 2.111 ms, N1
// 14.71 / 14.69 vs 14.50 / 14.63 ms, quant_mid 0.21 ms either way at C2.  The mid / small digests
// are not bound by these merge rounds.)
// Sorts a[0, P) (logical indices, PadIdx layout), P a power of two in [16, 16 * nthreads],
// by the nthreads threads t = 0.. of a workgroup (kWave = false: block barriers) or of one wave
// (kWave = true: wave-local LDS ordering only).
template <bool kWave>
__device__ void MergeSortLds(uint64_t* a, int P, int t) {
  auto sync = [] {
    if (kWave) WaveSync();
    else __syncthreads();
  };
  const bool act = t * kMsIpt < P;
  uint64_t r[kMsIpt];
  if (act) {
#pragma unroll
    for (int i = 0; i < kMsIpt; ++i) r[i] = a[PadIdx(t * kMsIpt + i)];
    SortNetwork16(r);
#pragma unroll
    for (int i = 0; i < kMsIpt; ++i) a[PadIdx(t * kMsIpt + i)] = r[i];
  }
  sync();
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
    sync();
    if (act) {
#pragma unroll
      for (int k = 0; k < kMsIpt; ++k) a[PadIdx(t * kMsIpt + k)] = r[k];
    }
    sync();
  }
}
__device__ __forceinline__ void BlockMergeSortLds(uint64_t* a, int P) { MergeSortLds<false>(a, P, threadIdx.x); }
__device__ __forceinline__ void WaveMergeSortLds(uint64_t* a, int P) { MergeSortLds<true>(a, P, threadIdx.x & 63); }
constexpr int kWaveSortMax = 64 * kMsIpt;  // 1024

constexpr int kMidMax = 4096;
constexpr int kMidCentroids = 2048;


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

constexpr int kNeed = 7 * 4;
constexpr int64_t kSeqMean = 16;

struct DigestShared {
  int64_t meta[4];
  int32_t need[kNeed];
  double mean[kNeed];
  double red[16];  // per-wave partial sums (workgroups of up to 1024 threads)
};

// Centroid boundaries precomputed by DigestChainKernel for a group assumed NaN-free (W = n);
// `starts` == nullptr: none.
struct PreChain {
  const uint32_t* starts;
  int64_t nc;
  int64_t W;
};


constexpr int kChainCap = 2048;
constexpr int kChainWaves = 4;

__device__ __forceinline__ PreChain PreChainAt(const uint32_t* starts_all, const int32_t* nc_all, uint32_t i, int64_t n) {
  PreChain p;
  p.starts = starts_all ? starts_all + static_cast<uint64_t>(i) * kChainCap : nullptr;
  p.nc = starts_all ? nc_all[i] : -1;
  p.W = n;
  return p;
}

// kStagePre: starts_buf is LDS; a precomputed chain is copied into it first (one coalesced
// pass), so the quantile searches and centroid ranges read LDS instead of chains of dependent
// global loads.
template <bool kStagePre = false, typename KeyAt>
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
  if (kStagePre && use_pre && pre.nc <= max_c) {  // the barrier below orders the copy
    for (int64_t j = t; j < pre.nc; j += blockDim.x) starts_buf[j] = pre.starts[j];
    starts = starts_buf;
  }
  if (t == 0) {
    int64_t nc;
    if (use_pre) nc = pre.nc;
    else nc = DigestBoundaries(W, starts_buf, max_c);
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


// Big groups: chunk sort (one workgroup per 4096-element chunk) into sort keys.
struct BigChunk {
  uint64_t off;    // absolute staging offset of the chunk
  uint64_t g_off;  // absolute staging offset of its group
  uint32_t len;    // <= kMidMax
  uint32_t g_n;    // group size
  uint32_t passes; // merge passes the group needs (ceil(log2(g_n / kMidMax)))
  uint32_t bidx;   // index of its group in the big-group list
};


struct BigGroup {
  uint64_t off;     // absolute staging offset of the group
  uint64_t n;
  uint32_t c0;      // its first chunk
  uint32_t nch;     // its chunk count
  uint32_t g;
  uint32_t passes;  // merge passes it needs: its sorted keys end in keysA (even) / keysB (odd)
};


// Groups above this many values select with 4096 bins and an 8192-key sample (SelNb).
constexpr uint64_t kSelLargeN = uint64_t(1) << 21;

// Floating-point sums in double-double (an error-free TwoSum per addition, the error words
// summed beside): a group's sum is then its exact sum to ~2^-100 relative, rounded once at the
// end, so it no longer depends on the order its values were staged in (that order is the
// consume's tile completion order, which differs run to run; plain double sums differed in the
// last bits).  The reference sums sequentially in double; both agree to its rounding.
// Compiled with -ffp-contract=off (the transformations need unfused operations).
// Determinism holds while a group's values span less than ~2^100 in magnitude (the low word
// keeps ~53 more bits below the high one); beyond that, or under heavy cancellation, the rounded
// result can still depend on the staging order.
// Non-finite sums: once hi is +-inf or NaN (an inf / NaN value, or an overflow) the error word
// is pinned to 0, so the result is the plain sequential sum's inf / NaN (the reference's), not
// the NaN that inf - inf inside the error term would give.
struct DD {
  double hi, lo;
};
__device__ __forceinline__ DD TwoSum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  const double e = (a - (s - bb)) + (b - bb);
  return DD{s, isfinite(s) ? e : 0.0};
}
__device__ __forceinline__ DD DDAdd(DD x, DD y) {
  const DD s = TwoSum(x.hi, y.hi);
  const double e = s.lo + (x.lo + y.lo);
  const double h = s.hi + e;
  return DD{h, isfinite(h) ? e - (h - s.hi) : 0.0};
}
__device__ __forceinline__ DD DDAddD(DD x, double b) { return DDAdd(x, DD{b, 0.0}); }
__device__ __forceinline__ DD WaveSumDD(DD v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = DDAdd(v, DD{__shfl_xor(v.hi, o, 64), __shfl_xor(v.lo, o, 64)});
  return v;
}
// The rounded sum (non-finite: the plain sum's inf / NaN, whose error words are meaningless).
__device__ __forceinline__ double DDValue(DD v) { return isfinite(v.hi) ? v.hi + v.lo : v.hi; }

}  // namespace pxg
