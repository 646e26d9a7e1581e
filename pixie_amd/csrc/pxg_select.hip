// The selection path of the quantile digests' big groups (groups above the mid classes):
// sample -> splitters, bin counts, plan, gather + inside sums, bin sorts, digests, per set of
// big groups (pxg_select.h BigSet).  Split out of pxg_finalize.hip, which orchestrates it
// (AggFinalizeTable: the early set of a fused split's designated groups, the late set of the
// classification's class 3).  Reference: the same QuantilesUDA digests (math_sketches.h:33-82)
// as the sort path; see the comment below for the algorithm.
#include <algorithm>

#include "pxg_agg_host.h"
#include "pxg_keys.h"
#include "pxg_quant.h"
#include "pxg_select.h"
#include "pxg_tdigest.h"

namespace pxg {

// ---------------------------------------------------------------------------------------
// Big groups by selection.  A digest reads at most 4 centroid means per quantile, each the
// mean of a known range of sorted ranks (the chain depends on W only), so a big group is never
// sorted.  Its values are binned by splitters taken from a sorted sample (BigSample), the bins
// are counted (BigHist), the bins holding the needed ranges' ends are chosen (BigPlan), their
// values gathered while the ranks strictly inside a range are summed in place (BigCollect),
// the gathered bins sorted (BigBinSort), and the means and quantiles formed (BigSelDigest).
// Centroids of <= kSeqMean values (every centroid while W <= ~10000) get the reference's
// incremental mean over their sorted values, as in BlockDigest; larger ones sum/count with a
// fixed summation order (deterministic).  A group the path cannot serve (NaN values, a bin to
// gather beyond LDS capacity: heavy duplicates, too many bins) is flagged; finalize then runs
// the full sort + merge path (BigChunkSort / BigMergeTile / BigDigest) for the big groups.
// ---------------------------------------------------------------------------------------
// 4096 bins keep the gathered bins of a multi-million-value group (the largest C2 group at
// 1B rows holds ~6.9M values: ~1.7K per bin) far below the largest LDS sort (16384 keys).
constexpr int kSelBins = 4096;
constexpr int kSelBinBits = 12;
constexpr int kSelSample = 8192;  // two samples per bin
constexpr int kSelMaxRanges = kNeed;
constexpr int kSelMaxColl = 256;
constexpr int kSelHugeThreads = 1024;
constexpr uint32_t kSelCollCap = kSelHugeThreads * kMsIpt;  // 16384
constexpr int kSelLists = 3;  // gathered bins: <= 1024 values (wave), <= 4096 (256 threads), larger (1024 threads)

// Bins actually used by a group of n values (the rest hold splitter ~0 and stay empty): <= 2048
// values per bin on average, so a gathered bin beyond kSelCollCap is a ~1e-6 event per bin.
// Groups under 16K values use ~16-32 values per bin (128..1024 bins): their sample (2 nb keys)
// and its sort stay a small fraction of the group (at 1B rows 1,872 of the 2,692 big groups hold
// 4K-16K values; a 2048-key sample of a 5000-value group cost almost a sort of the group).
// Groups above kSelLargeN (2M) values use all 4096 bins (an 8192-key sample, the 512-thread
// launch over BigSetup's list of them): with 2048 bins a 6.9M-value group averaged ~3.4K values
// per bin, and a gathered bin holds a Gamma(2)-distributed multiple of that (the splitters are
// every other sample), so one past kSelCollCap (4.9x the mean) sent the group to the sort path in
// ~5% of 1B-row finalizes (tools/n1_fallback.py: 2 of 40).  At 4096 bins that is 9.7x the mean
// (~1e-7 per bin).  Those groups are the designated ones of the fused split, whose selection
// runs off the critical path (the early set).
__device__ __forceinline__ int SelNb(uint64_t n) {
  if (n > kSelLargeN) return kSelBins;
  int nb = kSelBins / 4;
  while (nb > 128 && static_cast<uint64_t>(nb) * 16 > n) nb >>= 1;
  return nb;
}
constexpr uint8_t kTagColl = 0x80;

struct BigPlan {
  int32_t nc;        // centroids
  int32_t n_ranges;  // distinct centroids the quantiles read
  int32_t n_coll;    // bins to gather
  int32_t fallback;  // 1: the full sort path serves this group
  int32_t need_u[kNeed];  // DigestQuantile mean call (q * 4 + k) -> range
  int32_t rj[kSelMaxRanges];
  uint32_t rs[kSelMaxRanges], re[kSelMaxRanges];    // rank range [rs, re)
  uint32_t rbs[kSelMaxRanges], rbe[kSelMaxRanges];  // bins of its first and last rank
  uint16_t coll[kSelMaxColl];                       // bins to gather, ascending
};

static_assert(sizeof(BigPlan) % 4 == 0, "BigPlan is copied as words");

// Bin of a sort key: the last b with S[b] <= key (S[0] = 0, S non-decreasing).  A group using
// nb < kSelBins bins has S[b >= nb] = ~0: only an all-ones key lands there (bin kSelBins - 1),
// so the search runs over [0, nb) and then checks that one case.
__device__ __forceinline__ int SelBin(const uint64_t* S, uint64_t key, int nb) {
  int b = 0;
  for (int step = nb >> 1; step >= 1; step >>= 1)
    if (S[b + step] <= key) b += step;
  return key == ~0ULL ? kSelBins - 1 : b;
}
// Bin holding rank r: the last b with bs[b] <= r (bs = exclusive prefix of the bin counts;
// that bin is never empty since bs[b + 1] > r).
__device__ __forceinline__ int BinOfRank(const uint32_t* bs, uint32_t r) {
  int b = 0;
#pragma unroll
  for (int step = kSelBins / 2; step >= 1; step >>= 1)
    if (bs[b + step] <= r) b += step;
  return b;
}

// Guide table per group: kSelGuide equal-width buckets of the key range [lo, hi] = [S[1],
// S[nb - 1]] (bucket i starts at lo + (i << sh), sh the smallest shift that leaves fewer than
// kSelGuide buckets), entry i = SelBin of the bucket's start.  A key's bin then lies between
// the entries of its bucket and its successor: a few splitter reads instead of a 12-step
// search (bins are equi-depth, buckets equal-width; a bucket holds ~2 bins on average, ~6 at
// the densest part of a lognormal).  The search result is SelBin's, bit for bit.
constexpr int kSelGuideBits = 11;
constexpr int kSelGuide = 1 << kSelGuideBits;
constexpr int kSelGuideStride = kSelGuide + 2;  // u16 entries per group (kSelGuide + 1 used)

__device__ __forceinline__ int SelGuideShift(uint64_t span) {
  const int bits = span == 0 ? 0 : 64 - __clzll(static_cast<long long>(span));
  return bits > kSelGuideBits ? bits - kSelGuideBits : 0;
}
__device__ __forceinline__ uint64_t SelGuideStart(uint64_t lo, int i, int sh) {
  const uint64_t off = static_cast<uint64_t>(i) << sh;
  if ((off >> sh) != static_cast<uint64_t>(i)) return ~0ULL;
  const uint64_t v = lo + off;
  return v < lo ? ~0ULL : v;
}
// Per-group constants of the guided search (S in LDS with S[0] = 0, nb >= 2).
struct SelGuideK {
  uint64_t lo, hi;
  int sh, nb;
};
__device__ __forceinline__ SelGuideK SelGuideOf(const uint64_t* S, int nb) {
  SelGuideK g;
  g.lo = S[1];
  g.hi = S[nb - 1];
  g.sh = SelGuideShift(g.hi - g.lo);
  g.nb = nb;
  return g;
}
// Bracket [b, e] of a key's bin from the guide (b == e: decided).  Selects only: a branch
// here made the compiler copy the callers' whole per-value arrays on every path.
__device__ __forceinline__ void SelGuideBracket(const uint16_t* Gd, const SelGuideK& g, uint64_t key, int& b, int& e) {
  const bool below = key < g.lo, above = key >= g.hi, ones = key == ~0ULL;
  const int gi = (below || above) ? 0 : static_cast<int>((key - g.lo) >> g.sh);
  const int gb = Gd[gi], ge = Gd[gi + 1];
  const int fixed = ones ? kSelBins - 1 : below ? 0 : g.nb - 1;
  const bool dec = below || above;  // (ones implies above)
  b = dec ? fixed : gb;
  e = dec ? fixed : ge;
}
// Last index in [b, e] whose splitter is <= key (S[b] <= key holds): binary lifting, the
// rare wide brackets first, then three fixed steps.
// Branch-free steps (the probe index is clamped to e, so every load is in range and no step
// needs its own exec mask).
__device__ __forceinline__ int SelGuideFinish(const uint64_t* S, uint64_t key, int b, int e) {
  const int d = e - b;
  if (d > 7) {
    for (int step = 1 << (31 - __clz(d)); step >= 8; step >>= 1) {
      const int m = min(b + step, e);
      b = (b + step <= e && S[m] <= key) ? m : b;
    }
  }
#pragma unroll
  for (int step = 4; step >= 1; step >>= 1) {
    const int m = min(b + step, e);
    const uint64_t sm = S[m];
    b = (b + step <= e && sm <= key) ? m : b;
  }
  return b;
}

// Splitters: 2 * nb keys at evenly spaced positions of the group, sorted; S[b] = every second
// of them (b < nb), S[0] = 0, S[b >= nb] = ~0 (empty bins).  Two launches: groups sampling
// <= 4096 keys (256 threads, 35 KB of LDS) and the few sampling 8192 (512 threads, 70 KB), so
// the common case is not held to the large kernel's occupancy.
template <int NS>
__global__ void __launch_bounds__(NS / kMsIpt) BigSampleKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ nbig_p,
                                                               const uint64_t* __restrict__ vals, int arg_type, uint64_t* __restrict__ spl,
                                                               uint16_t* __restrict__ guide, const uint32_t* __restrict__ only,
                                                               const uint32_t* __restrict__ only_cnt) {
  // only != nullptr: block i serves big group only[i] (i < *only_cnt).
  if (blockIdx.x >= (only ? *only_cnt : *nbig_p)) return;
  const uint32_t bi = only ? only[blockIdx.x] : blockIdx.x;
  const BigGroup G = groups[bi];
  const int nb = SelNb(G.n), ns = 2 * nb;
  if (ns > NS || (NS > kSelSample / 2 && ns <= kSelSample / 2)) return;  // the other launch's group
  __shared__ uint64_t keys[PaddedLen(NS)];
  // ns is a power of two: run r starts at (2r + 1) n / (2 ns / kSampleRun) by a shift; every
  // load of a thread is issued before any is used.
  // Runs of kSampleRun consecutive values (one 64-byte line) at ns / kSampleRun evenly spaced
  // positions: 8x fewer lines fetched than single values, still spread over the whole group.
  // The splitters only shape the bins; every result is exact whichever sample is taken.
  constexpr int kSampleRun = 8;
  const int sh = __ffs(2 * (ns / kSampleRun)) - 1;
  constexpr int kPerT = NS / (NS / kMsIpt);
  uint64_t raw[kPerT];
#pragma unroll
  for (int q = 0; q < kPerT; ++q) {
    const int j = q * blockDim.x + threadIdx.x;
    const uint64_t r = static_cast<uint64_t>(j / kSampleRun);
    const uint64_t at = min(((2 * r + 1) * G.n) >> sh, G.n - kSampleRun) + static_cast<uint64_t>(j % kSampleRun);
    raw[q] = j < ns ? vals[G.off + at] : 0ULL;
  }
#pragma unroll
  for (int q = 0; q < kPerT; ++q) {
    const int j = q * blockDim.x + threadIdx.x;
    if (j < ns) keys[PadIdx(j)] = QKey(raw[q], arg_type);
  }
  __syncthreads();
  BlockMergeSortLds(keys, ns);
  uint64_t* S = spl + static_cast<uint64_t>(bi) * kSelBins;
  for (int b = threadIdx.x; b < kSelBins; b += blockDim.x) S[b] = b == 0 ? 0ULL : b < nb ? keys[PadIdx(2 * b)] : ~0ULL;
  auto Sk = [&](int b) -> uint64_t { return b == 0 ? 0ULL : keys[PadIdx(2 * b)]; };
  const uint64_t lo = Sk(1), hi = Sk(nb - 1);
  const int gsh = SelGuideShift(hi - lo);
  uint16_t* Gd = guide + static_cast<uint64_t>(bi) * kSelGuideStride;
  for (int i = threadIdx.x; i <= kSelGuide; i += blockDim.x) {
    const uint64_t v = SelGuideStart(lo, i, gsh);
    int b = 0;
    for (int step = nb >> 1; step >= 1; step >>= 1)
      if (Sk(b + step) <= v) b += step;
    Gd[i] = static_cast<uint16_t>(b);
  }
}

// Bin counts (and NaN count) per big group.  A workgroup takes cpb consecutive 4096-value
// chunks (a group's chunks are consecutive; cpb = SelChunksPerBlock): the splitters are loaded
// and the LDS counts flushed to the group's global histogram once per group it meets, not once
// per chunk.  Both BigHist and BigCollect load the next chunk while binning the current one,
// so one resident round of blocks (3 per CU: LDS and VGPRs) keeps the memory system busy.
// cpb is rounded up, so the grid never exceeds blocks_per_cu per CU (a second, partial round
// of blocks would run alone on part of the chip).
static uint32_t SelChunksPerBlock(uint32_t nchunks, int num_cus, uint32_t blocks_per_cu, uint32_t cap = 8) {
  const uint32_t slots = blocks_per_cu * static_cast<uint32_t>(num_cus);
  return std::max<uint32_t>(1, std::min<uint32_t>(cap, (nchunks + slots - 1) / slots));
}
// quant_sel_hist's cap on chunks per block (64: measured in round 3 against 8 / 16 / 32, fewer
// histogram flushes per group).
constexpr uint32_t kSelHistCap = 64;
template <bool kF64>
__global__ void __launch_bounds__(256) BigHistKernel(const BigChunk* __restrict__ chunks, const uint32_t* __restrict__ nchunks_p,
                                                     const uint64_t* __restrict__ vals, int arg_type, const uint64_t* __restrict__ spl,
                                                     const uint16_t* __restrict__ guide, uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ nan_cnt, uint32_t cpb, uint16_t* __restrict__ bin_out) {
  const uint32_t nchunks = *nchunks_p;
  const uint32_t c0 = blockIdx.x * cpb;
  if (c0 >= nchunks) return;
  const uint32_t c1 = min(nchunks, c0 + cpb);
  __shared__ uint64_t S[kSelBins];
  __shared__ uint32_t h[kSelBins];
  __shared__ uint16_t Gd[kSelGuide + 1];
  __shared__ uint32_t s_nan;
  constexpr int kPer = kMidMax / 256;
  uint32_t cur = 0xFFFFFFFFu;
  SelGuideK gk{0, 0, 0, 2};
  // The next chunk's values are loaded while the current one is binned.
  // Loads past a chunk's end re-read its last value (no exec-masked load branches; those
  // lanes are not counted).
  BigChunk c = chunks[c0];
  uint64_t raw[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) raw[k] = vals[c.off + min(k * 256 + static_cast<int>(threadIdx.x), static_cast<int>(c.len) - 1)];
  for (uint32_t ci = c0; ci < c1; ++ci) {
    const BigChunk cn = ci + 1 < c1 ? chunks[ci + 1] : c;  // the last chunk re-reads itself
    uint64_t rawn[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) rawn[k] = vals[cn.off + min(k * 256 + static_cast<int>(threadIdx.x), static_cast<int>(cn.len) - 1)];
    if (c.bidx != cur) {
      if (cur != 0xFFFFFFFFu) {  // flush the previous group's counts
        __syncthreads();
        uint32_t* H = hist + static_cast<uint64_t>(cur) * kSelBins;
        for (int b = threadIdx.x; b < kSelBins; b += 256)
          if (h[b]) atomicAdd(&H[b], h[b]);
        if (threadIdx.x == 0 && s_nan) atomicAdd(&nan_cnt[cur], s_nan);
        __syncthreads();
      }
      cur = c.bidx;
      const int nb = SelNb(c.g_n);
      const uint64_t* Sg = spl + static_cast<uint64_t>(cur) * kSelBins;
      const uint16_t* Gg = guide + static_cast<uint64_t>(cur) * kSelGuideStride;
      for (int b = threadIdx.x; b < kSelBins; b += 256) {
        S[b] = b < nb ? Sg[b] : ~0ULL;
        h[b] = 0;
      }
      for (int i = threadIdx.x; i <= kSelGuide; i += 256) Gd[i] = Gg[i];
      if (threadIdx.x == 0) s_nan = 0;
      __syncthreads();
      gk = SelGuideOf(S, nb);
    }
    // Every value's bracket, then the lifting steps (16 independent searches in flight), then
    // the LDS counts: an atomic between two searches would order the next one's reads behind it.
    // (Keys are recomputed from raw rather than kept: 32 fewer VGPRs, one more wave per SIMD.)
    uint32_t nn = 0;
    int bin[kPer], bend[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint64_t key = QKeyT<kF64>(raw[k]);
      const int i = k * 256 + threadIdx.x;
      nn += (i < static_cast<int>(c.len) && (key < kNegInfKey || key > kPosInfKey)) ? 1u : 0u;
      SelGuideBracket(Gd, gk, key, bin[k], bend[k]);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) bin[k] = SelGuideFinish(S, QKeyT<kF64>(raw[k]), bin[k], bend[k]);
    // Each value's bin, for BigCollect (which then needs neither the splitters nor the search).
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (k * 256 + static_cast<int>(threadIdx.x) < static_cast<int>(c.len)) bin_out[c.off + k * 256 + threadIdx.x] = static_cast<uint16_t>(bin[k]);
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (k * 256 + static_cast<int>(threadIdx.x) < static_cast<int>(c.len)) atomicAdd(&h[bin[k]], 1u);
    if (nn) atomicAdd(&s_nan, nn);
    c = cn;
#pragma unroll
    for (int k = 0; k < kPer; ++k) raw[k] = rawn[k];
  }
  __syncthreads();
  uint32_t* H = hist + static_cast<uint64_t>(cur) * kSelBins;
  for (int b = threadIdx.x; b < kSelBins; b += 256)  // bins >= nb only see all-ones keys
    if (h[b]) atomicAdd(&H[b], h[b]);
  if (threadIdx.x == 0 && s_nan) atomicAdd(&nan_cnt[cur], s_nan);
}

// Per big group: bin starts, the centroids the quantiles read (DigestQuantile's recording
// pass, as in BlockDigest), their rank ranges and bins, the bin tags (gather / inside range u)
// and the gather offsets.
__global__ void __launch_bounds__(256) BigPlanKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ nbig_p,
                                                     const uint32_t* __restrict__ chain_starts, const int32_t* __restrict__ chain_nc,
                                                     const uint32_t* __restrict__ hist, const uint32_t* __restrict__ nan_cnt,
                                                     uint32_t* __restrict__ bstart_all, uint8_t* __restrict__ tag_all,
                                                     uint32_t* __restrict__ cbase_all, BigPlan* __restrict__ plans,
                                                     unsigned int* __restrict__ n_fallback, uint32_t* __restrict__ bin_lists,
                                                     uint32_t list_cap, uint32_t* __restrict__ list_cnt) {
  if (blockIdx.x >= *nbig_p) return;
  __shared__ uint32_t bs[kSelBins + 1];
  __shared__ uint8_t tg[kSelBins];
  __shared__ uint32_t s_scan[256], s_scan2[256];
  __shared__ BigPlan P;
  __shared__ int32_t s_need[kNeed];
  __shared__ int s_fb;
  const int t = threadIdx.x;
  const uint32_t bi = blockIdx.x;
  const BigGroup G = groups[bi];
  const int64_t W = static_cast<int64_t>(G.n);
  const uint32_t* H = hist + static_cast<uint64_t>(bi) * kSelBins;
  const int32_t nc = chain_nc[bi];
  // The chain staged in LDS for the recording pass's searches (ordered by the barriers below).
  __shared__ uint32_t s_starts[kChainCap];
  {
    const uint32_t* gs = chain_starts + static_cast<uint64_t>(bi) * kChainCap;
    for (int j = t; j < nc; j += 256) s_starts[j] = gs[j];
  }
  const uint32_t* starts = s_starts;
  constexpr int kPer = kSelBins / 256;
  // exclusive scan of the bin counts
  uint32_t cnt[kPer], tot = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    cnt[k] = H[t * kPer + k];
    tot += cnt[k];
  }
  s_scan[t] = tot;
  if (t == 0) s_fb = (nan_cnt[bi] != 0 || nc < 0) ? 1 : 0;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t x = t >= o ? s_scan[t - o] : 0u;
    __syncthreads();
    s_scan[t] += x;
    __syncthreads();
  }
  {
    uint32_t run = s_scan[t] - tot;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      bs[t * kPer + k] = run;
      run += cnt[k];
    }
    if (t == 255) bs[kSelBins] = run;
  }
  if (t < kNeed) s_need[t] = -1;
  __syncthreads();
  if (s_fb) {
    if (t == 0) {
      P.fallback = 1;
      atomicAdd(n_fallback, 1u);
    }
    __syncthreads();
    if (t == 0) plans[bi].fallback = 1;
    return;
  }
  auto start = [&](int64_t j) -> int64_t { return starts[j]; };
  if (t < 7) {
    int k = 0;
    (void)DigestQuantile(kQuantileQ[t], nc, W, start, [&](int64_t j) -> double {
      if (k < 4) s_need[t * 4 + k] = static_cast<int32_t>(j);
      ++k;
      return 0.0;
    });
  }
  for (int b = t; b < kSelBins; b += 256) tg[b] = 0;
  __syncthreads();
  if (t == 0) {
    int nr = 0;
    for (int i = 0; i < kNeed; ++i) {
      const int32_t j = s_need[i];
      int u = -1;
      if (j >= 0) {
        for (int v = 0; v < nr; ++v)
          if (P.rj[v] == j) u = v;
        if (u < 0) {
          u = nr++;
          const uint32_t s = starts[j];
          const uint32_t e = j + 1 < nc ? starts[j + 1] : static_cast<uint32_t>(W);
          P.rj[u] = j;
          P.rs[u] = s;
          P.re[u] = e;
        }
      }
      P.need_u[i] = u;
    }
    P.n_ranges = nr;
    P.nc = nc;
    P.fallback = 0;
  }
  __syncthreads();
  if (t < P.n_ranges) {  // the ranges' end bins, one thread per range (12-step LDS searches)
    P.rbs[t] = static_cast<uint32_t>(BinOfRank(bs, P.rs[t]));
    P.rbe[t] = static_cast<uint32_t>(BinOfRank(bs, P.re[t] - 1));
  }
  __syncthreads();
  // Tags: the end bins of every range (every bin of a small range) are gathered; the bins
  // strictly inside a large range are summed in place.  Distinct ranges never share an inside
  // bin, so the writes below never disagree.
  for (int u = 0; u < P.n_ranges; ++u) {
    const uint32_t b0 = P.rbs[u], b1 = P.rbe[u];
    const bool small = P.re[u] - P.rs[u] <= static_cast<uint32_t>(kSeqMean);
    for (uint32_t b = b0 + t; b <= b1; b += 256) tg[b] = (small || b == b0 || b == b1) ? kTagColl : static_cast<uint8_t>(u + 1);
  }
  __syncthreads();
  // Gathered bins in ascending order and their offsets (relative to the group) in the
  // candidate buffer.
  uint32_t nf = 0, nv = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    if (tg[t * kPer + k] == kTagColl) {
      ++nf;
      nv += cnt[k];
    }
  }
  s_scan[t] = nf;
  s_scan2[t] = nv;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t x = t >= o ? s_scan[t - o] : 0u;
    const uint32_t y = t >= o ? s_scan2[t - o] : 0u;
    __syncthreads();
    s_scan[t] += x;
    s_scan2[t] += y;
    __syncthreads();
  }
  {
    uint32_t fi = s_scan[t] - nf, vo = s_scan2[t] - nv;
    bool over = false;
    uint32_t* cb = cbase_all + static_cast<uint64_t>(bi) * kSelBins;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int b = t * kPer + k;
      if (tg[b] == kTagColl) {
        if (fi < static_cast<uint32_t>(kSelMaxColl)) P.coll[fi] = static_cast<uint16_t>(b);
        over = over || cnt[k] > kSelCollCap;
        cb[b] = vo;
        ++fi;
        vo += cnt[k];
      }
    }
    if (over) s_fb = 1;
  }
  __syncthreads();
  const uint32_t n_coll = s_scan[255];
  if (t == 0) {
    P.n_coll = static_cast<int32_t>(n_coll);
    if (n_coll > static_cast<uint32_t>(kSelMaxColl)) s_fb = 1;
  }
  __syncthreads();
  if (t == 0 && s_fb) {
    P.fallback = 1;
    atomicAdd(n_fallback, 1u);
  }
  // The gathered bins join the global sort lists (<= kWaveSortMax values: list 0, one wave
  // each; <= kMidMax: list 1, one workgroup each; larger: list 2, one 1024-thread workgroup
  // each), entries (group << kSelBinBits) | bin.
  __shared__ uint32_t s_lc[kSelLists], s_lb[kSelLists];
  if (t < kSelLists) s_lc[t] = 0;
  __syncthreads();
  const bool listed = !s_fb && t < P.n_coll;
  uint32_t my_list = 0, my_pos = 0, my_entry = 0;
  if (listed) {
    const int b = P.coll[t];
    my_list = H[b] > static_cast<uint32_t>(kMidMax) ? 2u : H[b] > static_cast<uint32_t>(kWaveSortMax) ? 1u : 0u;
    my_pos = atomicAdd(&s_lc[my_list], 1u);
    my_entry = (bi << kSelBinBits) | static_cast<uint32_t>(b);
  }
  __syncthreads();
  if (t < kSelLists && s_lc[t]) s_lb[t] = atomicAdd(&list_cnt[t], s_lc[t]);
  __syncthreads();
  if (listed && H[P.coll[t]] > 1) bin_lists[my_list * list_cap + s_lb[my_list] + my_pos] = my_entry;
  else if (listed) bin_lists[my_list * list_cap + s_lb[my_list] + my_pos] = 0xFFFFFFFFu;  // nothing to sort
  uint32_t* bso = bstart_all + static_cast<uint64_t>(bi) * (kSelBins + 1);
  uint8_t* tgo = tag_all + static_cast<uint64_t>(bi) * kSelBins;
  for (int b = t; b <= kSelBins; b += 256) bso[b] = bs[b];
  for (int b = t; b < kSelBins; b += 256) tgo[b] = tg[b];
  __syncthreads();
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&P);
  uint32_t* dst = reinterpret_cast<uint32_t*>(plans + bi);
  for (int w = t; w < static_cast<int>(sizeof(BigPlan) / 4); w += 256) dst[w] = src[w];
}

// Gather the values of the tagged bins into the group's candidate region (any order: the bins
// are sorted next) and sum the values inside each large range per chunk, in double-double
// (pxg_quant.h DD): the group's range sums are then exact to ~2^-100 and rounded once in
// BigSelDigest, so they do not depend on the staging order of the group's values.
// A workgroup takes cpb consecutive chunks (as BigHistKernel); splitters and tags are reloaded
// only when the group changes.  Gather slots are taken in two steps: LDS counters per gathered
// bin, then one device atomic per bin and chunk reserves the bin's range — a device atomic per
// value put its round trip in almost every 64-value round (~6% of values are gathered).
template <bool kF64>
__global__ void __launch_bounds__(256) BigCollectKernel(const BigChunk* __restrict__ chunks, const uint32_t* __restrict__ nchunks_p,
                                                        const BigPlan* __restrict__ plans, const uint64_t* __restrict__ vals, int arg_type,
                                                        const uint16_t* __restrict__ bin_in, const uint8_t* __restrict__ tag_all,
                                                        const uint32_t* __restrict__ cbase_all, uint32_t* __restrict__ cursor_all,
                                                        uint64_t* __restrict__ cand, double* __restrict__ partial, uint32_t cpb) {
  const uint32_t nchunks = *nchunks_p;
  const uint32_t c0 = blockIdx.x * cpb;
  if (c0 >= nchunks) return;
  const uint32_t c1 = min(nchunks, c0 + cpb);
  __shared__ uint8_t tg[kSelBins];
  __shared__ double acc[4][kSelMaxRanges], acc_lo[4][kSelMaxRanges];
  __shared__ uint8_t cix[kSelBins];              // gathered bin -> its index in P.coll
  __shared__ uint16_t s_coll[kSelMaxColl];
  __shared__ uint32_t lcnt[kSelMaxColl], lbase[kSelMaxColl];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  constexpr int kRounds = kMidMax / 256;
  uint32_t cur = 0xFFFFFFFFu;
  for (int k = t; k < kSelMaxColl; k += 256) lcnt[k] = 0;  // (the loop's first barrier orders it)
  // (No next-chunk prefetch here: its 32 VGPRs cost a wave per SIMD and measured no faster.)
  for (uint32_t ci = c0; ci < c1; ++ci) {
    const BigChunk c = chunks[ci];
    uint64_t raw[kRounds];
    int bins[kRounds];  // from BigHist (bin_in: the same search over the same splitters)
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int i = min(wid * (kMidMax / 4) + r * 64 + lane, static_cast<int>(c.len) - 1);
      raw[r] = vals[c.off + i];
      bins[r] = bin_in[c.off + i];
    }
    const BigPlan* P = plans + c.bidx;
    if (!P->fallback) {  // uniform
      const int n_ranges = P->n_ranges, n_coll = P->n_coll;
      __syncthreads();  // the previous chunk's acc / tg / lbase readers are done
      if (c.bidx != cur) {
        cur = c.bidx;
        const uint8_t* Tg = tag_all + static_cast<uint64_t>(cur) * kSelBins;
        for (int b = t; b < kSelBins; b += 256) tg[b] = Tg[b];
        for (int k = t; k < n_coll; k += 256) {
          const int b = P->coll[k];
          s_coll[k] = static_cast<uint16_t>(b);
          cix[b] = static_cast<uint8_t>(k);
        }
      }
      if (t < 4 * kSelMaxRanges) {
        (&acc[0][0])[t] = 0.0;
        (&acc_lo[0][0])[t] = 0.0;
      }
      __syncthreads();
      const uint32_t* cb = cbase_all + static_cast<uint64_t>(cur) * kSelBins;
      uint32_t* cc = cursor_all + static_cast<uint64_t>(cur) * kSelBins;
      uint64_t* cg = cand + c.g_off;
      uint32_t ls[kRounds];  // gathered: (index in P.coll) << 16 | slot in this chunk's run
#pragma unroll
      for (int r = 0; r < kRounds; ++r) {
        const int i = wid * (kMidMax / 4) + r * 64 + lane;
        int u = -1;
        double v = 0.0;
        ls[r] = ~0u;
        if (i < static_cast<int>(c.len)) {
          const uint64_t key = QKeyT<kF64>(raw[r]);
          const int b = bins[r];
          const uint8_t tag = tg[b];
          if (tag == kTagColl) {
            const uint32_t ix = cix[b];
            ls[r] = (ix << 16) | atomicAdd(&lcnt[ix], 1u);
          } else if (tag != 0) {
            u = tag - 1;
            v = QVal(key);
          }
        }
        unsigned long long pend = __ballot(u >= 0);
        while (pend) {
          const int uu = __builtin_amdgcn_readlane(u, __ffsll(static_cast<long long>(pend)) - 1);
          const bool mine = u == uu;
          const DD sm = WaveSumDD(DD{mine ? v : 0.0, 0.0});
          if (lane == 0) {
            const DD x = DDAdd(DD{acc[wid][uu], acc_lo[wid][uu]}, sm);
            acc[wid][uu] = x.hi;
            acc_lo[wid][uu] = x.lo;
          }
          pend &= ~__ballot(mine);
        }
      }
      __syncthreads();
      for (int k = t; k < n_coll; k += 256) {  // reserve each gathered bin's run of this chunk
        const uint32_t cnt = lcnt[k];
        if (cnt) {
          const int b = s_coll[k];
          lbase[k] = cb[b] + atomicAdd(&cc[b], cnt);
          lcnt[k] = 0;
        }
      }
      for (int u = t; u < n_ranges; u += 256) {  // per range and chunk: high word, then low word
        DD x{acc[0][u], acc_lo[0][u]};
        for (int w = 1; w < 4; ++w) x = DDAdd(x, DD{acc[w][u], acc_lo[w][u]});
        partial[(static_cast<uint64_t>(ci) * kSelMaxRanges + u) * 2] = x.hi;
        partial[(static_cast<uint64_t>(ci) * kSelMaxRanges + u) * 2 + 1] = x.lo;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRounds; ++r)
        if (ls[r] != ~0u) cg[lbase[ls[r] >> 16] + (ls[r] & 0xFFFFu)] = QKeyT<kF64>(raw[r]);
    }
  }
}

// Sort the gathered bins of the big groups, grid-stride over the lists BigPlan filled: bins
// of <= 1024 values one per wave (BigBinSortKernel), larger ones one per workgroup
// (BigBinSortLargeKernel).
__device__ __forceinline__ uint64_t* BinOfEntry(uint32_t e, const BigGroup* __restrict__ groups, const uint32_t* __restrict__ hist,
                                                 const uint32_t* __restrict__ cbase_all, uint64_t* __restrict__ cand, int* n) {
  const uint32_t bi = e >> kSelBinBits, b = e & (kSelBins - 1u);
  *n = static_cast<int>(hist[static_cast<uint64_t>(bi) * kSelBins + b]);
  return cand + groups[bi].off + cbase_all[static_cast<uint64_t>(bi) * kSelBins + b];
}
__global__ void __launch_bounds__(256) BigBinSortKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ list_cnt, const uint32_t* __restrict__ hist,
                                                        const uint32_t* __restrict__ cbase_all, uint64_t* __restrict__ cand) {
  __shared__ uint64_t keys[4][PaddedLen(kWaveSortMax)];
  const uint32_t cnt = *list_cnt;
  const int lane = threadIdx.x & 63;
  uint64_t* s = keys[threadIdx.x >> 6];
  for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < cnt; j += gridDim.x * 4) {
    const uint32_t e = list[j];
    if (e == 0xFFFFFFFFu) continue;
    int n;
    uint64_t* a = BinOfEntry(e, groups, hist, cbase_all, cand, &n);
    int Pn = kMsIpt;
    while (Pn < n) Pn <<= 1;
    for (int i = lane; i < Pn; i += 64) s[PadIdx(i)] = i < n ? a[i] : ~0ULL;
    WaveSync();
    WaveMergeSortLds(s, Pn);
    for (int i = lane; i < n; i += 64) a[i] = s[PadIdx(i)];
    WaveSync();
  }
}
__global__ void __launch_bounds__(256) BigBinSortLargeKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ list,
                                                             const uint32_t* __restrict__ list_cnt, const uint32_t* __restrict__ hist,
                                                             const uint32_t* __restrict__ cbase_all, uint64_t* __restrict__ cand) {
  __shared__ uint64_t keys[PaddedLen(kMidMax)];
  const uint32_t cnt = *list_cnt;
  for (uint32_t j = blockIdx.x; j < cnt; j += gridDim.x) {
    const uint32_t e = list[j];
    if (e == 0xFFFFFFFFu) continue;
    int n;
    uint64_t* a = BinOfEntry(e, groups, hist, cbase_all, cand, &n);
    int Pn = kMsIpt;
    while (Pn < n) Pn <<= 1;
    for (int i = threadIdx.x; i < Pn; i += blockDim.x) keys[PadIdx(i)] = i < n ? a[i] : ~0ULL;
    __syncthreads();
    BlockMergeSortLds(keys, Pn);
    for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = keys[PadIdx(i)];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kSelHugeThreads) BigBinSortHugeKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ list,
                                                                         const uint32_t* __restrict__ list_cnt, const uint32_t* __restrict__ hist,
                                                                         const uint32_t* __restrict__ cbase_all, uint64_t* __restrict__ cand) {
  __shared__ uint64_t keys[PaddedLen(static_cast<int>(kSelCollCap))];
  const uint32_t cnt = *list_cnt;
  for (uint32_t j = blockIdx.x; j < cnt; j += gridDim.x) {
    const uint32_t e = list[j];
    if (e == 0xFFFFFFFFu) continue;
    int n;
    uint64_t* a = BinOfEntry(e, groups, hist, cbase_all, cand, &n);
    int Pn = kMsIpt;
    while (Pn < n) Pn <<= 1;
    for (int i = threadIdx.x; i < Pn; i += blockDim.x) keys[PadIdx(i)] = i < n ? a[i] : ~0ULL;
    __syncthreads();
    BlockMergeSortLds(keys, Pn);
    for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = keys[PadIdx(i)];
    __syncthreads();
  }
}

// Centroid means and the seven quantiles of every big group served by the selection path.
__global__ void __launch_bounds__(256) BigSelDigestKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ nbig_p,
                                                          const BigPlan* __restrict__ plans, const uint32_t* __restrict__ chain_starts,
                                                          const uint32_t* __restrict__ bstart_all, const uint32_t* __restrict__ cbase_all,
                                                          const uint64_t* __restrict__ cand, const double* __restrict__ partial,
                                                          double* __restrict__ out) {
  if (blockIdx.x >= *nbig_p) return;
  const uint32_t bi = blockIdx.x;
  if (plans[bi].fallback) return;
  __shared__ BigPlan P;
  __shared__ double mean_u[kSelMaxRanges];
  __shared__ double red[4], red_lo[4];
  __shared__ uint32_t s_starts[kChainCap];  // the chain, staged for the quantile searches
  const int t = threadIdx.x;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(plans + bi);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&P);
    for (int w = t; w < static_cast<int>(sizeof(BigPlan) / 4); w += 256) dst[w] = src[w];
  }
  __syncthreads();
  const BigGroup G = groups[bi];
  const int64_t W = static_cast<int64_t>(G.n);
  {
    const uint32_t* gs = chain_starts + static_cast<uint64_t>(bi) * kChainCap;
    for (int j = t; j < P.nc; j += 256) s_starts[j] = gs[j];  // (ordered by the barriers below)
  }
  const uint32_t* starts = s_starts;
  const uint32_t* bs = bstart_all + static_cast<uint64_t>(bi) * (kSelBins + 1);
  const uint32_t* cb = cbase_all + static_cast<uint64_t>(bi) * kSelBins;
  const uint64_t* cg = cand + G.off;
  if (t < P.n_ranges && P.re[t] - P.rs[t] <= static_cast<uint32_t>(kSeqMean)) {
    // CentroidMean reads ranks in increasing order: one bin search, then walk the bins.
    int cur_b = -1;
    auto rank_val_seq = [&](int64_t r) -> double {
      const uint32_t rr = static_cast<uint32_t>(r);
      if (cur_b < 0) cur_b = BinOfRank(bs, rr);
      while (bs[cur_b + 1] <= rr) ++cur_b;
      return QVal(cg[cb[cur_b] + (rr - bs[cur_b])]);
    };
    mean_u[t] = CentroidMean(rank_val_seq, P.rs[t], P.re[t]);
  }
  for (int u = 0; u < P.n_ranges; ++u) {  // uniform: large ranges, block sums
    const uint32_t s = P.rs[u], e = P.re[u];
    if (e - s <= static_cast<uint32_t>(kSeqMean)) continue;
    const uint32_t b0 = P.rbs[u], b1 = P.rbe[u];
    DD acc{0.0, 0.0};  // the range's end bins (sorted candidates) and its chunks' inside sums
    const uint32_t e0 = min(e, bs[b0 + 1]);
    for (uint32_t r = s + t; r < e0; r += 256) acc = DDAddD(acc, QVal(cg[cb[b0] + (r - bs[b0])]));
    if (b1 != b0)
      for (uint32_t r = bs[b1] + t; r < e; r += 256) acc = DDAddD(acc, QVal(cg[cb[b1] + (r - bs[b1])]));
    for (uint32_t k = t; k < G.nch; k += 256) {
      const uint64_t pi = (static_cast<uint64_t>(G.c0 + k) * kSelMaxRanges + u) * 2;
      acc = DDAdd(acc, DD{partial[pi], partial[pi + 1]});
    }
    acc = WaveSumDD(acc);
    if ((t & 63) == 0) {
      red[t >> 6] = acc.hi;
      red_lo[t >> 6] = acc.lo;
    }
    __syncthreads();
    if (t == 0) {
      DD x{red[0], red_lo[0]};
      for (int w = 1; w < 4; ++w) x = DDAdd(x, DD{red[w], red_lo[w]});
      mean_u[u] = DDValue(x) / static_cast<double>(e - s);
    }
    __syncthreads();
  }
  __syncthreads();
  if (t < 7) {
    auto start = [&](int64_t j) -> int64_t { return starts[j]; };
    int k = 0;
    out[static_cast<uint64_t>(G.g) * 7 + t] = DigestQuantile(kQuantileQ[t], P.nc, W, start, [&](int64_t) -> double {
      const int32_t u = P.need_u[t * 4 + (k < 4 ? k : 3)];
      ++k;
      return mean_u[u];
    });
  }
}


// The group ids of a set's big groups whose selection plan fell back (BigPlan::fallback).
__global__ void FallbackListKernel(const BigGroup* __restrict__ groups, const uint32_t* __restrict__ count, const BigPlan* __restrict__ plans,
                                   uint32_t* __restrict__ list, uint32_t* __restrict__ n_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *count) return;
  if (plans[i].fallback) list[atomicAdd(n_out, 1u)] = groups[i].g;
}


int32_t SelEnsure(const BigSet& S, uint64_t n, DevBuf& keysA, DevBuf& sel_bin) {
  const size_t nb = S.n_big;
  PXG_RETURN_IF_ERROR(keysA.Ensure(n * 8));
  PXG_RETURN_IF_ERROR(S.spl->Ensure(nb * kSelBins * 8 + nb * kSelGuideStride * 2 + 16));
  PXG_RETURN_IF_ERROR(S.cnt->Ensure(nb * kSelBins * 8 + nb * 4 + 16));
  PXG_RETURN_IF_ERROR(S.list->Ensure(nb * kSelMaxColl * kSelLists * 4 + 16));
  PXG_RETURN_IF_ERROR(S.bstart->Ensure(nb * (kSelBins + 1) * 4 + 16));
  PXG_RETURN_IF_ERROR(S.tag->Ensure(nb * kSelBins + 16));
  PXG_RETURN_IF_ERROR(S.cbase->Ensure(nb * kSelBins * 4 + 16));
  PXG_RETURN_IF_ERROR(S.plan->Ensure(nb * sizeof(BigPlan) + 16));
  PXG_RETURN_IF_ERROR(S.partial->Ensure(static_cast<size_t>(S.n_chunks) * kSelMaxRanges * 16 + 16));  // (high, low) words
  return sel_bin.Ensure(n * 2 + 16);  // per staged value its bin (BigHist -> BigCollect; sets are disjoint)
}

int32_t SelFront(Ctx* ctx, hipStream_t st, const BigSet& S, const SelIn& in) {
  const uint64_t* vals = in.vals;
  const int at = in.arg_type;
  const uint64_t nb = S.n_big;
  PXG_HIP(hipMemsetAsync(S.cnt->p, 0, nb * kSelBins * 8 + nb * 4 + 16, st));
  uint16_t* guide = reinterpret_cast<uint16_t*>(S.spl->as<uint64_t>() + nb * kSelBins);
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_sample", BigSampleKernel<kSelSample / 2>, dim3(S.n_big), dim3(kSelSample / 2 / kMsIpt), 0,
                               static_cast<const BigGroup*>(S.big), S.d_count, vals, at, S.spl->as<uint64_t>(), guide, nullptr, nullptr));
  const uint32_t n_large = static_cast<uint32_t>(std::min<uint64_t>(S.n_big, in.n / kSelLargeN + 1));  // groups above kSelLargeN: bound
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_sample", BigSampleKernel<kSelSample>, dim3(n_large), dim3(kSelSample / kMsIpt), 0,
                               static_cast<const BigGroup*>(S.big), S.d_count, vals, at, S.spl->as<uint64_t>(), guide, S.large_list,
                               S.large_cnt));
  const uint32_t cpb = SelChunksPerBlock(S.n_chunks, ctx->num_cus, 3, kSelHistCap);
  return LaunchOn(ctx, st, "quant_sel_hist", at == PXG_FLOAT64 ? BigHistKernel<true> : BigHistKernel<false>, dim3((S.n_chunks + cpb - 1) / cpb),
                  dim3(256), 0, static_cast<const BigChunk*>(S.chunks), S.d_meta, vals, at, S.spl->as<const uint64_t>(),
                  static_cast<const uint16_t*>(guide), S.cnt->as<uint32_t>(), S.cnt->as<uint32_t>() + 2 * nb * kSelBins, cpb,
                  (*in.sel_bin).as<uint16_t>());
}

int32_t SelBack(Ctx* ctx, hipStream_t st, const BigSet& S, const SelIn& in) {
  const uint64_t* vals = in.vals;
  const int at = in.arg_type;
  const uint64_t nb = S.n_big;
  uint32_t* hist = S.cnt->as<uint32_t>();
  uint32_t* cursor = hist + nb * kSelBins;
  uint32_t* nan_cnt = hist + 2 * nb * kSelBins;
  uint32_t* list_cnt = nan_cnt + nb;
  const uint32_t list_cap = static_cast<uint32_t>(nb * kSelMaxColl);
  uint32_t* lists = S.list->as<uint32_t>();
  const BigGroup* big = S.big;
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_plan", BigPlanKernel, dim3(S.n_big), dim3(256), 0, big, S.d_count, S.chain_starts,
                               S.chain_nc, static_cast<const uint32_t*>(hist), static_cast<const uint32_t*>(nan_cnt), S.bstart->as<uint32_t>(),
                               S.tag->as<uint8_t>(), S.cbase->as<uint32_t>(), S.plan->as<BigPlan>(), in.d_fallback, lists, list_cap, list_cnt));
  const uint32_t cpb = SelChunksPerBlock(S.n_chunks, ctx->num_cus, 3, 64);  // 3 resident per CU (LDS)
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_collect", at == PXG_FLOAT64 ? BigCollectKernel<true> : BigCollectKernel<false>,
                               dim3((S.n_chunks + cpb - 1) / cpb), dim3(256), 0, static_cast<const BigChunk*>(S.chunks), S.d_meta,
                               S.plan->as<const BigPlan>(), vals, at, (*in.sel_bin).as<const uint16_t>(), S.tag->as<const uint8_t>(),
                               S.cbase->as<const uint32_t>(), cursor, (*in.keysA).as<uint64_t>(), S.partial->as<double>(), cpb));
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_bin_sort", BigBinSortKernel,
                               dim3(std::min<uint32_t>(list_cap / 4 + 1, static_cast<uint32_t>(ctx->num_cus) * 4)), dim3(256), 0, big,
                               static_cast<const uint32_t*>(lists), static_cast<const uint32_t*>(list_cnt), static_cast<const uint32_t*>(hist),
                               S.cbase->as<const uint32_t>(), (*in.keysA).as<uint64_t>()));
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_bin_sort", BigBinSortLargeKernel,
                               dim3(std::min<uint32_t>(list_cap, static_cast<uint32_t>(ctx->num_cus))), dim3(256), 0, big,
                               static_cast<const uint32_t*>(lists + list_cap), static_cast<const uint32_t*>(list_cnt + 1),
                               static_cast<const uint32_t*>(hist), S.cbase->as<const uint32_t>(), (*in.keysA).as<uint64_t>()));
  PXG_RETURN_IF_ERROR(LaunchOn(ctx, st, "quant_sel_bin_sort", BigBinSortHugeKernel,
                               dim3(std::min<uint32_t>(list_cap, static_cast<uint32_t>(ctx->num_cus))), dim3(kSelHugeThreads), 0, big,
                               static_cast<const uint32_t*>(lists + 2 * list_cap), static_cast<const uint32_t*>(list_cnt + 2),
                               static_cast<const uint32_t*>(hist), S.cbase->as<const uint32_t>(), (*in.keysA).as<uint64_t>()));
  return LaunchOn(ctx, st, "quant_sel_digest", BigSelDigestKernel, dim3(S.n_big), dim3(256), 0, big, S.d_count, S.plan->as<const BigPlan>(),
                  S.chain_starts, S.bstart->as<const uint32_t>(), S.cbase->as<const uint32_t>(), (*in.keysA).as<const uint64_t>(),
                  S.partial->as<const double>(), in.out);
}

int32_t SelFallbackList(Ctx* ctx, const BigSet& S, uint32_t* list, uint32_t* count) {
  return Launch(ctx, "quant_fallback_list", FallbackListKernel, dim3((S.n_big + 255) / 256), dim3(256), 0, static_cast<const BigGroup*>(S.big),
                S.d_count, S.plan->as<const BigPlan>(), list, count);
}

}  // namespace pxg
