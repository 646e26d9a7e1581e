// Grouping of the staging records for agg finalize (pxg_finalize.hip): the stable LSD radix
// sort by dense group id, and the fused split that designates the largest groups and gives each
// its own bucket in the sort's first pass.  (The work replaced is agg_node.cc:273-349's flush +
// per-group finalize over AggHashMap values; how records get grouped is this implementation's
// choice.)  Entry points: pxg_sort.h.
#include <algorithm>
#include <cstdlib>

#include "pxg_agg_host.h"
#include "pxg_scan.h"
#include "pxg_sort.h"

namespace pxg {

constexpr int kRadixBlock = 256;
constexpr int kRadixItems = 12;
constexpr int kRadixTile = kRadixBlock * kRadixItems;
constexpr int kRadixBuckets = 1 << kRadixBits;
constexpr int kRsScanBlock = 256;


// Sort key of a staged record.  Pass 0 reads table slots and maps them through `rank` (slot ->
// dense group id; kDeferredSlot / empty -> G, which sorts last); later passes read dense ids.
__device__ __forceinline__ uint32_t DenseKey(uint32_t k, const uint32_t* __restrict__ rank, uint32_t cap, uint32_t G) {
  if (!rank) return k;
  return k < cap ? rank[k] : G;
}


// ---------------------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits, four kernels per pass: tile digit counts (RsHist),
// digit totals (RsTotal), tile offsets (RsScan: one workgroup per digit scans that digit's
// tile counts and adds the digit's base), and the scatter (RsScatter).  No tile ever waits on another: a decoupled look-back (one-sweep) was
// measured slower here, its inclusive prefixes advancing only a few tiles per device-scope
// round trip while ~1000 tiles start at once.
// ---------------------------------------------------------------------------------------

// Tile digit counts of one pass -> hist[tile * kRadixBuckets + d] (tile-major: one contiguous
// 1 KB row per workgroup; the digit-major layout cost one partial-line write per digit and
// tile, ~10M scattered writes per pass at 1B rows).  With a rank map (first pass) the dense keys are also written out, so the first scatter reads
// them instead of gathering again.
// A workgroup counts kHistTiles consecutive tiles: all their keys (and, in the first pass, their
// rank gathers) are in flight at once, then each tile's counts are taken in turn.  (Until round 6
// the gathers were guarded and compiled to one wait each; unconditional: 1B rows' fused-split
// histogram 0.45-0.47 -> 0.41-0.42 ms, C2's first histogram 0.057-0.063 -> 0.046-0.048 ms,
// profiles/r06_ab_rank_gathers.log.)  Four tiles
// per workgroup at >= 16K tiles (1B rows: the rank-gathering pass 0.59 -> 0.51 ms); one below,
// where four would leave too few workgroups (C2: 0.057 -> 0.085 ms).
template <int kHistTiles>
__global__ void __launch_bounds__(kRadixBlock) RsHistKernel(const uint32_t* __restrict__ keys, uint64_t n,
                                                            const uint32_t* __restrict__ rank, uint32_t cap, uint32_t G, int shift,
                                                            uint32_t* __restrict__ hist, uint32_t ntiles, uint32_t* __restrict__ dense_out) {
  // One LDS histogram per wave, plain LDS atomics (a hot digit serialises only within its wave;
  // the 8-ballot match of WaveHistAdd cost more ALU than the conflicts it saved here).
  constexpr int kWaves = kRadixBlock / 64;
  __shared__ uint32_t h[kWaves][kRadixBuckets];
  const int wid = threadIdx.x >> 6;
  const uint32_t tile0 = XcdRemap(blockIdx.x, gridDim.x) * kHistTiles;
  // 32-bit positions relative to the workgroup's first record (n < 2^32).
  const uint64_t base = static_cast<uint64_t>(tile0) * kRadixTile;
  const uint32_t rem = static_cast<uint32_t>(min(n - min(n, base), static_cast<uint64_t>(kHistTiles) * kRadixTile));
  const uint32_t* kp = keys + base;
  uint32_t kk[kHistTiles][kRadixItems];
#pragma unroll
  for (int j = 0; j < kHistTiles; ++j)
#pragma unroll
    for (int k = 0; k < kRadixItems; ++k) {
      const uint32_t i = j * kRadixTile + k * kRadixBlock + threadIdx.x;
      kk[j][k] = i < rem ? kp[i] : 0u;
    }
  if (rank) {
    // The rank gathers unconditional (clamped slot), so all of them are in flight together: a
    // guarded gather compiled to a branch and a wait per item.
#pragma unroll
    for (int j = 0; j < kHistTiles; ++j)
#pragma unroll
      for (int k = 0; k < kRadixItems; ++k) {
        const bool ok = kk[j][k] < cap;
        const uint32_t g = rank[ok ? kk[j][k] : 0u];
        kk[j][k] = ok ? g : G;
      }
    uint32_t* dp = dense_out + base;
#pragma unroll
    for (int j = 0; j < kHistTiles; ++j)
#pragma unroll
      for (int k = 0; k < kRadixItems; ++k) {
        const uint32_t i = j * kRadixTile + k * kRadixBlock + threadIdx.x;
        if (i < rem) dp[i] = kk[j][k];
      }
  }
#pragma unroll
  for (int j = 0; j < kHistTiles; ++j) {
    if (tile0 + j >= ntiles) break;  // uniform
#pragma unroll
    for (int w = 0; w < kWaves; ++w) h[w][threadIdx.x] = 0;  // kRadixBlock == kRadixBuckets
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRadixItems; ++k) {
      const uint32_t i = j * kRadixTile + k * kRadixBlock + threadIdx.x;
      if (i < rem) atomicAdd(&h[wid][(kk[j][k] >> shift) & (kRadixBuckets - 1)], 1u);
    }
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += h[w][threadIdx.x];
    hist[static_cast<uint64_t>(tile0 + j) * kRadixBuckets + threadIdx.x] = t;
    __syncthreads();
  }
}

// The tile offsets from the tile-major counts, in three coalesced kernels: per range of
// kRsTilesPerPart tiles the digit sums (RsPart), per digit the exclusive scan of those sums and
// the digit total (RsPartScan), per range the running offsets tile by tile plus the digit
// base (RsDown, in place: hist[tile][d] becomes the output position of the tile's first d).
constexpr uint32_t kRsTilesPerPart = 16;
__global__ void __launch_bounds__(kRadixBuckets) RsPartKernel(const uint32_t* __restrict__ hist, uint32_t ntiles,
                                                              uint32_t* __restrict__ part) {
  const uint32_t w = blockIdx.x, d = threadIdx.x;
  const uint32_t t0 = w * kRsTilesPerPart, t1 = min(ntiles, t0 + kRsTilesPerPart);
  uint32_t s = 0;
  for (uint32_t t = t0; t < t1; ++t) s += hist[static_cast<uint64_t>(t) * kRadixBuckets + d];
  part[static_cast<uint64_t>(w) * kRadixBuckets + d] = s;
}
__global__ void __launch_bounds__(kRsScanBlock) RsPartScanKernel(uint32_t* __restrict__ part, uint32_t nparts,
                                                                 uint32_t* __restrict__ ghist) {
  constexpr int kWaves = kRsScanBlock / 64;
  __shared__ uint32_t s_w[kWaves];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const uint32_t d = blockIdx.x;
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < nparts; i0 += kRsScanBlock) {
    const uint32_t i = i0 + t;
    const uint32_t c = i < nparts ? part[static_cast<uint64_t>(i) * kRadixBuckets + d] : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t before = carry;
    for (int w = 0; w < wid; ++w) before += s_w[w];
    uint32_t round = 0;
    for (int w = 0; w < kWaves; ++w) round += s_w[w];
    if (i < nparts) part[static_cast<uint64_t>(i) * kRadixBuckets + d] = before + incl - c;
    carry += round;
    __syncthreads();
  }
  if (t == 0) ghist[d] = carry;
}
__global__ void __launch_bounds__(kRadixBuckets) RsDownKernel(uint32_t* __restrict__ hist, uint32_t ntiles,
                                                              const uint32_t* __restrict__ part, const uint32_t* __restrict__ ghist) {
  __shared__ uint32_t s[kRadixBuckets];
  const uint32_t w = blockIdx.x, d = threadIdx.x;
  // digit base: exclusive scan of the digit totals (Hillis-Steele over 256 values)
  const uint32_t tot = ghist[d];
  s[d] = tot;
  __syncthreads();
  for (int o = 1; o < kRadixBuckets; o <<= 1) {
    const uint32_t x = d >= static_cast<uint32_t>(o) ? s[d - o] : 0u;
    __syncthreads();
    s[d] += x;
    __syncthreads();
  }
  uint32_t run = s[d] - tot + part[static_cast<uint64_t>(w) * kRadixBuckets + d];
  const uint32_t t0 = w * kRsTilesPerPart, t1 = min(ntiles, t0 + kRsTilesPerPart);
  for (uint32_t t = t0; t < t1; ++t) {
    uint32_t* h = hist + static_cast<uint64_t>(t) * kRadixBuckets + d;
    const uint32_t c = *h;
    *h = run;
    run += c;
  }
}

// Block d: digit d's total over all tiles (the digit bases come from these; per-tile atomics
// into 256 global totals were a contention point).
__global__ void __launch_bounds__(kRsScanBlock) RsTotalKernel(const uint32_t* __restrict__ hist, uint32_t ntiles,
                                                              uint32_t* __restrict__ ghist) {
  __shared__ uint32_t s[kRsScanBlock];
  const uint32_t* row = hist + static_cast<uint64_t>(blockIdx.x) * ntiles;
  uint32_t tot = 0;
  for (uint32_t i = threadIdx.x; i < ntiles; i += kRsScanBlock) tot += row[i];
  s[threadIdx.x] = tot;
  __syncthreads();
  for (int o = kRsScanBlock / 2; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) ghist[blockIdx.x] = s[0];
}

// Block d: exclusive scan of digit d's tile counts, plus the digit's global base.  Each wave
// scans a contiguous quarter of the row with coalesced loads (4 x 64 counts per step, a wave
// prefix by shuffles); the quarters' totals are combined through LDS first.
__global__ void __launch_bounds__(kRsScanBlock) RsScanKernel(uint32_t* __restrict__ hist, uint32_t ntiles,
                                                             const uint32_t* __restrict__ ghist) {
  constexpr int kWaves = kRsScanBlock / 64;
  constexpr int kU = 4;
  __shared__ uint32_t s[kRsScanBlock];
  __shared__ uint32_t s_w[kWaves];
  const int t = threadIdx.x, d = blockIdx.x;
  const int lane = t & 63, wid = t >> 6;
  // the digit base: sum of the totals of digits < d
  s[t] = t < d ? ghist[t] : 0u;
  __syncthreads();
  for (int o = kRsScanBlock / 2; o > 0; o >>= 1) {
    if (t < o) s[t] += s[t + o];
    __syncthreads();
  }
  const uint32_t carry = s[0];
  uint32_t* row = hist + static_cast<uint64_t>(d) * ntiles;
  const uint32_t per = (ntiles + kWaves - 1) / kWaves;
  const uint32_t q0 = min(ntiles, per * wid), q1 = min(ntiles, q0 + per);
  uint32_t tot = 0;
  for (uint32_t i = q0 + lane; i < q1; i += 64) tot += row[i];
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  if (lane == 0) s_w[wid] = tot;
  __syncthreads();
  uint32_t run = carry;
  for (int w = 0; w < wid; ++w) run += s_w[w];
  for (uint32_t i0 = q0; i0 < q1; i0 += 64 * kU) {
    uint32_t c[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t i = i0 + u * 64 + lane;
      c[u] = i < q1 ? row[i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      uint32_t incl = c[u];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      const uint32_t i = i0 + u * 64 + lane;
      if (i < q1) row[i] = run + incl - c[u];
      run += __shfl(incl, 63, 64);
    }
  }
}

// One pass.  Wave w of a block owns the contiguous quarter [w * kPerWave, (w + 1) * kPerWave)
// of the tile, in (k, lane) order, so a wave's running per-digit counts live in its own LDS
// slice and need no block barrier inside the item loop: ranks within a wave come from an
// 8-ballot match of the digit bits.  The tile is then reordered by digit in LDS and written
// out in digit runs (consecutive threads -> consecutive addresses) instead of one scattered
// store per item.  The first value stream is loaded up front so its latency overlaps the
// ranking.  (Round 6: loading stream v + 1 into the same registers right after stream v went to
// LDS, ahead of stream v's run writes, made the 9-stream partition sort slower: C3 without the
// filter, radix_scatter 7.0 -> 8.1 ms.  The guarded per-item loads of streams 1.. compile to one
// load and one wait per item; issuing a stream's 12 loads together (clamped rows) was slower
// too: C3 without the filter 7.14 -> 8.58 ms, 1B rows' fused split 1.07 -> 1.16 ms,
// profiles/r06_ab_loads.log.)
__global__ void __launch_bounds__(kRadixBlock) RsScatterKernel(const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout,
                                                               ConstValPtrs vin, ValPtrs vout, int nvals, uint64_t n, int shift,
                                                               const uint32_t* __restrict__ offs, uint32_t ntiles) {
  constexpr int kWaves = kRadixBlock / 64;
  constexpr int kPerWave = kRadixTile / kWaves;
  __shared__ uint32_t whist[kWaves][kRadixBuckets];
  __shared__ uint32_t dstart[kRadixBuckets];
  __shared__ uint32_t gofs[kRadixBuckets];
  __shared__ uint64_t s_buf[kRadixTile];
  __shared__ uint8_t s_dig[kRadixTile];
  uint32_t* s_key = reinterpret_cast<uint32_t*>(s_buf);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  const uint32_t tile = XcdRemap(blockIdx.x, gridDim.x);  // as in RsHistKernel
  for (int d = lane; d < kRadixBuckets; d += 64) whist[wid][d] = 0;
  gofs[threadIdx.x] = offs[static_cast<uint64_t>(tile) * kRadixBuckets + threadIdx.x];
  (void)ntiles;
  WaveSync();
  const uint64_t tile0 = static_cast<uint64_t>(tile) * kRadixTile;
  const uint64_t wbase = tile0 + static_cast<uint64_t>(wid) * kPerWave;
  const int tn = static_cast<int>(min(static_cast<uint64_t>(kRadixTile), n - tile0));
  uint32_t part[kRadixItems], keys[kRadixItems], dig[kRadixItems];
  uint64_t v0[kRadixItems];
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
    keys[k] = i < n ? kin[i] : 0u;
    v0[k] = (nvals > 0 && i < n) ? vin.p[0][i] : 0ULL;
  }
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
    const bool valid = i < n;
    const uint32_t d = (keys[k] >> shift) & (kRadixBuckets - 1);
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
    dig[k] = d;
  }
  __syncthreads();
  {
    const int d = threadIdx.x;  // kRadixBlock == kRadixBuckets
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += whist[w][d];
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
  for (int j = threadIdx.x; j < tn; j += kRadixBlock) {
    const uint32_t d = s_dig[j];
    kout[gofs[d] + (j - dstart[d])] = s_key[j];
  }
  for (int v = 0; v < nvals; ++v) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRadixItems; ++k) {
      const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
      if (i < n) s_buf[lpos[k]] = v == 0 ? v0[k] : vin.p[v][i];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < tn; j += kRadixBlock) {
      const uint32_t d = s_dig[j];
      vout.p[v][gofs[d] + (j - dstart[d])] = s_buf[j];
    }
  }
}

// Sorts n records (dense key = DenseKey(keys[i]), values vin[0..nvals)) stably by dense key
// into kbuf[0/1] / vbuf[0/1] (ping-pong); *skeys / *svals name the sorted streams.
constexpr int kRsMaxPasses = 4;
// shift0 / fixed_bits (partition sorts, pxg_hc.hip): sort by bits [shift0, shift0 + fixed_bits)
// of the raw keys instead (no rank map).
int32_t RadixSortStreams(Ctx* ctx, const uint32_t* keys, const uint32_t* rank, uint32_t cap, uint32_t G, ConstValPtrs vin,
                                int nvals, uint64_t n, uint32_t* kbuf[2], ValPtrs vbuf[2], RadixPassWs& ws, const uint32_t** skeys,
                                ConstValPtrs* svals, int shift0, int fixed_bits) {
  if (n == 0 || n >= (uint64_t(1) << 32)) return SetError(PXG_INVALID_ARGUMENT, "radix sort of %llu records", static_cast<unsigned long long>(n));
  int nbits = 1;
  while ((uint64_t(1) << nbits) < static_cast<uint64_t>(G) + 1) ++nbits;
  if (fixed_bits > 0) nbits = fixed_bits;
  const int passes = (nbits + kRadixBits - 1) / kRadixBits;
  if (passes > kRsMaxPasses) return SetError(PXG_INVALID_ARGUMENT, "radix sort of %u keys", G);
  const uint32_t ntiles = static_cast<uint32_t>((n + kRadixTile - 1) / kRadixTile);
  PXG_RETURN_IF_ERROR(ws.hist.Ensure(static_cast<size_t>(ntiles) * kRadixBuckets * 4));
  PXG_RETURN_IF_ERROR(ws.ghist.Ensure(static_cast<size_t>(kRsMaxPasses) * kRadixBuckets * 4));
  const uint32_t nparts = (ntiles + kRsTilesPerPart - 1) / kRsTilesPerPart;
  PXG_RETURN_IF_ERROR(ws.part.Ensure(static_cast<size_t>(nparts) * kRadixBuckets * 4));
  uint32_t* ghist = ws.ghist.as<uint32_t>();
  // With a rank map, the first histogram pass writes the dense keys into kbuf[1] (which the
  // first scatter does not write) and the scatters read those.
  const uint32_t* kin = keys;
  for (int p = 0; p < passes; ++p) {
    const int cur = p & 1;
    const bool gather = p == 0 && rank != nullptr;
    uint32_t* gh = ghist + p * kRadixBuckets;
    const int ht = ntiles >= 16384 ? 4 : 1;
    PXG_RETURN_IF_ERROR(Launch(ctx, gather ? "radix_hist_rank" : "radix_hist", ht == 4 ? RsHistKernel<4> : RsHistKernel<1>,
                               dim3((ntiles + ht - 1) / ht), dim3(kRadixBlock), 0, kin, n, gather ? rank : nullptr, cap,
                               G, shift0 + p * kRadixBits, ws.hist.as<uint32_t>(), ntiles, gather ? kbuf[1] : nullptr));
    if (gather) kin = kbuf[1];
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", RsPartKernel, dim3(nparts), dim3(kRadixBuckets), 0,
                               static_cast<const uint32_t*>(ws.hist.as<uint32_t>()), ntiles, ws.part.as<uint32_t>()));
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", RsPartScanKernel, dim3(kRadixBuckets), dim3(kRsScanBlock), 0, ws.part.as<uint32_t>(),
                               nparts, gh));
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", RsDownKernel, dim3(nparts), dim3(kRadixBuckets), 0, ws.hist.as<uint32_t>(), ntiles,
                               static_cast<const uint32_t*>(ws.part.as<uint32_t>()), static_cast<const uint32_t*>(gh)));
    PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scatter", RsScatterKernel, dim3(ntiles), dim3(kRadixBlock), 0, kin, kbuf[cur], vin, vbuf[cur],
                               nvals, n, shift0 + p * kRadixBits, ws.hist.as<const uint32_t>(), ntiles));
    kin = kbuf[cur];
    for (int v = 0; v < kMaxVals; ++v) vin.p[v] = vbuf[cur].p[v];
  }
  *skeys = kin;
  *svals = vin;
  return PXG_OK;
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
// A wave takes 256 consecutive keys per step (one 16-byte load per lane, the previous lane's last
// key by a shuffle), grid-stride over a resident grid: one thread per key meant 200K workgroups
// for the rest records at 1B rows, and with the early big set's kernels beside it the pass took
// 0.22 ms for 212 MB.
__device__ __forceinline__ void GroupHead(uint64_t i, uint64_t n, uint32_t k, uint32_t prev, uint32_t G, uint32_t* __restrict__ gstart) {
  if (i < n && k != prev) gstart[k < G ? k : G] = static_cast<uint32_t>(i);
}
__global__ void __launch_bounds__(256) GroupHeadsKernel(const uint32_t* __restrict__ keys, uint64_t n, uint32_t G, uint32_t* __restrict__ gstart) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 6;
  const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
  for (uint64_t w0 = ((static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6) * 256; w0 < n; w0 += nwaves * 256) {
    const uint64_t b = w0 + 4 * static_cast<uint64_t>(lane);
    uint32_t k0, k1, k2, k3;
    if (vec && b + 4 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(keys + b);
      k0 = v.x;
      k1 = v.y;
      k2 = v.z;
      k3 = v.w;
    } else {
      k0 = b < n ? keys[b] : ~0u;
      k1 = b + 1 < n ? keys[b + 1] : ~0u;
      k2 = b + 2 < n ? keys[b + 2] : ~0u;
      k3 = b + 3 < n ? keys[b + 3] : ~0u;
    }
    uint32_t prev = __shfl_up(k3, 1, 64);
    if (lane == 0) prev = w0 == 0 ? ~k0 : keys[w0 - 1];  // the first key always heads its group
    GroupHead(b, n, k0, prev, G, gstart);
    GroupHead(b + 1, n, k1, k0, G, gstart);
    GroupHead(b + 2, n, k2, k1, G, gstart);
    GroupHead(b + 3, n, k3, k2, G, gstart);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && n > 0 && keys[n - 1] < G) gstart[G] = static_cast<uint32_t>(n);
}

// ---------------------------------------------------------------------------------------
// Designation of the large groups for the fused split below.  Finalize only needs each group's
// records contiguous (every reduction and digest below works on a group's range; the quantile
// kernels sort the values they read).  A strided sample of the staging counts records per slot;
// the groups it says are large ("designated", at most max_big of them, the largest first) get
// the last group ids.  Group ids: the rest groups take [0, Gr) and the designated ones [Gr, G),
// both in slot order.  A group the sample misses goes through the rest sort; one it
// over-estimates is classified by its true count: the sample decides the cost, never the result.
// (Round 4's separate split pass over the staging, before the radix sort, is gone: the fused
// split does the same work inside the sort's first pass.)
// ---------------------------------------------------------------------------------------
constexpr uint32_t kSplitStride = 128;    // every 128th staged record is sampled
constexpr int kSampleTable = 4096;
constexpr int kSamplePerThread = 16;

// Sampled per-slot counts: each block aggregates 4096 samples in an LDS table, then adds its
// distinct slots' counts to scnt (one global atomic per distinct slot per block, so a hot
// group sees one per block, not one per sample).  A slot that finds no LDS entry within 32
// probes is dropped: such a block met thousands of distinct cold slots, none of them large.
__global__ void __launch_bounds__(256) SplitSampleKernel(const uint32_t* __restrict__ slot, uint64_t n, uint32_t cap,
                                                         uint32_t* __restrict__ scnt) {
  __shared__ uint32_t s_key[kSampleTable];
  __shared__ uint32_t s_cnt[kSampleTable];
  for (int i = threadIdx.x; i < kSampleTable; i += 256) {
    s_key[i] = 0xFFFFFFFFu;
    s_cnt[i] = 0;
  }
  __syncthreads();
  const uint64_t j0 = static_cast<uint64_t>(blockIdx.x) * 256 * kSamplePerThread;
  uint32_t sv[kSamplePerThread];
#pragma unroll
  for (int k = 0; k < kSamplePerThread; ++k) {
    const uint64_t r = (j0 + static_cast<uint64_t>(k) * 256 + threadIdx.x) * kSplitStride;
    sv[k] = r < n ? slot[r] : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int k = 0; k < kSamplePerThread; ++k) {
    const uint32_t x = sv[k];
    if (x >= cap) continue;
    uint32_t h = (x * 0x9E3779B1u) >> 20;
    for (int p = 0; p < 32; ++p) {
      uint32_t cur = __hip_atomic_load(&s_key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (cur == 0xFFFFFFFFu) {
        cur = atomicCAS(&s_key[h], 0xFFFFFFFFu, x);
        if (cur == 0xFFFFFFFFu) cur = x;
      }
      if (cur == x) {
        atomicAdd(&s_cnt[h], 1u);
        break;
      }
      h = (h + 1) & (kSampleTable - 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kSampleTable; i += 256)
    if (s_cnt[i]) atomicAdd(&scnt[s_key[i]], s_cnt[i]);
}

// lvl[l] = occupied slots whose sample count has floor(log2) == l: the designation threshold
// is raised by powers of two until at most max_big slots reach it, so the cap keeps the
// largest groups rather than the first ones in slot order.
__global__ void SplitLevelsKernel(const uint32_t* __restrict__ scnt, uint32_t cap, uint32_t* __restrict__ lvl) {
  __shared__ uint32_t s_l[32];
  if (threadIdx.x < 32) s_l[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = i < cap ? scnt[i] : 0u;
  if (c) atomicAdd(&s_l[31 - __clz(c)], 1u);
  __syncthreads();
  if (threadIdx.x < 32 && s_l[threadIdx.x]) atomicAdd(&lvl[threadIdx.x], s_l[threadIdx.x]);
}

__device__ __forceinline__ uint32_t SplitThreshold(const uint32_t* __restrict__ lvl, uint32_t min_samples, uint32_t max_big) {
  uint32_t above = 0;  // slots with a count >= 2^(l + 1)
  int L = 32;
  for (int l = 31; l >= 0; --l) {
    above += lvl[l];
    if (above > max_big) break;
    L = l;
  }
  const uint32_t p = L >= 32 ? 0xFFFFFFFFu : (1u << L);
  return max(min_samples, p);
}

// flags[slot] = designated << 32 | occupied (one u64 scan gives both ranks).
__global__ void SplitFlagsKernel(const unsigned long long* __restrict__ slots, uint32_t cap, const uint32_t* __restrict__ scnt,
                                 const uint32_t* __restrict__ lvl, uint32_t min_samples, uint32_t max_big, uint64_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const uint32_t t = SplitThreshold(lvl, min_samples, max_big);
  const bool occ = slots[i] != 0;
  const bool des = occ && scnt[i] >= t;
  flags[i] = (static_cast<uint64_t>(des) << 32) | static_cast<uint64_t>(occ);
}

__device__ __forceinline__ uint32_t SplitNd(const uint64_t* __restrict__ ftotal, uint32_t max_big) {
  return min(static_cast<uint32_t>(*ftotal >> 32), max_big);
}

// Group ids from the scanned flags: designated slots -> Gr + their rank, the rest -> their rank
// among the rest; gslot[id] = slot (so gslot[Gr + j] lists the designated slots by bucket).
__global__ void SplitIdsKernel(const unsigned long long* __restrict__ slots, uint32_t cap, const uint32_t* __restrict__ scnt,
                               const uint32_t* __restrict__ lvl, uint32_t min_samples, uint32_t max_big, const uint64_t* __restrict__ fscan,
                               const uint64_t* __restrict__ ftotal, uint32_t G, uint32_t* __restrict__ newid, uint32_t* __restrict__ gslot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap || slots[i] == 0) return;
  const uint32_t t = SplitThreshold(lvl, min_samples, max_big);
  const uint32_t nd = SplitNd(ftotal, max_big), Gr = G - nd;
  const uint64_t f = fscan[i];
  const uint32_t d_rank = static_cast<uint32_t>(f >> 32), o_rank = static_cast<uint32_t>(f);
  const bool des = scnt[i] >= t && d_rank < max_big;
  const uint32_t id = des ? Gr + d_rank : o_rank - min(d_rank, max_big);
  newid[i] = id;
  gslot[id] = i;
}

// ---------------------------------------------------------------------------------------
// Fused split (large aggregations): the staging split folded into the radix sort's first pass.
// The largest groups by a sample (at most kFsMaxU, "designated" as in the split above) get one
// bucket each in a 9-bit first pass whose other 256 buckets are the low digit of the remaining
// ("rest") groups' ids: one stable pass leaves every designated group contiguous and final, and
// the rest records sorted by their low digit, so only the rest records (~30 % at the north_star
// size) go through the remaining pass(es).  Final layout [rest by id | designated by id | no
// group], the same as the split's.  A 10-bit pass (767 designated groups, 73 % of the records at
// 1B rows) measured slower: ~1000 partial-line runs per 3072-record tile outran the L2's write
// combining (scatter 1.11 ms vs 0.83 ms with 512 buckets).
// ---------------------------------------------------------------------------------------
constexpr int kFsBits = 9;
constexpr int kFsBuckets = 1 << kFsBits;          // 512
constexpr int kFsRest = kRadixBuckets;            // buckets [0, 256): the rest's low digit
static_assert(kFsMaxU == kFsBuckets - kFsRest - 1, "designated buckets; the last one: no group");
constexpr int kFsBlock = 256;
constexpr int kFsItems = 12;
constexpr int kFsTile = kFsBlock * kFsItems;      // 3072 records (6144 with 512-thread workgroups: scatter 0.81 -> 1.11 ms at 1B rows)
static_assert(kFsBuckets % kFsBlock == 0, "buckets per thread");

__device__ __forceinline__ uint32_t FsBucket(uint32_t id, uint32_t Gr, uint32_t G, uint32_t nd) {
  return id < Gr ? (id & (kFsRest - 1)) : (id < G ? kFsRest + (id - Gr) : kFsRest + nd);
}

// Tile bucket counts -> hist[tile * kFsBuckets + b] (tile-major); the dense ids (newid[slot], G
// for a record without a group) to dense_out for the scatter.  (Gathering the ids again in the
// scatter instead of this round trip measured slower at 1B rows: hist 0.45 -> 0.41 ms, scatter
// 0.81 -> 1.04 ms.  Nontemporal stores: hist 0.456 -> 0.446 ms, the scatter's run writes
// 0.80 -> 1.60 ms.  Round 6: lanes of one bucket matched by 9 ballots, one LDS add per distinct
// bucket instead of an atomic per lane: N1 step 14.51 -> 14.70 ms, so the atomics stay.)
template <int kHistTiles>
__global__ void __launch_bounds__(kFsBlock) FsHistKernel(const uint32_t* __restrict__ slot, uint64_t n, const uint32_t* __restrict__ newid,
                                                         uint32_t cap, uint32_t G, const uint64_t* __restrict__ ftotal,
                                                         uint32_t* __restrict__ hist, uint32_t ntiles, uint32_t* __restrict__ dense_out) {
  constexpr int kWaves = kFsBlock / 64;
  __shared__ uint32_t h[kWaves][kFsBuckets];
  const int wid = threadIdx.x >> 6;
  const uint32_t nd = SplitNd(ftotal, kFsMaxU), Gr = G - nd;
  const uint32_t tile0 = XcdRemap(blockIdx.x, gridDim.x) * kHistTiles;
  const uint64_t base = static_cast<uint64_t>(tile0) * kFsTile;
  const uint32_t rem = static_cast<uint32_t>(min(n - min(n, base), static_cast<uint64_t>(kHistTiles) * kFsTile));
  const uint32_t* kp = slot + base;
  uint32_t kk[kHistTiles][kFsItems];
#pragma unroll
  for (int j = 0; j < kHistTiles; ++j)
#pragma unroll
    for (int k = 0; k < kFsItems; ++k) {
      const uint32_t i = j * kFsTile + k * kFsBlock + threadIdx.x;
      kk[j][k] = i < rem ? kp[i] : 0u;
    }
  // Every id gather issued before the first store (clamped slot, as in RsHistKernel): a guarded
  // gather followed by its store compiled to a wait per item.
#pragma unroll
  for (int j = 0; j < kHistTiles; ++j)
#pragma unroll
    for (int k = 0; k < kFsItems; ++k) {
      const bool ok = kk[j][k] < cap;
      const uint32_t g = newid[ok ? kk[j][k] : 0u];
      kk[j][k] = ok ? g : G;
    }
#pragma unroll
  for (int j = 0; j < kHistTiles; ++j)
#pragma unroll
    for (int k = 0; k < kFsItems; ++k) {
      const uint32_t i = j * kFsTile + k * kFsBlock + threadIdx.x;
      if (i < rem) dense_out[base + i] = kk[j][k];
    }
#pragma unroll
  for (int j = 0; j < kHistTiles; ++j) {
    if (tile0 + j >= ntiles) break;  // uniform
    for (int w = 0; w < kWaves; ++w)
      for (int d = threadIdx.x; d < kFsBuckets; d += kFsBlock) h[w][d] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kFsItems; ++k) {
      const uint32_t i = j * kFsTile + k * kFsBlock + threadIdx.x;
      if (i < rem) atomicAdd(&h[wid][FsBucket(kk[j][k], Gr, G, nd)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < kFsBuckets; d += kFsBlock) {
      uint32_t t = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) t += h[w][d];
      hist[static_cast<uint64_t>(tile0 + j) * kFsBuckets + d] = t;
    }
    __syncthreads();
  }
}

// Tile offsets of NB-bucket tile-major counts (the RsPart / RsPartScan / RsDown scheme for any
// bucket count): per 16-tile range the bucket sums; per bucket the scan of the range sums and
// the bucket total; the bucket bases (exclusive scan of the totals, base[NB] = the total); per
// range the running offsets, in place.
template <int NB>
__global__ void __launch_bounds__(256) XPartKernel(const uint32_t* __restrict__ hist, uint32_t ntiles, uint32_t* __restrict__ part) {
  const uint32_t w = blockIdx.x;
  const uint32_t t0 = w * kRsTilesPerPart, t1 = min(ntiles, t0 + kRsTilesPerPart);
  for (int d = threadIdx.x; d < NB; d += 256) {
    uint32_t s = 0;
    for (uint32_t t = t0; t < t1; ++t) s += hist[static_cast<uint64_t>(t) * NB + d];
    part[static_cast<uint64_t>(w) * NB + d] = s;
  }
}
template <int NB>
__global__ void __launch_bounds__(kRsScanBlock) XPartScanKernel(uint32_t* __restrict__ part, uint32_t nparts, uint32_t* __restrict__ tot) {
  constexpr int kWaves = kRsScanBlock / 64;
  __shared__ uint32_t s_w[kWaves];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const uint32_t d = blockIdx.x;
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < nparts; i0 += kRsScanBlock) {
    const uint32_t i = i0 + t;
    const uint32_t c = i < nparts ? part[static_cast<uint64_t>(i) * NB + d] : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t before = carry;
    for (int w = 0; w < wid; ++w) before += s_w[w];
    uint32_t round = 0;
    for (int w = 0; w < kWaves; ++w) round += s_w[w];
    if (i < nparts) part[static_cast<uint64_t>(i) * NB + d] = before + incl - c;
    carry += round;
    __syncthreads();
  }
  if (t == 0) tot[d] = carry;
}
template <int NB>
__global__ void __launch_bounds__(256) XBaseKernel(const uint32_t* __restrict__ tot, uint32_t* __restrict__ base) {
  constexpr int kPer = NB / 256;
  __shared__ uint32_t s_w[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    v[k] = tot[threadIdx.x * kPer + k];
    sum += v[k];
  }
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
  for (int w = 0; w < wid; ++w) run += s_w[w];
  if (threadIdx.x == 255) base[NB] = run + sum;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    base[threadIdx.x * kPer + k] = run;
    run += v[k];
  }
}
template <int NB>
__global__ void __launch_bounds__(256) XDownKernel(uint32_t* __restrict__ hist, uint32_t ntiles, const uint32_t* __restrict__ part,
                                                   const uint32_t* __restrict__ base) {
  const uint32_t w = blockIdx.x;
  const uint32_t t0 = w * kRsTilesPerPart, t1 = min(ntiles, t0 + kRsTilesPerPart);
  for (int d = threadIdx.x; d < NB; d += 256) {
    uint32_t run = base[d] + part[static_cast<uint64_t>(w) * NB + d];
    for (uint32_t t = t0; t < t1; ++t) {
      uint32_t* h = hist + static_cast<uint64_t>(t) * NB + d;
      const uint32_t c = *h;
      *h = run;
      run += c;
    }
  }
}

// The fused first pass (RsScatterKernel's scheme with 1024 buckets: 10-ballot wave ranks, the
// tile reordered by bucket in LDS, bucket runs written out).  Rest records (key and values) go to
// the rest sort's input [0, n_rest); designated records' values straight to their final position
// in vfin; records without a group are not written (nothing reads past gstart[G]).
__global__ void __launch_bounds__(kFsBlock) FsScatterKernel(const uint32_t* __restrict__ kin, uint64_t n, uint32_t G,
                                                            const uint64_t* __restrict__ ftotal, ConstValPtrs vin, int nvals,
                                                            const uint32_t* __restrict__ offs, uint32_t* __restrict__ kout, ValPtrs vrest,
                                                            ValPtrs vfin) {
  constexpr int kWaves = kFsBlock / 64;
  constexpr int kPerWave = kFsTile / kWaves;
  constexpr int kPerThr = kFsBuckets / kFsBlock;
  __shared__ uint32_t whist[kWaves][kFsBuckets];
  __shared__ uint32_t dstart[kFsBuckets];
  __shared__ uint32_t gofs[kFsBuckets];
  __shared__ uint64_t s_buf[kFsTile];
  __shared__ uint16_t s_dig[kFsTile];
  __shared__ uint32_t s_w[kWaves];
  uint32_t* s_key = reinterpret_cast<uint32_t*>(s_buf);
  const uint32_t nd = SplitNd(ftotal, kFsMaxU), Gr = G - nd;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  const uint32_t tile = XcdRemap(blockIdx.x, gridDim.x);
  for (int d = threadIdx.x; d < kFsBuckets; d += kFsBlock) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) whist[w][d] = 0;
    gofs[d] = offs[static_cast<uint64_t>(tile) * kFsBuckets + d];
  }
  __syncthreads();
  const uint64_t tile0 = static_cast<uint64_t>(tile) * kFsTile;
  const uint64_t wbase = tile0 + static_cast<uint64_t>(wid) * kPerWave;
  const int tn = static_cast<int>(min(static_cast<uint64_t>(kFsTile), n - tile0));
  uint32_t part[kFsItems], keys[kFsItems], dig[kFsItems];
  uint64_t v0[kFsItems];
#pragma unroll
  for (int k = 0; k < kFsItems; ++k) {
    const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
    keys[k] = i < n ? kin[i] : 0u;
    v0[k] = (nvals > 0 && i < n) ? vin.p[0][i] : 0ULL;
  }
#pragma unroll
  for (int k = 0; k < kFsItems; ++k) {
    const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
    const bool valid = i < n;
    const uint32_t d = FsBucket(keys[k], Gr, G, nd);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kFsBits; ++b) {
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
    dig[k] = d;
  }
  __syncthreads();
  {
    // Bucket starts inside the tile: thread t owns buckets [t * kPerThr, (t + 1) * kPerThr).
    uint32_t tot[kPerThr], sum = 0;
#pragma unroll
    for (int q = 0; q < kPerThr; ++q) {
      const int d = threadIdx.x * kPerThr + q;
      tot[q] = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) tot[q] += whist[w][d];
      sum += tot[q];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int w = 0; w < wid; ++w) run += s_w[w];
#pragma unroll
    for (int q = 0; q < kPerThr; ++q) {
      const int d = threadIdx.x * kPerThr + q;
      dstart[d] = run;
      uint32_t acc = run;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {  // in place: whist[w][d] becomes the start of (w, d)
        const uint32_t c = whist[w][d];
        whist[w][d] = acc;
        acc += c;
      }
      run += tot[q];
    }
  }
  __syncthreads();
  uint32_t lpos[kFsItems];
#pragma unroll
  for (int k = 0; k < kFsItems; ++k) {
    lpos[k] = whist[wid][dig[k]] + part[k];
    if (wbase + static_cast<uint64_t>(k) * 64 + lane < n) {
      s_key[lpos[k]] = keys[k];
      s_dig[lpos[k]] = static_cast<uint16_t>(dig[k]);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < tn; j += kFsBlock) {
    const uint32_t d = s_dig[j];
    if (d < static_cast<uint32_t>(kFsRest)) kout[gofs[d] + (j - dstart[d])] = s_key[j];
  }
  const uint32_t d_none = kFsRest + nd;
  for (int v = 0; v < nvals; ++v) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kFsItems; ++k) {
      const uint64_t i = wbase + static_cast<uint64_t>(k) * 64 + lane;
      if (i < n) s_buf[lpos[k]] = v == 0 ? v0[k] : vin.p[v][i];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < tn; j += kFsBlock) {
      const uint32_t d = s_dig[j];
      const uint32_t dst = gofs[d] + (j - dstart[d]);
      if (d < static_cast<uint32_t>(kFsRest)) vrest.p[v][dst] = s_buf[j];
      else if (d < d_none) vfin.p[v][dst] = s_buf[j];
    }
  }
}

// gstart of the designated groups and gstart[G]: gstart[Gr + j] = base[kFsRest + j], j <= nd.
__global__ void FsGstartKernel(const uint32_t* __restrict__ base, const uint64_t* __restrict__ ftotal, uint32_t G,
                               uint32_t* __restrict__ gstart) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nd = SplitNd(ftotal, kFsMaxU);
  if (j <= nd) gstart[G - nd + j] = base[kFsRest + j];
}

int32_t RadixSortPairs(Ctx* ctx, const uint32_t* keys, const uint32_t* rank, uint32_t cap, uint32_t G, const uint64_t* vals,
                       uint64_t n, RadixWs& ws, const uint32_t** skeys, const uint64_t** svals) {
  for (int b = 0; b < 2; ++b) {
    PXG_RETURN_IF_ERROR(ws.key[b].Ensure(n * 4 + 16));
    PXG_RETURN_IF_ERROR(ws.val[b].Ensure(n * 8 + 16));
  }
  ConstValPtrs vin;
  uint32_t* kbuf[2];
  ValPtrs vbuf[2];
  for (int v = 0; v < kMaxVals; ++v) {
    vin.p[v] = nullptr;
    vbuf[0].p[v] = vbuf[1].p[v] = nullptr;
  }
  vin.p[0] = vals;
  for (int b = 0; b < 2; ++b) {
    kbuf[b] = ws.key[b].as<uint32_t>();
    vbuf[b].p[0] = ws.val[b].as<uint64_t>();
  }
  PXG_RETURN_IF_ERROR(RadixSortStreams(ctx, keys, rank, cap, G, vin, 1, n, kbuf, vbuf, ws.rs, skeys, &vin));
  *svals = vin.p[0];
  return PXG_OK;
}

int32_t RadixSortBits(Ctx* ctx, const uint32_t* keys, int shift0, int nbits, const uint64_t* const* vals, int nvals, uint64_t n,
                      DevBuf kb[2], DevBuf vb[2], RadixPassWs& ws, const uint32_t** skeys, const uint64_t** svals) {
  if (nvals < 1 || nvals > kMaxVals) return SetError(PXG_INVALID_ARGUMENT, "radix sort of %d streams", nvals);
  for (int b = 0; b < 2; ++b) {
    PXG_RETURN_IF_ERROR(kb[b].Ensure(n * 4 + 16));
    PXG_RETURN_IF_ERROR(vb[b].Ensure(n * 8 * nvals + 16));
  }
  ConstValPtrs vin;
  uint32_t* kbuf[2];
  ValPtrs vbuf[2];
  for (int v = 0; v < kMaxVals; ++v) {
    vin.p[v] = v < nvals ? vals[v] : nullptr;
    for (int b = 0; b < 2; ++b) vbuf[b].p[v] = v < nvals ? vb[b].as<uint64_t>() + v * n : nullptr;
  }
  for (int b = 0; b < 2; ++b) kbuf[b] = kb[b].as<uint32_t>();
  PXG_RETURN_IF_ERROR(RadixSortStreams(ctx, keys, nullptr, 0, 0, vin, nvals, n, kbuf, vbuf, ws, skeys, &vin, shift0, nbits));
  *svals = vin.p[0];  // stream v at *svals + v * n
  return PXG_OK;
}

int32_t GroupStarts(Ctx* ctx, const uint32_t* skeys, uint64_t n, uint32_t G, uint32_t* gstart) {
  const int64_t waves = (static_cast<int64_t>(n) + 255) / 256;
  const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, static_cast<int64_t>(ctx->num_cus) * 8)));
  return Launch(ctx, "group_heads", GroupHeadsKernel, dim3(grid), dim3(256), 0, skeys, n, G, gstart);
}

// Fused split for large aggregations (PXG_FSPLIT=0 / 1 overrides the size rule).
// Measured (rocprof, same box): 1B rows (120M staged) finalize span 5.00 -> 4.84 ms; at C2 (12M
// staged) the extra sample / designation launches cost what the shorter rest pass saves.
constexpr uint64_t kFsMinStaged = uint64_t(1) << 25;
bool FusedSplitOn(uint64_t n) {
  const char* e = std::getenv("PXG_FSPLIT");
  if (e && e[0]) return e[0] != '0';
  return n >= kFsMinStaged;
}

// ---------------------------------------------------------------------------------------
// Entry points of the grouping for AggFinalizeTable (pxg_finalize.hip); pxg_sort.h documents them.
// ---------------------------------------------------------------------------------------
int32_t DenseIdsBySlot(Ctx* ctx, const unsigned long long* slots, uint32_t cap, uint32_t* rank, uint32_t* gslot, uint32_t* d_ngroups,
                       void* scan_tmp) {
  PXG_RETURN_IF_ERROR(Launch(ctx, "slot_flags", SlotFlagsKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0, slots, cap, rank));
  PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, rank, rank, cap, d_ngroups, scan_tmp));
  return Launch(ctx, "slot_gslot", SlotGslotKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0, slots, cap,
                static_cast<const uint32_t*>(rank), gslot);
}

int32_t DesignateLargeGroups(Ctx* ctx, const unsigned long long* slots, uint32_t cap, const uint32_t* st_slot, uint64_t n, uint32_t G,
                             DevBuf& split_cnt, DevBuf& split_flags, uint32_t* rank, uint32_t* gslot, uint32_t* d_ngroups, void* scan_tmp,
                             uint64_t** d_ftotal) {
  const uint32_t max_big = kFsMaxU;
  const uint32_t min_samples = std::max<uint32_t>(1, kFsMinRows / kSplitStride);
  PXG_RETURN_IF_ERROR(split_cnt.Ensure(static_cast<size_t>(cap) * 4 + 32 * 4));
  PXG_RETURN_IF_ERROR(split_flags.Ensure((static_cast<size_t>(cap) + 2) * 8));
  uint64_t* flags = split_flags.as<uint64_t>();
  uint64_t* ftotal = flags + cap;
  uint32_t* lvl = split_cnt.as<uint32_t>() + cap;
  PXG_HIP(hipMemsetAsync(split_cnt.p, 0, static_cast<size_t>(cap) * 4 + 32 * 4, ctx->stream));
  const uint64_t nsamp = (n + kSplitStride - 1) / kSplitStride;
  PXG_RETURN_IF_ERROR(Launch(ctx, "split_sample", SplitSampleKernel, dim3(GridFor(static_cast<int64_t>(nsamp), 256 * kSamplePerThread, 1 << 30)),
                             dim3(256), 0, st_slot, n, cap, split_cnt.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(Launch(ctx, "split_ids", SplitLevelsKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                             split_cnt.as<const uint32_t>(), cap, lvl));
  PXG_RETURN_IF_ERROR(Launch(ctx, "split_ids", SplitFlagsKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0, slots, cap,
                             split_cnt.as<const uint32_t>(), static_cast<const uint32_t*>(lvl), min_samples, max_big, flags));
  PXG_RETURN_IF_ERROR(ScanExclusiveU64(ctx, flags, flags, cap, ftotal, scan_tmp));
  PXG_RETURN_IF_ERROR(Launch(ctx, "split_ids", SplitIdsKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0, slots, cap,
                             split_cnt.as<const uint32_t>(), static_cast<const uint32_t*>(lvl), min_samples, max_big,
                             static_cast<const uint64_t*>(flags), static_cast<const uint64_t*>(ftotal), G, rank, gslot));
  // d_ngroups (the device's own group count, checked at the end of finalize) from the occupied total.
  PXG_HIP(hipMemcpyAsync(d_ngroups, ftotal, 4, hipMemcpyDeviceToDevice, ctx->stream));
  *d_ftotal = ftotal;
  return PXG_OK;
}

int32_t FusedSplitPass(Ctx* ctx, const uint32_t* st_slot, uint64_t n, const uint32_t* rank, uint32_t cap, uint32_t G, const uint64_t* d_ftotal,
                       ConstValPtrs vin, int nvs, DevBuf& split_hist, DevBuf& split_tot, DevBuf& fs_keys, RadixPassWs& rs, uint32_t* kout_rest,
                       ValPtrs vrest, ValPtrs vfin, const uint32_t** base_out) {
  const uint32_t ntiles = static_cast<uint32_t>((n + kFsTile - 1) / kFsTile);
  const uint32_t nparts = (ntiles + kRsTilesPerPart - 1) / kRsTilesPerPart;
  PXG_RETURN_IF_ERROR(split_hist.Ensure(static_cast<size_t>(ntiles) * kFsBuckets * 4));
  PXG_RETURN_IF_ERROR(rs.part.Ensure(static_cast<size_t>(nparts) * kFsBuckets * 4));
  PXG_RETURN_IF_ERROR(split_tot.Ensure(static_cast<size_t>(2 * kFsBuckets + 2) * 4));
  PXG_RETURN_IF_ERROR(fs_keys.Ensure(n * 4 + 16));
  uint32_t* hist = split_hist.as<uint32_t>();
  uint32_t* tot = split_tot.as<uint32_t>();
  uint32_t* base = tot + kFsBuckets;
  const int ht = ntiles >= 16384 ? 4 : 1;
  PXG_RETURN_IF_ERROR(Launch(ctx, "radix_hist_rank", ht == 4 ? FsHistKernel<4> : FsHistKernel<1>, dim3((ntiles + ht - 1) / ht), dim3(kFsBlock), 0,
                             st_slot, n, rank, cap, G, d_ftotal, hist, ntiles, fs_keys.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", XPartKernel<kFsBuckets>, dim3(nparts), dim3(256), 0, static_cast<const uint32_t*>(hist), ntiles,
                             rs.part.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", XPartScanKernel<kFsBuckets>, dim3(kFsBuckets), dim3(kRsScanBlock), 0, rs.part.as<uint32_t>(),
                             nparts, tot));
  PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", XBaseKernel<kFsBuckets>, dim3(1), dim3(256), 0, static_cast<const uint32_t*>(tot), base));
  PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scan", XDownKernel<kFsBuckets>, dim3(nparts), dim3(256), 0, hist, ntiles,
                             static_cast<const uint32_t*>(rs.part.as<uint32_t>()), static_cast<const uint32_t*>(base)));
  // n_rest (= base[kFsRest]) and the designated count to pinned memory; the scatter runs meanwhile.
  uint8_t* pin = static_cast<uint8_t*>(ctx->pinned);
  PXG_HIP(hipMemcpyAsync(pin + 104, base + kFsRest, 4, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipMemcpyAsync(pin + 112, d_ftotal, 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipEventRecord(ctx->ev_split, ctx->stream));
  PXG_RETURN_IF_ERROR(Launch(ctx, "radix_scatter", FsScatterKernel, dim3(ntiles), dim3(kFsBlock), 0, static_cast<const uint32_t*>(fs_keys.as<uint32_t>()),
                             n, G, d_ftotal, vin, nvs, static_cast<const uint32_t*>(hist), kout_rest, vrest, vfin));
  *base_out = base;
  return PXG_OK;
}

const uint32_t* FusedSplitDesignatedStarts(const uint32_t* base) { return base + kFsRest; }

int32_t FusedSplitGstart(Ctx* ctx, const uint32_t* base, const uint64_t* d_ftotal, uint32_t G, uint32_t* gstart) {
  return Launch(ctx, "group_heads", FsGstartKernel, dim3((kFsMaxU + 256) / 256), dim3(256), 0, base, d_ftotal, G, gstart);
}

}  // namespace pxg
