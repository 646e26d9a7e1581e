// High-cardinality aggregation: partitioned LDS hash tables instead of one global table.
//
// Reference: the same AggNode hash aggregation (agg_node.cc:209-271 AggHashMap lookup/insert,
// ConvertAggHashMapToRowBatch agg_node.cc:303-349).  With millions of groups (C3: ~5-7M
// (pod, remote_addr) groups from 12M selected rows) a global open-addressing table makes every
// row a chain of random HBM round trips (probe, representative-row compare, key publication,
// key extraction), so this mode restructures the work around partitions that fit in LDS:
//
//   consume  (AggConsumeFastKernel<..., HC>): one record per selected row (key words + values,
//            pxg_agg.h HcStageDev) written densely as word streams, plus its key-hash top half.
//   sort     the records by the top `pbits` hash bits (stable LSD radix passes over the
//            partition bits only, every record stream moved with coalesced loads and runs).
//   agg      one workgroup per partition (~1024 records, contiguous after the sort): an LDS
//            open-addressing table of kHcTable entries {tag, representative record}, exact key
//            compare against the representative, LDS integer atomics for count / sum / min /
//            max; the partition's groups are then emitted densely (one global atomic each).
//   keys     string keys: one scan of the lengths, one copy from a dense key scratch.
//
// Results are order-independent integer reductions, so they do not depend on the partition
// count or on the order threads meet in LDS.  A partition whose distinct keys overflow its
// table sets a flag and the whole pass reruns with 4x the partitions (the staged records are
// unchanged).
#include <algorithm>
#include <cstdlib>

#include "pxg_agg_host.h"
#include "pxg_keys.h"
#include "pxg_scan.h"
#include "pxg_sort.h"

namespace pxg {

constexpr int kHcBlock = 256;
constexpr uint64_t kHcMaxPartRecs = 4096;  // records per partition the first pass aims below (FinalizeHc)
constexpr int kHcTable = 1024;  // LDS entries per partition (~1024 records, ~300-400 groups at C3)
constexpr int kHcMaxAcc = 4;
constexpr int kHcKeyWords = 1 + kMaxKeys * kHcStrWords;
constexpr int kHcGroupsLog2 = 9;  // the first pass sizes partitions for ~2^kHcGroupsLog2 groups (~50 % table fill)

// kHcAddWide: an exact 128-bit two's-complement sum (low word in the accumulator, high word in
// its acc_hi array), for MEAN over INT64: MeanUDA accumulates `double sum += arg`
// (math_ops.h:586-589), which cannot wrap, so a 64-bit integer sum that passes 2^63 must not
// either.
enum HcAccOp : int32_t { kHcAdd = 0, kHcMin = 1, kHcMax = 2, kHcAddWide = 3 };

struct HcAggPlan {
  uint64_t n;  // records (the distance between two sorted record streams)
  int32_t stride, kwords, nk, n_udas, nacc, nhi;
  int32_t ktype[kMaxKeys], koff[kMaxKeys];
  int32_t uda_kind[kMaxUdas], uda_acc[kMaxUdas];
  int64_t uda_init[kMaxUdas];
  int32_t acc_op[kHcMaxAcc], acc_word[kHcMaxAcc];
  int32_t acc_hi[kHcMaxAcc];  // kHcAddWide: LDS array of the high words (nacc + j), else -1
  int32_t tail0;  // key 0's third word rides in the lengths word's high half (its stream is dropped)
};

struct HcOut {
  uint64_t* uda[kMaxUdas];
  uint8_t* states;           // export: each group's Serialize() states (srec bytes) instead of uda[]
  int32_t srec, soff[kMaxUdas];
  uint64_t* kfix[kMaxKeys];  // fixed-width keys (UINT128: 2 words per group, BOOLEAN: bytes)
  uint32_t* klen[kMaxKeys];  // STRING: lengths, turned into offsets by the scan
  uint64_t* kscr;            // the representative's key words, kwords per group (STRING keys), or null
  uint32_t g0;               // groups the table path already wrote
};

// FinalizeHc in export mode (ExportHcGroups): per partition group its Serialize() states at
// states + g * state_rec and its key words in the scratch (word j at kscr[j * plan.n + g]).
struct HcExport {
  uint8_t* states = nullptr;
  uint32_t groups = 0;
  const uint64_t* kscr = nullptr;
  HcAggPlan plan{};
};

// starts[p] = first sorted record of partition p (p in [0, P]); partition = key >> shift.
// Record i writes the starts of the partitions in (part(i - 1), part(i)] (part(-1) = -1,
// part(n) = P).  A wave takes 256 consecutive records per step (one 16-byte load per lane, the
// previous lane's last key by a shuffle) over a resident grid, as GroupHeadsKernel does.
__device__ __forceinline__ void HcPartFill(int64_t prev, int64_t cur, uint64_t i, uint32_t* __restrict__ starts) {
  for (int64_t p = prev + 1; p <= cur; ++p) starts[p] = static_cast<uint32_t>(i);
}
__global__ void __launch_bounds__(256) HcPartStartsKernel(const uint32_t* __restrict__ skeys, uint64_t n, int shift, uint32_t P,
                                                          uint32_t* __restrict__ starts) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 6;
  const bool vec = (reinterpret_cast<uintptr_t>(skeys) & 15) == 0;
  for (uint64_t w0 = ((static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6) * 256; w0 < n; w0 += nwaves * 256) {
    const uint64_t b = w0 + 4 * static_cast<uint64_t>(lane);
    uint32_t k[4];
    if (vec && b + 4 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(skeys + b);
      k[0] = v.x;
      k[1] = v.y;
      k[2] = v.z;
      k[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) k[j] = b + j < n ? skeys[b + j] : 0u;
    }
    int64_t p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = static_cast<int64_t>(k[j] >> shift);
    int64_t prev = static_cast<int64_t>(__shfl_up(static_cast<int>(p[3]), 1, 64));
    if (lane == 0) prev = w0 == 0 ? -1 : static_cast<int64_t>(skeys[w0 - 1] >> shift);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (b + j >= n) break;
      HcPartFill(prev, p[j], b + j, starts);
      prev = p[j];
    }
  }
  // record n: the partitions after the last record's (all of them when n == 0)
  if (blockIdx.x == 0 && threadIdx.x == 0) HcPartFill(n == 0 ? -1 : static_cast<int64_t>(skeys[n - 1] >> shift), static_cast<int64_t>(P), n, starts);
}

__device__ __forceinline__ unsigned long long HcAccInit(int op) {
  return op == kHcMin ? static_cast<unsigned long long>(INT64_MAX) : (op == kHcMax ? static_cast<unsigned long long>(INT64_MIN) : 0ULL);
}

// One group's key outputs from its representative's key words: STRING lengths (offsets after
// the scan), fixed-width keys, and the words into the key scratch (stream-major, so the string
// copy after the scan streams it).
template <int KW>
__device__ __forceinline__ void HcEmitKeys(const HcAggPlan& hp, const HcOut& out, uint32_t g, const uint64_t* w) {
  const uint32_t l = g - out.g0;
  if (out.kscr) {
#pragma unroll
    for (int j = 0; j < KW; ++j) out.kscr[static_cast<uint64_t>(j) * hp.n + l] = w[j];
  }
  if (out.states) return;  // export: the key words are all it needs
#pragma unroll
  for (int k = 0; k < kMaxKeys; ++k) {
    if (k >= hp.nk) break;
    const int t = hp.ktype[k];
    const int o = hp.koff[k];
    uint64_t k0 = 0, k1 = 0;
#pragma unroll
    for (int j = 1; j < KW; ++j) {
      k0 = j == o ? w[j] : k0;
      k1 = j == o + 1 ? w[j] : k1;
    }
    if (t == PXG_STRING) {
      out.klen[k][g] = static_cast<uint32_t>((w[0] >> (16 * k)) & 0xFFFF);
    } else if (t == PXG_UINT128) {
      out.kfix[k][2 * g] = k0;
      out.kfix[k][2 * g + 1] = k1;
    } else if (t == PXG_BOOLEAN) {
      reinterpret_cast<uint8_t*>(out.kfix[k])[g] = static_cast<uint8_t>(k0);
    } else {
      out.kfix[k][g] = k0;
    }
  }
}

// The 128-bit two's-complement integer hi:lo as a double.  Inside the int64 range it is the
// int64's conversion (exact rounding); beyond it |x| >= 2^63, so the two-term sum's rounding
// error stays within a few ulps (no cancellation).
__device__ __forceinline__ double WideToDouble(int64_t hi, uint64_t lo) {
  const bool fits = (hi == 0 && static_cast<int64_t>(lo) >= 0) || (hi == -1 && static_cast<int64_t>(lo) < 0);
  return fits ? static_cast<double>(static_cast<int64_t>(lo)) : static_cast<double>(hi) * 18446744073709551616.0 + static_cast<double>(lo);
}

// One group's UDA outputs (UDA Finalize, math_ops.h CountUDA / SumUDA / MeanUDA / MinUDA /
// MaxUDA).  MEAN over integer arguments divides the exact 128-bit integer sum (the reference
// accumulates the same values in a double; both agree to rounding, and neither wraps).
__device__ __forceinline__ void HcEmitVals(const HcAggPlan& hp, const HcOut& out, uint32_t g, uint32_t cnt, const unsigned long long* s_acc,
                                           int slot) {
  if (out.states) {  // export: Serialize() states (math_ops.h:583-772; MeanInfo {size, sum})
    uint8_t* st = out.states + static_cast<uint64_t>(g) * out.srec;
    for (int u = 0; u < hp.n_udas; ++u) {
      const int a = hp.uda_acc[u];
      const unsigned long long acc = a >= 0 ? s_acc[a * kHcTable + slot] : 0ULL;
      uint64_t v0 = acc, v1 = 0;
      switch (hp.uda_kind[u]) {
        case PXG_UDA_COUNT: v0 = cnt; break;
        case PXG_UDA_MEAN: {
          const int hi = a >= 0 ? hp.acc_hi[a] : -1;
          const int64_t h = hi >= 0 ? static_cast<int64_t>(s_acc[hi * kHcTable + slot]) : (static_cast<int64_t>(acc) >> 63);
          v0 = cnt;
          v1 = FBits(WideToDouble(h, acc));
          break;
        }
        case PXG_UDA_SUM: v0 = acc + static_cast<uint64_t>(hp.uda_init[u]); break;
        default: break;  // MIN / MAX (integer)
      }
      __builtin_memcpy(st + out.soff[u], &v0, 8);
      if (hp.uda_kind[u] == PXG_UDA_MEAN) __builtin_memcpy(st + out.soff[u] + 8, &v1, 8);
    }
    return;
  }
  for (int u = 0; u < hp.n_udas; ++u) {
    const int a = hp.uda_acc[u];
    const unsigned long long acc = a >= 0 ? s_acc[a * kHcTable + slot] : 0ULL;
    uint64_t v;
    switch (hp.uda_kind[u]) {
      case PXG_UDA_COUNT: v = cnt; break;
      case PXG_UDA_MEAN: {
        const int hi = a >= 0 ? hp.acc_hi[a] : -1;
        const int64_t h = hi >= 0 ? static_cast<int64_t>(s_acc[hi * kHcTable + slot]) : (static_cast<int64_t>(acc) >> 63);
        v = FBits(WideToDouble(h, acc) / static_cast<double>(cnt));
        break;
      }
      case PXG_UDA_SUM:
      case PXG_UDA_MINSUM: v = acc + static_cast<uint64_t>(hp.uda_init[u]); break;
      default: v = acc; break;  // MIN / MAX (integer)
    }
    out.uda[u][g] = v;
  }
}

// Linear probe of the partition table from `pos`: the slot of the record's group (inserting
// it when absent), or -1 when the table is full.  With `defer`, a tag match is returned as a
// candidate (*cand = true) without comparing keys, so the caller can issue the compares of
// several records at once; without it every tag match is compared here.
template <int KW>
__device__ __forceinline__ int HcProbe(unsigned long long* s_ent, uint32_t pos, unsigned long long mine, const uint64_t* w,
                                       const HcAggPlan& hp, const uint64_t* __restrict__ rec, bool defer, bool* cand) {
  const uint32_t tag = static_cast<uint32_t>(mine >> 32);
  *cand = false;
  for (int probe = 0; probe < kHcTable; ++probe) {
    unsigned long long cur = __hip_atomic_load(&s_ent[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0) {
      unsigned long long expected = 0;
      if (__hip_atomic_compare_exchange_strong(&s_ent[pos], &expected, mine, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP))
        return static_cast<int>(pos);
      cur = expected;
    }
    if (static_cast<uint32_t>(cur >> 32) == tag) {
      if (defer) {
        *cand = true;
        return static_cast<int>(pos);
      }
      const uint64_t* q = rec + static_cast<uint32_t>(cur);
      bool eq = true;
#pragma unroll
      for (int j = 0; j < KW; ++j) eq = eq && q[j * hp.n] == w[j];
      if (eq) return static_cast<int>(pos);
    }
    pos = (pos + 1) & (kHcTable - 1);
  }
  return -1;
}

// Probe hash of a record's key words (any function of the words works: the partition came
// from the consume hash, this only spreads a partition's keys over its LDS table).
template <int KW>
__device__ __forceinline__ uint64_t HcWordsHash(const uint64_t* w) {
  uint64_t h = 0x9E3779B97F4A7C15ULL;
#pragma unroll
  for (int j = 0; j < KW; ++j) h = Fmix64(h ^ (w[j] + 0xC2B2AE3D27D4EB4FULL * (j + 1)));
  return h;
}

// One workgroup per partition (grid-stride).  meta[0]: groups emitted, meta[1]: overflow flag.
// A partition's records are contiguous in the sorted streams (`rec`, stream j at rec + j * n).
// Records are taken kHcR per thread at a time: their key words are all requested before the
// first LDS probe, and the representative compares of the batch are issued together after
// every record has found its candidate slot.  KW: key words per record (hp.kwords), a template
// so the batch's registers are sized exactly.
constexpr int kHcR = 4;  // (8 measured slower in round 6: C3 hc_agg 0.51 -> 0.88 ms, C3 full 2.79 -> 3.77 ms)
template <int KW>
__global__ void __launch_bounds__(kHcBlock) HcAggKernel(HcAggPlan hp, const uint64_t* __restrict__ rec,
                                                       const uint32_t* __restrict__ starts, uint32_t nparts, HcOut out,
                                                       uint32_t* __restrict__ meta) {
  extern __shared__ unsigned long long s_dyn[];
  unsigned long long* s_ent = s_dyn;                                  // [kHcTable]: tag << 32 | rep record
  unsigned long long* s_acc = s_dyn + kHcTable;                       // [nacc][kHcTable]
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_dyn + kHcTable * (1 + hp.nacc + hp.nhi));  // [kHcTable]
  constexpr int kWaves = kHcBlock / 64;
  constexpr int kPerThr = kHcTable / kHcBlock;
  __shared__ uint32_t s_wsum[kWaves];
  __shared__ uint32_t s_gbase;
  __shared__ int s_ovf;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t n = hp.n;
  for (uint32_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const uint32_t s = starts[p], e = starts[p + 1];
    for (int t = threadIdx.x; t < kHcTable; t += kHcBlock) {
      s_ent[t] = 0;
      s_cnt[t] = 0;
      for (int a = 0; a < hp.nacc; ++a) s_acc[a * kHcTable + t] = HcAccInit(hp.acc_op[a]);
      for (int a = 0; a < hp.nhi; ++a) s_acc[(hp.nacc + a) * kHcTable + t] = 0;
    }
    if (threadIdx.x == 0) s_ovf = 0;
    __syncthreads();
    // A partition of at most one batch keeps its records in registers through the emit, and
    // each group's representative writes the group's keys from them.
    const bool single = e - s <= static_cast<uint32_t>(kHcBlock * kHcR);
    uint64_t w[kHcR][KW];
    bool live[kHcR];
    int slot[kHcR];
#pragma unroll
    for (int q = 0; q < kHcR; ++q) {
      live[q] = false;
      slot[q] = -1;
    }
    for (uint32_t b0 = s; b0 < e; b0 += kHcBlock * kHcR) {
#pragma unroll
      for (int q = 0; q < kHcR; ++q) {
        const uint32_t i = b0 + q * kHcBlock + threadIdx.x;
        const uint32_t ii = i < e ? i : s;  // in range, ignored
#pragma unroll
        for (int j = 0; j < KW; ++j) w[q][j] = rec[j * n + ii];
        live[q] = i < e && w[q][0] != kHcHole;
      }
      bool cand[kHcR];
      unsigned long long mine[kHcR];
#pragma unroll
      for (int q = 0; q < kHcR; ++q) {
        slot[q] = -1;
        cand[q] = false;
        const uint64_t h = HcWordsHash<KW>(w[q]);
        mine[q] = (static_cast<unsigned long long>(static_cast<uint32_t>(h >> 32) | 0x80000000u) << 32) |
                  (b0 + q * kHcBlock + threadIdx.x);
        if (!live[q]) continue;
        slot[q] = HcProbe<KW>(s_ent, static_cast<uint32_t>(h) & (kHcTable - 1), mine[q], w[q], hp, rec, true, &cand[q]);
      }
      // The candidates' representative key words, all requested before the compares (a
      // non-candidate reads the partition's first record and ignores it).
      bool eq[kHcR];
#pragma unroll
      for (int q = 0; q < kHcR; ++q) {
        const uint32_t ri = cand[q] ? static_cast<uint32_t>(s_ent[slot[q]]) : s;
        eq[q] = true;
#pragma unroll
        for (int j = 0; j < KW; ++j) eq[q] = eq[q] && rec[j * n + ri] == w[q][j];
      }
#pragma unroll
      for (int q = 0; q < kHcR; ++q) {
        if (!cand[q] || eq[q]) continue;
        // a tag collision: keep probing past it, comparing as we go
        bool c2;
        slot[q] = HcProbe<KW>(s_ent, (static_cast<uint32_t>(slot[q]) + 1) & (kHcTable - 1), mine[q], w[q], hp, rec, false, &c2);
      }
#pragma unroll
      for (int q = 0; q < kHcR; ++q) {
        if (live[q] && slot[q] < 0) s_ovf = 1;
        if (live[q] && slot[q] >= 0) atomicAdd(&s_cnt[slot[q]], 1u);
      }
      for (int a = 0; a < hp.nacc; ++a) {
        const int op = hp.acc_op[a];
        const uint64_t* vs = rec + static_cast<uint64_t>(hp.acc_word[a]) * n;
        uint64_t x[kHcR];
#pragma unroll
        for (int q = 0; q < kHcR; ++q) {
          const uint32_t i = b0 + q * kHcBlock + threadIdx.x;
          x[q] = vs[i < e ? i : s];
        }
#pragma unroll
        for (int q = 0; q < kHcR; ++q) {
          if (!live[q] || slot[q] < 0) continue;
          unsigned long long* dst = &s_acc[a * kHcTable + slot[q]];
          if (op == kHcAdd) {
            atomicAdd(dst, x[q]);
          } else if (op == kHcAddWide) {
            // low word, then the carry out of it plus the sign extension of x into the high word
            const unsigned long long old = atomicAdd(dst, x[q]);
            const unsigned long long inc = static_cast<unsigned long long>(static_cast<int64_t>(x[q]) >> 63) + (old + x[q] < old ? 1ULL : 0ULL);
            if (inc) atomicAdd(&s_acc[hp.acc_hi[a] * kHcTable + slot[q]], inc);
          } else if (op == kHcMin) atomicMin(reinterpret_cast<long long*>(dst), static_cast<long long>(x[q]));
          else atomicMax(reinterpret_cast<long long*>(dst), static_cast<long long>(x[q]));
        }
      }
    }
    __syncthreads();
    if (s_ovf) {  // uniform: the host reruns with more partitions
      if (threadIdx.x == 0) atomicOr(&meta[1], 1u);
      __syncthreads();
      continue;
    }
    // Emit: thread t owns entries [t * kPerThr, (t + 1) * kPerThr); a block scan of the counts
    // and one global atomic place the partition's groups.
    uint32_t occ = 0;
#pragma unroll
    for (int k = 0; k < kPerThr; ++k) occ |= (s_ent[threadIdx.x * kPerThr + k] != 0 ? 1u : 0u) << k;
    const uint32_t c = static_cast<uint32_t>(__popc(occ));
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t y = s_wsum[w];
      wbase += w < wid ? y : 0u;
      tot += y;
    }
    if (threadIdx.x == 0) s_gbase = tot ? atomicAdd(&meta[0], tot) : 0u;
    __syncthreads();
    uint32_t g = out.g0 + s_gbase + wbase + incl - c;
#pragma unroll
    for (int k = 0; k < kPerThr; ++k) {
      if (!((occ >> k) & 1u)) continue;
      const int sl = threadIdx.x * kPerThr + k;
      HcEmitVals(hp, out, g, s_cnt[sl], s_acc, sl);
      if (single) {
        s_cnt[sl] = g;  // the group's output row, for its representative below
      } else {
        const uint32_t ri = static_cast<uint32_t>(s_ent[sl]);
        uint64_t rw[KW];
#pragma unroll
        for (int j = 0; j < KW; ++j) rw[j] = rec[j * n + ri];
        HcEmitKeys<KW>(hp, out, g, rw);
      }
      ++g;
    }
    if (single) {
      __syncthreads();
#pragma unroll
      for (int q = 0; q < kHcR; ++q) {
        if (!live[q] || slot[q] < 0) continue;
        const uint32_t i = s + q * kHcBlock + threadIdx.x;
        if (static_cast<uint32_t>(s_ent[slot[q]]) == i) HcEmitKeys<KW>(hp, out, s_cnt[slot[q]], w[q]);
      }
    }
    __syncthreads();  // the next partition reuses the LDS table
  }
}

struct HcKeyCopy {
  int32_t kw[kMaxKeys];     // the key's words in the scratch
  uint32_t* off[kMaxKeys];  // R.key_offsets[k] + g0 (null: not a STRING key)
  uint8_t* data[kMaxKeys];  // R.key_data[k]
  uint32_t dbase[kMaxKeys]; // bytes the table path wrote before (offsets are rebased by it)
};

// String key bytes of every group (local group l) from the key scratch HcEmitKeys wrote
// (word j of group l at kscr[j * kcap + l]).
__global__ void HcKeyCopyKernel(const uint64_t* __restrict__ kscr, uint64_t kcap, uint32_t ngroups, int nk, HcKeyCopy kc, HcAggPlan hp) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l > ngroups) return;
  const uint64_t lens = l < ngroups ? kscr[l] : 0;
  for (int k = 0; k < nk; ++k) {
    uint32_t* off = kc.off[k];
    if (!off) continue;
    if (l == ngroups) {  // the total (written by the scan)
      if (kc.dbase[k]) off[l] += kc.dbase[k];
      continue;
    }
    const uint32_t len = static_cast<uint32_t>((lens >> (16 * k)) & 0xFFFF);
    uint64_t kw[kHcStrWords];
#pragma unroll
    for (int j = 0; j < kHcStrWords; ++j) kw[j] = j < kc.kw[k] ? kscr[static_cast<uint64_t>(hp.koff[k] + j) * kcap + l] : 0;
    if (k == 0 && hp.tail0) kw[2] = lens >> 32;  // (kc.kw[0] == 2)
    const uint32_t o = off[l] + kc.dbase[k];
    if (kc.dbase[k]) off[l] = o;
    CopyBytesOverlap(kc.data[k] + o, reinterpret_cast<const uint8_t*>(kw), len);
  }
}

using HcAggFn = void (*)(HcAggPlan, const uint64_t*, const uint32_t*, uint32_t, HcOut, uint32_t*);
static HcAggFn HcAggFor(int kwords) {
  switch (kwords) {
    case 1: return HcAggKernel<1>;
    case 2: return HcAggKernel<2>;
    case 3: return HcAggKernel<3>;
    case 4: return HcAggKernel<4>;
    case 5: return HcAggKernel<5>;
    case 6: return HcAggKernel<6>;
    case 7: return HcAggKernel<7>;
    case 8: return HcAggKernel<8>;
    case 9: return HcAggKernel<9>;
    case 10: return HcAggKernel<10>;
    case 11: return HcAggKernel<11>;
    case 12: return HcAggKernel<12>;
    default: return HcAggKernel<13>;
  }
}
static_assert(kHcKeyWords == 13, "HcAggFor covers 1..13 key words");

// The partition pass's record layout.  With `compact`, a STRING key keeps only the words its
// longest staged value needs (the rest of its streams are all zero: C3's remote_addr fits 2 of
// its 3 words), so the sort moves and hc_agg reads fewer streams; src[j] names the staged stream
// of compacted word j.  Without it (spill) the staged layout as is.
static HcAggPlan MakeHcPlan(const Agg& a, bool compact = false, int32_t* src = nullptr, int32_t* kwc = nullptr) {
  HcAggPlan hp;
  std::memset(&hp, 0, sizeof(hp));
  hp.nk = a.n_keys;
  hp.n_udas = a.n_udas;
  int w = 1;
  if (src) src[0] = 0;
  for (int k = 0; k < a.n_keys; ++k) {
    hp.ktype[k] = a.key_types[k];
    int kw = a.hc_layout.kw[k];
    if (compact && a.key_types[k] == PXG_STRING) kw = std::min<int>(kw, static_cast<int>((a.hc_maxlen_h[k] + 7) / 8));
    // (consume writes bytes 16-19 of key 0 into the lengths word when there are <= 2 keys)
    if (compact && k == 0 && a.key_types[0] == PXG_STRING && a.n_keys <= 2 && kw == 3 && a.hc_maxlen_h[0] <= 20) {
      kw = 2;
      hp.tail0 = 1;
    }
    hp.koff[k] = w;
    if (kwc) kwc[k] = kw;
    for (int j = 0; j < kw; ++j)
      if (src) src[w + j] = a.hc_layout.koff[k] + j;
    w += kw;
  }
  hp.kwords = w;
  for (int v = 0; v < a.n_vals; ++v)
    if (src) src[w + v] = a.hc_layout.kwords + v;
  hp.stride = w + a.n_vals;
  for (int u = 0; u < a.n_udas; ++u) {
    const int kind = a.uda_kind[u];
    hp.uda_kind[u] = kind;
    hp.uda_init[u] = a.hplan.uda_init[u];
    hp.uda_acc[u] = -1;
    if (kind == PXG_UDA_COUNT) continue;
    const int i = hp.nacc++;
    hp.uda_acc[u] = i;
    hp.acc_op[i] = kind == PXG_UDA_MIN ? kHcMin : (kind == PXG_UDA_MAX ? kHcMax : (kind == PXG_UDA_MEAN ? kHcAddWide : kHcAdd));
    hp.acc_word[i] = hp.kwords + a.uda_val[u];
  }
  for (int i = 0; i < hp.nacc; ++i) hp.acc_hi[i] = hp.acc_op[i] == kHcAddWide ? hp.nacc + hp.nhi++ : -1;
  return hp;
}

int32_t Agg::FinalizeHc(HcExport* ex) {
  AggResult& R = res;
  const uint64_t n = hc_n;
  const uint32_t g0 = ex ? 0u : static_cast<uint32_t>(R.n_groups);
  if (ex) ex->groups = 0;
  if (!ex) R.ready = false;
  if (n == 0) {
    if (!ex) R.ready = true;
    return PXG_OK;
  }
  int32_t src[kHcMaxStride];
  int32_t kwc[kMaxKeys];
  HcAggPlan hp = MakeHcPlan(*this, true, src, kwc);
  hp.n = n;
  const uint64_t* streams[kHcMaxStride];
  for (int j = 0; j < hp.stride; ++j) streams[j] = hc_rec.as<const uint64_t>() + static_cast<uint64_t>(src[j]) * hc_cap;
  FinalizeWs& w = ws;
  PXG_RETURN_IF_ERROR(w.hc_meta.Ensure(64));
  // Result buffers for up to n more groups, keeping the table path's g0 groups.
  const uint64_t cap_g = static_cast<uint64_t>(g0) + n;
  uint64_t dbase[kMaxKeys] = {0};
  for (int u = 0; u < n_udas && !ex; ++u) PXG_RETURN_IF_ERROR(R.uda_out[u].Reserve(cap_g * 8, static_cast<size_t>(g0) * 8, ctx->stream));
  for (int k = 0; k < n_keys && !ex; ++k) {
    const int t = key_types[k];
    if (t == PXG_STRING) {
      // (the payload is reserved after the partition pass, from its group count)
      dbase[k] = static_cast<uint64_t>(R.key_data_len[k]);
      PXG_RETURN_IF_ERROR(R.key_offsets[k].Reserve((cap_g + 1) * 4, static_cast<size_t>(g0) * 4, ctx->stream));
    } else {
      const size_t wd = t == PXG_UINT128 ? 16 : 8;
      PXG_RETURN_IF_ERROR(R.key_fixed[k].Reserve(cap_g * wd, static_cast<size_t>(g0) * wd, ctx->stream));
    }
  }
  HcOut out;
  std::memset(&out, 0, sizeof(out));
  if (ex) {
    out.states = ex->states;
    out.srec = hplan_x.state_rec;
    for (int u = 0; u < n_udas; ++u) out.soff[u] = hplan_x.state_off[u];
  } else {
    for (int u = 0; u < n_udas; ++u) out.uda[u] = R.uda_out[u].as<uint64_t>();
    for (int k = 0; k < n_keys; ++k) {
      if (key_types[k] == PXG_STRING) out.klen[k] = R.key_offsets[k].as<uint32_t>();
      else out.kfix[k] = R.key_fixed[k].as<uint64_t>();
    }
  }
  bool any_str_key = false;
  for (int k = 0; k < n_keys; ++k) any_str_key = any_str_key || key_types[k] == PXG_STRING;
  if (any_str_key || ex) {  // (an export rebuilds every group's key record from the scratch)
    PXG_RETURN_IF_ERROR(w.hc_kscr.Ensure(n * static_cast<uint64_t>(hp.kwords) * 8 + 16));
    out.kscr = w.hc_kscr.as<uint64_t>();
  }
  out.g0 = g0;
  static_assert(kHcTable == kHcTableEntries, "LDS budget and table size disagree");
  const size_t lds = HcAggLdsBytes(hp.nacc, hp.nhi);
  if (lds > HcMaxDynLds()) return SetError(PXG_INTERNAL, "hc_agg needs %zu bytes of LDS", lds);
  uint32_t* meta = w.hc_meta.as<uint32_t>();
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + 192);
  // The first pass aims at ~2^kHcGroupsLog2 groups per partition (a half-full LDS table) from
  // the expected group count: the hint or the last run (both count every group), else the
  // records (all distinct).  Sizing by records alone gave ~1024 groups per partition for
  // near-unique keys, i.e. about half the partitions overflowed and the pass ran twice.
  uint64_t est = std::max<uint64_t>(last_groups, hint_groups > 0 ? static_cast<uint64_t>(hint_groups) : 0);
  if (est == 0 || est > n) est = n;
  int pbits = 1;
  while (pbits < 28 && (est >> (pbits + kHcGroupsLog2)) > 0) ++pbits;
  // ... and at most ~kHcMaxPartRecs records per partition: a workgroup's batches over a long
  // partition are latency-bound (tools/hc_pbits_ab.py, C3 without the filter, 100M records of
  // 6.4M groups: 14 bits by groups, 6100 records per partition -> 15 bits: hc_agg 3.78 -> 2.78 ms,
  // step 16.3 -> 15.5 ms; 16 bits measured slower again, 16.1 ms).  The filtered C3 (12M records)
  // keeps its 14 bits (13 / 15 / 16 bits: 3.46 / 3.36 / 3.84 ms against 3.11).
  while (pbits < 28 && (n >> pbits) > kHcMaxPartRecs) ++pbits;
  const char* fe = std::getenv("PXG_HC_PBITS");  // tests: the first pass's partition count
  const int forced = fe ? std::atoi(fe) : 0;
  if (forced > 0 && forced <= 28) pbits = forced;
  uint32_t G = 0;
  last_hc_reruns = 0;
  for (;;) {
    const uint32_t P = 1u << pbits;
    const int shift = 32 - pbits;
    const uint32_t* sk = nullptr;
    const uint64_t* srec = nullptr;
    PXG_RETURN_IF_ERROR(RadixSortBits(ctx, hc_key.as<const uint32_t>(), shift, pbits, streams, hp.stride, n, w.hc_k, w.hc_v, w.rs, &sk,
                                      &srec));
    PXG_RETURN_IF_ERROR(w.hc_starts.Ensure((static_cast<size_t>(P) + 1) * 4));
    {
      const int64_t waves = (static_cast<int64_t>(n) + 255) / 256;
      const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, static_cast<int64_t>(ctx->num_cus) * 8)));
      PXG_RETURN_IF_ERROR(Launch(ctx, "hc_part_starts", HcPartStartsKernel, dim3(grid), dim3(256), 0, sk, n, shift, P, w.hc_starts.as<uint32_t>()));
    }
    PXG_HIP(hipMemsetAsync(meta, 0, 8, ctx->stream));
    const uint32_t grid = std::min<uint32_t>(P, 1u << 16);
    PXG_RETURN_IF_ERROR(Launch(ctx, "hc_agg", HcAggFor(hp.kwords), dim3(grid), dim3(kHcBlock), lds, hp, srec, w.hc_starts.as<const uint32_t>(), P,
                               out, meta));
    PXG_HIP(hipMemcpyAsync(pin, meta, 8, hipMemcpyDeviceToHost, ctx->stream));
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    G = pin[0];
    if (pin[1] == 0) break;
    if (pbits >= 28) return SetError(PXG_INTERNAL, "high-cardinality partitions overflow their LDS tables at 2^28 partitions");
    pbits = std::min(28, pbits + 2);
    ++last_hc_reruns;
  }
  last_hc_pbits = pbits;
  if (ex) {
    ex->groups = G;
    ex->kscr = out.kscr;
    ex->plan = hp;
    return PXG_OK;
  }
  // String keys: lengths -> offsets (scan), then the bytes.  Payload bound: G groups of at most
  // kHcStrWords words per key (int32 Arrow offsets: < 2 GiB per column; bounding by the G groups
  // rather than the n records lets 100M records of 10M groups through).
  for (int k = 0; k < n_keys; ++k) {
    if (key_types[k] != PXG_STRING) continue;
    const uint64_t need = dbase[k] + static_cast<uint64_t>(G) * 8 * kHcStrWords;
    if (need >= (uint64_t(1) << 31)) return SetError(PXG_UNIMPLEMENTED, "string key column over 2 GiB");
    PXG_RETURN_IF_ERROR(R.key_data[k].Reserve(need + 16, dbase[k], ctx->stream));
  }
  bool any_str = false;
  HcKeyCopy kc;
  std::memset(&kc, 0, sizeof(kc));
  for (int k = 0; k < n_keys; ++k) {
    if (key_types[k] != PXG_STRING) continue;
    uint32_t* off = R.key_offsets[k].as<uint32_t>() + g0;
    if (G == 0) {
      // No partition groups (e.g. every staged key was long and took the table path): the
      // offsets end where the table path's bytes end.
      PXG_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(off), static_cast<int>(dbase[k]), 1, ctx->stream));
      continue;
    }
    any_str = true;
    PXG_RETURN_IF_ERROR(w.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(G) + 1) + 64));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, off, off, G, off + G, w.scan.p));
    kc.off[k] = off;
    kc.kw[k] = kwc[k];
    kc.data[k] = R.key_data[k].as<uint8_t>();
    kc.dbase[k] = static_cast<uint32_t>(dbase[k]);
  }
  uint32_t* pin32 = pin + 4;
  if (any_str && G > 0) {
    PXG_RETURN_IF_ERROR(Launch(ctx, "hc_key_copy", HcKeyCopyKernel, dim3(GridFor(static_cast<int64_t>(G) + 1, 256, 1 << 30)), dim3(256), 0,
                               static_cast<const uint64_t*>(out.kscr), hp.n, G, n_keys, kc, hp));
    for (int k = 0; k < n_keys; ++k)
      if (kc.off[k]) PXG_HIP(hipMemcpyAsync(pin32 + k, kc.off[k] + G, 4, hipMemcpyDeviceToHost, ctx->stream));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  for (int k = 0; k < n_keys; ++k)
    if (kc.off[k]) R.key_data_len[k] = G > 0 ? pin32[k] : static_cast<int64_t>(dbase[k]);
  R.n_groups = static_cast<int64_t>(g0) + G;
  R.ready = true;
  return PXG_OK;
}

// ---------------------------------------------------------------------------------------
// Spill: partition records -> table state (arena keys, slots, staging records), so export /
// import (which work on the table state) see every group.
// ---------------------------------------------------------------------------------------
// Pass 1: each live record's compact arena record (pxg_keys.h layout) in its fixed-size arena
// slot.  A separate launch from the inserts: a thread that meets another record's slot word reads
// that record's key bytes, which are only guaranteed visible (across XCDs, whose L2s are not
// coherent with relaxed atomics) after the kernel that wrote them has ended.
__global__ void __launch_bounds__(256) HcSpillArenaKernel(HcAggPlan hp, const uint64_t* __restrict__ rec, uint64_t rcap, uint64_t n,
                                                          int32_t rec_words, uint64_t abase, uint64_t* __restrict__ arena) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t lens = rec[i];
  if (lens == kHcHole) return;
  uint64_t* ar = arena + abase + i * static_cast<uint64_t>(rec_words);
  int wo = 0;
  for (int k = 0; k < hp.nk; ++k) {
    const int t = hp.ktype[k];
    const uint64_t* kw = rec + static_cast<uint64_t>(hp.koff[k]) * rcap + i;
    if (t == PXG_STRING) {
      const uint32_t len = static_cast<uint32_t>((lens >> (16 * k)) & 0xFFFF);
      ar[wo] = len;
      const int nw = static_cast<int>((len + 7) >> 3);
      for (int j = 0; j < nw; ++j) ar[wo + 1 + j] = kw[j * rcap];
      wo += 1 + nw;
    } else if (t == PXG_UINT128) {
      ar[wo] = kw[0];
      ar[wo + 1] = kw[rcap];
      wo += 2;
    } else {
      ar[wo] = kw[0];
      wo += 1;
    }
  }
}

// Pass 2: find-or-insert every live record's arena record, and its staging record.
__global__ void __launch_bounds__(256) HcSpillKernel(const AggPlanDev* __restrict__ plan, HcAggPlan hp, const uint64_t* __restrict__ rec,
                                                     uint64_t rcap, uint64_t n, int32_t rec_words, uint64_t abase, const uint64_t* __restrict__ arena,
                                                     unsigned long long* __restrict__ slots, uint32_t mask, uint32_t* __restrict__ st_slot,
                                                     StageDev stg, int nv, unsigned int* __restrict__ counters) {
  __shared__ unsigned int s_ins;
  if (threadIdx.x == 0) s_ins = 0;
  __syncthreads();
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t lens = i < n ? rec[i] : kHcHole;
  const bool live = lens != kHcHole;
  uint32_t slot = kDeferredSlot;
  if (live) {
    const uint64_t at = abase + i * static_cast<uint64_t>(rec_words);
    const uint64_t* ar = arena + at;
    KeySet mine;
    LoadKeysArena(plan, ar, mine);
    const uint64_t h = HashKeys(plan, mine);
    const uint32_t tag = SlotTag(h);
    const unsigned long long desired = MakeSlotWord(tag, kKindArena, static_cast<uint32_t>(at));
    uint32_t pos = static_cast<uint32_t>(h) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
      unsigned long long w = __hip_atomic_load(&slots[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0) {
        unsigned long long expected = 0;
        if (__hip_atomic_compare_exchange_strong(&slots[pos], &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          atomicAdd(&s_ins, 1u);
          slot = pos;
          break;
        }
        w = expected;
      }
      if (static_cast<uint32_t>(w >> 33) == tag) {
        KeySet other;
        LoadKeysArena(plan, arena + static_cast<uint32_t>(w), other);
        if (KeysEqual(plan, mine, other)) {
          slot = pos;
          break;
        }
      }
      pos = (pos + 1) & mask;
    }
    if (slot == kDeferredSlot) atomicOr(&counters[9], 1u);  // table full: cannot happen at <= 25% fill
  }
  // Staging records of the live rows, compacted per wave (one cursor atomic per wave).
  const int lane = threadIdx.x & 63;
  const unsigned long long m = __ballot(live);
  if (m) {
    const int leader = __ffsll(static_cast<long long>(m)) - 1;
    unsigned long long b = 0;
    if (lane == leader) b = atomicAdd(stg.cursor, static_cast<unsigned long long>(__popcll(m)));
    b = __shfl(b, leader, 64);
    if (live) {
      const uint64_t sp = b + __popcll(m & ((1ULL << lane) - 1));
      st_slot[sp] = slot;
      for (int v = 0; v < nv; ++v) stg.vals[v][sp] = rec[static_cast<uint64_t>(hp.kwords + v) * rcap + i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_ins) atomicAdd(&counters[0], s_ins);
}

static uint32_t HcNextPow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return static_cast<uint32_t>(std::min<uint64_t>(p, uint64_t(1) << 31));
}

int32_t Agg::SpillHc() {
  if (!hc_active) return PXG_OK;
  hc_active = false;
  const uint64_t n = hc_n;
  hc_n = 0;
  if (n == 0) return PXG_OK;
  const HcAggPlan hp = MakeHcPlan(*this);
  int32_t rec_words = 0;
  for (int k = 0; k < n_keys; ++k) rec_words += key_types[k] == PXG_STRING ? 1 + kHcStrWords : hc_layout.kw[k];
  const uint64_t abase = arena_words;
  if (abase + n * rec_words >= (uint64_t(1) << 32)) return SetError(PXG_RESOURCE_UNAVAILABLE, "key arena exceeds 32 GiB");
  PXG_RETURN_IF_ERROR(arena.Reserve((abase + n * rec_words) * 8 + kArenaSlack, abase * 8, ctx->stream));
  const uint64_t want = 4 * (inserted + n);
  if (want > (uint64_t(1) << 31)) return SetError(PXG_RESOURCE_UNAVAILABLE, "group table would exceed 2^31 slots");
  if (want > cap) PXG_RETURN_IF_ERROR(Grow(HcNextPow2(want)));
  PXG_RETURN_IF_ERROR(EnsureStage(st_n + n));
  uint8_t* cb = counters.as<uint8_t>();
  PXG_HIP(hipMemsetAsync(cb + 36, 0, 4, ctx->stream));
  PXG_HIP(hipMemsetAsync(cb + 48, 0, 8, ctx->stream));  // the record cursor, mirrored into hc_n by PublishNew
  StageDev stg;
  std::memset(&stg, 0, sizeof(stg));
  for (int v = 0; v < n_vals; ++v) stg.vals[v] = st_val[v].as<uint64_t>();
  stg.cursor = reinterpret_cast<unsigned long long*>(cb + 16);
  const dim3 grid(GridFor(static_cast<int64_t>(n), 256, 1 << 30));
  PXG_RETURN_IF_ERROR(Launch(ctx, "hc_spill_arena", HcSpillArenaKernel, grid, dim3(256), 0, hp, hc_rec.as<const uint64_t>(), hc_cap, n,
                             rec_words, abase, arena.as<uint64_t>()));
  PXG_RETURN_IF_ERROR(Launch(ctx, "hc_spill", HcSpillKernel, grid, dim3(256), 0,
                             d_plan.as<const AggPlanDev>(), hp, hc_rec.as<const uint64_t>(), hc_cap, n, rec_words, abase,
                             arena.as<const uint64_t>(), slots.as<unsigned long long>(), cap - 1,
                             st_slot.as<uint32_t>(), stg, n_vals, counters.as<unsigned int>()));
  arena_words = abase + n * rec_words;
  uint8_t* pin = static_cast<uint8_t*>(ctx->pinned) + 224;
  PXG_HIP(hipMemcpyAsync(pin, cb, 40, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  uint32_t groups = 0, err = 0;
  std::memcpy(&groups, pin, 4);
  std::memcpy(&err, pin + 36, 4);
  std::memcpy(&st_n, pin + 16, 8);
  if (err) return SetError(PXG_INTERNAL, "group table full while spilling partition records");
  inserted = groups;
  state_version++;
  return PXG_OK;
}

// Export of a high-cardinality run without the spill: the partition groups are aggregated as in
// FinalizeHc (states instead of results), and each group's key record is rebuilt from the key
// scratch into the arena past its live words; eslots[g_table + l] names it (arena word offset,
// as a table slot word would).  The export then treats table groups and partition groups alike.
__global__ void __launch_bounds__(256) HcGroupArenaKernel(HcAggPlan hp, const uint64_t* __restrict__ kscr, uint32_t G, int32_t rec_words,
                                                          uint64_t abase, uint64_t* __restrict__ arena, unsigned long long* __restrict__ eslots) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= G) return;
  const uint64_t n = hp.n;
  const uint64_t lens = kscr[l];
  const uint64_t at = abase + static_cast<uint64_t>(l) * rec_words;
  uint64_t* ar = arena + at;
  int wo = 0;
  for (int k = 0; k < hp.nk; ++k) {
    const int t = hp.ktype[k];
    const uint64_t* kw = kscr + static_cast<uint64_t>(hp.koff[k]) * n + l;
    if (t == PXG_STRING) {
      const uint32_t len = static_cast<uint32_t>((lens >> (16 * k)) & 0xFFFF);
      ar[wo] = len;
      const int nw = static_cast<int>((len + 7) >> 3);
      for (int j = 0; j < nw; ++j) ar[wo + 1 + j] = (k == 0 && hp.tail0 && j == 2) ? (lens >> 32) : kw[j * n];
      wo += 1 + nw;
    } else if (t == PXG_UINT128) {
      ar[wo] = kw[0];
      ar[wo + 1] = kw[n];
      wo += 2;
    } else {
      ar[wo] = kw[0];
      wo += 1;
    }
  }
  eslots[l] = at;
}

int32_t Agg::ExportHcGroups(uint32_t g_table, DevBuf* states, DevBuf* eslots, uint32_t* n_hc, uint64_t* key_words) {
  *n_hc = 0;
  *key_words = 0;
  if (!hc_active || hc_n == 0) return PXG_OK;
  const uint64_t srec = static_cast<uint64_t>(hplan_x.state_rec);
  PXG_RETURN_IF_ERROR(states->Reserve((static_cast<uint64_t>(g_table) + hc_n) * srec + 16, static_cast<uint64_t>(g_table) * srec, ctx->stream));
  HcExport ex;
  ex.states = states->as<uint8_t>() + static_cast<uint64_t>(g_table) * srec;
  PXG_RETURN_IF_ERROR(FinalizeHc(&ex));
  const uint32_t G = ex.groups;
  if (G == 0) return PXG_OK;
  int32_t rec_words = 0;
  for (int k = 0; k < n_keys; ++k) rec_words += key_types[k] == PXG_STRING ? 1 + kHcStrWords : hc_layout.kw[k];
  const uint64_t abase = arena_words;
  if (abase + static_cast<uint64_t>(G) * rec_words >= (uint64_t(1) << 32)) return SetError(PXG_RESOURCE_UNAVAILABLE, "key arena exceeds 32 GiB");
  // Scratch past the live words: arena_words is not advanced (the records serve this export only).
  PXG_RETURN_IF_ERROR(arena.Reserve((abase + static_cast<uint64_t>(G) * rec_words) * 8 + kArenaSlack, abase * 8, ctx->stream));
  PXG_RETURN_IF_ERROR(eslots->Reserve((static_cast<uint64_t>(g_table) + G) * 8 + 16, static_cast<uint64_t>(g_table) * 8, ctx->stream));
  PXG_RETURN_IF_ERROR(Launch(ctx, "hc_export_keys", HcGroupArenaKernel, dim3(GridFor(G, 256, 1 << 30)), dim3(256), 0, ex.plan, ex.kscr, G, rec_words,
                             abase, arena.as<uint64_t>(), eslots->as<unsigned long long>() + g_table));
  *n_hc = G;
  *key_words = static_cast<uint64_t>(G) * rec_words;
  return PXG_OK;
}

int32_t AggFinalizeImpl(Agg* a) {
  if (a->merged) return a->FinalizeMerged();  // imported partial states (pxg_partial.hip)
  PXG_RETURN_IF_ERROR(AggFinalizeTable(a));  // the table path (high-cardinality mode: rows with long keys)
  if (!a->hc_active) return PXG_OK;
  return a->FinalizeHc();
}

}  // namespace pxg
