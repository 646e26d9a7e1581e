// Fused Filter -> Map -> BlockingAgg consume path, key arena publication and table growth.
//
// Reference loops replaced: filter predicate (filter_node.cc:135-153),
// compaction (filter_node.cc:78-130), map UDF row loop (udf_wrapper.h:102-133), group-key
// extraction + hash probe (agg_node.cc:209-271) and the per-row UDA value buffering
// (agg_node.cc:258-268).  One launch streams every row of the table once.
#include <algorithm>
#include <cstdlib>

#include "pxg_agg_host.h"
#include "pxg_keys.h"
#include "pxg_program.h"
#include "pxg_scan.h"

namespace pxg {

constexpr int kConsumeBlock = 256;
constexpr int kGenericTile = 4096;   // rows per workgroup tile of the generic kernel (16 per thread)
// Rows per workgroup tile of the fast kernel: 16384, or 32768 when the launch has enough
// tiles for >= 8 rounds of resident workgroups (fewer phase-2 barriers per row; at 100M rows the
// larger tiles lose more to the last round's imbalance than they gain: 1.42 -> 1.79 ms at
// 32768, while 1B rows go 13.16 -> 12.93 ms; 65536 tiles: 13.59 ms).  Row offsets within a tile
// are u16 in LDS.
constexpr int kConsumeTile = 16384;
constexpr int kConsumeTileMax = 32768;
constexpr int kSelCap = 16384;       // selected rows collected before phase 2 runs (LDS)
// (The fast kernel runs 4 waves per SIMD, limited by both LDS (34.9 KB per workgroup) and
// VGPRs (~125).  Forcing 5 -- a 12288-row selection buffer and amdgpu_waves_per_eu(5) --
// spilled 32-93 VGPRs to scratch: C2 consume 1.30 -> 2.09 ms.)
constexpr int kSubRows = 8192;       // rows per phase-1 sub-batch (32 per thread in flight)

struct TileRange {
  int64_t tile0;  // first tile index of this range
  int64_t lo;     // local row range within the chunk
  int64_t hi;
  int32_t chunk;
  int32_t tile_rows;  // rows per tile (fast kernel; the generic kernel uses kGenericTile)
};

constexpr uint32_t kMaxProbe = 256;  // longer probe sequences defer the row (table grows)

// Probe for the row's group; insert it (CAS of an empty slot word) when absent.  Inserts are
// counted in the workgroup's LDS counter (`s_ins`) and flushed once per tile, so no per-row
// atomic ever targets a shared global address.  The table fill check reads the flushed global
// count: it is a soft guard that keeps probe sequences short; a full or overlong probe defers.
__device__ __forceinline__ uint32_t FindOrInsert(const AggPlanDev* __restrict__ plan, const DevChunk* __restrict__ chunks,
                                                 const KeySet& keys, uint64_t h, uint32_t rowref, const AggTableDev& tab,
                                                 unsigned int* s_ins) {
  const uint32_t tag = SlotTag(h);
  uint32_t pos = static_cast<uint32_t>(h) & tab.mask;
  const uint32_t max_probe = min(tab.mask + 1, kMaxProbe);
  for (uint32_t probe = 0; probe < max_probe; ++probe) {
    unsigned long long w = __hip_atomic_load(&tab.slots[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == 0) {
      const unsigned int ins = __hip_atomic_load(&tab.counters[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + *s_ins;
      if (ins >= tab.limit) return kDeferredSlot;
      unsigned long long expected = 0;
      const unsigned long long desired = MakeSlotWord(tag, 0, rowref);
      if (__hip_atomic_compare_exchange_strong(&tab.slots[pos], &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        atomicAdd(s_ins, 1u);
        return pos;
      }
      w = expected;
    }
    if (static_cast<uint32_t>(w >> 33) == tag) {
      KeySet rep;
      const uint32_t ref = static_cast<uint32_t>(w);
      if (w & kKindArena) {
        LoadKeysArena(plan, tab.arena + ref, rep);
      } else {
        LoadKeysRow(plan, chunks[ref >> kChunkShift], static_cast<int64_t>(ref & (kChunkRows - 1)), rep);
      }
      if (KeysEqual(plan, keys, rep)) return pos;
    }
    pos = (pos + 1) & tab.mask;
  }
  return kDeferredSlot;
}

__device__ __forceinline__ void ProcessRow(const AggPlanDev* __restrict__ plan, const DevChunk* __restrict__ chunks,
                                           const DevChunk& ch, uint32_t chunk_idx, int64_t local, const AggTableDev& tab,
                                           const StageDev& stg, uint64_t pos, unsigned int* s_ins) {
  KeySet k;
  LoadKeysRow(plan, ch, local, k);
  const uint64_t h = HashKeys(plan, k);
  const uint32_t rowref = (chunk_idx << kChunkShift) | static_cast<uint32_t>(local);
  const uint32_t slot = FindOrInsert(plan, chunks, k, h, rowref, tab, s_ins);
  // Deferred rows: one list append per wave (ballot + leader atomic).
  const unsigned long long dm = __ballot(slot == kDeferredSlot);
  if (dm) {
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll(static_cast<long long>(dm)) - 1;
    unsigned int base = 0;
    if (lane == leader) base = atomicAdd(&tab.counters[2], static_cast<unsigned int>(__popcll(dm)));
    base = __shfl(base, leader, 64);
    if (slot == kDeferredSlot) {
      const unsigned int at = base + __popcll(dm & ((1ULL << lane) - 1));
      tab.deferred[at] = rowref;
      tab.deferred_pos[at] = static_cast<uint32_t>(pos);
    }
  }
  stg.slot[pos] = slot;
  const int nv = plan->n_vals;
  for (int v = 0; v < nv; ++v) {
    uint64_t x;
    if (plan->val_kind[v] == kValMinOf2) {
      const int64_t a = static_cast<int64_t>(EvalProgram(&plan->vals[v], ch, local, plan->col_types).a);
      const int64_t b = static_cast<int64_t>(EvalProgram(&plan->vals2[v], ch, local, plan->col_types).a);
      x = static_cast<uint64_t>(a < b ? a : b);
    } else {
      x = EvalProgram(&plan->vals[v], ch, local, plan->col_types).a;
    }
    stg.vals[v][pos] = x;
  }
}

// One workgroup per tile of 4096 rows (grid-stride).  Phase 1 evaluates the predicate for all
// 16 rows of each thread first (16 independent loads in flight), then compacts the passing
// rows into LDS: per-wave ballots, one LDS prefix over the 4 waves; phase 2 processes the
// compacted rows densely and appends one staging record per row (one cursor atomic per tile).
__global__ void __launch_bounds__(kConsumeBlock) AggConsumeKernel(const AggPlanDev* __restrict__ plan,
                                                                  const DevChunk* __restrict__ chunks,
                                                                  const TileRange* __restrict__ ranges, int nranges,
                                                                  int64_t ntiles, AggTableDev tab, StageDev stg,
                                                                  uint32_t /*nchunks: signature shared with the fast path*/) {
  constexpr int kPer = kGenericTile / kConsumeBlock;
  constexpr int kWaves = kConsumeBlock / 64;
  __shared__ int32_t s_sel[kGenericTile];
  __shared__ uint32_t s_wcnt[kWaves];
  __shared__ unsigned int s_ins;
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  const uint32_t bid = XcdRemap(blockIdx.x, gridDim.x);
  if (threadIdx.x == 0) s_ins = 0;
  for (int64_t t = bid; t < ntiles; t += gridDim.x) {
    int ri = 0;
    while (ri + 1 < nranges && ranges[ri + 1].tile0 <= t) ++ri;
    const TileRange rg = ranges[ri];
    const DevChunk& ch = chunks[rg.chunk];
    const int64_t row0 = rg.lo + (t - rg.tile0) * kGenericTile;
    const int64_t row1 = min(row0 + kGenericTile, rg.hi);
    // Rows of this thread: row0 + k*256 + tid (coalesced per k).
    bool pass[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int64_t r = row0 + k * kConsumeBlock + threadIdx.x;
      pass[k] = r < row1;
      if (pass[k] && plan->has_filter) pass[k] = EvalProgram(&plan->filter, ch, r, plan->col_types).a != 0;
    }
    unsigned long long m[kPer];
    uint32_t wtot = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      m[k] = __ballot(pass[k]);
      wtot += static_cast<uint32_t>(__popcll(m[k]));
    }
    if (lane == 0) s_wcnt[wid] = wtot;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t c = s_wcnt[w];
      wbase += w < wid ? c : 0;
      total += c;
    }
    // Flush the previous tile's insert count and reserve this tile's staging range.
    if (threadIdx.x == 0) {
      if (s_ins) {
        atomicAdd(&tab.counters[0], s_ins);
        s_ins = 0;
      }
      s_base = total ? atomicAdd(stg.cursor, static_cast<unsigned long long>(total)) : 0ULL;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (pass[k]) s_sel[wbase + __popcll(m[k] & lanemask_lt)] = k * kConsumeBlock + threadIdx.x;
      wbase += static_cast<uint32_t>(__popcll(m[k]));
    }
    __syncthreads();
    const uint64_t base = s_base;
    for (uint32_t i = threadIdx.x; i < total; i += kConsumeBlock)
      ProcessRow(plan, chunks, ch, static_cast<uint32_t>(rg.chunk), row0 + s_sel[i], tab, stg, base + i, &s_ins);
    __syncthreads();
  }
  if (threadIdx.x == 0 && s_ins) atomicAdd(&tab.counters[0], s_ins);
}

// Re-process deferred rows (already past the filter) after the table grew.  Each row fills in
// the slot of the staging record it already has (its values were staged with it), so a
// deferral never adds records: the staging holds exactly one record per selected row.
__global__ void __launch_bounds__(kConsumeBlock) AggConsumeListKernel(const AggPlanDev* __restrict__ plan,
                                                                      const DevChunk* __restrict__ chunks,
                                                                      const uint32_t* __restrict__ list,
                                                                      const uint32_t* __restrict__ list_pos, uint32_t n,
                                                                      AggTableDev tab, StageDev stg) {
  __shared__ unsigned int s_ins;
  if (threadIdx.x == 0) s_ins = 0;
  for (uint32_t t0 = blockIdx.x * kConsumeBlock; t0 < n; t0 += gridDim.x * kConsumeBlock) {
    if (threadIdx.x == 0 && s_ins) {
      atomicAdd(&tab.counters[0], s_ins);
      s_ins = 0;
    }
    __syncthreads();
    const uint32_t i = t0 + threadIdx.x;
    if (i < n) {
      const uint32_t ref = list[i];
      const uint32_t c = ref >> kChunkShift;
      ProcessRow(plan, chunks, chunks[c], c, static_cast<int64_t>(ref & (kChunkRows - 1)), tab, stg, list_pos[i], &s_ins);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && s_ins) atomicAdd(&tab.counters[0], s_ins);
}

// ---------------------------------------------------------------------------------------
// Fast path: every group key is a bare column, the filter and every value stream are one of
// the two fast shapes.  Keys live in registers as realigned, tail-masked 8-byte words, so a
// string key costs two memory round trips (offsets, then every payload word at once) instead
// of one per word, and equality against the group's representative key is word compares of
// registers.  No interpreter stack, so no scratch and a small register budget.  The hash is
// bit-identical to HashKeys (rehash, import and the generic kernel share the table).
// Rows with a string key longer than kFastStrWords words are deferred to the generic kernel.
// ---------------------------------------------------------------------------------------
constexpr int kFastStrWords = 6;

template <int NK>
struct FastKeys {
  uint64_t w[NK][kFastStrWords];  // STRING: payload words; fixed: w[0] (UINT128: w[0], w[1])
  uint32_t len[NK];               // STRING byte length (0 for fixed types)
};

// Payload words of a string of len <= 8 * kFastStrWords bytes at p, tail-masked.  The bytes
// are fetched with 16-byte loads straight from the (unaligned) string start: gfx950 serves
// unaligned global loads in hardware, so no realignment shifts are needed (<= 3 loads; every
// load of a divergent wave costs address-processing time per lane).  Payload buffers carry a
// 16-byte pad, so the over-read of the last load stays in bounds.
constexpr int kFast16 = kFastStrWords / 2;
__device__ __forceinline__ void LoadStrWords(const uint8_t* p, uint32_t len, uint64_t* w) {
  const uint32_t n16 = (len + 15) >> 4;
#pragma unroll
  for (int i = 0; i < kFast16; ++i) {
    ulonglong2 v = make_ulonglong2(0, 0);
    if (static_cast<uint32_t>(i) < n16) __builtin_memcpy(&v, p + 16 * i, 16);
    w[2 * i] = v.x;
    w[2 * i + 1] = v.y;
  }
#pragma unroll
  for (int j = 0; j < kFastStrWords; ++j) {
    const int rem = static_cast<int>(len) - 8 * j;
    w[j] = rem >= 8 ? w[j] : (rem > 0 ? (w[j] & ((1ULL << (rem * 8)) - 1)) : 0);
  }
}

// offsets[r] and offsets[r + 1] with one 12-byte load from the 8-byte aligned pair start.
__device__ __forceinline__ void LoadOffsetPair(const int32_t* __restrict__ offs, int64_t r, int32_t* o0, int32_t* o1) {
  struct __attribute__((packed, aligned(4))) I3 { int32_t a, b, c; };
  const I3 v = *reinterpret_cast<const I3*>(offs + (r & ~int64_t(1)));
  const bool odd = (r & 1) != 0;
  *o0 = odd ? v.b : v.a;
  *o1 = odd ? v.c : v.b;
}

// First round trip of a row's keys: the offset pair of every STRING key (start, length) and the
// value of every fixed-width key.  Phase 2 issues it one row ahead, so it overlaps the previous
// row's probe instead of heading each row's dependent load chain.
// Key type i of the plan; S: the kernel is specialised for plans whose keys are all STRING (C2,
// C3's (pod, remote_addr)), which drops the fixed-width branches and their registers.
template <bool S>
__device__ __forceinline__ int KeyT(const AggPlanDev* __restrict__ plan, int i) {
  return S ? static_cast<int>(PXG_STRING) : plan->key_types[i];
}

template <int NK>
struct KeyHeads {
  int32_t o0[NK];
  uint32_t len[NK];
  uint64_t a[NK], b[NK];
};

template <int NK, bool S = false>
__device__ __forceinline__ void LoadKeyHeads(const AggPlanDev* __restrict__ plan, const DevChunk& ch, int64_t r, KeyHeads<NK>& h) {
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    const int t = KeyT<S>(plan, i);
    const DevCol& col = ch.cols[plan->keys[i].col];
    if (t == PXG_STRING) {
      int32_t o0, o1;
      LoadOffsetPair(col.offsets, r, &o0, &o1);
      h.o0[i] = o0;
      h.len[i] = static_cast<uint32_t>(o1 - o0);
      h.a[i] = h.b[i] = 0;
    } else {
      h.o0[i] = 0;
      const Val v = LoadCol(col, t, r);
      // A computed fixed-width key (kShapeColOpConst over an 8-byte integer column, e.g.
      // bin(time_, 10 s) = t - t % b, math_ops.h:512-527) is applied to the loaded value.
      h.a[i] = plan->keys[i].shape == kShapeCol ? v.a : ApplyShape(&plan->keys[i], v.a);
      h.b[i] = v.b;
      h.len[i] = 0;
    }
  }
}

// Second round trip: the string payload words.  Returns false when a string key is too long for
// the register path.
template <int NK, bool S = false>
__device__ __forceinline__ bool LoadKeyBodies(const AggPlanDev* __restrict__ plan, const DevChunk& ch, const KeyHeads<NK>& h,
                                              FastKeys<NK>& k) {
  const uint8_t* ptr[NK];
  bool ok = true;
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    k.len[i] = h.len[i];
    if (KeyT<S>(plan, i) == PXG_STRING) {
      ptr[i] = ch.cols[plan->keys[i].col].data + h.o0[i];
      ok = ok && h.len[i] <= 8u * kFastStrWords;
    } else {
      k.w[i][0] = h.a[i];
      k.w[i][1] = h.b[i];
    }
  }
  if (!ok) return false;
#pragma unroll
  for (int i = 0; i < NK; ++i)
    if (KeyT<S>(plan, i) == PXG_STRING) LoadStrWords(ptr[i], k.len[i], k.w[i]);
  return true;
}

template <int NK, bool S = false>
__device__ __forceinline__ uint64_t HashFastKeys(const AggPlanDev* __restrict__ plan, const FastKeys<NK>& k) {
  uint64_t h = 0x243F6A8885A308D3ULL;
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    const int t = KeyT<S>(plan, i);
    uint64_t hk;
    if (t == PXG_STRING) {
      uint64_t s = 0x13198A2E03707344ULL;
#pragma unroll
      for (int j = 0; j < kFastStrWords; ++j) {
        if (8u * j < k.len[i]) {
          s = (s ^ k.w[i][j]) * 0x9E3779B97F4A7C15ULL;
          s ^= s >> 29;
        }
      }
      hk = Fmix64(s ^ (static_cast<uint64_t>(k.len[i]) * 0xC2B2AE3D27D4EB4FULL));
    } else if (t == PXG_UINT128) {
      hk = Fmix64(k.w[i][0] ^ Fmix64(k.w[i][1] + 0xA4093822299F31D0ULL));
    } else {
      hk = Fmix64(k.w[i][0] + 0x082EFA98EC4E6C89ULL);
    }
    h = Fmix64(h * 0x9E3779B97F4A7C15ULL + hk);
  }
  return h;
}

template <int NK, bool S = false>
__device__ __forceinline__ bool FastKeysEqual(const AggPlanDev* __restrict__ plan, const FastKeys<NK>& x, const FastKeys<NK>& y) {
  bool eq = true;
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    const int t = KeyT<S>(plan, i);
    if (t == PXG_STRING) {
      eq = eq && x.len[i] == y.len[i];
#pragma unroll
      for (int j = 0; j < kFastStrWords; ++j) eq = eq && x.w[i][j] == y.w[i][j];
    } else {
      eq = eq && x.w[i][0] == y.w[i][0] && (t != PXG_UINT128 || x.w[i][1] == y.w[i][1]);
    }
  }
  return eq;
}

// Equality against an arena key record (pxg_keys.h layout).  The record's word offsets are
// taken from the probing key's own lengths (a record with different lengths is unequal
// anyway), so every word is requested at once; the over-read stays inside kArenaSlack.
template <int NK, bool S = false>
__device__ __forceinline__ bool FastKeysEqualArena(const AggPlanDev* __restrict__ plan, const FastKeys<NK>& x,
                                                   const uint64_t* __restrict__ rec) {
  bool eq = true;
  int w = 0;
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    const int t = KeyT<S>(plan, i);
    if (t == PXG_STRING) {
      eq = eq && rec[w] == x.len[i];
      const int nw = static_cast<int>((x.len[i] + 7) >> 3);
#pragma unroll
      for (int j = 0; j < kFastStrWords; ++j)
        if (j < nw) eq = eq && rec[w + 1 + j] == x.w[i][j];
      w += 1 + nw;
    } else if (t == PXG_UINT128) {
      eq = eq && rec[w] == x.w[i][0] && rec[w + 1] == x.w[i][1];
      w += 2;
    } else {
      eq = eq && rec[w] == x.w[i][0];
      w += 1;
    }
  }
  return eq;
}

// Key-column base pointers of one chunk.  The consume kernel keeps them in LDS for the first
// kLdsChunks chunks, so comparing against a group's representative row does not first fetch
// the row's chunk descriptor from global memory (one dependent round trip less per probe).
constexpr int kLdsChunks = 64;
template <int NK>
struct KeyCols {
  const int32_t* off[NK];  // STRING offsets
  const uint8_t* dat[NK];  // STRING payload, or the values of a fixed-width key
};

template <int NK, bool S = false>
__device__ __forceinline__ KeyCols<NK> KeyColsOf(const AggPlanDev* __restrict__ plan, const DevChunk& ch) {
  KeyCols<NK> kc;
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    const DevCol& col = ch.cols[plan->keys[i].col];
    kc.off[i] = col.offsets;
    kc.dat[i] = KeyT<S>(plan, i) == PXG_STRING ? col.data : col.values;
  }
  return kc;
}

// Equality against the keys of row r (a group's representative row), compared word by word
// as the row's payload words arrive; nothing of the row's key is kept in registers.
template <int NK, bool S = false>
__device__ __forceinline__ bool FastKeysEqualRow(const AggPlanDev* __restrict__ plan, const KeyCols<NK>& kc, int64_t r,
                                                 const FastKeys<NK>& x) {
  bool eq = true;
  const uint8_t* ptr[NK];
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    const int t = KeyT<S>(plan, i);
    if (t == PXG_STRING) {
      int32_t o0, o1;
      LoadOffsetPair(kc.off[i], r, &o0, &o1);
      ptr[i] = kc.dat[i] + o0;
      eq = eq && static_cast<uint32_t>(o1 - o0) == x.len[i];
    } else {
      DevCol c;
      c.values = kc.dat[i];
      c.offsets = nullptr;
      c.data = nullptr;
      const Val v = LoadCol(c, t, r);
      const uint64_t a = plan->keys[i].shape == kShapeCol ? v.a : ApplyShape(&plan->keys[i], v.a);
      eq = eq && a == x.w[i][0] && (t != PXG_UINT128 || v.b == x.w[i][1]);
    }
  }
  if (!eq) return false;
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    if (KeyT<S>(plan, i) != PXG_STRING) continue;
    uint64_t w[kFastStrWords];
    LoadStrWords(ptr[i], x.len[i], w);
#pragma unroll
    for (int j = 0; j < kFastStrWords; ++j) eq = eq && w[j] == x.w[i][j];
  }
  return eq;
}

// Key compare against the probe record at the probed position (pxg_agg.h): 1 equal, 0 not,
// -1 when the record does not hold this slot word (never published: imported / spilled groups).
// One 16-byte load for the header and one per chunk of used key words, all issued at once and
// all in the record's 128-byte line; unused words are zero on both sides, so whole chunks compare.
template <int NK>
__device__ __forceinline__ int RecordEqual(const uint64_t* __restrict__ rec, unsigned long long w, const FastKeys<NK>& k) {
  static_assert(NK <= kRecMaxKeys && 2 + NK * kRecKeyWords <= kRecWords, "record layout");
  constexpr int kChunks = (2 + NK * kRecKeyWords + 1) / 2;
  const ulonglong2* r2 = reinterpret_cast<const ulonglong2*>(rec);
  uint32_t nw[NK];
#pragma unroll
  for (int i = 0; i < NK; ++i) nw[i] = (k.len[i] + 7) >> 3;
  uint64_t c[2 * kChunks];
#pragma unroll
  for (int ci = 0; ci < kChunks; ++ci) {
    bool need = ci == 0;
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int lo = 2 + kRecKeyWords * i;
      need = need || (2 * ci + 1 >= lo && 2 * ci < lo + static_cast<int>(nw[i]));
    }
    ulonglong2 v = make_ulonglong2(0, 0);
    if (need) v = r2[ci];
    c[2 * ci] = v.x;
    c[2 * ci + 1] = v.y;
  }
  if (c[0] != w) return -1;
  uint64_t lens = 0;
#pragma unroll
  for (int i = 0; i < NK; ++i) lens |= static_cast<uint64_t>(k.len[i]) << (16 * i);
  bool eq = c[1] == lens;
#pragma unroll
  for (int i = 0; i < NK; ++i)
#pragma unroll
    for (int j = 0; j < kRecKeyWords; ++j) eq = eq && c[2 + kRecKeyWords * i + j] == k.w[i][j];
  return eq ? 1 : 0;
}

// In-launch probe record of a group whose slot still holds its row word (RROW consumes): written
// by the inserting lane and by a lane that confirmed the group against its representative row,
// from the key in its registers.  Words 1..15 first, then (after their stores are acknowledged)
// word 0 = the slot word, so a line that shows the slot word already holds the key; a reader
// that sees a stale line (its L1 / L2 copy from before, or another XCD's copy not written back
// yet) sees word 0 != the slot word and compares against the representative row instead.  Only
// a record that EQUALS the probe key is trusted (a record is never taken as proof of inequality
// in-launch), so a line caught mid-write can cost a slow compare but never a wrong group.
template <int NK>
__device__ __forceinline__ void WriteRowRecord(uint64_t* __restrict__ rec, unsigned long long w, const FastKeys<NK>& k) {
  uint64_t lens = 0;
#pragma unroll
  for (int i = 0; i < NK; ++i) lens |= static_cast<uint64_t>(k.len[i]) << (16 * i);
  uint64_t r[kRecWords];
#pragma unroll
  for (int t = 0; t < kRecWords; ++t) r[t] = 0;
#pragma unroll
  for (int i = 0; i < NK; ++i)
#pragma unroll
    for (int j = 0; j < kRecKeyWords; ++j) r[2 + kRecKeyWords * i + j] = k.w[i][j];
  rec[1] = lens;
  ulonglong2* d = reinterpret_cast<ulonglong2*>(rec);
#pragma unroll
  for (int t = 1; t < kRecWords / 2; ++t) d[t] = make_ulonglong2(r[2 * t], r[2 * t + 1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  rec[0] = w;
}

// TAGONLY: timing-only diagnostic (PXG_DIAG_CONSUME=1): a tag match is taken as the group without
// the representative compare, which prices that compare (tools/consume_diag.py; wrong groups on
// a tag collision, never followed by a checked finalize).
template <int NK, bool S = false, bool TAGONLY = false, bool REC = false, bool RROW = false>
__device__ __forceinline__ uint32_t FastFindOrInsert(const AggPlanDev* __restrict__ plan, const DevChunk* __restrict__ chunks,
                                                     const KeyCols<NK>* __restrict__ s_kc, uint32_t n_lds_chunks,
                                                     const FastKeys<NK>& keys, uint64_t h, uint32_t rowref,
                                                     const AggTableDev& tab, unsigned int* s_ins) {
  const uint32_t tag = SlotTag(h);
  uint32_t pos = static_cast<uint32_t>(h) & tab.mask;
  const uint32_t max_probe = min(tab.mask + 1, kMaxProbe);
  uint32_t probe = 0;
  while (probe < max_probe) {
    // Phase A: walk slot words only, to the first empty slot or tag match.  Lanes of a wave
    // leave this cheap loop at different probe lengths but meet again for phase B, so the
    // (expensive) key comparison runs once per wave in the common case instead of once per
    // probe step.  Plain (cacheable) loads: within a launch a slot word only ever changes
    // 0 -> final value (by CAS), so a non-zero word is final and a stale 0 costs only the CAS.
    unsigned long long w = tab.slots[pos];
    while (w != 0 && static_cast<uint32_t>(w >> 33) != tag) {
      if (++probe >= max_probe) return kDeferredSlot;
      pos = (pos + 1) & tab.mask;
      w = tab.slots[pos];
    }
    if (w == 0) {
      const unsigned int ins = __hip_atomic_load(&tab.counters[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + *s_ins;
      if (ins >= tab.limit) return kDeferredSlot;
      unsigned long long expected = 0;
      const unsigned long long desired = MakeSlotWord(tag, 0, rowref);
      if (__hip_atomic_compare_exchange_strong(&tab.slots[pos], &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        atomicAdd(s_ins, 1u);
        if constexpr (RROW) WriteRowRecord<NK>(tab.prec + static_cast<uint64_t>(pos) * kRecWords, desired, keys);
        return pos;
      }
      w = expected;  // lost the race: the winner's word decides below
    }
    // Phase B: exact key comparison against the slot's representative.
    if (TAGONLY && static_cast<uint32_t>(w >> 33) == tag) return pos;
    if (static_cast<uint32_t>(w >> 33) == tag) {
      const uint32_t ref = static_cast<uint32_t>(w);
      bool eq;
      if (w & kKindArena) {
        int r = -1;
        if constexpr (REC) r = RecordEqual<NK>(tab.prec + static_cast<uint64_t>(pos) * kRecWords, w, keys);
        eq = r >= 0 ? r == 1 : FastKeysEqualArena<NK, S>(plan, keys, tab.arena + ref);
      } else {
        int r = -1;
        if constexpr (RROW) r = RecordEqual<NK>(tab.prec + static_cast<uint64_t>(pos) * kRecWords, w, keys);
        if (r == 1) {
          eq = true;  // the in-launch record equals this key (see WriteRowRecord)
        } else {
          const uint32_t c = ref >> kChunkShift;
          const KeyCols<NK> kc = c < n_lds_chunks ? s_kc[c] : KeyColsOf<NK, S>(plan, chunks[c]);
          eq = FastKeysEqualRow<NK, S>(plan, kc, static_cast<int64_t>(ref & (kChunkRows - 1)), keys);
          if constexpr (RROW)
            if (eq && r < 0) WriteRowRecord<NK>(tab.prec + static_cast<uint64_t>(pos) * kRecWords, w, keys);
        }
      }
      if (eq) return pos;
    }
    ++probe;
    pos = (pos + 1) & tab.mask;
  }
  return kDeferredSlot;
}

// MODE: 0 = production; 1 / 2 / 3 are timing-only diagnostic builds: 1 probes without the
// representative compare (tag match = hit), 2 stops after the filter, 3 after key load + hash
// (garbage slots; tools/consume_diag.py; never followed by a checked finalize).
//
// One workgroup per tile of rg.tile_rows rows (grid-stride).  Phase 1 runs in sub-batches of
// kSubRows rows: every thread evaluates the predicate for 32 rows (32 independent loads in
// flight), then the passing rows are compacted into LDS with per-wave ballots and one LDS
// prefix over the 4 waves.  Phase 2 processes the compacted rows densely and appends one
// staging record per row (one cursor atomic per flush).  Large tiles matter: the block barrier
// that ends phase 2 waits for the slowest probe chain of the block, and more rows per barrier
// amortise that wait (4096 -> 8192 -> 16384 rows per tile: 1.80 -> 1.64 -> 1.38 ms at C2).
// Phase 2 is flushed early when the selection buffer could overflow (selectivity > 1/2).
//
// HC (high-cardinality mode, pxg_hc.hip): phase 2 writes one partition record per row instead
// of probing the global table; a row with a STRING key longer than kHcStrWords words leaves a
// hole there and takes the table path (a staging record whose slot the generic list kernel
// fills in, like any deferred row), so the two paths hold disjoint key sets.
// REC: published slots compare against the probe records (all-STRING keys, <= 2 keys; the table
// passes prec).
template <int NK, int MODE, bool PAIRS = false, bool HC = false, bool REC = false, bool RROW = false>
__global__ void __launch_bounds__(kConsumeBlock) AggConsumeFastKernel(const AggPlanDev* __restrict__ plan,
                                                                      const DevChunk* __restrict__ chunks,
                                                                      const TileRange* __restrict__ ranges, int nranges,
                                                                      int64_t ntiles, AggTableDev tab, StageDev stg,
                                                                      uint32_t nchunks) {
  constexpr bool S = (MODE & 4) != 0;  // all keys STRING
  constexpr int kPer = kSubRows / kConsumeBlock;

  constexpr int kWaves = kConsumeBlock / 64;
  constexpr int kCap = kSelCap;
  __shared__ uint16_t s_sel[kCap];
  __shared__ uint32_t s_wcnt[2][kWaves];
  __shared__ unsigned int s_ins;
  __shared__ unsigned long long s_base;
  __shared__ KeyCols<NK> s_kc[kLdsChunks];
  __shared__ unsigned int s_mlen[NK];  // HC: the workgroup's longest STRING key per key
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (HC && threadIdx.x < NK) s_mlen[threadIdx.x] = 0;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  const uint32_t bid = XcdRemap(blockIdx.x, gridDim.x);
  const int nv = plan->n_vals;
  if (threadIdx.x == 0) s_ins = 0;
  const uint32_t n_lds_chunks = min(nchunks, static_cast<uint32_t>(kLdsChunks));
  int64_t flo = 0, fhi = 0;
  bool fneg = false;
  // (Not compiled into the mixed-key partition-record kernels: their register budget could not
  // take it, C5's consume 1.37 -> 2.11 ms with no filter at all.)
  const bool frange = !PAIRS && (!HC || S) && plan->has_filter && FilterRange(&plan->filter, plan->col_types[plan->filter.col], &flo, &fhi, &fneg);
  for (uint32_t c = threadIdx.x; c < n_lds_chunks; c += kConsumeBlock) s_kc[c] = KeyColsOf<NK, S>(plan, chunks[c]);
  __syncthreads();
  for (int64_t t = bid; t < ntiles; t += gridDim.x) {
    int ri = 0;
    while (ri + 1 < nranges && ranges[ri + 1].tile0 <= t) ++ri;
    const TileRange rg = ranges[ri];
    const DevChunk& ch = chunks[rg.chunk];
    const int64_t row0 = rg.lo + (t - rg.tile0) * rg.tile_rows;
    const int64_t row1 = min(row0 + rg.tile_rows, rg.hi);
    const int kSubBatches = rg.tile_rows / kSubRows;
    // The filter column streamed two rows per lane with 16-byte loads (an 8-byte column, even
    // tile start): 8-byte loads stream at ~3.7 TB/s on gfx950, 16-byte ones at ~5.7 TB/s
    // (tools/stream_probe.hip, profiles/r03_stream_probe*.log).  Uniform per tile.
    // PAIRS: chosen on the host (an 8-byte filter column, every range starting at an even row).
    uint32_t total = 0;
#pragma unroll 1
    for (int sb = 0; sb < kSubBatches; ++sb) {
      const int64_t sb0 = row0 + static_cast<int64_t>(sb) * kSubRows;
      uint32_t wtot = 0;
      uint32_t wbase = total, sbtot = 0;
      if constexpr (PAIRS) {
        constexpr int kPairs = kPer / 2;
        const uint64_t* fv = reinterpret_cast<const uint64_t*>(ch.cols[plan->filter.col].values);
        // Pass bits per lane (bit k: pair k), not ballot words: 2 registers instead of 32
        // scalar pairs live across the barrier; the ballots are re-taken after it.
        uint32_t be = 0, bo = 0;
        const ulonglong2* fv2 = reinterpret_cast<const ulonglong2*>(fv);
        const DevProgram* fp = &plan->filter;
        const int64_t r0 = sb0 + 2 * static_cast<int64_t>(threadIdx.x);
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
          const int64_t r = r0 + 2 * k * kConsumeBlock;
          ulonglong2 v = make_ulonglong2(0, 0);
          if (r + 1 < row1) v = fv2[r >> 1];
          else if (r < row1) v.x = fv[r];
          be |= static_cast<uint32_t>(r < row1 && ApplyShape(fp, v.x) != 0) << k;
          bo |= static_cast<uint32_t>(r + 1 < row1 && ApplyShape(fp, v.y) != 0) << k;
        }
        // The wave's count as a lane reduction (no ballot words live across the barrier).
        uint32_t c = static_cast<uint32_t>(__popc(be) + __popc(bo));
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        wtot = c;
        if (lane == 0) s_wcnt[sb & 1][wid] = wtot;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
          const uint32_t c = s_wcnt[sb & 1][w];
          wbase += w < wid ? c : 0;
          sbtot += c;
        }
        // Row order inside the wave: lane l's even row follows both rows of every lower lane.
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
          const bool pe = (be >> k) & 1u, po = (bo >> k) & 1u;
          const unsigned long long me = __ballot(pe), mo = __ballot(po);
          const uint32_t at = wbase + static_cast<uint32_t>(__popcll(me & lanemask_lt) + __popcll(mo & lanemask_lt));
          const uint16_t off = static_cast<uint16_t>(sb * kSubRows + 2 * (k * kConsumeBlock + threadIdx.x));
          if (pe) s_sel[at] = off;
          if (po) s_sel[at + (pe ? 1 : 0)] = static_cast<uint16_t>(off + 1);
          wbase += static_cast<uint32_t>(__popcll(me) + __popcll(mo));
        }
      } else {
        bool pass[kPer];
        if (frange) {
          // An integer range filter: the kPer loads (clamped rows) all issued before the first
          // compare.  The generic loop below dispatches on the shape per row and waits for each
          // load before the next.
          const int64_t* fv = reinterpret_cast<const int64_t*>(ch.cols[plan->filter.col].values);
          constexpr int kFB = kPer / 2;
#pragma unroll
          for (int h = 0; h < kPer; h += kFB) {
            int64_t v[kFB];
#pragma unroll
            for (int k = 0; k < kFB; ++k) {
              const int64_t r = sb0 + (h + k) * kConsumeBlock + threadIdx.x;
              v[k] = fv[r < row1 ? r : row1 - 1];
            }
#pragma unroll
            for (int k = 0; k < kFB; ++k) {
              const int64_t r = sb0 + (h + k) * kConsumeBlock + threadIdx.x;
              pass[h + k] = r < row1 && ((v[k] >= flo && v[k] <= fhi) != fneg);
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < kPer; ++k) {
            const int64_t r = sb0 + k * kConsumeBlock + threadIdx.x;
            pass[k] = r < row1;
            if (pass[k] && plan->has_filter) pass[k] = EvalShape(&plan->filter, ch, r, plan->col_types) != 0;
          }
        }
        unsigned long long m[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
          m[k] = __ballot(pass[k]);
          wtot += static_cast<uint32_t>(__popcll(m[k]));
        }
        if (lane == 0) s_wcnt[sb & 1][wid] = wtot;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
          const uint32_t c = s_wcnt[sb & 1][w];
          wbase += w < wid ? c : 0;
          sbtot += c;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
          if (pass[k]) s_sel[wbase + __popcll(m[k] & lanemask_lt)] = static_cast<uint16_t>(sb * kSubRows + k * kConsumeBlock + threadIdx.x);
          wbase += static_cast<uint32_t>(__popcll(m[k]));
        }
      }
      total += sbtot;
      if (sb + 1 < kSubBatches && total + kSubRows <= kCap) continue;
      // Phase 2 over the rows collected so far.
      if (threadIdx.x == 0) {
        if (s_ins) {
          atomicAdd(&tab.counters[0], s_ins);
          s_ins = 0;
        }
        s_base = total ? atomicAdd(HC ? stg.hc.cursor : stg.cursor, static_cast<unsigned long long>(total)) : 0ULL;
      }
      __syncthreads();
      const uint64_t base = s_base;
      KeyHeads<NK> heads = {};
      if ((MODE & 3) != 2 && threadIdx.x < total) LoadKeyHeads<NK, S>(plan, ch, row0 + s_sel[threadIdx.x], heads);
      for (uint32_t i = threadIdx.x; i < total; i += kConsumeBlock) {
        const int64_t local = row0 + s_sel[i];
        const uint64_t pos = base + i;
        if constexpr (HC) {
          uint64_t x[kHcMaxVals];
#pragma unroll
          for (int v = 0; v < kHcMaxVals; ++v) x[v] = v < nv ? EvalShape(&plan->vals[v], ch, local, plan->col_types) : 0;
          FastKeys<NK> k;
          bool fit = LoadKeyBodies<NK, S>(plan, ch, heads, k);
          if (i + kConsumeBlock < total) LoadKeyHeads<NK, S>(plan, ch, row0 + s_sel[i + kConsumeBlock], heads);
#pragma unroll
          for (int q = 0; q < NK; ++q) fit = fit && (KeyT<S>(plan, q) != PXG_STRING || k.len[q] <= 8u * kHcStrWords);
          uint64_t* r = stg.hc.rec + pos;
          const uint64_t cap = stg.hc.cap;
          if (fit) {
            const uint64_t h = HashFastKeys<NK, S>(plan, k);
            uint64_t lens = 0;
#pragma unroll
            for (int q = 0; q < NK; ++q) {
              lens |= static_cast<uint64_t>(k.len[q]) << (16 * q);
              if (KeyT<S>(plan, q) == PXG_STRING) atomicMax(&s_mlen[q], k.len[q]);
            }
            // Bytes 16-19 of a first STRING key also ride in the lengths word's spare half
            // (<= 2 keys): when no staged first key is longer than 20 bytes, the partition pass
            // drops that key's third word stream (MakeHcPlan, tail0).
            if (NK <= 2 && KeyT<S>(plan, 0) == PXG_STRING) lens |= (k.w[0][2] & 0xFFFFFFFFULL) << 32;
            r[0] = lens;
#pragma unroll
            for (int q = 0; q < NK; ++q) {
#pragma unroll
              for (int j = 0; j < kHcStrWords; ++j)
                if (j < stg.hc.kw[q]) r[(stg.hc.koff[q] + j) * cap] = k.w[q][j];
            }
#pragma unroll
            for (int v = 0; v < kHcMaxVals; ++v)
              if (v < nv) r[(stg.hc.kwords + v) * cap] = x[v];
            stg.hc.key[pos] = static_cast<uint32_t>(h >> 32);
          } else {
            r[0] = kHcHole;
            stg.hc.key[pos] = 0xFFFFFFFFu;
          }
          // Rows with a long key: a staging record for the table path, deferred (one cursor and
          // one list append per wave).
          const unsigned long long lm = __ballot(!fit);
          if (lm) {
            const int leader = __ffsll(static_cast<long long>(lm)) - 1;
            const unsigned int cnt = static_cast<unsigned int>(__popcll(lm));
            unsigned long long sb = 0;
            unsigned int db = 0;
            if (lane == leader) {
              sb = atomicAdd(stg.cursor, static_cast<unsigned long long>(cnt));
              db = atomicAdd(&tab.counters[2], cnt);
            }
            sb = __shfl(sb, leader, 64);
            db = __shfl(db, leader, 64);
            if (!fit) {
              const unsigned int rk = static_cast<unsigned int>(__popcll(lm & lanemask_lt));
              const uint64_t sp = sb + rk;
#pragma unroll
              for (int v = 0; v < kHcMaxVals; ++v)
                if (v < nv) stg.vals[v][sp] = x[v];
              stg.slot[sp] = kDeferredSlot;
              tab.deferred[db + rk] = (static_cast<uint32_t>(rg.chunk) << kChunkShift) | static_cast<uint32_t>(local);
              tab.deferred_pos[db + rk] = static_cast<uint32_t>(sp);
            }
          }
          continue;
        }
        // Value streams first: independent of the key chain, their loads overlap it.
        for (int v = 0; v < nv; ++v) stg.vals[v][pos] = EvalShape(&plan->vals[v], ch, local, plan->col_types);
        FastKeys<NK> k;
        uint32_t slot = kDeferredSlot;
        const uint32_t rowref = (static_cast<uint32_t>(rg.chunk) << kChunkShift) | static_cast<uint32_t>(local);
        bool have_keys = false;
        if ((MODE & 3) != 2) {
          have_keys = LoadKeyBodies<NK, S>(plan, ch, heads, k);
          // the next row's heads, in flight during this row's hash and probe
          if (i + kConsumeBlock < total) LoadKeyHeads<NK, S>(plan, ch, row0 + s_sel[i + kConsumeBlock], heads);
        }
        if ((MODE & 3) == 2) {
          slot = 0;
        } else if (have_keys) {
          const uint64_t h = HashFastKeys<NK, S>(plan, k);
          if ((MODE & 3) == 3) {
            stg.slot[pos] = static_cast<uint32_t>(h);
            continue;
          }
          slot = FastFindOrInsert<NK, S, (MODE & 3) == 1, REC && S && NK <= kRecMaxKeys, RROW && S && NK <= kRecMaxKeys>(
              plan, chunks, s_kc, n_lds_chunks, k, h, rowref, tab, &s_ins);
        }
        const unsigned long long dm = __ballot(slot == kDeferredSlot);
        if (dm) {
          const int leader = __ffsll(static_cast<long long>(dm)) - 1;
          unsigned int dbase = 0;
          if (lane == leader) dbase = atomicAdd(&tab.counters[2], static_cast<unsigned int>(__popcll(dm)));
          dbase = __shfl(dbase, leader, 64);
          if (slot == kDeferredSlot) {
            const unsigned int at = dbase + __popcll(dm & lanemask_lt);
            tab.deferred[at] = rowref;
            tab.deferred_pos[at] = static_cast<uint32_t>(pos);
          }
        }
        stg.slot[pos] = slot;
      }
      __syncthreads();  // s_sel / s_base are rewritten next
      total = 0;
    }
  }
  if (threadIdx.x == 0 && s_ins) atomicAdd(&tab.counters[0], s_ins);
  if constexpr (HC) {
    __syncthreads();
    if (threadIdx.x < NK && s_mlen[threadIdx.x]) atomicMax(&stg.hc.maxlen[threadIdx.x], s_mlen[threadIdx.x]);
  }
}

// ---------------------------------------------------------------------------------------
// Publication: every slot still holding a row reference (kind 0) gets its key copied into the
// arena.  sizes[i] = (1 << 40) | words, so one exclusive scan yields both the record offsets
// and (total >> 40) the number of published groups.
constexpr int kPublishCountShift = 40;
__global__ void AggPublishSizesKernel(const AggPlanDev* __restrict__ plan, const DevChunk* __restrict__ chunks,
                                      const unsigned long long* __restrict__ slots, uint32_t cap, uint64_t* __restrict__ sizes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const unsigned long long w = slots[i];
  uint64_t s = 0;
  if (w != 0 && !(w & kKindArena)) {
    const uint32_t ref = static_cast<uint32_t>(w);
    KeySet k;
    LoadKeysRow(plan, chunks[ref >> kChunkShift], static_cast<int64_t>(ref & (kChunkRows - 1)), k);
    s = (uint64_t(1) << kPublishCountShift) | KeyRecordWords(plan, k);
  }
  sizes[i] = s;
}

// The probe record of a published group (all-STRING keys): its slot word, the lengths, the key
// words tail-masked and zero-padded (word 0 = 0, i.e. no record, when a key is too long).
__device__ __forceinline__ void WriteProbeRecord(const AggPlanDev* __restrict__ plan, const KeySet& k, unsigned long long word,
                                                 uint64_t* __restrict__ rec) {
  uint64_t r[kRecWords];
#pragma unroll
  for (int t = 0; t < kRecWords; ++t) r[t] = 0;
  r[0] = word;
#pragma unroll
  for (int i = 0; i < kRecMaxKeys; ++i) {
    if (i >= plan->n_keys) break;
    const uint32_t len = static_cast<uint32_t>(k.v[i].b);
    if (len > 8u * kRecKeyWords) r[0] = 0;
    r[1] |= static_cast<uint64_t>(len & 0xFFFF) << (16 * i);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(k.v[i].a);
#pragma unroll
    for (int j = 0; j < kRecKeyWords; ++j)
      if (8u * j < len && len <= 8u * kRecKeyWords) r[2 + kRecKeyWords * i + j] = LoadWordU(src + 8 * j) & TailMask(len - 8u * j);
  }
  ulonglong2* d = reinterpret_cast<ulonglong2*>(rec);
#pragma unroll
  for (int t = 0; t < kRecWords / 2; ++t) d[t] = make_ulonglong2(r[2 * t], r[2 * t + 1]);
}

// Probe records of every published slot (after a rehash moved the slots).
__global__ void RecordsFromArenaKernel(const AggPlanDev* __restrict__ plan, const unsigned long long* __restrict__ slots, uint32_t cap,
                                       const uint64_t* __restrict__ arena, uint64_t* __restrict__ prec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const unsigned long long w = slots[i];
  if (!(w & kKindArena)) return;
  KeySet k;
  LoadKeysArena(plan, arena + static_cast<uint32_t>(w), k);
  WriteProbeRecord(plan, k, w, prec + static_cast<uint64_t>(i) * kRecWords);
}

// total != null: the speculative launch (issued before the host has read the scanned total).
// It writes nothing unless the new records fit the arena as reserved (arena_bytes, with the
// slack) and keep 32-bit offsets; every thread reads the same total, so the whole grid agrees.
__global__ void AggPublishWriteKernel(const AggPlanDev* __restrict__ plan, const DevChunk* __restrict__ chunks,
                                      unsigned long long* __restrict__ slots, uint32_t cap, const uint64_t* __restrict__ offs,
                                      uint64_t base, uint64_t* __restrict__ arena, uint64_t* __restrict__ prec,
                                      const uint64_t* __restrict__ total, uint64_t arena_bytes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  if (total) {
    const uint64_t words = *total & ((uint64_t(1) << kPublishCountShift) - 1);
    if ((base + words) * 8 + kArenaSlack > arena_bytes || base + words >= (uint64_t(1) << 32)) return;
  }
  const unsigned long long w = slots[i];
  if (w == 0 || (w & kKindArena)) return;
  const uint32_t ref = static_cast<uint32_t>(w);
  KeySet k;
  LoadKeysRow(plan, chunks[ref >> kChunkShift], static_cast<int64_t>(ref & (kChunkRows - 1)), k);
  const uint64_t at = base + (offs[i] & ((uint64_t(1) << kPublishCountShift) - 1));
  WriteKeyRecord(plan, k, arena + at);
  const unsigned long long nw = MakeSlotWord(static_cast<uint32_t>(w >> 33), kKindArena, static_cast<uint32_t>(at));
  slots[i] = nw;
  if (prec) WriteProbeRecord(plan, k, nw, prec + static_cast<uint64_t>(i) * kRecWords);
}

__global__ void AggRehashKernel(const AggPlanDev* __restrict__ plan, const unsigned long long* __restrict__ old_slots,
                                uint32_t old_cap, unsigned long long* __restrict__ new_slots, uint32_t new_mask,
                                const uint64_t* __restrict__ arena, uint32_t* __restrict__ remap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap) return;
  const unsigned long long w = old_slots[i];
  if (w == 0) return;
  KeySet k;
  LoadKeysArena(plan, arena + static_cast<uint32_t>(w), k);
  const uint64_t h = HashKeys(plan, k);
  uint32_t p = static_cast<uint32_t>(h) & new_mask;
  for (uint32_t probe = 0; probe <= new_mask; ++probe) {
    unsigned long long expected = 0;
    if (__hip_atomic_compare_exchange_strong(&new_slots[p], &expected, w, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
      remap[i] = p;
      return;
    }
    p = (p + 1) & new_mask;
  }
}

__global__ void StageRemapKernel(uint32_t* __restrict__ slot, uint64_t n, const uint32_t* __restrict__ remap) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  if (s != kDeferredSlot) slot[i] = remap[s];
}

// ---------------------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------------------
static uint32_t NextPow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return static_cast<uint32_t>(std::min<uint64_t>(p, uint64_t(1) << 31));
}

static AggTableDev TableDev(Agg* a, int defer_buf) {
  AggTableDev t;
  t.slots = a->slots.as<unsigned long long>();
  t.mask = a->cap - 1;
  t.limit = a->cap / 2;
  t.counters = a->counters.as<unsigned int>();
  t.deferred = a->deferred[defer_buf].as<uint32_t>();
  t.deferred_pos = a->deferred_pos[defer_buf].as<uint32_t>();
  t.arena = a->arena.as<uint64_t>();
  t.prec = a->rec_ok && a->rec_cap == a->cap ? a->prec.as<uint64_t>() : nullptr;
  return t;
}

static StageDev StageDevOf(Agg* a) {
  StageDev s;
  s.slot = a->st_slot.as<uint32_t>();
  for (int v = 0; v < kMaxVals; ++v) s.vals[v] = v < a->n_vals ? a->st_val[v].as<uint64_t>() : nullptr;
  s.cursor = reinterpret_cast<unsigned long long*>(a->counters.as<uint8_t>() + 16);
  s.hc = a->hc_layout;
  s.hc.rec = a->hc_rec.as<uint64_t>();
  s.hc.key = a->hc_key.as<uint32_t>();
  s.hc.cap = a->hc_cap;
  s.hc.cursor = reinterpret_cast<unsigned long long*>(a->counters.as<uint8_t>() + 48);
  s.hc.maxlen = a->hc_maxlen.as<unsigned int>();
  return s;
}

int32_t Agg::EnsureTable(uint32_t want) {
  if (slots.p) return PXG_OK;
  cap = want;
  PXG_RETURN_IF_ERROR(slots.Alloc(static_cast<size_t>(cap) * 8));
  PXG_HIP(hipMemsetAsync(slots.p, 0, static_cast<size_t>(cap) * 8, ctx->stream));
  return PXG_OK;
}

// Probe records sized with the table (rec_ok plans only; at most kRecMaxCap slots).  Fresh
// buffers are cleared: a record is valid only while its word 0 equals its slot's word.
constexpr uint32_t kRecMaxCap = uint32_t(1) << 22;
int32_t Agg::EnsureRecords() {
  if (!rec_ok || cap > kRecMaxCap) {
    rec_cap = 0;
    return PXG_OK;
  }
  if (rec_cap == cap) return PXG_OK;
  prec.Free();
  PXG_RETURN_IF_ERROR(prec.Alloc(static_cast<size_t>(cap) * kRecWords * 8));
  PXG_HIP(hipMemsetAsync(prec.p, 0, static_cast<size_t>(cap) * kRecWords * 8, ctx->stream));
  rec_cap = cap;
  rec_dirty = false;
  return PXG_OK;
}

// After a rehash the slots moved: clear the records and write one per published slot again.
int32_t Agg::RebuildRecords() {
  if (!rec_ok || rec_cap == 0) return PXG_OK;
  PXG_RETURN_IF_ERROR(EnsureRecords());
  if (rec_cap != cap) return PXG_OK;
  PXG_HIP(hipMemsetAsync(prec.p, 0, static_cast<size_t>(cap) * kRecWords * 8, ctx->stream));
  PXG_RETURN_IF_ERROR(Launch(ctx, "agg_records", RecordsFromArenaKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                             d_plan.as<const AggPlanDev>(), slots.as<const unsigned long long>(), cap, arena.as<const uint64_t>(),
                             prec.as<uint64_t>()));
  rec_dirty = true;
  return PXG_OK;
}

int32_t Agg::EnsureStage(uint64_t need) {
  // Capacity is whatever the buffers hold now (finalize swaps staging with same-size buffers).
  st_cap = st_slot.bytes / 4;
  for (int v = 0; v < n_vals; ++v) st_cap = std::min<uint64_t>(st_cap, st_val[v].bytes / 8);
  if (need <= st_cap) return PXG_OK;
  uint64_t c = std::max<uint64_t>(need, st_cap * 2);
  PXG_RETURN_IF_ERROR(st_slot.Reserve(c * 4, st_n * 4, ctx->stream));
  for (int v = 0; v < n_vals; ++v) PXG_RETURN_IF_ERROR(st_val[v].Reserve(c * 8, st_n * 8, ctx->stream));
  st_cap = c;
  return PXG_OK;
}

int32_t Agg::EnsureHc(uint64_t need) {
  if (need <= hc_cap) return PXG_OK;
  const uint64_t c = std::max<uint64_t>(need, hc_cap * 2);
  const int sw = hc_layout.stride;
  DevBuf nr;
  PXG_RETURN_IF_ERROR(nr.Alloc(c * sw * 8 + 64));
  if (hc_n > 0)  // stream j moves from j * hc_cap to j * c
    for (int j = 0; j < sw; ++j)
      PXG_HIP(hipMemcpyAsync(nr.as<uint64_t>() + j * c, hc_rec.as<uint64_t>() + j * hc_cap, hc_n * 8, hipMemcpyDeviceToDevice, ctx->stream));
  PXG_RETURN_IF_ERROR(hc_key.Reserve(c * 4 + 16, hc_n * 4, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  hc_rec = std::move(nr);
  hc_cap = c;
  return PXG_OK;
}

int64_t HcMinGroups() {
  const char* e = std::getenv("PXG_HC_MIN_GROUPS");
  return e ? std::atoll(e) : (int64_t(1) << 20);
}

bool Agg::HcNext() const {
  const int64_t m = HcMinGroups();
  return hc_ok && m > 0 && std::max<int64_t>(hint_groups, static_cast<int64_t>(last_groups)) >= m && !EnvFlag("PXG_NO_HC");
}

int32_t Agg::Grow(uint32_t new_cap) {
  if (new_cap <= cap) return PXG_OK;
  DevBuf ns;
  PXG_RETURN_IF_ERROR(ns.Alloc(static_cast<size_t>(new_cap) * 8));
  PXG_HIP(hipMemsetAsync(ns.p, 0, static_cast<size_t>(new_cap) * 8, ctx->stream));
  DevBuf remap;
  PXG_RETURN_IF_ERROR(remap.Alloc(static_cast<size_t>(cap) * 4));
  PXG_RETURN_IF_ERROR(Launch(ctx, "agg_rehash", AggRehashKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                             d_plan.as<const AggPlanDev>(), slots.as<const unsigned long long>(), cap,
                             ns.as<unsigned long long>(), new_cap - 1, arena.as<const uint64_t>(), remap.as<uint32_t>()));
  if (st_n > 0) {
    PXG_RETURN_IF_ERROR(Launch(ctx, "stage_remap", StageRemapKernel, dim3(GridFor(static_cast<int64_t>(st_n), 256, 1 << 30)), dim3(256), 0,
                               st_slot.as<uint32_t>(), st_n, remap.as<const uint32_t>()));
  }
  PXG_RETURN_IF_ERROR(MaccFollowGrow(this, slots.as<const unsigned long long>(), cap, remap.as<const uint32_t>(), new_cap));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  slots = std::move(ns);
  cap = new_cap;
  return RebuildRecords();
}

// Publish every kind-0 slot into the arena; reads back the group count, the deferred count
// and the staging cursor with one synchronisation.
int32_t Agg::PublishNew(Table* t, uint32_t* n_deferred) {
  const size_t sz_bytes = static_cast<size_t>(cap + 1) * 8;
  const size_t need = sz_bytes + 64 + ScanScratchBytes(cap);
  PXG_RETURN_IF_ERROR(scratch.Ensure(need));
  uint64_t* sizes = scratch.as<uint64_t>();
  uint64_t* total = reinterpret_cast<uint64_t*>(scratch.as<uint8_t>() + sz_bytes);
  void* sc = scratch.as<uint8_t>() + sz_bytes + 64;
  const DevChunk* chunks = t->d_chunks.as<const DevChunk>();
  PXG_RETURN_IF_ERROR(Launch(ctx, "agg_publish_sizes", AggPublishSizesKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                             d_plan.as<const AggPlanDev>(), chunks, slots.as<const unsigned long long>(), cap, sizes));
  PXG_RETURN_IF_ERROR(ScanExclusiveU64(ctx, sizes, sizes, cap, total, sc));
  uint8_t* pin = static_cast<uint8_t*>(ctx->pinned);
  {
    const SmallCopy rb[3] = {{total, 0, 8}, {counters.p, 8, 56}, {hc_maxlen.p, 64, static_cast<uint32_t>(sizeof(hc_maxlen_h))}};
    PXG_RETURN_IF_ERROR(ReadbackSmall(ctx, ctx->stream, rb, hc_active ? 3 : 2));
  }
  uint64_t* rec_p = rec_ok && rec_cap == cap ? prec.as<uint64_t>() : nullptr;
  // With an arena already reserved, the write goes out before the read-back is waited on, and
  // the host waits only for the read-back: the write runs during the host's round trip (the C2
  // trace had the stream idle ~33 us here). It skips itself when the records do not fit; the host
  // then reserves and launches it again below.
  const uint64_t spec_bytes = arena.p ? arena.bytes : 0;
  if (spec_bytes) {
    PXG_HIP(hipEventRecord(ctx->ev_pub, ctx->stream));
    PXG_RETURN_IF_ERROR(Launch(ctx, "agg_publish_write", AggPublishWriteKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                               d_plan.as<const AggPlanDev>(), chunks, slots.as<unsigned long long>(), cap,
                               static_cast<const uint64_t*>(sizes), arena_words, arena.as<uint64_t>(), rec_p,
                               static_cast<const uint64_t*>(total), spec_bytes));
    PXG_HIP(hipEventSynchronize(ctx->ev_pub));
  } else {
    PXG_HIP(hipStreamSynchronize(ctx->stream));
  }
  uint8_t c[56];
  uint64_t tot = 0;
  std::memcpy(&tot, pin, 8);
  std::memcpy(c, pin + 8, 56);
  std::memcpy(n_deferred, c + 8, 4);
  std::memcpy(&st_n, c + 16, 8);
  std::memcpy(&hc_n, c + 48, 8);
  if (hc_active) std::memcpy(hc_maxlen_h, pin + 64, sizeof(hc_maxlen_h));

  const uint64_t n_new = tot >> kPublishCountShift;
  const uint64_t words = tot & ((uint64_t(1) << kPublishCountShift) - 1);
  uint32_t dev_groups = 0;  // exact: every successful insert CAS is counted (per-tile flushes)
  std::memcpy(&dev_groups, c, 4);
  if (n_new > 0) {
    // Slot words hold 32-bit arena offsets: refuse before any record is written (the
    // speculative launch checks the same bound on the device).
    if (arena_words + words >= (uint64_t(1) << 32)) return SetError(PXG_RESOURCE_UNAVAILABLE, "key arena exceeds 32 GiB");
    const bool written = spec_bytes && (arena_words + words) * 8 + kArenaSlack <= spec_bytes;
    if (!written) {
      PXG_RETURN_IF_ERROR(arena.Reserve((arena_words + words) * 8 + kArenaSlack, arena_words * 8, ctx->stream));
      PXG_RETURN_IF_ERROR(Launch(ctx, "agg_publish_write", AggPublishWriteKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                                 d_plan.as<const AggPlanDev>(), chunks, slots.as<unsigned long long>(), cap,
                                 static_cast<const uint64_t*>(sizes), arena_words, arena.as<uint64_t>(), rec_p,
                                 static_cast<const uint64_t*>(nullptr), uint64_t(0)));
    }
    if (rec_p) rec_dirty = true;
    arena_words += words;
  }
  // The device insert counter is exact (every successful insert CAS is counted).
  inserted = std::max<uint64_t>(inserted + n_new, dev_groups);
  // The device-side fill count restarts from the exact number of groups.
  PXG_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(counters.p), static_cast<int>(inserted), 1, ctx->stream));
  return PXG_OK;
}

static int32_t CheckTableTypes(const Agg& a, const Table& t) {
  for (auto& cr : a.col_refs) {
    if (cr.first >= t.ncols) return SetError(PXG_INVALID_ARGUMENT, "program references column %d; table has %d", cr.first, t.ncols);
    if (t.types[cr.first] != cr.second)
      return SetError(PXG_INVALID_ARGUMENT, "column %d has type %d; program expects %d", cr.first, t.types[cr.first], cr.second);
  }
  return PXG_OK;
}

int32_t Agg::ConsumeRange(Table* t, int64_t begin, int64_t end) {
  HostClock clk;
  PXG_RETURN_IF_ERROR(CheckTableTypes(*this, *t));
  PXG_RETURN_IF_ERROR(t->EnsureDeviceDescriptors());
  clk.Mark("consume: descriptors");
  if (t->chunks.size() > 255) return SetError(PXG_UNIMPLEMENTED, "tables are limited to 255 chunks per agg consume");
  int64_t tile_rows = fast_nk > 0 ? kConsumeTile : kGenericTile;
  if (fast_nk > 0) {
    const int64_t rounds8 = static_cast<int64_t>(ctx->num_cus) * 4 * 8;  // 4 resident workgroups per CU
    while (tile_rows < kConsumeTileMax && (end - begin) / (2 * tile_rows) >= rounds8) tile_rows *= 2;
    static const int64_t forced = [] {  // tests: PXG_CONSUME_TILE=32768 / 65536 at small sizes
      const char* e = std::getenv("PXG_CONSUME_TILE");
      const int64_t v = e ? std::atoll(e) : 0;
      return (v == 16384 || v == 32768 || v == 65536) ? v : 0;
    }();
    if (forced) tile_rows = forced;
  }
  static const int diag = [] {
    const char* e = std::getenv("PXG_DIAG_CONSUME");
    return e ? std::atoi(e) : 0;
  }();
  // 16-byte filter pair loads measured slower in this kernel (tools/ab_run.sh, r03: C2 1.44 vs
  // 1.52 ms, 1B rows 12.7 vs 13.9 ms): opt-in only (PXG_PAIRS=1).
  bool all_str = true;
  for (int i = 0; i < n_keys; ++i) all_str = all_str && key_types[i] == PXG_STRING;
  // 16-byte pair loads of the filter column: an 8-byte column, every tile starting at an even
  // row (device column buffers are allocated 256-byte aligned).
  bool pairs_ok = hplan.has_filter;
  if (pairs_ok) {
    const int ft = hplan.col_types[hplan.filter.col];
    pairs_ok = ft == PXG_INT64 || ft == PXG_FLOAT64 || ft == PXG_TIME64NS;
    for (const auto& c : t->chunks) {  // every range's first row (tiles start there)
      const int64_t lo = std::max(begin, c->row_base) - c->row_base;
      if (lo < c->nrows && c->row_base < end) pairs_ok = pairs_ok && (lo & 1) == 0;
    }
    for (const auto& c : t->chunks) pairs_ok = pairs_ok && (reinterpret_cast<uintptr_t>(c->cols[hplan.filter.col].values.p) & 15) == 0;
  }
  const bool pairs = pairs_ok && EnvFlag("PXG_PAIRS");
  // Tile ranges of [b, e) in `rs` (tiles of `tr` rows, appended; tile0 counted from t0).
  auto make_ranges = [&](int64_t b, int64_t e, int64_t tr, std::vector<TileRange>* rs) {
    int64_t nt = 0;
    for (size_t c = 0; c < t->chunks.size(); ++c) {
      const Chunk& ch = *t->chunks[c];
      const int64_t lo = std::max(b, ch.row_base) - ch.row_base;
      const int64_t hi = std::min(e, ch.row_base + ch.nrows) - ch.row_base;
      if (lo >= hi) continue;
      TileRange r;
      r.tile0 = nt;
      r.lo = lo;
      r.hi = hi;
      r.chunk = static_cast<int32_t>(c);
      r.tile_rows = static_cast<int32_t>(tr);
      rs->push_back(r);
      nt += (hi - lo + tr - 1) / tr;
    }
    return nt;
  };
  std::vector<TileRange> ranges;
  const int64_t ntiles = make_ranges(begin, end, tile_rows, &ranges);
  if (ranges.empty()) return PXG_OK;
  const int64_t rows = end - begin;
  if (st_n + static_cast<uint64_t>(rows) >= (uint64_t(1) << 32))
    return SetError(PXG_UNIMPLEMENTED, "more than 2^32 staged rows in one aggregation");
  // High-cardinality mode is decided once per run, at its first consume.
  if (st_n == 0 && hc_n == 0 && inserted == 0 && arena_words == 0) hc_active = HcNext();
  if (hc_active) {
    if (hc_n + static_cast<uint64_t>(rows) >= (uint64_t(1) << 32) - 1)
      return SetError(PXG_UNIMPLEMENTED, "more than 2^32 staged rows in one aggregation");
    PXG_RETURN_IF_ERROR(EnsureHc(hc_n + static_cast<uint64_t>(rows)));
  }
  PXG_RETURN_IF_ERROR(EnsureStage(st_n + static_cast<uint64_t>(rows)));
  PXG_RETURN_IF_ERROR(deferred[0].Ensure(static_cast<size_t>(rows) * 4 + 16));
  PXG_RETURN_IF_ERROR(deferred_pos[0].Ensure(static_cast<size_t>(rows) * 4 + 16));
  clk.Mark("consume: staging ensure");
  // The tile ranges of a repeated consume (same table, same rows) are already on the device.
  auto upload = [&](DevBuf& dr, std::vector<uint8_t>& cache, const std::vector<TileRange>& rs) -> int32_t {
    const size_t rbytes = rs.size() * sizeof(TileRange);
    if (rbytes != cache.size() || std::memcmp(cache.data(), rs.data(), rbytes) != 0) {
      PXG_RETURN_IF_ERROR(dr.Ensure(rbytes));
      PXG_HIP(hipMemcpyAsync(dr.p, rs.data(), rbytes, hipMemcpyHostToDevice, ctx->stream));
      PXG_HIP(hipStreamSynchronize(ctx->stream));  // `rs` is pageable and goes out of scope
      cache.assign(reinterpret_cast<const uint8_t*>(rs.data()), reinterpret_cast<const uint8_t*>(rs.data()) + rbytes);
    }
    return PXG_OK;
  };
  // Workgroups per CU of the grid (PXG_CONSUME_BPC: experiments).  4 (round 5, tools/
  // consume_diag.py sweep on one box): C2 1.287 ms (8: 1.310, 6: 1.463, 3: 1.371), 1B rows
  // 10.70 ms (8: 10.80).
  static const int64_t bpc = [] {
    const char* e = std::getenv("PXG_CONSUME_BPC");
    const int64_t v = e ? std::atoll(e) : 0;
    return v > 0 ? v : 4;
  }();
  // Probe records (pxg_agg.h) for all-STRING keys; PXG_NO_PREC=1 turns them off (tests compare).
  const bool rec = rec_ok && !hc_active && diag == 0 && fast_nk > 0 && fast_nk <= kRecMaxKeys && all_str && !EnvFlag("PXG_NO_PREC");
  if (rec) PXG_RETURN_IF_ERROR(EnsureRecords());
  using KernFn = void (*)(const AggPlanDev*, const DevChunk*, const TileRange*, int, int64_t, AggTableDev, StageDev, uint32_t);
  auto pick = [&](bool with_rec, bool with_rrow = false) -> KernFn {
    KernFn kern = AggConsumeKernel;
    switch (fast_nk * 4 + (diag & 3)) {
#define PXG_FAST_CASE(nk)                                           \
  case nk * 4 + 0: kern = AggConsumeFastKernel<nk, 0>; break;       \
  case nk * 4 + 1: kern = all_str ? AggConsumeFastKernel<nk, 5> : AggConsumeFastKernel<nk, 1>; break; \
  case nk * 4 + 2: kern = AggConsumeFastKernel<nk, 2>; break;       \
  case nk * 4 + 3: kern = AggConsumeFastKernel<nk, 3>; break;
      PXG_FAST_CASE(1)
      PXG_FAST_CASE(2)
      PXG_FAST_CASE(3)
      PXG_FAST_CASE(4)
#undef PXG_FAST_CASE
      default: break;
    }
    if (hc_active) {  // partition records (fast_nk > 0 by eligibility)
      switch (fast_nk * 2 + (all_str ? 1 : 0)) {
#define PXG_HC_CASE(nk)                                                     \
  case nk * 2 + 0: return AggConsumeFastKernel<nk, 0, false, true>;         \
  case nk * 2 + 1: return AggConsumeFastKernel<nk, 4, false, true>;
        PXG_HC_CASE(1)
        PXG_HC_CASE(2)
        PXG_HC_CASE(3)
        PXG_HC_CASE(4)
#undef PXG_HC_CASE
        default: break;
      }
    }
    if (fast_nk == 0 || (diag & 3) != 0) return kern;
    if (all_str) {  // all-STRING keys: the specialised production kernels (PXG_PAIRS=1: 16-byte filter loads)
      switch (fast_nk) {
        case 1:
          kern = with_rrow  ? AggConsumeFastKernel<1, 4, false, false, true, true>
                 : with_rec ? AggConsumeFastKernel<1, 4, false, false, true>
                            : (pairs ? AggConsumeFastKernel<1, 4, true> : AggConsumeFastKernel<1, 4>);
          break;
        case 2:
          kern = with_rrow  ? AggConsumeFastKernel<2, 4, false, false, true, true>
                 : with_rec ? AggConsumeFastKernel<2, 4, false, false, true>
                            : (pairs ? AggConsumeFastKernel<2, 4, true> : AggConsumeFastKernel<2, 4>);
          break;
        case 3: kern = pairs ? AggConsumeFastKernel<3, 4, true> : AggConsumeFastKernel<3, 4>; break;
        case 4: kern = pairs ? AggConsumeFastKernel<4, 4, true> : AggConsumeFastKernel<4, 4>; break;
        default: break;
      }
    }
    return kern;
  };
  // One launch over `rs` (nt tiles), its publication, and the retry rounds of deferred rows.
  auto run = [&](DevBuf& dr, std::vector<uint8_t>& cache, const std::vector<TileRange>& rs, int64_t nt, KernFn kern,
                 const char* name) -> int32_t {
    PXG_RETURN_IF_ERROR(upload(dr, cache, rs));
    PXG_HIP(hipMemsetAsync(counters.as<uint8_t>() + 8, 0, 4, ctx->stream));  // deferred count
    const int grid = static_cast<int>(std::min<int64_t>(nt, static_cast<int64_t>(ctx->num_cus) * bpc));
    PXG_RETURN_IF_ERROR(Launch(ctx, name, kern, dim3(grid), dim3(kConsumeBlock), 0, d_plan.as<const AggPlanDev>(),
                               t->d_chunks.as<const DevChunk>(), dr.as<const TileRange>(), static_cast<int>(rs.size()), nt, TableDev(this, 0),
                               StageDevOf(this), static_cast<uint32_t>(t->chunks.size())));
    clk.Mark("consume: launch");
    uint32_t n_def = 0;
    PXG_RETURN_IF_ERROR(PublishNew(t, &n_def));
    clk.Mark("consume: kernel + publish");
    int buf = 0;
    for (int round = 0; n_def > 0; ++round) {
      // Rows are deferred by a full table / overlong probe, or (fast path) by a long string key.
      // Grow unless this is the first retry and the table still has room for every deferred row.
      // Growth is sized by groups, not rows: deferred rows mostly repeat groups, so the table
      // grows geometrically (x4 per round, from at least 4x the groups it holds) and the retry
      // defers again while it is still too small; 4 * (groups + deferred rows) caps it.
      const uint64_t want = static_cast<uint64_t>(inserted) + n_def;
      if (round > 0 || fast_nk == 0 || want > static_cast<uint64_t>(cap) * 3 / 8) {
        const uint64_t geo = std::max<uint64_t>(static_cast<uint64_t>(cap) * 4, static_cast<uint64_t>(inserted) * 4);
        PXG_RETURN_IF_ERROR(Grow(NextPow2(std::min<uint64_t>(geo, 4 * want))));
      }
      PXG_RETURN_IF_ERROR(deferred[1 - buf].Ensure(static_cast<size_t>(n_def) * 4 + 16));
      PXG_RETURN_IF_ERROR(deferred_pos[1 - buf].Ensure(static_cast<size_t>(n_def) * 4 + 16));
      PXG_HIP(hipMemsetAsync(counters.as<uint8_t>() + 8, 0, 4, ctx->stream));
      PXG_RETURN_IF_ERROR(Launch(ctx, "agg_consume_list", AggConsumeListKernel, dim3(GridFor(n_def, kConsumeBlock, ctx->num_cus * 8)),
                                 dim3(kConsumeBlock), 0, d_plan.as<const AggPlanDev>(), t->d_chunks.as<const DevChunk>(),
                                 deferred[buf].as<const uint32_t>(), deferred_pos[buf].as<const uint32_t>(), n_def,
                                 TableDev(this, 1 - buf), StageDevOf(this)));
      PXG_RETURN_IF_ERROR(PublishNew(t, &n_def));
      buf = 1 - buf;
    }
    return PXG_OK;
  };
  // Probe records build up inside the launch (WriteRowRecord): the inserting lane writes its
  // group's record, lanes that confirm a group against its representative row write it where
  // their XCD had none, and published groups of earlier consumes keep their publication records.
  // (Round 4 published the hot groups with a separate prefix launch over ~1/32 of the range
  // first: 0.43 ms at 1B rows, break-even at 100M; the in-launch records replaced it.)
  if (rec && rec_cap == cap) {
    PXG_RETURN_IF_ERROR(run(d_ranges, last_ranges, ranges, ntiles, pick(true, true), "agg_consume"));
    rec_dirty = true;
  } else {
    PXG_RETURN_IF_ERROR(run(d_ranges, last_ranges, ranges, ntiles, pick(false), "agg_consume"));
  }
  // Keep the table at most ~37% full for the next consume.
  if (inserted > static_cast<uint64_t>(cap) * 3 / 8) PXG_RETURN_IF_ERROR(Grow(NextPow2(static_cast<uint64_t>(inserted) * 4)));
  return PXG_OK;
}

}  // namespace pxg

using namespace pxg;

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
static void CollectColRefs(const pxg_program& p, std::vector<std::pair<int32_t, int32_t>>* refs) {
  for (int i = 0; i < p.n_insns; ++i)
    if (p.insns[i].op == PXG_OP_COL) refs->push_back({p.insns[i].arg, p.insns[i].type});
    else if (p.insns[i].op == PXG_OP_STATE_WORD) refs->push_back({p.insns[i].arg, PXG_STRING});
}

static bool SameProgram(const pxg_program& a, const pxg_program& b) {
  if (a.n_insns != b.n_insns || a.result_type != b.result_type || a.pool_len != b.pool_len) return false;
  for (int i = 0; i < a.n_insns; ++i) {
    const pxg_insn &x = a.insns[i], &y = b.insns[i];
    if (x.op != y.op || x.type != y.type || x.arg != y.arg || x.imm != y.imm) return false;
  }
  return a.pool_len == 0 || std::memcmp(a.pool, b.pool, a.pool_len) == 0;
}

static int32_t UdaOutType(int kind, int arg_type) {
  switch (kind) {
    case PXG_UDA_COUNT: return PXG_INT64;
    case PXG_UDA_SUM: return arg_type == PXG_FLOAT64 ? PXG_FLOAT64 : PXG_INT64;
    case PXG_UDA_MEAN: return PXG_FLOAT64;
    case PXG_UDA_MEAN_MERGE: return PXG_FLOAT64;
    case PXG_UDA_MIN:
    case PXG_UDA_MAX: return arg_type;
    case PXG_UDA_QUANTILES: return PXG_FLOAT64;
    case PXG_UDA_MINSUM: return PXG_INT64;
    default: return PXG_DATA_TYPE_UNKNOWN;
  }
}

// Device UDA registry: (kind, arg type) signatures supported on the device, mirroring the
// builtin registrations (math_ops.cc:228-250, math_sketches.cc:25-28).
static bool UdaSupported(int kind, int arg) {
  switch (kind) {
    case PXG_UDA_COUNT: return arg >= PXG_BOOLEAN && arg <= PXG_TIME64NS;
    case PXG_UDA_SUM: return arg == PXG_FLOAT64 || arg == PXG_INT64 || arg == PXG_BOOLEAN;
    case PXG_UDA_MEAN: return arg == PXG_FLOAT64 || arg == PXG_INT64 || arg == PXG_BOOLEAN;
    case PXG_UDA_MEAN_MERGE: return arg == PXG_FLOAT64;
    case PXG_UDA_MIN:
    case PXG_UDA_MAX: return arg == PXG_FLOAT64 || arg == PXG_INT64 || arg == PXG_TIME64NS;
    case PXG_UDA_QUANTILES: return arg == PXG_FLOAT64 || arg == PXG_INT64;
    case PXG_UDA_MINSUM: return arg == PXG_INT64;
    default: return false;
  }
}

// The consume fast path takes bare-column group keys and fast-shape filter / value programs
// over fixed-width columns (AggConsumeFastKernel); returns its key count, 0 if not eligible.
static int32_t FastPathKeys(const AggPlanDev& p) {
  if (p.n_keys < 1 || p.n_keys > kMaxKeys) return 0;
  for (int k = 0; k < p.n_keys; ++k) {
    const int t = p.key_types[k];
    if (t < PXG_BOOLEAN || t > PXG_TIME64NS) return 0;
    if (p.keys[k].shape == kShapeCol) continue;
    // col op const over an 8-byte integer column giving an 8-byte integer (bin(), arithmetic):
    // the kernel loads the column at its own width and applies the shape.
    const int ct = p.col_types[p.keys[k].col];
    const bool int8 = (ct == PXG_INT64 || ct == PXG_TIME64NS) && (t == PXG_INT64 || t == PXG_TIME64NS);
    if (p.keys[k].shape != kShapeColOpConst || !int8 || p.keys[k].conv != 0) return 0;
  }
  auto fixed_shape = [&](const DevProgram& q) {
    if (q.shape != kShapeCol && q.shape != kShapeColOpConst) return false;
    const int ct = p.col_types[q.col];
    return ct != PXG_STRING && ct != PXG_UINT128 && ct != PXG_DATA_TYPE_UNKNOWN;
  };
  if (p.has_filter && !fixed_shape(p.filter)) return 0;
  for (int v = 0; v < p.n_vals; ++v)
    if (p.val_kind[v] != kValProgram || !fixed_shape(p.vals[v])) return 0;
  return p.n_keys;
}

extern "C" int32_t pxg_agg_create(pxg_ctx* ctx, const pxg_agg_spec* spec, pxg_agg** out) {
  if (!ctx || !spec || !out) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  if (spec->n_keys < 0 || spec->n_keys > kMaxKeys) return SetError(PXG_UNIMPLEMENTED, "at most %d group keys", kMaxKeys);
  if (spec->n_udas < 0 || spec->n_udas > kMaxUdas) return SetError(PXG_UNIMPLEMENTED, "at most %d aggregate expressions", kMaxUdas);
  auto holder = std::make_unique<pxg_agg>();
  Agg& a = holder->impl;
  a.ctx = &ctx->impl;
  a.n_keys = spec->n_keys;
  a.n_udas = spec->n_udas;
  a.windowed = spec->windowed != 0;
  a.has_filter = spec->filter != nullptr;
  a.emit_states = spec->emit_states != 0;
  std::memset(&a.hplan, 0, sizeof(a.hplan));
  std::vector<uint8_t> pool;
  std::vector<std::pair<DevProgram*, size_t>> pool_fix;
  size_t off = 0;
  a.hplan.n_keys = a.n_keys;
  a.hplan.n_udas = a.n_udas;
  a.hplan.has_filter = a.has_filter ? 1 : 0;
  if (a.has_filter) {
    if (spec->filter->result_type != PXG_BOOLEAN) return SetError(PXG_INVALID_ARGUMENT, "filter must be BOOLEAN");
    PXG_RETURN_IF_ERROR(CompileProgram(*spec->filter, nullptr, kMaxCols, &a.hplan.filter, &pool, &off));
    pool_fix.push_back({&a.hplan.filter, off});
    CollectColRefs(*spec->filter, &a.col_refs);
  }
  for (int k = 0; k < a.n_keys; ++k) {
    const pxg_program& p = spec->keys[k];
    if (p.result_type == PXG_STRING && !(p.n_insns == 1 && p.insns && p.insns[0].op == PXG_OP_COL))
      return SetError(PXG_UNIMPLEMENTED, "computed STRING group keys are not supported on device");
    PXG_RETURN_IF_ERROR(CompileProgram(p, nullptr, kMaxCols, &a.hplan.keys[k], &pool, &off));
    pool_fix.push_back({&a.hplan.keys[k], off});
    a.hplan.key_types[k] = p.result_type;
    a.key_types.push_back(p.result_type);
    CollectColRefs(p, &a.col_refs);
  }
  std::vector<const pxg_program*> val_progs, val_progs2;
  std::vector<int> val_kinds;
  // A plain (kValProgram) stream for p, shared with an earlier identical one.
  auto plain_stream = [&](const pxg_program& p, int32_t type, int* vi) -> int32_t {
    for (size_t j = 0; j < val_progs.size(); ++j) {
      if (val_kinds[j] == kValProgram && SameProgram(*val_progs[j], p)) {
        *vi = static_cast<int>(j);
        return PXG_OK;
      }
    }
    if (static_cast<int>(val_progs.size()) >= kMaxVals) return SetError(PXG_UNIMPLEMENTED, "too many distinct UDA arguments");
    *vi = static_cast<int>(val_progs.size());
    val_progs.push_back(&p);
    val_progs2.push_back(&p);
    val_kinds.push_back(kValProgram);
    a.val_type.push_back(type);
    return PXG_OK;
  };
  int32_t state_off = 0;
  for (int u = 0; u < a.n_udas; ++u) {
    const pxg_uda_spec& us = spec->udas[u];
    if (!UdaSupported(us.kind, us.arg_type)) return SetError(PXG_UNIMPLEMENTED, "UDA kind %d with arg type %d has no device implementation", us.kind, us.arg_type);
    a.uda_kind.push_back(us.kind);
    a.uda_arg_type.push_back(us.arg_type);
    a.uda_out_type.push_back(UdaOutType(us.kind, us.arg_type));
    a.uda_init.push_back(us.init_i64);
    a.uda_has_init.push_back(us.has_init);
    int vi = -1, vi2 = -1;
    if (a.emit_states) {  // Serialize() sizes (math_ops.h:583-772)
      if (us.kind == PXG_UDA_QUANTILES || us.kind == PXG_UDA_MINSUM || us.kind == PXG_UDA_MEAN_MERGE)
        return SetError(PXG_UNIMPLEMENTED, "UDA kind %d has no Serialize: it cannot be partially aggregated", us.kind);
      a.hplan.state_off[u] = state_off;
      state_off += us.kind == PXG_UDA_MEAN ? 16 : 8;
    }
    if (us.kind == PXG_UDA_MEAN_MERGE) {
      if (us.arg.result_type != PXG_FLOAT64 || us.arg2.result_type != PXG_INT64)
        return SetError(PXG_INVALID_ARGUMENT, "MEAN_MERGE takes a FLOAT64 sum and an INT64 size");
      PXG_RETURN_IF_ERROR(plain_stream(us.arg, PXG_FLOAT64, &vi));
      PXG_RETURN_IF_ERROR(plain_stream(us.arg2, PXG_INT64, &vi2));
    } else if (us.kind != PXG_UDA_COUNT) {
      if (us.arg.result_type != us.arg_type) return SetError(PXG_INVALID_ARGUMENT, "UDA %d arg type mismatch", u);
      const int vk = us.kind == PXG_UDA_MINSUM ? kValMinOf2 : kValProgram;
      for (size_t j = 0; j < val_progs.size(); ++j) {
        if (val_kinds[j] == vk && SameProgram(*val_progs[j], us.arg) &&
            (vk != kValMinOf2 || SameProgram(*val_progs2[j], us.arg2))) {
          vi = static_cast<int>(j);
          break;
        }
      }
      if (vi < 0) {
        if (static_cast<int>(val_progs.size()) >= kMaxVals) return SetError(PXG_UNIMPLEMENTED, "too many distinct UDA arguments");
        vi = static_cast<int>(val_progs.size());
        val_progs.push_back(&us.arg);
        val_progs2.push_back(&us.arg2);
        val_kinds.push_back(vk);
        a.val_type.push_back(us.arg_type);
      }
    }
    a.uda_val.push_back(vi);
    a.hplan.uda_kind[u] = us.kind;
    a.hplan.uda_val[u] = vi;
    a.hplan.uda_val2[u] = vi2;
    a.hplan.uda_arg_type[u] = us.arg_type;
    a.hplan.uda_init[u] = us.has_init ? us.init_i64 : 0;
  }
  a.n_vals = static_cast<int32_t>(val_progs.size());
  a.hplan.n_vals = a.n_vals;
  a.state_rec = state_off;
  a.hplan.state_rec = state_off;
  a.hplan.emit_states = a.emit_states ? 1 : 0;
  for (int v = 0; v < a.n_vals; ++v) {
    a.hplan.val_kind[v] = val_kinds[v];
    a.hplan.val_type[v] = a.val_type[v];
    PXG_RETURN_IF_ERROR(CompileProgram(*val_progs[v], nullptr, kMaxCols, &a.hplan.vals[v], &pool, &off));
    pool_fix.push_back({&a.hplan.vals[v], off});
    CollectColRefs(*val_progs[v], &a.col_refs);
    if (val_kinds[v] == kValMinOf2) {
      PXG_RETURN_IF_ERROR(CompileProgram(*val_progs2[v], nullptr, kMaxCols, &a.hplan.vals2[v], &pool, &off));
      pool_fix.push_back({&a.hplan.vals2[v], off});
      CollectColRefs(*val_progs2[v], &a.col_refs);
    }
  }
  for (auto& cr : a.col_refs) {
    if (cr.first < 0 || cr.first >= kMaxCols) return SetError(PXG_INVALID_ARGUMENT, "column index %d out of range", cr.first);
    a.hplan.col_types[cr.first] = cr.second;
  }
  PXG_RETURN_IF_ERROR(a.d_pool.Alloc(pool.size() + 16));
  if (!pool.empty()) PXG_HIP(hipMemcpy(a.d_pool.p, pool.data(), pool.size(), hipMemcpyHostToDevice));
  for (auto& pf : pool_fix) pf.first->pool = a.d_pool.as<uint8_t>() + pf.second;
  PXG_RETURN_IF_ERROR(a.d_plan.Alloc(sizeof(AggPlanDev)));
  // Exchange states (pxg_xchg.hip): Serialize() sizes of every non-quantile UDA
  // (math_ops.h:583-772: count / sum / min / max 8 bytes, MeanInfo 16).
  {
    a.hplan_x = a.hplan;
    bool ok = !a.windowed && !a.emit_states && a.n_keys > 0;
    int32_t so = 0, mw = 0;
    for (int u = 0; u < a.n_udas; ++u) {
      const int k = a.uda_kind[u];
      a.hplan_x.state_off[u] = 0;
      a.macc_off[u] = -1;
      if (k == PXG_UDA_QUANTILES) {
        if (a.x_qval >= 0 && a.x_qval != a.uda_val[u]) ok = false;
        a.x_qval = a.uda_val[u];
        continue;
      }
      if (k == PXG_UDA_MINSUM || k == PXG_UDA_MEAN_MERGE) ok = false;
      a.hplan_x.state_off[u] = so;
      so += k == PXG_UDA_MEAN ? 16 : 8;
      a.macc_off[u] = mw;
      mw += k == PXG_UDA_MEAN ? 2 : 1;
    }
    a.hplan_x.state_rec = so;
    a.hplan_x.emit_states = 0;
    a.macc_words = mw + 1;  // + the flags word
    a.x_ok = ok;
    PXG_RETURN_IF_ERROR(a.d_plan_x.Alloc(sizeof(AggPlanDev)));
  }
  a.fast_nk = FastPathKeys(a.hplan);
  {
    bool all_str = a.fast_nk > 0;
    for (int k = 0; k < a.n_keys; ++k) all_str = all_str && a.key_types[k] == PXG_STRING;
    a.rec_ok = all_str && a.fast_nk <= kRecMaxKeys;
  }
  // High-cardinality mode: fast-path keys, integer SUM / MEAN / MINSUM and integer MIN / MAX (LDS
  // integer atomics: order-independent, so the partition tables give deterministic results),
  // at most kHcMaxVals value streams and 4 accumulated UDAs.
  {
    bool ok = a.fast_nk > 0 && !a.windowed && !a.emit_states && a.n_vals <= kHcMaxVals && kMaxVals >= kHcMaxStride;
    int acc = 0, wide = 0;  // wide: MEAN accumulators, which also keep a high-word LDS array
    for (int u = 0; u < a.n_udas && ok; ++u) {
      const int k = a.uda_kind[u], at = a.uda_arg_type[u];
      const bool int_arg = at == PXG_INT64 || at == PXG_BOOLEAN;
      switch (k) {
        case PXG_UDA_COUNT: break;
        case PXG_UDA_SUM:
        case PXG_UDA_MEAN: ok = int_arg; ++acc; wide += k == PXG_UDA_MEAN; break;
        case PXG_UDA_MINSUM: ++acc; break;
        case PXG_UDA_MIN:
        case PXG_UDA_MAX: ok = at == PXG_INT64 || at == PXG_TIME64NS; ++acc; break;
        default: ok = false;
      }
    }
    // LDS of one hc_agg workgroup: kHcTable x (8 B entry + 8 B per accumulator and per MEAN high
    // word + 4 B count), within HcMaxDynLds (4 MEANs: 77,824 B; gfx950 allows 160 KiB per workgroup).
    a.hc_ok = ok && acc <= 4 && HcAggLdsBytes(acc, wide) <= HcMaxDynLds();
    int32_t w = 1;
    for (int k = 0; k < a.n_keys; ++k) {
      const int t = a.key_types[k];
      a.hc_layout.koff[k] = w;
      a.hc_layout.kw[k] = t == PXG_STRING ? kHcStrWords : (t == PXG_UINT128 ? 2 : 1);
      w += a.hc_layout.kw[k];
    }
    a.hc_layout.kwords = w;
    a.hc_layout.stride = w + a.n_vals;
    a.hc_ok = a.hc_ok && a.hc_layout.stride <= kHcMaxStride;
  }
  a.hint_groups = spec->expected_groups;
  PXG_HIP(hipMemcpy(a.d_plan.p, &a.hplan, sizeof(AggPlanDev), hipMemcpyHostToDevice));
  PXG_HIP(hipMemcpy(a.d_plan_x.p, &a.hplan_x, sizeof(AggPlanDev), hipMemcpyHostToDevice));
  PXG_RETURN_IF_ERROR(a.counters.Alloc(64));
  PXG_HIP(hipMemsetAsync(a.counters.p, 0, 64, a.ctx->stream));
  PXG_RETURN_IF_ERROR(a.hc_maxlen.Alloc(sizeof(a.hc_maxlen_h)));
  PXG_HIP(hipMemsetAsync(a.hc_maxlen.p, 0, sizeof(a.hc_maxlen_h), a.ctx->stream));
  const int64_t expected = spec->expected_groups > 0 ? spec->expected_groups : 4096;
  // The smallest table that holds the expected groups at <= 3/8 load, the fill the post-consume
  // growth rule keeps (ConsumeRange): an exact hint (the engine's group-count statistics) never
  // triggers a rehash, and the table is no larger than that, since publication, finalize's
  // dense ranking and every reset sweep all of it (C3, 5.07M groups: 32M -> 16M slots, step
  // 7.96 -> 7.18 ms at an exact hint; the probe kernel itself is unchanged).
  a.min_cap = NextPow2(std::max<uint64_t>(static_cast<uint64_t>(expected) * 8 / 3 + 1, 1024));
  // A high-cardinality run keeps only the rows with long keys in the table.
  if (a.HcNext()) a.min_cap = 1 << 16;
  PXG_RETURN_IF_ERROR(a.EnsureTable(a.min_cap));
  PXG_RETURN_IF_ERROR(a.arena.Alloc(1 << 16));
  PXG_HIP(hipStreamSynchronize(a.ctx->stream));
  *out = holder.release();
  return PXG_OK;
}

extern "C" int32_t pxg_agg_destroy(pxg_agg* agg) {
  if (!agg) return PXG_OK;
  hipStreamSynchronize(agg->impl.ctx->stream);
  delete agg;
  return PXG_OK;
}

extern "C" int32_t pxg_agg_consume(pxg_agg* agg, pxg_table* table, int64_t begin, int64_t end) {
  if (!agg || !table) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Table& t = table->impl;
  PXG_RETURN_IF_ERROR(t.FlushStage());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "row range [%lld,%lld) outside table of %lld rows", (long long)begin, (long long)end, (long long)t.nrows);
  if (t.ctx != agg->impl.ctx) return SetError(PXG_INVALID_ARGUMENT, "table and agg belong to different contexts");
  if (agg->impl.merged) return SetError(PXG_FAILED_PRECONDITION, "this aggregation holds merged partial states; reset it before consuming rows");
  agg->impl.res.ready = false;
  agg->impl.state_version++;
  return agg->impl.ConsumeRange(&t, begin, end);
}

extern "C" int32_t pxg_agg_info(pxg_agg* agg, pxg_agg_stats* st) {
  if (!agg || !st) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  const Agg& a = agg->impl;
  st->table_capacity = a.cap;
  st->groups = static_cast<int64_t>(a.inserted);
  st->rows_selected = static_cast<int64_t>(a.hc_active ? a.hc_n : a.st_n);
  st->key_arena_bytes = static_cast<int64_t>(a.arena_words * 8);
  st->staging_capacity = static_cast<int64_t>(a.st_cap);
  st->fast_path_keys = a.fast_nk;
  st->big_sort_groups = static_cast<int32_t>(a.last_big_sort_groups);
  st->hc_mode = a.hc_active ? 1 : 0;
  st->hc_partition_bits = a.last_hc_pbits;
  st->hc_reruns = a.last_hc_reruns;
  return PXG_OK;
}

extern "C" int32_t pxg_agg_rows_selected(pxg_agg* agg, int64_t* rows) {
  if (!agg || !rows) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  *rows = static_cast<int64_t>(agg->impl.hc_active ? agg->impl.hc_n : agg->impl.st_n);
  return PXG_OK;
}

extern "C" int32_t pxg_agg_reset(pxg_agg* agg) {
  if (!agg) return SetError(PXG_INVALID_ARGUMENT, "agg is null");
  Agg& a = agg->impl;
  // A table grown far beyond what the last run needed (e.g. an agg reused by a later, smaller
  // query) is shrunk, so publication and finalize do not keep sweeping empty slots.
  // The group count of the last run survives the reset that ends it (the engine resets an agg
  // after its emit and again when a later query takes it from the cache; sizing by the second
  // reset's zero count shrank C5's 3M-group table back to the hint every query: 5 rehash rounds).
  if (a.hc_active && a.res.ready && a.res.n_groups > 0) a.last_groups = static_cast<uint64_t>(a.res.n_groups);
  else if (a.inserted > 0) a.last_groups = a.inserted;
  const uint32_t fit = NextPow2(std::max<uint64_t>(a.HcNext() ? 0 : a.last_groups * 4, a.min_cap));
  if (a.cap > 16 * static_cast<uint64_t>(fit)) {
    PXG_HIP(hipStreamSynchronize(a.ctx->stream));
    a.slots.Free();
    a.cap = fit;
    PXG_RETURN_IF_ERROR(a.slots.Alloc(static_cast<size_t>(a.cap) * 8));
  }
  // Slots, dirty probe records (a record is valid only for a slot word of its own run), counters
  // and the HC key-length maxima, zeroed by one launch (four memsets cost ~22 us of stream time
  // per C2 step), stream-ordered before the next consume.
  {
    void* zp[4] = {a.slots.p, a.counters.p, a.hc_maxlen.p, a.prec.p};
    size_t zb[4] = {static_cast<size_t>(a.cap) * 8, 64, sizeof(a.hc_maxlen_h), static_cast<size_t>(a.cap) * kRecWords * 8};
    const bool recs = a.rec_dirty && a.rec_cap == a.cap;
    PXG_RETURN_IF_ERROR(ZeroRanges(a.ctx, a.ctx->stream, zp, zb, recs ? 4 : 3));
    if (recs) a.rec_dirty = false;
  }
  std::memset(a.hc_maxlen_h, 0, sizeof(a.hc_maxlen_h));
  a.st_n = 0;
  a.hc_n = 0;
  a.hc_active = false;
  a.merged = false;    // accumulators are re-initialised by the next merged import
  a.macc_cap = 0;
  a.x_parts_seen = 0;
  a.xc.valid = false;
  a.arena_words = 0;
  a.inserted = 0;
  a.state_version++;
  a.res.Clear();
  return PXG_OK;
}
