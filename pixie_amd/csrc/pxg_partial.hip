// Partial aggregation export/import: the PEM-partial / Kelvin-finalize split
// (planpb AggregateOperator.partial_agg / finalize_results, src/carnot/planpb/plan.proto:250-257;
// the splitter that creates it: src/carnot/planner/distributed/splitter/partial_op_mgr/
// partial_op_mgr.cc:69-83) mapped onto the GPUs of one node.
//
// An agg's state after consume is (group table + key arena, staging records).  Export
// partitions it by hash(group key) into n_parts self-describing byte buffers; import merges a
// buffer into another agg (on any device): its groups are found-or-inserted into the table by
// exact key equality and its staged records are appended, remapped onto the local slots.
// Finalize then runs unchanged, so count/sum/mean/min/max and quantiles of the union are the
// single-node results (UDA Merge semantics, math_ops.h:590-593,633,668-672,710-714,747;
// math_sketches.h:38).  QuantilesUDA has no Serialize (math_sketches.h:33-82), so the
// reference could not split it into partial states at all: its inputs travel as values.
//
// Part layout (8-byte aligned sections):
//   PartHeader (64 B)
//   koff  u64[n_groups]        word offset of each group's key record within `keys`
//   keys  u64[key_words]       arena-format key records (pxg_keys.h)
//   gid   u32[n_rows] (+pad)   group index (into koff) of each staged record
//   vals  u64[n_vals][n_rows]  staged value streams, stream-major
#include <algorithm>

#include "pxg_agg_host.h"
#include "pxg_keys.h"
#include "pxg_scan.h"
#include "pxg_tdigest.h"

namespace pxg {

constexpr uint32_t kPartMagic = 0x50475850u;  // "PXGP"
constexpr uint32_t kPartVersion = 1;
constexpr int kMaxParts = 63;                  // digit 63 = "not exported" sentinel

struct PartHeader {
  uint32_t magic;
  uint32_t version;
  uint32_t n_keys;
  uint32_t n_vals;
  uint64_t n_groups;
  uint64_t n_rows;
  uint64_t key_words;
  uint64_t plan_sig;
  uint64_t reserved[2];
};
static_assert(sizeof(PartHeader) == 64, "PartHeader is 64 bytes");

// Exchange v2 part header (partial states; layout below, XLayoutOf).
constexpr uint32_t kXMagic = 0x58475850u;  // "PXGX"
constexpr uint32_t kXVersion = 3;
constexpr int kXCentCapH = 2048;  // = kXCentCap (pxg_finalize.hip)
constexpr uint64_t kXFlagDigest = 1;
constexpr int kXWtShift = 48;
constexpr int kXMaxParts = 64;  // parts one merged run may import (pxg_finalize.hip kXParts)

struct XHeader {
  uint32_t magic;
  uint32_t version;
  uint32_t n_keys;
  uint32_t state_rec;
  uint64_t n_groups;
  uint64_t n_items;
  uint64_t key_words;
  uint64_t plan_sig;
  uint64_t has_q;
  uint64_t item_words;  // words of the items region (raw value 1, centroid 2)
};
static_assert(sizeof(XHeader) == 64, "XHeader is 64 bytes");

static bool IsXPart(const void* hdr_host) {
  uint32_t m = 0;
  std::memcpy(&m, hdr_host, 4);
  return m == kXMagic;
}


__host__ __device__ static inline uint64_t Align8(uint64_t x) { return (x + 7) & ~uint64_t(7); }

struct PartLayout {
  uint64_t koff, keys, gid, vals, bytes;
};
static PartLayout LayoutOf(uint64_t n_groups, uint64_t n_rows, uint64_t key_words, int n_vals) {
  PartLayout L;
  L.koff = sizeof(PartHeader);
  L.keys = L.koff + n_groups * 8;
  L.gid = L.keys + key_words * 8;
  L.vals = L.gid + Align8(n_rows * 4);
  L.bytes = L.vals + static_cast<uint64_t>(n_vals) * n_rows * 8;
  return L;
}

// Signature of what a part carries: key types and staged value-stream types.
static uint64_t PlanSig(const Agg& a) {
  uint64_t h = 1469598103934665603ULL;
  auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ULL; };
  mix(static_cast<uint64_t>(a.n_keys));
  for (int t : a.key_types) mix(static_cast<uint64_t>(t));
  mix(static_cast<uint64_t>(a.n_vals));
  for (int t : a.val_type) mix(static_cast<uint64_t>(t));
  return h;
}

__device__ __forceinline__ uint32_t PartOfHash(uint64_t h, uint32_t n_parts) {
  return static_cast<uint32_t>(((h >> 32) * static_cast<uint64_t>(n_parts)) >> 32);
}

// ---------------------------------------------------------------------------------------
// Stable partition by a small digit (< 64): per-tile histograms, one scan, stable scatter of
// item indices (ballot-matched ranks within a wave, LDS counts across waves).
// ---------------------------------------------------------------------------------------
constexpr int kPartBlock = 256;
constexpr int kPartItems = 16;
constexpr int kPartTile = kPartBlock * kPartItems;
constexpr int kPartBuckets = 64;
constexpr int kPartBits = 6;

__global__ void __launch_bounds__(kPartBlock) PartHistKernel(const uint8_t* __restrict__ digit, uint64_t n,
                                                             uint32_t* __restrict__ hist, uint32_t nblocks) {
  __shared__ uint32_t h[kPartBuckets];
  if (threadIdx.x < kPartBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kPartTile;
  for (int k = 0; k < kPartItems; ++k) {
    const uint64_t i = base + static_cast<uint64_t>(k) * kPartBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[digit[i]], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kPartBuckets) hist[static_cast<uint64_t>(threadIdx.x) * nblocks + blockIdx.x] = h[threadIdx.x];
}

__global__ void __launch_bounds__(kPartBlock) PartScatterKernel(const uint8_t* __restrict__ digit, uint64_t n,
                                                                const uint32_t* __restrict__ offs, uint32_t nblocks,
                                                                uint32_t* __restrict__ out) {
  __shared__ uint32_t running[kPartBuckets];
  __shared__ uint32_t wcnt[kPartBlock / 64][kPartBuckets];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  if (threadIdx.x < kPartBuckets) running[threadIdx.x] = offs[static_cast<uint64_t>(threadIdx.x) * nblocks + blockIdx.x];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kPartTile;
  for (int k = 0; k < kPartItems; ++k) {
    for (int i = threadIdx.x; i < (kPartBlock / 64) * kPartBuckets; i += kPartBlock) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t i = base + static_cast<uint64_t>(k) * kPartBlock + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = valid ? digit[i] : 0u;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kPartBits; ++b) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long m = __ballot(valid && bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t rank = static_cast<uint32_t>(__popcll(peers & lanemask_lt));
    if (valid && rank == 0) wcnt[wid][d] = static_cast<uint32_t>(__popcll(peers));
    __syncthreads();
    if (valid) {
      uint32_t pre = 0;
      for (int w = 0; w < wid; ++w) pre += wcnt[w][d];
      out[running[d] + pre + rank] = static_cast<uint32_t>(i);
    }
    __syncthreads();
    if (threadIdx.x < kPartBuckets) {
      uint32_t s = 0;
      for (int w = 0; w < kPartBlock / 64; ++w) s += wcnt[w][threadIdx.x];
      running[threadIdx.x] += s;
    }
    __syncthreads();
  }
}

// starts[b] = first output position of bucket b (b <= kPartBuckets; starts[64] = n).
__global__ void PartStartsKernel(const uint32_t* __restrict__ scanned, uint32_t nblocks, uint64_t n, uint64_t* __restrict__ starts) {
  const int b = threadIdx.x;
  if (b < kPartBuckets) starts[b] = scanned[static_cast<uint64_t>(b) * nblocks];
  if (b == kPartBuckets) starts[b] = n;
}

// ---------------------------------------------------------------------------------------
// Export kernels.
// ---------------------------------------------------------------------------------------
__global__ void SlotPartKernel(const AggPlanDev* __restrict__ plan, const unsigned long long* __restrict__ slots, uint32_t cap,
                               const uint64_t* __restrict__ arena, uint32_t n_parts, uint8_t* __restrict__ part_of,
                               uint32_t* __restrict__ words) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap) return;
  const unsigned long long w = slots[s];
  if (w == 0) {
    part_of[s] = kMaxParts;
    words[s] = 0;
    return;
  }
  KeySet k;
  LoadKeysArena(plan, arena + static_cast<uint32_t>(w), k);
  part_of[s] = static_cast<uint8_t>(PartOfHash(HashKeys(plan, k), n_parts));
  words[s] = KeyRecordWords(plan, k);
}

// Sorted group list -> per-group key-record words (for the offset scan) and each slot's rank
// within its part.
__global__ void GroupRankKernel(const uint32_t* __restrict__ slist, uint64_t ng, const uint8_t* __restrict__ part_of,
                                const uint32_t* __restrict__ words, const uint64_t* __restrict__ gstarts,
                                uint64_t* __restrict__ kw, uint32_t* __restrict__ grank) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= ng) return;
  const uint32_t s = slist[j];
  kw[j] = words[s];
  grank[s] = static_cast<uint32_t>(j - gstarts[part_of[s]]);
}

__global__ void RowDigitKernel(const uint32_t* __restrict__ st_slot, uint64_t n, uint32_t cap, const uint8_t* __restrict__ part_of,
                               uint8_t* __restrict__ digit) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = st_slot[i];
  digit[i] = s < cap ? part_of[s] : static_cast<uint8_t>(kMaxParts);
}

struct PartDst {
  uint8_t* base;           // dst buffer
  const uint64_t* poff;    // [n_parts] byte offset of each part in dst
  const uint64_t* layout;  // [n_parts][4] koff, keys, gid, vals section offsets within the part
  const uint64_t* nrows;   // [n_parts] rows per part (vals stride)
};

__global__ void WriteGroupsKernel(const uint32_t* __restrict__ slist, uint64_t ng, const uint8_t* __restrict__ part_of,
                                  const uint64_t* __restrict__ gstarts, const uint64_t* __restrict__ koff_g,
                                  const unsigned long long* __restrict__ slots, const uint64_t* __restrict__ arena,
                                  const uint32_t* __restrict__ words, PartDst dst) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= ng) return;
  const uint32_t s = slist[j];
  const uint32_t p = part_of[s];
  const uint64_t local = j - gstarts[p];
  const uint64_t kbase = koff_g[gstarts[p]];
  const uint64_t rel = koff_g[j] - kbase;
  uint8_t* part = dst.base + dst.poff[p];
  reinterpret_cast<uint64_t*>(part + dst.layout[p * 4 + 0])[local] = rel;
  uint64_t* keys = reinterpret_cast<uint64_t*>(part + dst.layout[p * 4 + 1]) + rel;
  const uint64_t* rec = arena + static_cast<uint32_t>(slots[s]);
  const uint32_t nw = words[s];
  for (uint32_t w = 0; w < nw; ++w) keys[w] = rec[w];
}

struct ConstVals {
  const uint64_t* p[kMaxVals];
};

__global__ void WriteRowsKernel(const uint32_t* __restrict__ rlist, uint64_t nr, const uint32_t* __restrict__ st_slot,
                                const uint8_t* __restrict__ part_of, const uint32_t* __restrict__ grank,
                                const uint64_t* __restrict__ rstarts, ConstVals vals, int n_vals, PartDst dst) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= nr) return;
  const uint32_t i = rlist[j];
  const uint32_t s = st_slot[i];
  const uint32_t p = part_of[s];
  const uint64_t local = j - rstarts[p];
  uint8_t* part = dst.base + dst.poff[p];
  reinterpret_cast<uint32_t*>(part + dst.layout[p * 4 + 2])[local] = grank[s];
  uint64_t* v0 = reinterpret_cast<uint64_t*>(part + dst.layout[p * 4 + 3]);
  const uint64_t stride = dst.nrows[p];
  for (int v = 0; v < n_vals; ++v) v0[static_cast<uint64_t>(v) * stride + local] = vals.p[v][i];
}

// ---------------------------------------------------------------------------------------
// Import kernels.
// ---------------------------------------------------------------------------------------
// Find-or-insert an arena key record (kind-1 slot word).  The caller sized the table so that
// it stays <= 25% full: the probe always terminates at an empty or matching slot.
__global__ void ImportKeysKernel(const AggPlanDev* __restrict__ plan, unsigned long long* __restrict__ slots, uint32_t mask,
                                 const uint64_t* __restrict__ arena, uint64_t base, const uint64_t* __restrict__ koff, uint64_t ng,
                                 uint32_t* __restrict__ remap, unsigned int* __restrict__ n_inserted,
                                 unsigned int* __restrict__ err) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  const uint64_t at = base + koff[g];
  KeySet k;
  LoadKeysArena(plan, arena + at, k);
  const uint64_t h = HashKeys(plan, k);
  const uint32_t tag = SlotTag(h);
  const unsigned long long desired = MakeSlotWord(tag, kKindArena, static_cast<uint32_t>(at));
  uint32_t pos = static_cast<uint32_t>(h) & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    unsigned long long w = __hip_atomic_load(&slots[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == 0) {
      unsigned long long expected = 0;
      if (__hip_atomic_compare_exchange_strong(&slots[pos], &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        atomicAdd(n_inserted, 1u);
        remap[g] = pos;
        return;
      }
      w = expected;
    }
    if (static_cast<uint32_t>(w >> 33) == tag) {
      KeySet rep;
      LoadKeysArena(plan, arena + static_cast<uint32_t>(w), rep);
      if (KeysEqual(plan, k, rep)) {
        remap[g] = pos;
        return;
      }
    }
    pos = (pos + 1) & mask;
  }
  atomicOr(err, 1u);
  remap[g] = kDeferredSlot;
}

__global__ void ImportRowsKernel(const uint32_t* __restrict__ gid, uint64_t nr, uint64_t ng, const uint32_t* __restrict__ remap,
                                 uint32_t* __restrict__ st_slot, unsigned int* __restrict__ err) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  const uint32_t g = gid[i];
  if (g >= ng) {
    atomicOr(err, 2u);
    st_slot[i] = kDeferredSlot;
    return;
  }
  st_slot[i] = remap[g];
}

// ---------------------------------------------------------------------------------------
// Host side.
// ---------------------------------------------------------------------------------------
static int32_t Partition(Ctx* ctx, const uint8_t* digit, uint64_t n, uint32_t* out, uint64_t* d_starts, DevBuf* hist, DevBuf* scan) {
  const uint32_t nblocks = static_cast<uint32_t>(std::max<uint64_t>(1, (n + kPartTile - 1) / kPartTile));
  const uint64_t nh = static_cast<uint64_t>(kPartBuckets) * nblocks;
  PXG_RETURN_IF_ERROR(hist->Ensure(nh * 4 + 64));
  PXG_RETURN_IF_ERROR(scan->Ensure(ScanScratchBytes(static_cast<int64_t>(nh)) + 64));
  if (n > 0) {
    PXG_RETURN_IF_ERROR(Launch(ctx, "part_hist", PartHistKernel, dim3(nblocks), dim3(kPartBlock), 0, digit, n, hist->as<uint32_t>(), nblocks));
  } else {
    PXG_HIP(hipMemsetAsync(hist->p, 0, nh * 4, ctx->stream));
  }
  PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, hist->as<uint32_t>(), hist->as<uint32_t>(), static_cast<int64_t>(nh), nullptr, scan->p));
  if (n > 0)
    PXG_RETURN_IF_ERROR(Launch(ctx, "part_scatter", PartScatterKernel, dim3(nblocks), dim3(kPartBlock), 0, digit, n,
                               hist->as<const uint32_t>(), nblocks, out));
  return Launch(ctx, "part_starts", PartStartsKernel, dim3(1), dim3(128), 0, hist->as<const uint32_t>(), nblocks, n, d_starts);
}

int32_t Agg::PrepareExport(int32_t n_parts) {
  ExportCache& X = xc;
  if (X.valid && X.n_parts == n_parts && X.version == state_version) return PXG_OK;
  X.valid = false;
  const uint64_t n = st_n;
  PXG_RETURN_IF_ERROR(X.part_of.Ensure(cap + 16));
  PXG_RETURN_IF_ERROR(X.words.Ensure(static_cast<size_t>(cap) * 4 + 16));
  PXG_RETURN_IF_ERROR(X.slist.Ensure(static_cast<size_t>(cap) * 4 + 16));
  PXG_RETURN_IF_ERROR(X.grank.Ensure(static_cast<size_t>(cap) * 4 + 16));
  PXG_RETURN_IF_ERROR(X.starts.Ensure(2 * (kPartBuckets + 1) * 8 + 64));
  uint64_t* gstarts = X.starts.as<uint64_t>();
  uint64_t* rstarts = gstarts + kPartBuckets + 1;
  PXG_RETURN_IF_ERROR(Launch(ctx, "export_slot_part", SlotPartKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0,
                             d_plan.as<const AggPlanDev>(), slots.as<const unsigned long long>(), cap, arena.as<const uint64_t>(),
                             static_cast<uint32_t>(n_parts), X.part_of.as<uint8_t>(), X.words.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(Partition(ctx, X.part_of.as<const uint8_t>(), cap, X.slist.as<uint32_t>(), gstarts, &X.hist, &X.scan));
  // Occupied slots come first (parts 0..n_parts-1), then the empty-slot sentinel bucket.
  uint64_t hg[kPartBuckets + 1];
  PXG_HIP(hipMemcpyAsync(hg, gstarts, sizeof(hg), hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  const uint64_t ng = hg[n_parts];
  PXG_RETURN_IF_ERROR(X.koff.Ensure((ng + 1) * 8 + 64));
  PXG_RETURN_IF_ERROR(X.scan2.Ensure(ScanScratchBytes(static_cast<int64_t>(ng + 1)) + 64));
  uint64_t* koff = X.koff.as<uint64_t>();
  if (ng > 0) {
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_group_rank", GroupRankKernel, dim3(GridFor(static_cast<int64_t>(ng), 256, 1 << 30)), dim3(256), 0,
                               X.slist.as<const uint32_t>(), ng, X.part_of.as<const uint8_t>(), X.words.as<const uint32_t>(), gstarts, koff,
                               X.grank.as<uint32_t>()));
  }
  PXG_RETURN_IF_ERROR(ScanExclusiveU64(ctx, koff, koff, static_cast<int64_t>(ng), koff + ng, X.scan2.p));
  // Rows.
  PXG_RETURN_IF_ERROR(X.rdigit.Ensure(n + 16));
  PXG_RETURN_IF_ERROR(X.rlist.Ensure(n * 4 + 16));
  if (n > 0)
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_row_digit", RowDigitKernel, dim3(GridFor(static_cast<int64_t>(n), 256, 1 << 30)), dim3(256), 0,
                               st_slot.as<const uint32_t>(), n, cap, X.part_of.as<const uint8_t>(), X.rdigit.as<uint8_t>()));
  PXG_RETURN_IF_ERROR(Partition(ctx, X.rdigit.as<const uint8_t>(), n, X.rlist.as<uint32_t>(), rstarts, &X.hist, &X.scan));
  // Key-word totals at each part boundary.
  std::vector<uint64_t> kstart(n_parts + 1);
  uint64_t hr[kPartBuckets + 1];
  PXG_HIP(hipMemcpyAsync(hr, rstarts, sizeof(hr), hipMemcpyDeviceToHost, ctx->stream));
  for (int p = 0; p <= n_parts; ++p) PXG_HIP(hipMemcpyAsync(&kstart[p], koff + hg[p], 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  X.g_start.assign(hg, hg + n_parts + 1);
  X.r_start.assign(hr, hr + n_parts + 1);
  X.k_start = kstart;
  X.n_parts = n_parts;
  X.version = state_version;
  X.valid = true;
  return PXG_OK;
}

int32_t Agg::ExportPartial(int32_t n_parts, void* dst, int64_t dst_capacity, int64_t* part_offsets, int64_t* part_bytes) {
  PXG_RETURN_IF_ERROR(PrepareExport(n_parts));
  ExportCache& X = xc;
  std::vector<PartHeader> hdr(n_parts);
  std::vector<uint64_t> poff(n_parts), lay(4 * n_parts), nrows(n_parts);
  uint64_t off = 0;
  const uint64_t sig = PlanSig(*this);
  for (int p = 0; p < n_parts; ++p) {
    const uint64_t ng = X.g_start[p + 1] - X.g_start[p];
    const uint64_t nr = X.r_start[p + 1] - X.r_start[p];
    const uint64_t kw = X.k_start[p + 1] - X.k_start[p];
    const PartLayout L = LayoutOf(ng, nr, kw, n_vals);
    PartHeader& H = hdr[p];
    std::memset(&H, 0, sizeof(H));
    H.magic = kPartMagic;
    H.version = kPartVersion;
    H.n_keys = static_cast<uint32_t>(n_keys);
    H.n_vals = static_cast<uint32_t>(n_vals);
    H.n_groups = ng;
    H.n_rows = nr;
    H.key_words = kw;
    H.plan_sig = sig;
    poff[p] = off;
    lay[4 * p + 0] = L.koff;
    lay[4 * p + 1] = L.keys;
    lay[4 * p + 2] = L.gid;
    lay[4 * p + 3] = L.vals;
    nrows[p] = nr;
    part_offsets[p] = static_cast<int64_t>(off);
    part_bytes[p] = static_cast<int64_t>(L.bytes);
    off += Align8(L.bytes);
  }
  if (dst == nullptr) return PXG_OK;
  if (static_cast<uint64_t>(dst_capacity) < off)
    return SetError(PXG_INVALID_ARGUMENT, "export buffer holds %lld bytes; %llu needed", (long long)dst_capacity, (unsigned long long)off);
  // Part descriptors -> device (one small staging copy, kept alive until the sync below).
  std::vector<uint64_t> desc;
  desc.insert(desc.end(), poff.begin(), poff.end());
  desc.insert(desc.end(), lay.begin(), lay.end());
  desc.insert(desc.end(), nrows.begin(), nrows.end());
  PXG_RETURN_IF_ERROR(X.desc.Ensure(desc.size() * 8 + 64));
  PXG_HIP(hipMemcpyAsync(X.desc.p, desc.data(), desc.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  uint8_t* base = static_cast<uint8_t*>(dst);
  for (int p = 0; p < n_parts; ++p)
    PXG_HIP(hipMemcpyAsync(base + poff[p], &hdr[p], sizeof(PartHeader), hipMemcpyHostToDevice, ctx->stream));
  PartDst D;
  D.base = base;
  D.poff = X.desc.as<const uint64_t>();
  D.layout = D.poff + n_parts;
  D.nrows = D.layout + 4 * n_parts;
  const uint64_t ng = X.g_start[n_parts];
  const uint64_t nr = X.r_start[n_parts];
  const uint64_t* gstarts = X.starts.as<const uint64_t>();
  const uint64_t* rstarts = gstarts + kPartBuckets + 1;
  if (ng > 0)
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_write_groups", WriteGroupsKernel, dim3(GridFor(static_cast<int64_t>(ng), 256, 1 << 30)), dim3(256), 0,
                               X.slist.as<const uint32_t>(), ng, X.part_of.as<const uint8_t>(), gstarts, X.koff.as<const uint64_t>(),
                               slots.as<const unsigned long long>(), arena.as<const uint64_t>(), X.words.as<const uint32_t>(), D));
  if (nr > 0) {
    ConstVals cv;
    for (int v = 0; v < kMaxVals; ++v) cv.p[v] = v < n_vals ? st_val[v].as<const uint64_t>() : nullptr;
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_write_rows", WriteRowsKernel, dim3(GridFor(static_cast<int64_t>(nr), 256, 1 << 30)), dim3(256), 0,
                               X.rlist.as<const uint32_t>(), nr, st_slot.as<const uint32_t>(), X.part_of.as<const uint8_t>(),
                               X.grank.as<const uint32_t>(), rstarts, cv, n_vals, D));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}

// Merge n exported parts (part i at src + offs[i], sizes[i] bytes) in one pass: every header is
// read back with one synchronisation, the arena / table / staging are sized once for all of
// them, each part's keys and rows are imported by its own kernels, and one final readback
// collects the insert count and error flags -- two host round trips for any number of parts.
int32_t Agg::ImportPartials(const void* src, int32_t n, const int64_t* offs, const int64_t* sizes) {
  if (n <= 0) return PXG_OK;
  std::vector<PartHeader> H(static_cast<size_t>(n));
  const uint8_t* base8 = static_cast<const uint8_t*>(src);
  for (int i = 0; i < n; ++i) {
    if (sizes[i] < static_cast<int64_t>(sizeof(PartHeader)))
      return SetError(PXG_INVALID_ARGUMENT, "partial buffer of %lld bytes has no header", (long long)sizes[i]);
    PXG_HIP(hipMemcpyAsync(&H[i], base8 + offs[i], sizeof(PartHeader), hipMemcpyDeviceToHost, ctx->stream));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  // Exchange v2 parts (partial states) have their own header and merge.
  int nx = 0;
  for (int i = 0; i < n; ++i) nx += IsXPart(&H[i]) ? 1 : 0;
  if (nx == n) {
    std::vector<XHeader> XH(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) std::memcpy(&XH[i], &H[i], sizeof(XHeader));
    return ImportPartialsV2(base8, n, offs, sizes, XH.data());
  }
  if (nx > 0) return SetError(PXG_INVALID_ARGUMENT, "row parts and partial-state parts cannot be imported together");
  if (merged) return SetError(PXG_FAILED_PRECONDITION, "row parts cannot join an aggregation that merged partial states");
  uint64_t tot_groups = 0, tot_rows = 0, tot_words = 0;
  std::vector<PartLayout> L(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    const PartHeader& h = H[i];
    if (h.magic != kPartMagic || h.version != kPartVersion)
      return SetError(PXG_INVALID_ARGUMENT, "not a pxg partial-agg buffer (magic %08x version %u)", h.magic, h.version);
    if (h.plan_sig != PlanSig(*this) || h.n_keys != static_cast<uint32_t>(n_keys) || h.n_vals != static_cast<uint32_t>(n_vals))
      return SetError(PXG_INVALID_ARGUMENT, "partial buffer was exported by an aggregation with different key/value types");
    L[i] = LayoutOf(h.n_groups, h.n_rows, h.key_words, n_vals);
    if (static_cast<uint64_t>(sizes[i]) < L[i].bytes)
      return SetError(PXG_INVALID_ARGUMENT, "partial buffer truncated: %lld of %llu bytes", (long long)sizes[i], (unsigned long long)L[i].bytes);
    if (h.n_groups == 0 && h.n_rows != 0) return SetError(PXG_INVALID_ARGUMENT, "partial buffer has rows but no groups");
    tot_groups += h.n_groups;
    tot_rows += h.n_rows;
    tot_words += h.key_words;
  }
  state_version++;
  res.ready = false;
  if (tot_groups == 0) return PXG_OK;
  // Keys -> arena (all parts back to back), then find-or-insert.  The table is sized for <= 25%
  // fill after the import.
  const uint64_t abase = arena_words;
  if (abase + tot_words >= (uint64_t(1) << 32)) return SetError(PXG_RESOURCE_UNAVAILABLE, "key arena exceeds 32 GiB");
  PXG_RETURN_IF_ERROR(arena.Reserve((abase + tot_words) * 8 + kArenaSlack, abase * 8, ctx->stream));
  uint64_t want = 4 * (inserted + tot_groups);
  if (want > cap) {
    uint64_t c = cap;
    while (c < want) c <<= 1;
    if (c > (uint64_t(1) << 31)) return SetError(PXG_RESOURCE_UNAVAILABLE, "group table would exceed 2^31 slots");
    PXG_RETURN_IF_ERROR(Grow(static_cast<uint32_t>(c)));
  }
  PXG_RETURN_IF_ERROR(xc.remap.Ensure(tot_groups * 4 + 16));
  if (tot_rows > 0) PXG_RETURN_IF_ERROR(EnsureStage(st_n + tot_rows));
  uint8_t* meta = counters.as<uint8_t>();
  unsigned int* d_ins = reinterpret_cast<unsigned int*>(meta + 32);
  unsigned int* d_err = reinterpret_cast<unsigned int*>(meta + 36);
  PXG_HIP(hipMemsetAsync(meta + 32, 0, 8, ctx->stream));
  uint64_t kw = abase, g0 = 0, r0 = st_n;
  for (int i = 0; i < n; ++i) {
    const PartHeader& h = H[i];
    const uint8_t* p = base8 + offs[i];
    if (h.n_groups == 0) continue;
    uint32_t* remap = xc.remap.as<uint32_t>() + g0;
    PXG_HIP(hipMemcpyAsync(arena.as<uint64_t>() + kw, p + L[i].keys, h.key_words * 8, hipMemcpyDeviceToDevice, ctx->stream));
    PXG_RETURN_IF_ERROR(Launch(ctx, "import_keys", ImportKeysKernel, dim3(GridFor(static_cast<int64_t>(h.n_groups), 256, 1 << 30)), dim3(256), 0,
                               d_plan.as<const AggPlanDev>(), slots.as<unsigned long long>(), cap - 1, arena.as<const uint64_t>(), kw,
                               reinterpret_cast<const uint64_t*>(p + L[i].koff), h.n_groups, remap, d_ins, d_err));
    if (h.n_rows > 0) {
      PXG_RETURN_IF_ERROR(Launch(ctx, "import_rows", ImportRowsKernel, dim3(GridFor(static_cast<int64_t>(h.n_rows), 256, 1 << 30)), dim3(256), 0,
                                 reinterpret_cast<const uint32_t*>(p + L[i].gid), h.n_rows, h.n_groups,
                                 static_cast<const uint32_t*>(remap), st_slot.as<uint32_t>() + r0, d_err));
      for (int v = 0; v < n_vals; ++v)
        PXG_HIP(hipMemcpyAsync(st_val[v].as<uint64_t>() + r0, p + L[i].vals + static_cast<uint64_t>(v) * h.n_rows * 8, h.n_rows * 8,
                               hipMemcpyDeviceToDevice, ctx->stream));
    }
    kw += h.key_words;
    g0 += h.n_groups;
    r0 += h.n_rows;
  }
  arena_words = kw;
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + 240);
  PXG_HIP(hipMemcpyAsync(pin, meta + 32, 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  const uint32_t r_ins = pin[0], r_err = pin[1];
  if (r_err & 1u) return SetError(PXG_INTERNAL, "group table full during partial import");
  if (r_err & 2u) return SetError(PXG_INVALID_ARGUMENT, "partial buffer has a row whose group index is out of range");
  inserted += r_ins;
  st_n += tot_rows;
  // Keep the device fill counter and staging cursor exact (the consume kernel reads both).
  uint64_t* pin64 = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(ctx->pinned) + 248);
  *pin64 = st_n;
  PXG_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(counters.p), static_cast<int>(inserted), 1, ctx->stream));
  PXG_HIP(hipMemcpyAsync(counters.as<uint8_t>() + 16, pin64, 8, hipMemcpyHostToDevice, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}

int32_t Agg::ImportPartial(const void* src, int64_t nbytes) {
  const int64_t off = 0;
  return ImportPartials(src, 1, &off, &nbytes);
}

// ---------------------------------------------------------------------------------------
// Exchange v2: partial UDA states (partial_op_mgr.cc:69-83, math_ops.h:590-609,
// math_sketches.h:38).  Per group a part carries the group's key record, its Serialize() state
// record (count / sum / min / max 8 bytes, MeanInfo {size, sum} 16 bytes; hplan_x), and its
// quantile contribution: the raw values when this rank holds <= 8 * delta of them (kept
// bit-exact: a group of <= 8000 values anywhere is <= 8000 on every rank), else the centroid
// list of its single-pass digest (<= 2 * delta centroids; CentroidListKernel).  The owner merges
// states into per-slot accumulators and digests with DigestMergeKernel (pxg_finalize.hip).
//
// Part layout (8-byte aligned sections):
//   XHeader (64 B) | koff u64[G] | keys u64[KW] | states u8[G * state_rec] | gid u32[I] (pad) |
//   vals u64[I] | wts u64[I]   (wts: centroid weight, 0 for a raw value)
// ---------------------------------------------------------------------------------------


// Part layout: header, per group its key record offset (words), the key records, the state
// records, per group its items' start (kXItemShift: item index, low 32 bits: word, bit 63: the
// items are centroids) plus one end entry, then the items: a raw value is one word, a centroid
// two (mean bits, weight).  Raw values (the common case, groups <= 8 * delta values) thus cost
// 8 bytes each, as little as a shipped row value.
constexpr int kXItemShift = 32;
constexpr uint64_t kXCentFlag = uint64_t(1) << 63;
struct XLayout {
  uint64_t koff, keys, states, gofs, items, bytes;
};
__host__ __device__ static XLayout XLayoutOf(uint64_t ng, uint64_t nw, uint64_t kw, uint64_t srec, bool has_q) {
  XLayout L;
  L.koff = sizeof(XHeader);
  L.keys = L.koff + ng * 8;
  L.states = L.keys + kw * 8;
  L.gofs = L.states + Align8(ng * srec);
  L.items = L.gofs + (has_q ? (ng + 1) * 8 : 0);
  L.bytes = L.items + (has_q ? nw * 8 : 0);
  return L;
}

static uint64_t XPlanSig(const Agg& a) {
  uint64_t h = PlanSig(a) ^ 0x9E3779B97F4A7C15ULL;
  for (int u = 0; u < a.n_udas; ++u) h = (h ^ static_cast<uint64_t>(a.uda_kind[u] * 31 + a.uda_arg_type[u])) * 1099511628211ULL;
  return h;
}

__global__ void XBigIndexKernel(const uint32_t* __restrict__ big_g, uint32_t nbig, int32_t* __restrict__ xbig) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nbig) xbig[big_g[b]] = static_cast<int32_t>(b);
}

// Per dense group: its part, key-record words and item count.
__global__ void XGroupPartKernel(const AggPlanDev* __restrict__ plan, const unsigned long long* __restrict__ slots,
                                 const uint32_t* __restrict__ gslot, uint32_t G, const uint64_t* __restrict__ arena, uint32_t n_parts,
                                 const uint32_t* __restrict__ gstart, const int32_t* __restrict__ xbig, const int32_t* __restrict__ xcnt,
                                 int has_q, uint8_t* __restrict__ gpart, uint64_t* __restrict__ kw, uint64_t* __restrict__ ic) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  KeySet k;
  LoadKeysArena(plan, arena + static_cast<uint32_t>(slots[gslot[g]]), k);
  gpart[g] = static_cast<uint8_t>(PartOfHash(HashKeys(plan, k), n_parts));
  kw[g] = KeyRecordWords(plan, k);
  uint64_t items = 0, words = 0;
  if (has_q) {
    const int32_t b = xbig ? xbig[g] : -1;
    const int32_t nc = b >= 0 ? xcnt[b] : -1;
    items = nc > 0 ? static_cast<uint64_t>(nc) : (nc == 0 ? 1 : gstart[g + 1] - gstart[g]);
    words = nc > 0 ? 2 * items : items;
  }
  ic[g] = (items << kXItemShift) | words;  // both fields scanned at once (no carry: words < 2^32)
}

struct XDst {
  uint8_t* base;
  const uint64_t* poff;    // [n_parts] byte offset of each part
  const uint64_t* layout;  // [n_parts][6] koff, keys, states, gofs, items, -
  const uint64_t* nitems;  // [n_parts]
  const int64_t* fail;     // device layout: seg[0] < 0 = the layout refused the export (nothing written)
};

// One wave per listed group (part order): key record, state record, items.
__global__ void XWriteGroupsKernel(const uint32_t* __restrict__ glist, uint64_t ng, const uint8_t* __restrict__ gpart,
                                   const uint64_t* __restrict__ gstarts, const uint64_t* __restrict__ koff_j, const uint64_t* __restrict__ ioff_j,
                                   const unsigned long long* __restrict__ slots, const uint32_t* __restrict__ gslot,
                                   const uint64_t* __restrict__ arena, const AggPlanDev* __restrict__ plan, const uint8_t* __restrict__ states,
                                   uint32_t srec, const uint32_t* __restrict__ gstart, const uint64_t* __restrict__ vals,
                                   const int32_t* __restrict__ xbig, const int32_t* __restrict__ xcnt, const uint64_t* __restrict__ xcent,
                                   int has_q, XDst dst) {
  const uint64_t j = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (j >= ng) return;
  if (dst.fail && dst.fail[0] < 0) return;
  const uint32_t g = glist[j];
  const uint32_t p = gpart[g];
  const uint64_t local = j - gstarts[p];
  uint8_t* part = dst.base + dst.poff[p];
  const uint64_t* L = dst.layout + 6 * p;
  const uint64_t k0 = koff_j[gstarts[p]], i0 = ioff_j[gstarts[p]];
  const uint64_t krel = koff_j[j] - k0, irel = ioff_j[j] - i0;
  const uint64_t* rec = arena + static_cast<uint32_t>(slots[gslot[g]]);
  const uint64_t nkw = koff_j[j + 1] - koff_j[j];
  if (lane == 0) reinterpret_cast<uint64_t*>(part + L[0])[local] = krel;
  for (uint64_t w = lane; w < nkw; w += 64) reinterpret_cast<uint64_t*>(part + L[1])[krel + w] = rec[w];
  for (uint32_t b = lane; b < srec; b += 64) part[L[2] + local * srec + b] = states[static_cast<uint64_t>(g) * srec + b];
  if (!has_q) return;
  const int32_t b = xbig ? xbig[g] : -1;
  const int32_t nc = b >= 0 ? xcnt[b] : -1;
  uint64_t* gofs = reinterpret_cast<uint64_t*>(part + L[3]);
  if (lane == 0) {
    gofs[local] = irel | (nc > 0 ? kXCentFlag : 0);
    if (j + 1 == gstarts[p + 1]) gofs[local + 1] = ioff_j[j + 1] - i0;  // the part's end entry
  }
  uint64_t* ov = reinterpret_cast<uint64_t*>(part + L[4]) + (irel & 0xFFFFFFFFu);
  const uint64_t nw = (ioff_j[j + 1] - ioff_j[j]) & 0xFFFFFFFFu;
  if (nc > 0) {  // the centroid list: (mean bits, weight) pairs
    const uint64_t* c = xcent + static_cast<uint64_t>(b) * kXCentCapH * 2;
    for (uint64_t w = lane; w < nw; w += 64) ov[w] = c[w];
  } else if (nc == 0) {  // every value NaN: one NaN stands for the group (add() skips it)
    if (lane == 0) ov[0] = 0x7FF8000000000000ULL;
  } else {
    for (uint64_t i = lane; i < nw; i += 64) ov[i] = vals[gstart[g] + i];
  }
}

// Owner side: per-slot state accumulators (macc_words u64 per slot: each UDA's words at its
// offset, then a flags word), initialised to every UDA's identity.
struct UdaOutX {
  uint64_t* p[kMaxUdas];
};

struct XAccPlan {
  int32_t n_udas, words;
  int32_t kind[kMaxUdas], at[kMaxUdas], off[kMaxUdas], soff[kMaxUdas];
  int64_t init[kMaxUdas];
};

__device__ __forceinline__ uint64_t XAccInit(int kind, int at) {
  if (kind == PXG_UDA_MIN) return at == PXG_FLOAT64 ? static_cast<uint64_t>(OrderedFromDouble(FBits(kDblMax))) : static_cast<uint64_t>(INT64_MAX);
  if (kind == PXG_UDA_MAX) return at == PXG_FLOAT64 ? static_cast<uint64_t>(OrderedFromDouble(FBits(kDblMin))) : static_cast<uint64_t>(INT64_MIN);
  return 0;
}

__global__ void XAccInitKernel(XAccPlan xp, uint64_t* __restrict__ macc, uint32_t cap) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  uint64_t* r = macc + i * xp.words;
  for (int w = 0; w < xp.words; ++w) r[w] = 0;
  for (int u = 0; u < xp.n_udas; ++u)
    if (xp.off[u] >= 0) r[xp.off[u]] = XAccInit(xp.kind[u], xp.at[u]);
}

__global__ void XAccRemapKernel(XAccPlan xp, const unsigned long long* __restrict__ old_slots, uint32_t old_cap,
                                const uint32_t* __restrict__ remap, const uint64_t* __restrict__ src, uint64_t* __restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap || old_slots[i] == 0) return;
  const uint64_t* a = src + static_cast<uint64_t>(i) * xp.words;
  uint64_t* b = dst + static_cast<uint64_t>(remap[i]) * xp.words;
  for (int w = 0; w < xp.words; ++w) b[w] = a[w];
}

// Merge one part's state records into the accumulators (UDA Merge, math_ops.h:590-593 count,
// 633 sum, 668-672 mean, 710-714 min, 747 max).  INT64 sums wrap as the reference's do; float
// sums and mean sums are added in arrival order (within the 1e-6 bar).
__global__ void XImportStatesKernel(XAccPlan xp, const uint8_t* __restrict__ states, uint32_t srec, uint64_t ng,
                                    const uint32_t* __restrict__ remap, uint64_t* __restrict__ macc) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  const uint32_t slot = remap[g];
  if (slot == kDeferredSlot) return;
  uint64_t* r = macc + static_cast<uint64_t>(slot) * xp.words;
  const uint8_t* st = states + g * srec;
  for (int u = 0; u < xp.n_udas; ++u) {
    const int o = xp.off[u];
    if (o < 0) continue;
    uint64_t v0, v1 = 0;
    __builtin_memcpy(&v0, st + xp.soff[u], 8);
    switch (xp.kind[u]) {
      case PXG_UDA_COUNT: atomicAdd(reinterpret_cast<unsigned long long*>(r + o), static_cast<unsigned long long>(v0)); break;
      case PXG_UDA_SUM:
        if (xp.at[u] == PXG_FLOAT64) atomicAdd(reinterpret_cast<double*>(r + o), AsF(v0));
        else atomicAdd(reinterpret_cast<unsigned long long*>(r + o), static_cast<unsigned long long>(v0));
        break;
      case PXG_UDA_MEAN:  // MeanInfo {uint64 size; double sum}
        __builtin_memcpy(&v1, st + xp.soff[u] + 8, 8);
        atomicAdd(reinterpret_cast<unsigned long long*>(r + o), static_cast<unsigned long long>(v0));
        atomicAdd(reinterpret_cast<double*>(r + o + 1), AsF(v1));
        break;
      case PXG_UDA_MIN:
        atomicMin(reinterpret_cast<long long*>(r + o), xp.at[u] == PXG_FLOAT64 ? OrderedFromDouble(v0) : static_cast<long long>(v0));
        break;
      case PXG_UDA_MAX:
        atomicMax(reinterpret_cast<long long*>(r + o), xp.at[u] == PXG_FLOAT64 ? OrderedFromDouble(v0) : static_cast<long long>(v0));
        break;
      default: break;
    }
  }
}

// Items of one part -> staging weights (part index on top) and digest flags of their slots.
// One wave per imported group: its items into staging records (slot, value, part << 48 | weight;
// weight 0 = a raw value), and the digest flag of a slot that received centroids.
__global__ void XImportItemsKernel(const uint64_t* __restrict__ gofs, const uint64_t* __restrict__ items, uint64_t ng, uint64_t ni,
                                   uint64_t nw, const uint32_t* __restrict__ remap, uint64_t part, uint32_t* __restrict__ st_slot,
                                   uint64_t* __restrict__ st_val, uint64_t* __restrict__ st_wt, uint64_t* __restrict__ macc, int32_t words,
                                   unsigned int* __restrict__ err) {
  const uint64_t g = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (g >= ng) return;
  const uint64_t a = gofs[g], e = gofs[g + 1] & ~kXCentFlag;
  const bool cent = (a & kXCentFlag) != 0;
  const uint64_t i0 = (a & ~kXCentFlag) >> kXItemShift, i1 = e >> kXItemShift;
  const uint64_t w0 = a & 0xFFFFFFFFu, w1 = e & 0xFFFFFFFFu;
  if (i1 < i0 || i1 > ni || w1 < w0 || w1 > nw || (w1 - w0) != (cent ? 2 : 1) * (i1 - i0)) {
    if (lane == 0) atomicOr(err, 2u);
    return;
  }
  const uint32_t slot = remap[g];
  for (uint64_t i = lane; i < i1 - i0; i += 64) {
    st_slot[i0 + i] = slot;
    if (cent) {
      st_val[i0 + i] = items[w0 + 2 * i];
      st_wt[i0 + i] = (part << kXWtShift) | items[w0 + 2 * i + 1];
    } else {
      st_val[i0 + i] = items[w0 + i];
      st_wt[i0 + i] = part << kXWtShift;
    }
  }
  if (cent && lane == 0 && slot != kDeferredSlot)
    atomicOr(reinterpret_cast<unsigned long long*>(macc + static_cast<uint64_t>(slot) * words + words - 1),
             static_cast<unsigned long long>(kXFlagDigest));
}

// Plans without quantiles stage one placeholder item per imported group (so the grouping and
// the key output run as for any aggregation; every output is then taken from the accumulators).
__global__ void XPlaceholderKernel(const uint32_t* __restrict__ remap, uint64_t ng, uint32_t* __restrict__ st_slot,
                                   uint64_t* __restrict__ st_wt) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  st_slot[g] = remap[g];
  st_wt[g] = 0;
}

// Merged finalize: every non-quantile output from the accumulators of the group's slot, and the
// list of groups whose quantiles need the merged digest.
__global__ void XFinalizeStatesKernel(XAccPlan xp, const uint32_t* __restrict__ gslot, uint32_t G, const uint64_t* __restrict__ macc,
                                      UdaOutX out, uint32_t* __restrict__ dlist, uint32_t* __restrict__ dcount) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const uint64_t* r = macc + static_cast<uint64_t>(gslot[g]) * xp.words;
  for (int u = 0; u < xp.n_udas; ++u) {
    const int o = xp.off[u];
    if (o < 0) continue;
    uint64_t v = r[o];
    switch (xp.kind[u]) {
      case PXG_UDA_MEAN: v = FBits(AsF(r[o + 1]) / static_cast<double>(r[o])); break;
      case PXG_UDA_MIN:
      case PXG_UDA_MAX:
        if (xp.at[u] == PXG_FLOAT64) v = DoubleFromOrdered(static_cast<int64_t>(v));
        break;
      default: break;
    }
    out.p[u][g] = v;
  }
  if (dlist && (r[xp.words - 1] & kXFlagDigest)) dlist[atomicAdd(dcount, 1u)] = g;
}
static XAccPlan XAccPlanOf(const Agg& a) {
  XAccPlan xp;
  std::memset(&xp, 0, sizeof(xp));
  xp.n_udas = a.n_udas;
  xp.words = a.macc_words;
  for (int u = 0; u < a.n_udas; ++u) {
    xp.kind[u] = a.uda_kind[u];
    xp.at[u] = a.uda_arg_type[u];
    xp.off[u] = a.macc_off[u];
    xp.soff[u] = a.hplan_x.state_off[u];
    xp.init[u] = a.uda_init[u];
  }
  return xp;
}

bool ExchangeV2(const Agg& a) { return a.x_ok && !EnvFlag("PXG_XCHG_V1"); }
size_t XHeaderBytes() { return sizeof(XHeader); }

// Accumulators sized with the table (a fresh table: identities everywhere).
int32_t Agg::EnsureMacc() {
  if (macc_cap == cap) return PXG_OK;
  if (macc_cap != 0) return SetError(PXG_INTERNAL, "state accumulators out of step with the table");
  PXG_RETURN_IF_ERROR(macc.Ensure(static_cast<size_t>(cap) * macc_words * 8 + 64));
  PXG_RETURN_IF_ERROR(Launch(ctx, "import_states", XAccInitKernel, dim3(GridFor(cap, 256, 1 << 30)), dim3(256), 0, XAccPlanOf(*this),
                             macc.as<uint64_t>(), cap));
  macc_cap = cap;
  return PXG_OK;
}

// Grow() of a merged aggregation: its accumulator rows follow their slots.
int32_t MaccFollowGrow(Agg* a, const unsigned long long* old_slots, uint32_t old_cap, const uint32_t* remap, uint32_t new_cap) {
  if (!a->merged || a->macc_cap != old_cap) return PXG_OK;
  DevBuf nm;
  PXG_RETURN_IF_ERROR(nm.Alloc(static_cast<size_t>(new_cap) * a->macc_words * 8 + 64));
  const XAccPlan xp = XAccPlanOf(*a);
  PXG_RETURN_IF_ERROR(Launch(a->ctx, "import_states", XAccInitKernel, dim3(GridFor(new_cap, 256, 1 << 30)), dim3(256), 0, xp,
                             nm.as<uint64_t>(), new_cap));
  PXG_RETURN_IF_ERROR(Launch(a->ctx, "import_states", XAccRemapKernel, dim3(GridFor(old_cap, 256, 1 << 30)), dim3(256), 0, xp, old_slots,
                             old_cap, remap, a->macc.as<const uint64_t>(), nm.as<uint64_t>()));
  PXG_HIP(hipStreamSynchronize(a->ctx->stream));
  a->macc = std::move(nm);
  a->macc_cap = new_cap;
  return PXG_OK;
}

__global__ void XGatherU64Kernel(const uint32_t* __restrict__ idx, uint64_t n, const uint64_t* __restrict__ src, uint64_t* __restrict__ dst) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}
// Part boundaries of the group / key-word / item scans (one readback).
__global__ void XPartBoundsKernel(const uint64_t* __restrict__ gstarts, int n_parts, const uint64_t* __restrict__ koff_j,
                                  const uint64_t* __restrict__ ioff_j, uint64_t* __restrict__ out) {
  const int p = threadIdx.x;
  if (p > n_parts) return;
  const uint64_t j = gstarts[p];
  out[p] = j;
  out[n_parts + 1 + p] = koff_j[j];
  out[2 * (n_parts + 1) + p] = ioff_j[j];
}

// The export finalize's deferred checks (AggFinalizeTable ends an export without a host wait):
// `m` holds a host copy of ws.meta's first 24 bytes, taken after the stream passed the export.
int32_t Agg::CheckExportFinalize(const uint8_t* m) {
  if (!x_check_pending) return PXG_OK;  // (the finalize returned before its kernels: nothing staged)
  x_check_pending = false;
  uint32_t g_dev = 0, err = 0;
  std::memcpy(&g_dev, m + 8, 4);
  std::memcpy(&err, m + 16, 4);
  if (err) return SetError(PXG_INTERNAL, "t-digest centroid capacity exceeded");
  if (g_dev != x_check_groups) return SetError(PXG_INTERNAL, "group table holds %u groups, host mirror says %u", g_dev, x_check_groups);
  return PXG_OK;
}

// eslots[g] = the table slot word of table group g (its arena record offset in the low word).
__global__ void XTableSlotsKernel(const unsigned long long* __restrict__ slots, const uint32_t* __restrict__ gslot, uint32_t G,
                                  unsigned long long* __restrict__ eslots, uint32_t* __restrict__ egslot, uint32_t Gt) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < G) eslots[g] = slots[gslot[g]];
  if (g < Gt) egslot[g] = g;
}

// Export grouping (no host wait; the finalize waits once for its class counts when the plan has
// quantiles): the local finalize in export mode, each group's part, key-record words and items,
// the groups in part order, and per part (+ total) the group / key-word / item starts at
// xc.starts + kPartBuckets + 1 (device).
int32_t Agg::ExportGroupV2(int32_t n_parts) {
  ExportCache& X = xc;
  X.valid = false;
  const bool has_q = x_qval >= 0;
  {
    // 1. The local finalize in export mode: grouping, per-group states, big groups' centroid lists.
    PXG_RETURN_IF_ERROR(ws.meta.Ensure(64));  // read back by the callers even when nothing was staged
    x_check_pending = false;
    export_x = true;
    const int32_t rc = AggFinalizeTable(this);
    export_x = false;
    res.ready = false;
    if (rc != PXG_OK) return rc;
    const uint64_t Gtab = static_cast<uint64_t>(res.n_groups);
    // A high-cardinality run exports its partition groups beside the table groups (no spill):
    // aggregated to states by the partition pass, key records rebuilt as arena scratch.
    X.e_slots = slots.as<const unsigned long long>();
    X.e_gslot = ws.gslot.as<const uint32_t>();
    X.hc_key_words = 0;
    uint64_t G = Gtab;
    if (hc_active) {
      uint32_t n_hc = 0;
      PXG_RETURN_IF_ERROR(ExportHcGroups(static_cast<uint32_t>(Gtab), &ws.xstates, &X.eslots, &n_hc, &X.hc_key_words));
      G = Gtab + n_hc;
      if (G >= (uint64_t(1) << 32)) return SetError(PXG_UNIMPLEMENTED, "export of 2^32 groups");
      // (ExportHcGroups already sized eslots when it wrote partition groups; otherwise there is
      // nothing in it to keep.)
      PXG_RETURN_IF_ERROR(X.eslots.Reserve(G * 8 + 16, 0, ctx->stream));
      PXG_RETURN_IF_ERROR(X.egslot.Ensure(G * 4 + 16));
      if (G > 0)
        PXG_RETURN_IF_ERROR(Launch(ctx, "export_group_rank", XTableSlotsKernel, dim3(GridFor(static_cast<int64_t>(G), 256, 1 << 30)), dim3(256), 0,
                                   slots.as<const unsigned long long>(), ws.gslot.as<const uint32_t>(), static_cast<uint32_t>(Gtab),
                                   X.eslots.as<unsigned long long>(), X.egslot.as<uint32_t>(), static_cast<uint32_t>(G)));
      X.e_slots = X.eslots.as<const unsigned long long>();
      X.e_gslot = X.egslot.as<const uint32_t>();
    }
    // Items and item words both stay below 2^31: the group offset word keeps the item index in
    // bits 32..62 and the centroid flag in bit 63 (kXCentFlag).
    if (st_n + uint64_t(2) * kXCentCapH * x_nbig >= (uint64_t(1) << 31))
      return SetError(PXG_UNIMPLEMENTED, "exchange parts hold fewer than 2^31 items and item words");
    X.G = G;
    PXG_RETURN_IF_ERROR(X.part_of.Ensure(G + 16));
    PXG_RETURN_IF_ERROR(X.koff.Ensure((2 * G + 2) * 8 + 64));   // kw, then koff_j
    PXG_RETURN_IF_ERROR(X.words.Ensure((2 * G + 2) * 8 + 64));  // ic, then ioff_j
    PXG_RETURN_IF_ERROR(X.slist.Ensure(G * 4 + 16));            // glist
    PXG_RETURN_IF_ERROR(X.grank.Ensure(G * 4 + 16));            // xbig
    PXG_RETURN_IF_ERROR(X.starts.Ensure(4 * (kPartBuckets + 1) * 8 + 64));
    uint64_t* gstarts = X.starts.as<uint64_t>();
    uint64_t* bounds = gstarts + kPartBuckets + 1;
    int32_t* xbig = nullptr;
    if (has_q && x_nbig > 0 && G > 0) {
      xbig = reinterpret_cast<int32_t*>(X.grank.p);
      PXG_HIP(hipMemsetAsync(xbig, 0xFF, G * 4, ctx->stream));
      PXG_RETURN_IF_ERROR(Launch(ctx, "export_group_rank", XBigIndexKernel, dim3(GridFor(x_nbig, 256, 1 << 30)), dim3(256), 0,
                                 ws.lists.as<const uint32_t>() + 3 * G, x_nbig, xbig));
    }
    uint64_t* kw = X.koff.as<uint64_t>();
    uint64_t* koff_j = kw + G + 1;
    uint64_t* ic = X.words.as<uint64_t>();
    uint64_t* ioff_j = ic + G + 1;
    if (G > 0)
      PXG_RETURN_IF_ERROR(Launch(ctx, "export_slot_part", XGroupPartKernel, dim3(GridFor(static_cast<int64_t>(G), 256, 1 << 30)), dim3(256), 0,
                                 d_plan.as<const AggPlanDev>(), X.e_slots, X.e_gslot,
                                 static_cast<uint32_t>(G), arena.as<const uint64_t>(), static_cast<uint32_t>(n_parts),
                                 ws.gstart.as<const uint32_t>(), static_cast<const int32_t*>(xbig),
                                 static_cast<const int32_t*>(ws.xcnt.as<int32_t>()), has_q ? 1 : 0, X.part_of.as<uint8_t>(), kw, ic));
    PXG_RETURN_IF_ERROR(Partition(ctx, X.part_of.as<const uint8_t>(), G, X.slist.as<uint32_t>(), gstarts, &X.hist, &X.scan));
    PXG_RETURN_IF_ERROR(X.scan2.Ensure(ScanScratchBytes(static_cast<int64_t>(G) + 1) + 64));
    if (G > 0) {
      PXG_RETURN_IF_ERROR(Launch(ctx, "export_group_rank", XGatherU64Kernel, dim3(GridFor(static_cast<int64_t>(G), 256, 1 << 30)), dim3(256), 0,
                                 X.slist.as<const uint32_t>(), G, static_cast<const uint64_t*>(kw), koff_j));
      PXG_RETURN_IF_ERROR(Launch(ctx, "export_group_rank", XGatherU64Kernel, dim3(GridFor(static_cast<int64_t>(G), 256, 1 << 30)), dim3(256), 0,
                                 X.slist.as<const uint32_t>(), G, static_cast<const uint64_t*>(ic), ioff_j));
    }
    PXG_RETURN_IF_ERROR(ScanExclusiveU64(ctx, koff_j, koff_j, static_cast<int64_t>(G), koff_j + G, X.scan2.p));
    PXG_RETURN_IF_ERROR(ScanExclusiveU64(ctx, ioff_j, ioff_j, static_cast<int64_t>(G), ioff_j + G, X.scan2.p));
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_group_rank", XPartBoundsKernel, dim3(1), dim3(kPartBuckets + 1), 0,
                               static_cast<const uint64_t*>(gstarts), n_parts, static_cast<const uint64_t*>(koff_j),
                               static_cast<const uint64_t*>(ioff_j), bounds));
  }
  return PXG_OK;
}

int32_t Agg::ExportPartialV2(int32_t n_parts, void* dst, int64_t dst_capacity, int64_t* part_offsets, int64_t* part_bytes) {
  ExportCache& X = xc;
  if (merged) return SetError(PXG_FAILED_PRECONDITION, "an aggregation that merged imported states cannot be exported again");
  const bool has_q = x_qval >= 0;
  const uint32_t srec = static_cast<uint32_t>(hplan_x.state_rec);
  if (!(X.valid && X.v2 && X.n_parts == n_parts && X.version == state_version)) {
    PXG_RETURN_IF_ERROR(ExportGroupV2(n_parts));
    const uint64_t* bounds = X.starts.as<const uint64_t>() + kPartBuckets + 1;
    // Part bounds and the finalize's deferred checks in one readback.
    std::vector<uint64_t> hb(3 * (n_parts + 1) + 3);
    PXG_HIP(hipMemcpyAsync(hb.data(), bounds, 3 * (n_parts + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    PXG_HIP(hipMemcpyAsync(hb.data() + 3 * (n_parts + 1), ws.meta.p, 24, hipMemcpyDeviceToHost, ctx->stream));
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    PXG_RETURN_IF_ERROR(CheckExportFinalize(reinterpret_cast<const uint8_t*>(hb.data() + 3 * (n_parts + 1))));
    X.g_start.assign(hb.begin(), hb.begin() + n_parts + 1);
    X.k_start.assign(hb.begin() + n_parts + 1, hb.begin() + 2 * (n_parts + 1));
    X.r_start.assign(hb.begin() + 2 * (n_parts + 1), hb.begin() + 3 * (n_parts + 1));
    X.n_parts = n_parts;
    X.version = state_version;
    X.v2 = true;
    X.valid = true;
  }
  std::vector<XHeader> hdr(n_parts);
  std::vector<uint64_t> poff(n_parts), lay(6 * n_parts), nit(n_parts);
  uint64_t off = 0;
  const uint64_t sig = XPlanSig(*this);
  for (int p = 0; p < n_parts; ++p) {
    const uint64_t ng = X.g_start[p + 1] - X.g_start[p];
    const uint64_t ni = (X.r_start[p + 1] >> kXItemShift) - (X.r_start[p] >> kXItemShift);
    const uint64_t nw = (X.r_start[p + 1] & 0xFFFFFFFFu) - (X.r_start[p] & 0xFFFFFFFFu);
    const uint64_t kwp = X.k_start[p + 1] - X.k_start[p];
    const XLayout L = XLayoutOf(ng, nw, kwp, srec, has_q);
    XHeader& H = hdr[p];
    std::memset(&H, 0, sizeof(H));
    H.magic = kXMagic;
    H.version = kXVersion;
    H.n_keys = static_cast<uint32_t>(n_keys);
    H.state_rec = srec;
    H.n_groups = ng;
    H.n_items = ni;
    H.key_words = kwp;
    H.plan_sig = sig;
    H.has_q = has_q ? 1 : 0;
    H.item_words = nw;
    poff[p] = off;
    const uint64_t l6[6] = {L.koff, L.keys, L.states, L.gofs, L.items, 0};
    for (int k = 0; k < 6; ++k) lay[6 * p + k] = l6[k];
    nit[p] = ni;
    part_offsets[p] = static_cast<int64_t>(off);
    part_bytes[p] = static_cast<int64_t>(L.bytes);
    off += Align8(L.bytes);
  }
  if (dst == nullptr) return PXG_OK;
  if (static_cast<uint64_t>(dst_capacity) < off)
    return SetError(PXG_INVALID_ARGUMENT, "export buffer holds %lld bytes; %llu needed", (long long)dst_capacity, (unsigned long long)off);
  std::vector<uint64_t> desc;
  desc.insert(desc.end(), poff.begin(), poff.end());
  desc.insert(desc.end(), lay.begin(), lay.end());
  desc.insert(desc.end(), nit.begin(), nit.end());
  PXG_RETURN_IF_ERROR(X.desc.Ensure(desc.size() * 8 + 64));
  PXG_HIP(hipMemcpyAsync(X.desc.p, desc.data(), desc.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  uint8_t* base = static_cast<uint8_t*>(dst);
  for (int p = 0; p < n_parts; ++p) PXG_HIP(hipMemcpyAsync(base + poff[p], &hdr[p], sizeof(XHeader), hipMemcpyHostToDevice, ctx->stream));
  XDst D;
  D.base = base;
  D.poff = X.desc.as<const uint64_t>();
  D.layout = D.poff + n_parts;
  D.nitems = D.layout + 6 * n_parts;
  D.fail = nullptr;
  const uint64_t G = X.G;
  if (G > 0) {
    const bool has_big = has_q && x_nbig > 0;
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_write_groups", XWriteGroupsKernel, dim3(GridFor(static_cast<int64_t>(G) * 64, 256, 1 << 30)),
                               dim3(256), 0, X.slist.as<const uint32_t>(), G, X.part_of.as<const uint8_t>(), X.starts.as<const uint64_t>(),
                               static_cast<const uint64_t*>(X.koff.as<uint64_t>() + G + 1), static_cast<const uint64_t*>(X.words.as<uint64_t>() + G + 1),
                               X.e_slots, X.e_gslot, arena.as<const uint64_t>(),
                               d_plan.as<const AggPlanDev>(), ws.xstates.as<const uint8_t>(), srec, ws.gstart.as<const uint32_t>(), x_vals,
                               has_big ? static_cast<const int32_t*>(reinterpret_cast<int32_t*>(X.grank.p)) : nullptr,
                               static_cast<const int32_t*>(ws.xcnt.as<int32_t>()), static_cast<const uint64_t*>(ws.xcent.as<uint64_t>()),
                               has_q ? 1 : 0, D));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}


// The layout ExportPartialV2 computes on the host, on the device: one thread walks the parts
// (<= kPartBuckets) from the device bounds, writes the descriptor XWriteGroupsKernel reads, each
// part's header (into the part and into hdr_out), and each part's aligned byte count.
// The export finalize's deferred checks (Agg::CheckExportFinalize, from ws.meta) and the send
// buffer's capacity are checked here first: on a failure every part's count becomes -1 and
// nothing is written (XWriteGroupsKernel sees seg_out[0] < 0), so a rank announces its failure
// to its peers in the {bytes, header} exchange instead of dropping out of the collective, and a
// group count that differs from the host's sizing can never write past the buffer.
struct XHdrConst {
  uint32_t n_keys, srec;
  uint64_t plan_sig;
  int32_t has_q;
  int32_t check;          // the finalize's checks are pending (x_check_pending)
  uint32_t check_groups;  // the host's group count (x_check_groups)
  uint64_t cap;           // send buffer bytes
};
__global__ void XLayoutDevKernel(const uint64_t* __restrict__ bounds, int32_t n_parts, XHdrConst hc, const uint8_t* __restrict__ meta,
                                 uint8_t* __restrict__ base, uint64_t* __restrict__ desc, int64_t* __restrict__ seg_out,
                                 uint8_t* __restrict__ hdr_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t* g_start = bounds;
  const uint64_t* k_start = bounds + n_parts + 1;
  const uint64_t* r_start = bounds + 2 * (n_parts + 1);
  uint64_t* poff = desc;
  uint64_t* lay = desc + n_parts;
  uint64_t* nit = lay + 6 * n_parts;
  bool ok = true;
  if (hc.check) {
    const uint32_t g_dev = *reinterpret_cast<const uint32_t*>(meta + 8);
    const uint32_t err = *reinterpret_cast<const uint32_t*>(meta + 16);
    ok = err == 0 && g_dev == hc.check_groups;
  }
  uint64_t total = 0;
  for (int p = 0; p < n_parts; ++p) {
    const uint64_t nw = (r_start[p + 1] & 0xFFFFFFFFu) - (r_start[p] & 0xFFFFFFFFu);
    total += Align8(XLayoutOf(g_start[p + 1] - g_start[p], nw, k_start[p + 1] - k_start[p], hc.srec, hc.has_q != 0).bytes);
  }
  if (!ok || total > hc.cap) {
    for (int p = 0; p < n_parts; ++p) {
      seg_out[p] = -1;
      uint64_t* d1 = reinterpret_cast<uint64_t*>(hdr_out + 64 * static_cast<uint64_t>(p));
      for (int w = 0; w < 8; ++w) d1[w] = 0;
    }
    return;
  }
  uint64_t off = 0;
  for (int p = 0; p < n_parts; ++p) {
    const uint64_t ng = g_start[p + 1] - g_start[p];
    const uint64_t ni = (r_start[p + 1] >> kXItemShift) - (r_start[p] >> kXItemShift);
    const uint64_t nw = (r_start[p + 1] & 0xFFFFFFFFu) - (r_start[p] & 0xFFFFFFFFu);
    const uint64_t kwp = k_start[p + 1] - k_start[p];
    const XLayout L = XLayoutOf(ng, nw, kwp, hc.srec, hc.has_q != 0);
    XHeader H;
    __builtin_memset(&H, 0, sizeof(H));
    H.magic = kXMagic;
    H.version = kXVersion;
    H.n_keys = hc.n_keys;
    H.state_rec = hc.srec;
    H.n_groups = ng;
    H.n_items = ni;
    H.key_words = kwp;
    H.plan_sig = hc.plan_sig;
    H.has_q = hc.has_q ? 1 : 0;
    H.item_words = nw;
    poff[p] = off;
    lay[6 * p + 0] = L.koff;
    lay[6 * p + 1] = L.keys;
    lay[6 * p + 2] = L.states;
    lay[6 * p + 3] = L.gofs;
    lay[6 * p + 4] = L.items;
    lay[6 * p + 5] = 0;
    nit[p] = ni;
    const uint64_t* hw = reinterpret_cast<const uint64_t*>(&H);
    uint64_t* d0 = reinterpret_cast<uint64_t*>(base + off);
    uint64_t* d1 = reinterpret_cast<uint64_t*>(hdr_out + 64 * static_cast<uint64_t>(p));
    for (int w = 0; w < 8; ++w) {
      d0[w] = hw[w];
      d1[w] = hw[w];
    }
    const uint64_t seg = Align8(L.bytes);
    seg_out[p] = static_cast<int64_t>(seg);
    off += seg;
  }
}

int32_t Agg::ExportPartialDev(int32_t n_parts, DevBuf* send, int64_t* seg_dev, uint8_t* hdr_dev) {
  // Tests only (tests/test_comm_gpu.py): PXG_TEST_EXPORT_FAIL=host fails this rank's export before
  // anything is issued, =device makes the device layout refuse it (a forced group-count mismatch).
  const char* inject = std::getenv("PXG_TEST_EXPORT_FAIL");
  if (inject && std::strcmp(inject, "host") == 0) return SetError(PXG_INTERNAL, "export failure injected (PXG_TEST_EXPORT_FAIL=host)");
  const bool inject_dev = inject && std::strcmp(inject, "device") == 0;
  if (merged) return SetError(PXG_FAILED_PRECONDITION, "an aggregation that merged imported states cannot be exported again");
  if (n_parts < 1 || n_parts > kPartBuckets) return SetError(PXG_INVALID_ARGUMENT, "%d parts", n_parts);
  ExportCache& X = xc;
  const bool has_q = x_qval >= 0;
  const uint32_t srec = static_cast<uint32_t>(hplan_x.state_rec);
  // The grouping of a host-layout export of the same state is reused (pxg_agg_export_partial
  // just ran for these parts); otherwise the export finalize runs here.
  if (!(X.valid && X.v2 && X.n_parts == n_parts && X.version == state_version)) PXG_RETURN_IF_ERROR(ExportGroupV2(n_parts));
  const uint64_t G = X.G;
  // Host bound of the parts' total: headers, per-group offsets / states / item offsets, every
  // group's key record (<= the arena), items (raw values <= staged rows, <= 2 * kXCentCapH words
  // per centroid list), alignment.
  const uint64_t bound = static_cast<uint64_t>(n_parts) * (sizeof(XHeader) + 32) + G * (24 + Align8(srec)) + 8 * (arena_words + X.hc_key_words) +
                         8 * (st_n + uint64_t(2) * kXCentCapH * x_nbig) + 64;
  PXG_RETURN_IF_ERROR(send->Ensure(bound));
  PXG_RETURN_IF_ERROR(X.desc.Ensure(static_cast<size_t>(8 * n_parts) * 8 + 64));
  XHdrConst hc;
  hc.n_keys = static_cast<uint32_t>(n_keys);
  hc.srec = srec;
  hc.plan_sig = XPlanSig(*this);
  hc.has_q = has_q ? 1 : 0;
  hc.check = x_check_pending || inject_dev ? 1 : 0;
  hc.check_groups = x_check_groups + (inject_dev ? 1u : 0u);
  hc.cap = send->bytes;
  PXG_RETURN_IF_ERROR(Launch(ctx, "export_layout", XLayoutDevKernel, dim3(1), dim3(64), 0,
                             X.starts.as<const uint64_t>() + kPartBuckets + 1, n_parts, hc, ws.meta.as<const uint8_t>(), send->as<uint8_t>(),
                             X.desc.as<uint64_t>(), seg_dev, hdr_dev));
  XDst D;
  D.base = send->as<uint8_t>();
  D.poff = X.desc.as<const uint64_t>();
  D.layout = D.poff + n_parts;
  D.nitems = D.layout + 6 * n_parts;
  D.fail = seg_dev;
  if (G > 0) {
    const bool has_big = has_q && x_nbig > 0;
    PXG_RETURN_IF_ERROR(Launch(ctx, "export_write_groups", XWriteGroupsKernel, dim3(GridFor(static_cast<int64_t>(G) * 64, 256, 1 << 30)),
                               dim3(256), 0, X.slist.as<const uint32_t>(), G, X.part_of.as<const uint8_t>(), X.starts.as<const uint64_t>(),
                               static_cast<const uint64_t*>(X.koff.as<uint64_t>() + G + 1), static_cast<const uint64_t*>(X.words.as<uint64_t>() + G + 1),
                               X.e_slots, X.e_gslot, arena.as<const uint64_t>(),
                               d_plan.as<const AggPlanDev>(), ws.xstates.as<const uint8_t>(), srec, ws.gstart.as<const uint32_t>(), x_vals,
                               has_big ? static_cast<const int32_t*>(reinterpret_cast<int32_t*>(X.grank.p)) : nullptr,
                               static_cast<const int32_t*>(ws.xcnt.as<int32_t>()), static_cast<const uint64_t*>(ws.xcent.as<uint64_t>()),
                               has_q ? 1 : 0, D));
  }
  return PXG_OK;
}

int32_t Agg::ImportPartialsV2(const uint8_t* base8, int32_t n, const int64_t* offs, const int64_t* sizes, const void* hdrs) {
  const XHeader* H = static_cast<const XHeader*>(hdrs);
  if (!x_ok) return SetError(PXG_UNIMPLEMENTED, "this aggregation's UDAs cannot merge exchanged states");
  if (!merged && (st_n > 0 || inserted > 0 || hc_active))
    return SetError(PXG_FAILED_PRECONDITION, "exchanged states merge into an aggregation without consumed rows (reset it first)");
  const uint32_t srec = static_cast<uint32_t>(hplan_x.state_rec);
  const bool has_q = x_qval >= 0;
  uint64_t tot_groups = 0, tot_items = 0, tot_words = 0;
  std::vector<XLayout> L(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    const XHeader& h = H[i];
    if (h.version != kXVersion || h.plan_sig != XPlanSig(*this) || h.n_keys != static_cast<uint32_t>(n_keys) || h.state_rec != srec ||
        h.has_q != (has_q ? 1u : 0u))
      return SetError(PXG_INVALID_ARGUMENT, "partial-state buffer was exported by an aggregation with a different plan");
    L[i] = XLayoutOf(h.n_groups, h.item_words, h.key_words, srec, has_q);
    if (static_cast<uint64_t>(sizes[i]) < L[i].bytes)
      return SetError(PXG_INVALID_ARGUMENT, "partial buffer truncated: %lld of %llu bytes", (long long)sizes[i], (unsigned long long)L[i].bytes);
    tot_groups += h.n_groups;
    tot_items += has_q ? h.n_items : h.n_groups;
    tot_words += h.key_words;
  }
  // The merged digest tells the parts apart by the part index in the weights' top bits, and
  // DigestMergeKernel keeps one segment per part for at most kXMaxParts parts per merged run.
  int32_t parts_here = 0;
  for (int i = 0; i < n; ++i) parts_here += H[i].n_groups > 0 ? 1 : 0;
  if (has_q && x_parts_seen + parts_here > kXMaxParts)
    return SetError(PXG_UNIMPLEMENTED, "a merged aggregation takes at most %d imported parts (%d so far, %d more)", kXMaxParts, x_parts_seen,
                    parts_here);
  merged = true;
  state_version++;
  res.ready = false;
  if (tot_groups == 0) return PXG_OK;
  const uint64_t abase = arena_words;
  if (abase + tot_words >= (uint64_t(1) << 32)) return SetError(PXG_RESOURCE_UNAVAILABLE, "key arena exceeds 32 GiB");
  PXG_RETURN_IF_ERROR(arena.Reserve((abase + tot_words) * 8 + kArenaSlack, abase * 8, ctx->stream));
  uint64_t want = 4 * (inserted + tot_groups);
  if (want > cap) {
    uint64_t c = cap;
    while (c < want) c <<= 1;
    if (c > (uint64_t(1) << 31)) return SetError(PXG_RESOURCE_UNAVAILABLE, "group table would exceed 2^31 slots");
    PXG_RETURN_IF_ERROR(Grow(static_cast<uint32_t>(c)));
  }
  PXG_RETURN_IF_ERROR(EnsureMacc());
  PXG_RETURN_IF_ERROR(xc.remap.Ensure(tot_groups * 4 + 16));
  PXG_RETURN_IF_ERROR(EnsureStage(st_n + tot_items));
  PXG_RETURN_IF_ERROR(st_wt.Reserve((st_n + tot_items) * 8 + 16, st_n * 8, ctx->stream));
  uint8_t* meta = counters.as<uint8_t>();
  unsigned int* d_ins = reinterpret_cast<unsigned int*>(meta + 32);
  unsigned int* d_err = reinterpret_cast<unsigned int*>(meta + 36);
  PXG_HIP(hipMemsetAsync(meta + 32, 0, 8, ctx->stream));
  const XAccPlan xp = XAccPlanOf(*this);
  uint64_t kw = abase, g0 = 0, r0 = st_n;
  for (int i = 0; i < n; ++i) {
    const XHeader& h = H[i];
    const uint8_t* p = base8 + offs[i];
    if (h.n_groups == 0) continue;
    uint32_t* remap = xc.remap.as<uint32_t>() + g0;
    PXG_HIP(hipMemcpyAsync(arena.as<uint64_t>() + kw, p + L[i].keys, h.key_words * 8, hipMemcpyDeviceToDevice, ctx->stream));
    PXG_RETURN_IF_ERROR(Launch(ctx, "import_keys", ImportKeysKernel, dim3(GridFor(static_cast<int64_t>(h.n_groups), 256, 1 << 30)), dim3(256), 0,
                               d_plan.as<const AggPlanDev>(), slots.as<unsigned long long>(), cap - 1, arena.as<const uint64_t>(), kw,
                               reinterpret_cast<const uint64_t*>(p + L[i].koff), h.n_groups, remap, d_ins, d_err));
    if (srec > 0)
      PXG_RETURN_IF_ERROR(Launch(ctx, "import_states", XImportStatesKernel, dim3(GridFor(static_cast<int64_t>(h.n_groups), 256, 1 << 30)),
                                 dim3(256), 0, xp, p + L[i].states, srec, h.n_groups, static_cast<const uint32_t*>(remap), macc.as<uint64_t>()));
    const uint64_t part = static_cast<uint64_t>(x_parts_seen++);  // < kXMaxParts (checked above)
    if (has_q && h.n_items > 0) {
      PXG_RETURN_IF_ERROR(Launch(ctx, "import_rows", XImportItemsKernel, dim3(GridFor(static_cast<int64_t>(h.n_groups) * 64, 256, 1 << 30)),
                                 dim3(256), 0, reinterpret_cast<const uint64_t*>(p + L[i].gofs), reinterpret_cast<const uint64_t*>(p + L[i].items),
                                 h.n_groups, h.n_items, h.item_words, static_cast<const uint32_t*>(remap), part, st_slot.as<uint32_t>() + r0,
                                 st_val[x_qval].as<uint64_t>() + r0, st_wt.as<uint64_t>() + r0, macc.as<uint64_t>(), macc_words, d_err));
      r0 += h.n_items;
    } else if (!has_q) {
      PXG_RETURN_IF_ERROR(Launch(ctx, "import_rows", XPlaceholderKernel, dim3(GridFor(static_cast<int64_t>(h.n_groups), 256, 1 << 30)), dim3(256), 0,
                                 static_cast<const uint32_t*>(remap), h.n_groups, st_slot.as<uint32_t>() + r0, st_wt.as<uint64_t>() + r0));
      r0 += h.n_groups;
    }
    kw += h.key_words;
    g0 += h.n_groups;
  }
  arena_words = kw;
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + 240);
  PXG_HIP(hipMemcpyAsync(pin, meta + 32, 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  const uint32_t r_ins = pin[0], r_err = pin[1];
  if (r_err & 1u) return SetError(PXG_INTERNAL, "group table full during partial import");
  if (r_err & 2u) return SetError(PXG_INVALID_ARGUMENT, "partial buffer has an item whose group index is out of range");
  inserted += r_ins;
  st_n = r0;
  // The device insert count and staging cursor follow (stream-ordered memsets: no host buffer).
  PXG_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(counters.p), static_cast<int>(inserted), 1, ctx->stream));
  PXG_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(counters.as<uint8_t>() + 16), static_cast<int>(st_n & 0xFFFFFFFFu), 1, ctx->stream));
  PXG_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(counters.as<uint8_t>() + 20), static_cast<int>(st_n >> 32), 1, ctx->stream));
  return PXG_OK;
}

// Finalize of a merged aggregation: the ordinary finalize over the imported items (grouping, key
// output, and the quantiles of groups that arrived as raw values only), then every non-quantile
// output from the accumulators and the merged digests of the groups that received centroids.
int32_t Agg::FinalizeMerged() {
  PXG_RETURN_IF_ERROR(AggFinalizeTable(this));
  const uint32_t G = static_cast<uint32_t>(res.n_groups);
  if (G == 0) return PXG_OK;
  UdaOutX uo;
  for (int u = 0; u < kMaxUdas; ++u) uo.p[u] = u < n_udas ? res.uda_out[u].as<uint64_t>() : nullptr;
  const bool has_q = x_qval >= 0;
  PXG_RETURN_IF_ERROR(ws.dlist.Ensure(static_cast<size_t>(G) * 4 + 64));
  uint32_t* dcount = ws.dlist.as<uint32_t>() + G;
  PXG_HIP(hipMemsetAsync(dcount, 0, 4, ctx->stream));
  PXG_RETURN_IF_ERROR(Launch(ctx, "merged_states", XFinalizeStatesKernel, dim3(GridFor(G, 256, 1 << 30)), dim3(256), 0, XAccPlanOf(*this),
                             ws.gslot.as<const uint32_t>(), G, macc.as<const uint64_t>(), uo, has_q ? ws.dlist.as<uint32_t>() : nullptr,
                             dcount));
  if (has_q) PXG_RETURN_IF_ERROR(LaunchDigestMerge(this, ws.dlist.as<const uint32_t>(), dcount, G));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}

}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_agg_export_partial(pxg_agg* agg, int32_t n_parts, void* dst, int64_t dst_capacity, int64_t* part_offsets,
                                          int64_t* part_bytes) {
  if (!agg || !part_offsets || !part_bytes) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  if (n_parts < 1 || n_parts > kMaxParts) return SetError(PXG_INVALID_ARGUMENT, "n_parts must be in [1, %d]", kMaxParts);
  if (ExchangeV2(agg->impl)) return agg->impl.ExportPartialV2(n_parts, dst, dst_capacity, part_offsets, part_bytes);
  PXG_RETURN_IF_ERROR(agg->impl.SpillHc());  // v1 row parts are cut from the table state
  return agg->impl.ExportPartial(n_parts, dst, dst_capacity, part_offsets, part_bytes);
}

// The device-laid-out export that pxg_agg_alltoall sends (ExportPartialDev: sizes, headers and
// part layout computed on the device), into an aggregation-owned device buffer; one wait brings
// back the sizes, the headers and the export finalize's checks.
extern "C" int32_t pxg_agg_export_partial_dev(pxg_agg* agg, int32_t n_parts, void** parts, int64_t* part_bytes, uint8_t* headers) {
  if (!agg || !parts || !part_bytes) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  if (n_parts < 1 || n_parts > kMaxParts) return SetError(PXG_INVALID_ARGUMENT, "n_parts must be in [1, %d]", kMaxParts);
  Agg& a = agg->impl;
  if (!ExchangeV2(a)) return SetError(PXG_FAILED_PRECONDITION, "the device layout exports partial states (exchange v2) only");
  Agg::ExportCache& X = a.xc;
  const size_t hb = XHeaderBytes();
  PXG_RETURN_IF_ERROR(X.dcnt.Ensure(static_cast<size_t>(n_parts) * (8 + hb) + 64));
  int64_t* d_seg = X.dcnt.as<int64_t>();
  uint8_t* d_hdr = reinterpret_cast<uint8_t*>(d_seg + n_parts);
  PXG_RETURN_IF_ERROR(a.ExportPartialDev(n_parts, &X.dsend, d_seg, d_hdr));
  std::vector<uint8_t> h(static_cast<size_t>(n_parts) * (8 + hb) + 24);
  PXG_HIP(hipMemcpyAsync(h.data(), d_seg, static_cast<size_t>(n_parts) * (8 + hb), hipMemcpyDeviceToHost, a.ctx->stream));
  PXG_HIP(hipMemcpyAsync(h.data() + static_cast<size_t>(n_parts) * (8 + hb), a.ws.meta.p, 24, hipMemcpyDeviceToHost, a.ctx->stream));
  PXG_HIP(hipStreamSynchronize(a.ctx->stream));
  PXG_RETURN_IF_ERROR(a.CheckExportFinalize(h.data() + static_cast<size_t>(n_parts) * (8 + hb)));
  std::memcpy(part_bytes, h.data(), static_cast<size_t>(n_parts) * 8);
  for (int p = 0; p < n_parts; ++p)
    if (part_bytes[p] < 0) return SetError(PXG_INTERNAL, "device export refused its parts (send buffer of %zu bytes)", X.dsend.bytes);
  if (headers) std::memcpy(headers, h.data() + static_cast<size_t>(n_parts) * 8, static_cast<size_t>(n_parts) * hb);
  *parts = X.dsend.p;
  return PXG_OK;
}

extern "C" int32_t pxg_agg_import_partial(pxg_agg* agg, const void* src, int64_t nbytes) {
  if (!agg || !src) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  PXG_RETURN_IF_ERROR(agg->impl.SpillHc());
  return agg->impl.ImportPartial(src, nbytes);
}

extern "C" int32_t pxg_agg_import_partials(pxg_agg* agg, const void* src, int32_t n_parts, const int64_t* part_offsets,
                                           const int64_t* part_bytes) {
  if (!agg || (n_parts > 0 && (!src || !part_offsets || !part_bytes)) || n_parts < 0)
    return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  PXG_RETURN_IF_ERROR(agg->impl.SpillHc());
  return agg->impl.ImportPartials(src, n_parts, part_offsets, part_bytes);
}
