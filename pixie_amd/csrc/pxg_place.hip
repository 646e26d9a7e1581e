// Grouping of the staged records by group without a sort (finalize; SURVEY.md §8a A13/A17, the
// per-group value buffers that AggNode::HashRowBatch appends to, agg_node.cc:235-271, which
// EvaluatePartialAggregates and ConvertAggHashMapToRowBatch then read group by group,
// agg_node.cc:273-349).
//
// The stable LSD radix sort (pxg_finalize.hip) moves every record twice per 8-bit digit (two
// passes at 65K groups) plus a rank-gathering histogram pass: ~56 B of traffic per staged row.
// Nothing downstream needs row order inside a group (count / sum / min / max are order-free, a
// mean's float sum already follows the consume's tile completion order, and quantile digests of
// <= 8000 values sort their values), so a counting placement does: per tile of kPlaceTile records
// a workgroup-local LDS hash table counts records per table slot, and
//   1. PlaceCount   adds each tile's per-slot counts to a global count per slot (one device atomic
//                   per distinct slot of the tile, not per record);
//   2. a scan of the counts in slot order gives every slot's start, i.e. the records of dense
//      group g (the rank of its slot among the occupied ones) start at gstart[g];
//   3. PlaceScatter recounts the tile, reserves each distinct slot's range with one device atomic
//      on the slot's cursor, and writes every record's value streams to start + local rank, the
//      records of one slot in a tile landing in one contiguous range.
// ~24 B of traffic per staged row with one value stream.  Merged (exchange owner) and export
// finalizes keep the radix sort: their digest merge needs each part's items contiguous.
#include "pxg_agg_host.h"
#include "pxg_place.h"
#include "pxg_scan.h"

namespace pxg {

namespace {

constexpr int kPlaceBlock = 256;
constexpr int kPlaceItems = 16;
constexpr int kPlaceTile = kPlaceBlock * kPlaceItems;  // 4096 records per workgroup
constexpr int kPlaceHBits = 13;
constexpr int kPlaceH = 1 << kPlaceHBits;              // LDS table entries (load <= 1/2)
constexpr uint32_t kPlaceEmpty = 0xFFFFFFFFu;

// The LDS entry of `key` (inserted if absent).  Keys are table slots (< cap) or cap (records
// without a group), never kPlaceEmpty.
__device__ __forceinline__ uint32_t PlaceFind(uint32_t* s_key, uint32_t key) {
  uint32_t h = (key * 0x9E3779B1u) >> (32 - kPlaceHBits);
  while (true) {
    uint32_t cur = *static_cast<volatile uint32_t*>(s_key + h);
    if (cur == key) return h;
    if (cur == kPlaceEmpty) {
      cur = atomicCAS(s_key + h, kPlaceEmpty, key);
      if (cur == kPlaceEmpty || cur == key) return h;
    }
    h = (h + 1) & (kPlaceH - 1);
  }
}

__device__ __forceinline__ void PlaceLoadKeys(const uint32_t* __restrict__ slot, uint64_t n, uint32_t cap, uint64_t t0,
                                              uint32_t (&k)[kPlaceItems]) {
#pragma unroll
  for (int j = 0; j < kPlaceItems; ++j) {
    const uint64_t i = t0 + static_cast<uint64_t>(j) * kPlaceBlock + threadIdx.x;
    k[j] = i < n ? min(slot[i], cap) : kPlaceEmpty;
  }
}

__global__ void __launch_bounds__(kPlaceBlock) PlaceCountKernel(const uint32_t* __restrict__ slot, uint64_t n, uint32_t cap,
                                                                uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_key[kPlaceH];
  __shared__ uint32_t s_cnt[kPlaceH];
  for (int e = threadIdx.x; e < kPlaceH; e += kPlaceBlock) {
    s_key[e] = kPlaceEmpty;
    s_cnt[e] = 0;
  }
  const uint64_t t0 = static_cast<uint64_t>(XcdRemap(blockIdx.x, gridDim.x)) * kPlaceTile;
  uint32_t k[kPlaceItems];
  PlaceLoadKeys(slot, n, cap, t0, k);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPlaceItems; ++j)
    if (k[j] != kPlaceEmpty) atomicAdd(&s_cnt[PlaceFind(s_key, k[j])], 1u);
  __syncthreads();
  for (int e = threadIdx.x; e < kPlaceH; e += kPlaceBlock) {
    const uint32_t key = s_key[e];
    if (key != kPlaceEmpty) atomicAdd(&cnt[key], s_cnt[e]);
  }
}

// starts (the scanned counts, slot order) -> gstart of the dense groups; gstart[G] = the first
// record without a group.
__global__ void PlaceGstartKernel(const unsigned long long* __restrict__ slots, uint32_t cap, const uint32_t* __restrict__ rank,
                                  const uint32_t* __restrict__ starts, uint32_t G, uint32_t* __restrict__ gstart) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap && slots[i] != 0) gstart[rank[i]] = starts[i];
  if (i == cap) gstart[G] = starts[cap];
}

__global__ void __launch_bounds__(kPlaceBlock) PlaceScatterKernel(const uint32_t* __restrict__ slot, uint64_t n, uint32_t cap,
                                                                  uint32_t* __restrict__ cursor, PlaceVals vin, PlaceOut vout,
                                                                  int nvals) {
  __shared__ uint32_t s_key[kPlaceH];
  __shared__ uint32_t s_cnt[kPlaceH];  // local counts, then the tile's base per entry
  for (int e = threadIdx.x; e < kPlaceH; e += kPlaceBlock) {
    s_key[e] = kPlaceEmpty;
    s_cnt[e] = 0;
  }
  const uint64_t t0 = static_cast<uint64_t>(XcdRemap(blockIdx.x, gridDim.x)) * kPlaceTile;
  uint32_t k[kPlaceItems];
  PlaceLoadKeys(slot, n, cap, t0, k);
  __syncthreads();
  uint32_t ent[kPlaceItems], r[kPlaceItems];
#pragma unroll
  for (int j = 0; j < kPlaceItems; ++j) {
    ent[j] = 0;
    r[j] = 0;
    if (k[j] != kPlaceEmpty) {
      ent[j] = PlaceFind(s_key, k[j]);
      r[j] = atomicAdd(&s_cnt[ent[j]], 1u);
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kPlaceH; e += kPlaceBlock) {
    const uint32_t key = s_key[e];
    if (key != kPlaceEmpty) s_cnt[e] = atomicAdd(&cursor[key], s_cnt[e]);
  }
  __syncthreads();
  for (int v = 0; v < nvals; ++v) {
    const uint64_t* __restrict__ src = vin.p[v];
    uint64_t* __restrict__ dst = vout.p[v];
    uint64_t x[kPlaceItems];
#pragma unroll
    for (int j = 0; j < kPlaceItems; ++j) {
      const uint64_t i = t0 + static_cast<uint64_t>(j) * kPlaceBlock + threadIdx.x;
      x[j] = k[j] != kPlaceEmpty ? src[i] : 0ULL;
    }
#pragma unroll
    for (int j = 0; j < kPlaceItems; ++j)
      if (k[j] != kPlaceEmpty) dst[s_cnt[ent[j]] + r[j]] = x[j];
  }
}

}  // namespace

int32_t PlaceBySlot(Ctx* ctx, const uint32_t* st_slot, uint64_t n, uint32_t cap, const unsigned long long* slots, const uint32_t* rank,
                    uint32_t G, PlaceVals vin, int nvals, PlaceOut vout, uint32_t* gstart, DevBuf& cnt_buf, void* scan_tmp) {
  if (n == 0 || n >= (uint64_t(1) << 32)) return SetError(PXG_INVALID_ARGUMENT, "placement of %llu records", static_cast<unsigned long long>(n));
  if (nvals > kMaxVals) return SetError(PXG_INVALID_ARGUMENT, "%d value streams", nvals);
  PXG_RETURN_IF_ERROR(cnt_buf.Ensure((static_cast<size_t>(cap) + 2) * 4 + 64));
  uint32_t* cnt = cnt_buf.as<uint32_t>();
  PXG_HIP(hipMemsetAsync(cnt, 0, (static_cast<size_t>(cap) + 1) * 4, ctx->stream));
  const uint32_t ntiles = static_cast<uint32_t>((n + kPlaceTile - 1) / kPlaceTile);
  PXG_RETURN_IF_ERROR(Launch(ctx, "place_count", PlaceCountKernel, dim3(ntiles), dim3(kPlaceBlock), 0, st_slot, n, cap, cnt));
  PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, cnt, cnt, static_cast<int64_t>(cap) + 1, cnt + cap + 1, scan_tmp));
  PXG_RETURN_IF_ERROR(Launch(ctx, "place_gstart", PlaceGstartKernel, dim3(GridFor(static_cast<int64_t>(cap) + 1, 256, 1 << 30)), dim3(256), 0,
                             slots, cap, rank, static_cast<const uint32_t*>(cnt), G, gstart));
  PXG_RETURN_IF_ERROR(Launch(ctx, "place_scatter", PlaceScatterKernel, dim3(ntiles), dim3(kPlaceBlock), 0, st_slot, n, cap, cnt, vin, vout,
                             nvals));
  return PXG_OK;
}

}  // namespace pxg
