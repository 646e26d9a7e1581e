// Device-wide exclusive scan (used for compaction offsets, string offsets, radix sort).
#pragma once

#include "pxg_internal.h"

namespace pxg {

constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;  // per thread
constexpr int kScanTile = kScanBlock * kScanItems;

// Exclusive scan of n values of type T (uint32/uint64/int64) from `in` into `out`
// (out may alias in).  If total != nullptr the grand total is written there (device memory).
// Scratch must hold ScanScratchBytes(n) bytes.
size_t ScanScratchBytes(int64_t n);
int32_t ScanExclusiveU64(Ctx* ctx, const uint64_t* in, uint64_t* out, int64_t n, uint64_t* total, void* scratch);
int32_t ScanExclusiveU32(Ctx* ctx, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total, void* scratch);
// The same on another stream of ctx (its own scratch: scans on different streams may overlap).
int32_t ScanExclusiveU32On(Ctx* ctx, hipStream_t stream, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total,
                           void* scratch);

}  // namespace pxg
