// The selection path of the quantile digests' big groups (pxg_select.hip), as AggFinalizeTable
// (pxg_finalize.hip) drives it.
#pragma once

#include "pxg_internal.h"
#include "pxg_quant.h"

namespace pxg {

// One set of big groups for the selection / sort paths: its group and chunk lists (device, with
// their device counts), host upper bounds for the grids, its chains and selection workspace.
// Finalize runs two: the designated groups of a fused split (early, from the first pass) and
// the other big groups (after the classification).
struct BigSet {
  BigGroup* big = nullptr;
  BigChunk* chunks = nullptr;
  const uint32_t* d_count = nullptr;  // groups in the set
  const uint32_t* d_meta = nullptr;   // [0] chunks, [1] largest group (BigSetupKernel)
  uint32_t n_big = 0, n_chunks = 0;   // host bounds of both (grids; exact after the meta readback)
  uint64_t big_max = 0;               // largest group (host; the sort path's merge-pass count)
  const uint32_t* chain_starts = nullptr;
  const int32_t* chain_nc = nullptr;
  DevBuf *spl = nullptr, *cnt = nullptr, *list = nullptr, *bstart = nullptr, *tag = nullptr, *cbase = nullptr, *plan = nullptr,
         *partial = nullptr;
  const uint32_t* large_list = nullptr;  // set indices of the groups above kSelLargeN values (BigSetupKernel)
  const uint32_t* large_cnt = nullptr;
};


// One quantile UDA's inputs to the selection path: its value stream (staging order after the
// grouping), the staged row count (workspace sizes), the shared workspace (candidate keys, the
// per-value bins), the fallback counter and the UDA's 7-double output.
struct SelIn {
  const uint64_t* vals = nullptr;
  int arg_type = 0;
  uint64_t n = 0;
  DevBuf* keysA = nullptr;
  DevBuf* sel_bin = nullptr;
  unsigned int* d_fallback = nullptr;
  double* out = nullptr;
};

// Workspace of a set, grown to its host bounds (keysA: n keys, sel_bin: n bins).
int32_t SelEnsure(const BigSet& S, uint64_t n, DevBuf& keysA, DevBuf& sel_bin);
// First half on stream st (needs the grouped values and the set's chunk list only): sample,
// splitters, bin counts.
int32_t SelFront(Ctx* ctx, hipStream_t st, const BigSet& S, const SelIn& in);
// Second half (st ordered after the set's boundary chains): plan, gather + inside sums, bin
// sorts, digests into in.out; groups it cannot serve are flagged (BigPlan) and counted.
int32_t SelBack(Ctx* ctx, hipStream_t st, const BigSet& S, const SelIn& in);
// The group ids of the set's flagged groups appended to list (count: device counter).
int32_t SelFallbackList(Ctx* ctx, const BigSet& S, uint32_t* list, uint32_t* count);

}  // namespace pxg
