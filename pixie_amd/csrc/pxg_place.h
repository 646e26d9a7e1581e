// Counting placement of staged records by table slot (pxg_place.hip): the finalize's grouping
// without a sort when row order inside a group does not matter.
#pragma once

#include "pxg_agg.h"
#include "pxg_internal.h"

namespace pxg {

struct PlaceVals {
  const uint64_t* p[kMaxVals];
};
struct PlaceOut {
  uint64_t* p[kMaxVals];
};

// Groups n staged records (table slot st_slot[i]; kDeferredSlot or any slot >= cap: no group)
// by dense group id (rank[slot] of an occupied slot, slots[] != 0): value stream v of the records
// of group g lands in vout.p[v][gstart[g] .. gstart[g + 1]), records without a group after
// gstart[G].  Order inside a group is unspecified.  cnt_buf: grow-only workspace (cap + 2 words);
// scan_tmp: ScanScratchBytes(cap + 1) bytes.  Stream-ordered on ctx->stream.
int32_t PlaceBySlot(Ctx* ctx, const uint32_t* st_slot, uint64_t n, uint32_t cap, const unsigned long long* slots, const uint32_t* rank,
                    uint32_t G, PlaceVals vin, int nvals, PlaceOut vout, uint32_t* gstart, DevBuf& cnt_buf, void* scan_tmp);

}  // namespace pxg
