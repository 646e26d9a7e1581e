// Partial aggregation export/import (planpb AggregateOperator.partial_agg / finalize_results,
// src/carnot/planpb/plan.proto:250-257).  See DESIGN.md §5 for the wire format.
#include "pxg_agg_host.h"

using namespace pxg;

extern "C" int32_t pxg_agg_export_partial(pxg_agg* agg, int32_t n_parts, void* dst, int64_t dst_capacity, int64_t* part_offsets,
                                          int64_t* part_bytes) {
  (void)agg; (void)n_parts; (void)dst; (void)dst_capacity; (void)part_offsets; (void)part_bytes;
  return SetError(PXG_UNIMPLEMENTED, "partial export not implemented yet");
}

extern "C" int32_t pxg_agg_import_partial(pxg_agg* agg, const void* src, int64_t nbytes) {
  (void)agg; (void)src; (void)nbytes;
  return SetError(PXG_UNIMPLEMENTED, "partial import not implemented yet");
}
