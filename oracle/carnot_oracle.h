// ORACLE / TEST INFRASTRUCTURE ONLY.
//
// C ABI of the CPU restatement of Pixie Carnot's columnar hot path.  Only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
// (pixie_amd/, include/pxg.h) never links or calls it.  Restated reference files:
//   src/carnot/exec/{filter_node.cc:78-171, map_node.cc:47-71, agg_node.cc:43-542,
//   expression_evaluator.cc:61-342, row_tuple.h:71-252, memory_source_node.cc:92-124,
//   exec_graph.cc:52-331}, src/carnot/udf/udf_wrapper.h:60-438,
//   src/carnot/funcs/builtins/{math_ops.h, math_ops.cc:52-250, math_sketches.h:33-82,
//   json_ops.h:131-153}, src/carnot/plan/{operators.cc:59-395, scalar_expression.cc:232-348}.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// One column of one RowBatch, Arrow-like layout (BOOLEAN: one byte per value; UINT128: 16 B
// per value as {low u64, high u64}; STRING: int32 offsets[length+1] + bytes).
typedef struct {
  int32_t type;  // px.types.DataType
  int64_t length;
  const void* values;
  const int32_t* offsets;
  const uint8_t* data;
} oracle_column;

// A table as a sequence of RowBatches (batch-major: cols[b * ncols + c]).
typedef struct {
  const char* name;
  int32_t ncols;
  const char* const* col_names;
  const int32_t* col_types;
  int32_t nbatches;
  const oracle_column* cols;
  // Optional per-batch flags (bit0 eow, bit1 eos).  When given, the source emits exactly these
  // flags (the reference's ExecNodeTester feeds batches with explicit eow/eos,
  // src/carnot/exec/test_utils.h:319-480); otherwise MemorySourceNode semantics apply.
  const uint8_t* batch_flags;
} oracle_table;

// Execute a planpb.Plan given in protobuf-JSON form over the given tables.  Result tables are
// serialized into *out (PXRB format, see tests/pxrb.py) and released with oracle_free.
// Returns a px.statuspb.Code; on error a message is written into errbuf.
int32_t oracle_execute_plan(const char* plan_json, int32_t ntables, const oracle_table* tables,
                            uint8_t** out, int64_t* out_len, char* errbuf, int32_t errlen);

// Same, timing only the execution window (first GenerateNext .. last emit), in seconds.
int32_t oracle_execute_plan_timed(const char* plan_json, int32_t ntables,
                                  const oracle_table* tables, double* seconds, int64_t* out_rows,
                                  char* errbuf, int32_t errlen);

// Same, with every given batch re-sliced into RowBatches of batch_rows rows (0: as given);
// columns passed with no buffers are not materialised (the plan must not read them).
int32_t oracle_execute_plan_timed_rebatched(const char* plan_json, int32_t ntables,
                                            const oracle_table* tables, int64_t batch_rows,
                                            double* seconds, int64_t* out_rows, char* errbuf,
                                            int32_t errlen);

// Execute with every batch re-sliced into batch_rows-row RowBatches (0: as given), timing the
// execution window into *seconds (may be NULL) and returning the result tables as PXRB.
int32_t oracle_execute_plan_rebatched(const char* plan_json, int32_t ntables, const oracle_table* tables,
                                      int64_t batch_rows, double* seconds, uint8_t** out, int64_t* out_len,
                                      char* errbuf, int32_t errlen);

// Midpoint empirical ranks of candidate quantile values within their groups (rank-bound parity
// for groups whose reference digest depends on insertion order); see carnot_oracle.cc.
int32_t oracle_group_ranks(const oracle_column* keys, int32_t nk, const uint8_t* sel, const double* vals,
                           int64_t n, int32_t nq, const uint8_t* qkeys, const int64_t* qoffs,
                           const double* qv, int32_t per_q, double* out, int64_t* qcount);

void oracle_free(uint8_t* p);

// QuantilesUDA on a value sequence (math_sketches.h:36-54): out[7] = p01,p10,p25,p50,p75,p90,p99.
void oracle_tdigest_quantiles(const double* vals, int64_t n, double* out7);
// Two digests built from a and b, then merged (QuantilesUDA::Merge), then the quantiles.
/* The single-pass digest of n values (TDigest::FromValuesOnce): centroid means / weights into
 * means / weights (capacity cap), their count into *nc (-1 if cap is too small). */
void oracle_tdigest_centroids(const double* vals, int64_t n, double* means, double* weights, int64_t cap, int64_t* nc);
/* quantiles() x7 of a digest built as TDigest::merge_batch over nparts contributions, part i
 * being kind[i] == 0: counts[i] raw values (unprocessed), == 1: counts[i] centroids (means in
 * data, weights in weights), all concatenated in part order. */
void oracle_tdigest_batch_quantiles(int32_t nparts, const int32_t* kind, const int64_t* counts, const double* data,
                                    const double* weights, double* out7);
/* The same, with centroid-list part i carrying its rank's true extremes mins[i] / maxs[i]. */
void oracle_tdigest_batch_quantiles_mm(int32_t nparts, const int32_t* kind, const int64_t* counts, const double* data,
                                       const double* weights, const double* mins, const double* maxs, double* out7);
void oracle_tdigest_merge_quantiles(const double* a, int64_t na, const double* b, int64_t nb,
                                    double* out7);
// The JSON string QuantilesUDA::Finalize would produce (rapidjson Writer bytes, json_number.h).
int32_t oracle_quantiles_json(const double* vals, int64_t n, char* buf, int32_t buflen);
// The oracle's own rendering (json_number.h) of n groups of 7 quantile values: each group's JSON
// followed by a NUL, back to back; returns the bytes needed (writes at most cap).
int64_t oracle_quantiles_json_render(const double* q7, int64_t n, char* buf, int64_t cap);
// pluck_float64 (json_ops.h:131-153).
double oracle_pluck_float64(const char* json, const char* key);

#ifdef __cplusplus
}
#endif
