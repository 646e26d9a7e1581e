/*
 * pxcarnot.h — C ABI of the C++ host engine above libpxg (libpxcarnot.so).
 *
 * This is the host side of the drop-in: it takes an unmodified, PxL-compiled
 * px.carnot.planpb.Plan in its binary wire format, builds the execution graph the way
 * ExecutionGraph::Init does (src/carnot/exec/exec_graph.cc:52-104), with the GPU node classes
 * at the operator switch, and runs it over RowBatches of host tables.  The node classes keep
 * the reference's ExecNode NVI (Init / Prepare / Open / ConsumeNext / Close,
 * src/carnot/exec/exec_node.h:145-315) and resolve every ScalarFunc / AggregateExpression by
 * (name, registry arg types) like udf::Registry (src/carnot/udf/registry.cc:172-198).
 *
 * Reference interfaces replaced:
 *   pxc_execute_plan   Carnot::ExecutePlan for one plan fragment
 *                      (src/carnot/carnot.cc:221-333) over MemorySource tables
 *                      (src/carnot/exec/memory_source_node.cc:54-124).
 *   pxc_explain_plan   the lowering step alone (no device): which nodes the operator switch
 *                      picks, fused chains, compiled device programs.
 *   pxc_store_*        table_store::TableStore::AddTable / Table::TransferRecordBatch
 *                      (src/table_store/table/table.cc:174-200) with the tables in HBM.
 *
 * Errors: px.statuspb.Code values (src/common/base/statuspb/status.proto:27-52);
 * pxc_last_error() has the message.  There is no CPU execution path: a plan whose operators
 * or UDF/UDA signatures have no device implementation fails with UNIMPLEMENTED / NOT_FOUND.
 */
#ifndef PXCARNOT_H_
#define PXCARNOT_H_

#include <stdint.h>

#include "pxg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A MemorySource table as a sequence of RowBatches (batch-major: cols[b * ncols + c]).
 * batch_flags (optional): bit0 eow, bit1 eos per batch; when NULL the source behaves like
 * MemorySourceNode (eow = eos = true on the last batch). */
typedef struct {
  const char* name;
  int32_t ncols;
  int32_t nbatches;
  const int32_t* col_types;
  const pxg_column_view* cols;
  const uint8_t* batch_flags;
} pxc_table;

/* Threading: every pxc_* call that takes an engine holds the engine's lock for its duration,
 * so concurrent callers are serialised (the store, group-count hints, aggregation cache and
 * the engine's device stream are shared by all queries on one engine).  For concurrent query
 * execution, create one engine per query thread (Carnot runs each query on its own task,
 * src/vizier/services/agent/manager/exec.cc:84-97). */
typedef struct pxc_engine pxc_engine;

int32_t pxc_engine_create(int32_t device, pxc_engine** out);
int32_t pxc_engine_destroy(pxc_engine* engine);

/* Executes the first plan fragment of a binary planpb.Plan.  Every sink's RowBatches are
 * serialised into *out (PXRB layout: tests/oracle_client.py::parse_pxrb), released with
 * pxc_free. */
int32_t pxc_execute_plan(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables,
                         const pxc_table* tables, uint8_t** out, int64_t* out_len);

/* RowBatches for one GRPCSourceOperator node (grpc_source_node.cc:52-87), as the
 * schemapb.RowBatchData payloads of the TransferResultChunkRequests it received, in order. */
typedef struct {
  uint64_t grpc_source_id;  /* the GRPCSource's plan node id (GRPCSinkOperator.grpc_source_id) */
  int32_t nmessages;
  int32_t reserved;
  const uint8_t* const* messages;
  const int64_t* lengths;
} pxc_grpc_input;

/* pxc_execute_plan for fragments with GRPC sources / sinks (the PEM -> Kelvin hop,
 * grpc_sink_node.cc:276-330).  GRPC sources read `inputs`; every GRPCSinkOperator whose
 * destination is a grpc_source_id serialises its RowBatches (split at the reference's 1 MiB
 * request limit) as schemapb.RowBatchData into *grpc_out: "PXGS" u32 magic, u32 nsinks, then
 * per sink u64 destination id, u32 nmessages, (u32 length, bytes)*.  Released with pxc_free.
 * Sinks to a result table are returned in *out as by pxc_execute_plan. */
int32_t pxc_execute_plan_grpc(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables,
                              const pxc_table* tables, int32_t ninputs, const pxc_grpc_input* inputs, uint8_t** out,
                              int64_t* out_len, uint8_t** grpc_out, int64_t* grpc_out_len);

/* RowBatch::ToProto / FromProto (src/table_store/schema/row_batch.cc:161-224): one RowBatch of
 * host Arrow-layout columns <-> schemapb.RowBatchData wire bytes (the canonical proto3
 * encoding).  from_proto returns the batch in PXRB layout (one sink "rowbatch", one batch). */
int32_t pxc_rowbatch_to_proto(int32_t ncols, const pxg_column_view* cols, int64_t nrows, int32_t eow, int32_t eos,
                              uint8_t** out, int64_t* out_len);
int32_t pxc_rowbatch_from_proto(const uint8_t* msg, int64_t len, uint8_t** out, int64_t* out_len);

/* Lowering only (no device): a text description of the node graph and device programs. */
int32_t pxc_explain_plan(const uint8_t* plan, int64_t plan_len, int32_t ntables, const pxc_table* tables,
                         char** out);

/* HBM-resident table store (table_store::TableStore / Table, src/table_store/table/table.h:71-199):
 * named device tables owned by the engine that persist across queries.  A MemorySource whose
 * name is not among the call's host tables reads the stored table straight from HBM; a fused
 * Filter/Map -> blocking Agg chain over it consumes the device table in place (no per-query
 * upload).  Appends are host Arrow-layout batches, coalesced by the device table's pinned
 * staging into large chunks (the hot -> cold compaction of table.cc:409-427 happens at append).
 * When the table has a column named "time_" its rows must arrive in non-decreasing time_
 * order (the order Stirling pushes), which lets MemorySource start_time / stop_time select
 * [first row >= start, first row > stop) by a device binary search (table.cc:56-95,310-336). */
int32_t pxc_store_create_table(pxc_engine* engine, const char* name, int32_t ncols, const int32_t* types,
                               const char* const* names);
int32_t pxc_store_append(pxc_engine* engine, const char* name, const pxg_column_view* cols, int64_t nrows);
int32_t pxc_store_drop_table(pxc_engine* engine, const char* name);
/* Rows in the table, -1 when there is no such table. */
int64_t pxc_store_num_rows(pxc_engine* engine, const char* name);
/* The device table itself (owned by the store), NULL when absent. */
pxg_table* pxc_store_device_table(pxc_engine* engine, const char* name);
/* The engine's device context (owned by the engine): libpxg calls on stored tables use it. */
pxg_ctx* pxc_engine_ctx(pxc_engine* engine);
/* pxc_explain_plan with the engine's stored tables visible. */
int32_t pxc_engine_explain_plan(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables,
                                const pxc_table* tables, char** out);

/* The engine's own lowering of a plan's (fused Filter/Map ->) aggregation as a pxg_agg over a
 * device table named table_name with the given column types (the MemorySource is lowered as
 * over a stored device table).  *n_keys / *n_udas and uda_kinds[0..n_udas) (pxg_uda_kind,
 * capacity 16) describe its result columns.  Release with pxg_agg_destroy. */
int32_t pxc_plan_create_agg(pxg_ctx* ctx, const uint8_t* plan, int64_t plan_len, const char* table_name,
                            int32_t ncols, const int32_t* types, int64_t expected_groups, pxg_agg** out,
                            int32_t* n_keys, int32_t* n_udas, int32_t* uda_kinds);
/* Execution statistics (ExecNodeStats, src/carnot/exec/exec_node.h:41-125; carnot.cc:379-420).
 * With analyze on, every later query collects per-node total / self time and extra metrics as
 * well as the always-kept rows / bytes / batches in and out.  pxc_engine_last_stats returns the
 * last query's stats as a JSON object (malloc'ed, NUL-terminated; release with pxc_free):
 * {"bytes_processed", "rows_processed" (the sources' output, exec_graph.cc:333-347),
 *  "nodes": [{"node_id", "name", "bytes_output", "records_output", "batches_output",
 *             "bytes_input", "records_input", "batches_input", "total_execution_time_ns",
 *             "self_execution_time_ns", "extra_metrics", "extra_info"}, ...]} (field names of
 * queryresultspb.OperatorExecutionStats). */
int32_t pxc_engine_set_analyze(pxc_engine* engine, int32_t on);
int32_t pxc_engine_last_stats(pxc_engine* engine, char** out, int64_t* out_len);
void pxc_free(void* p);
/* QuantilesUDA::Finalize JSON (math_sketches.h:40-54, bytes as rapidjson's Writer emits them)
 * for n groups of 7 doubles (p01..p99): one buffer of n NUL-terminated strings (pxc_free). */
int32_t pxc_quantiles_json(const double* q7, int64_t n, char** out, int64_t* out_len);
const char* pxc_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* PXCARNOT_H_ */
