/*
 * pxg.h — C ABI of the MI355X-native Carnot columnar hot path (libpxg.so).
 *
 * This is the drop-in boundary.  The reference has no FFI for this path: its
 * Filter/Map/Agg nodes call the UDF registry in-process.  These entry points are what the
 * reference-side GPU exec nodes (GpuFilterNode / GpuMapNode / GpuAggNode, added at the
 * operator switch in src/carnot/exec/exec_graph.cc:66-80) would bind; INTEGRATION.md shows
 * that binding.  Plain pointers and sizes only; no torch / C++ types cross the ABI.
 *
 * Reference interfaces replaced (file:line under /root/reference):
 *   pxg_table_*            table_store::Table + RowBatch column buffers
 *                          (src/table_store/table/table.h:71-199,
 *                           src/table_store/schema/row_batch.h:40-129) — HBM-resident copy.
 *   pxg_filter             FilterNode::ConsumeNextImpl (src/carnot/exec/filter_node.cc:132-171)
 *                          + VectorNativeScalarExpressionEvaluator
 *                          (src/carnot/exec/expression_evaluator.cc:191-275).
 *   pxg_map                MapNode::ConsumeNextImpl (src/carnot/exec/map_node.cc:64-71)
 *                          + ArrowNativeScalarExpressionEvaluator (expression_evaluator.cc:277-342).
 *   pxg_agg_*              AggNode (src/carnot/exec/agg_node.cc:88-542) with the builtin UDAs
 *                          count/sum/mean/min/max (src/carnot/funcs/builtins/math_ops.h:583-772)
 *                          and quantiles (src/carnot/funcs/builtins/math_sketches.h:33-82);
 *                          pxg_agg_consume with a filter program = the fused
 *                          MemorySource -> Filter -> Map -> BlockingAgg chain.
 *   pxg_agg_export_partial /
 *   pxg_agg_import_partial partial_agg / finalize_results split
 *                          (src/carnot/planpb/plan.proto:250-257), exchanged between GPUs.
 *
 * Error convention: every call returns a px.statuspb.Code value
 * (src/common/base/statuspb/status.proto:27-52); pxg_last_error() gives the message of the
 * last failing call on the calling thread.  No C++ exception crosses the ABI.
 *
 * Threading: a pxg_ctx owns one HIP stream; all work issued through a ctx is stream-ordered
 * and asynchronous unless the call says it synchronises.  Handles are not thread-safe; use one
 * ctx per query thread (exec_graph.cc:177-289 drives one query on one thread).
 */
#ifndef PXG_H_
#define PXG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PXG_ABI_VERSION 1

/* px.types.DataType (src/shared/types/typespb/types.proto:26-34). */
enum pxg_data_type {
  PXG_DATA_TYPE_UNKNOWN = 0,
  PXG_BOOLEAN = 1,
  PXG_INT64 = 2,
  PXG_UINT128 = 3,
  PXG_FLOAT64 = 4,
  PXG_STRING = 5,
  PXG_TIME64NS = 6
};

/* px.statuspb.Code (src/common/base/statuspb/status.proto:27-52). */
enum pxg_code {
  PXG_OK = 0,
  PXG_CANCELLED = 1,
  PXG_UNKNOWN = 2,
  PXG_INVALID_ARGUMENT = 3,
  PXG_DEADLINE_EXCEEDED = 4,
  PXG_NOT_FOUND = 5,
  PXG_ALREADY_EXISTS = 6,
  PXG_PERMISSION_DENIED = 7,
  PXG_UNAUTHENTICATED = 8,
  PXG_INTERNAL = 9,
  PXG_UNIMPLEMENTED = 10,
  PXG_RESOURCE_UNAVAILABLE = 11,
  PXG_SYSTEM = 12,
  PXG_FAILED_PRECONDITION = 13
};

/* ---------------------------------------------------------------------------------------
 * Columns.  Arrow layout per column (Pixie never sets validity bitmaps):
 *   INT64 / TIME64NS / FLOAT64 : 8-byte values
 *   UINT128                    : 16-byte values {low u64, high u64}
 *   BOOLEAN                    : one byte per value (0/1); the host node unpacks Arrow bits
 *   STRING                     : int32 offsets[length+1] + UTF-8 bytes
 * ------------------------------------------------------------------------------------- */
typedef struct {
  int32_t type;           /* pxg_data_type */
  int32_t reserved;
  int64_t length;         /* rows */
  const void* values;     /* fixed-width types */
  const int32_t* offsets; /* STRING */
  const uint8_t* data;    /* STRING payload */
} pxg_column_view;

/* Host-visible output column.  Buffers are allocated by the library; release with
 * pxg_result_free (which frees every column of one result). */
typedef struct {
  int32_t type;
  int32_t reserved;
  int64_t length;
  void* values;
  int32_t* offsets;
  uint8_t* data;
  int64_t data_len;
} pxg_column_out;

/* ---------------------------------------------------------------------------------------
 * Expression programs: a typed postfix program compiled by the host node from a
 * plan::ScalarExpression after resolving each ScalarFunc against the device UDF registry
 * (udf::Registry::GetScalarUDFDefinition(name, arg types), src/carnot/udf/registry.cc:172-198).
 * Every stack slot carries a statically known type; mixed-type UDF signatures are compiled
 * with explicit conversions (the same C++ usual arithmetic conversions the reference's
 * FixedSizedValueType operators perform, src/shared/types/types.h:72-104).
 * ------------------------------------------------------------------------------------- */
enum pxg_opcode {
  PXG_OP_NOP = 0,
  PXG_OP_COL = 1,      /* push column[arg] (type = column type)                          */
  PXG_OP_CONST = 2,    /* push imm (BOOLEAN/INT64/TIME64NS: integer, FLOAT64: bits);
                          STRING: arg = pool offset, imm = length; UINT128: arg=pool off  */
  PXG_OP_I2F = 3,      /* int64 -> double                                                */
  PXG_OP_B2I = 4,      /* bool -> int64                                                  */
  PXG_OP_I2B = 5,      /* int64 -> bool (x != 0)                                         */
  PXG_OP_F2I = 6,      /* double -> int64, truncating (static_cast<int64_t>)             */
  PXG_OP_ADD_I = 10, PXG_OP_SUB_I = 11, PXG_OP_MUL_I = 12, PXG_OP_MOD_I = 13,
  PXG_OP_BIN_I = 14,   /* a - a % b (BinUDF, math_ops.h:512-527)                         */
  PXG_OP_NEG_I = 15, PXG_OP_INV_I = 16,
  PXG_OP_ADD_F = 20, PXG_OP_SUB_F = 21, PXG_OP_MUL_F = 22, PXG_OP_DIV_F = 23,
  PXG_OP_NEG_F = 24,
  PXG_OP_EQ_I = 30, PXG_OP_NE_I = 31, PXG_OP_LT_I = 32, PXG_OP_LE_I = 33,
  PXG_OP_GT_I = 34, PXG_OP_GE_I = 35,
  PXG_OP_EQ_F = 40, PXG_OP_NE_F = 41, PXG_OP_LT_F = 42, PXG_OP_LE_F = 43,
  PXG_OP_GT_F = 44, PXG_OP_GE_F = 45,
  PXG_OP_APPROX_EQ_F = 46, /* |a-b| <  DBL_EPSILON (ApproxEqualUDF)                      */
  PXG_OP_APPROX_NE_F = 47, /* |a-b| >  DBL_EPSILON (ApproxNotEqualUDF)                   */
  PXG_OP_EQ_S = 50, PXG_OP_NE_S = 51, PXG_OP_LT_S = 52, PXG_OP_LE_S = 53,
  PXG_OP_GT_S = 54, PXG_OP_GE_S = 55,
  PXG_OP_EQ_U = 60, PXG_OP_NE_U = 61,
  PXG_OP_AND = 70, PXG_OP_OR = 71, PXG_OP_NOT = 72,
  /* push the little-endian 8-byte word at byte offset imm of STRING column[arg], as `type`
   * (INT64 / TIME64NS / FLOAT64); 0 when the string is shorter than imm + 8.  Reads a UDA state
   * out of a serialized_expressions column (UDA::Deserialize, udf.h:98-100).             */
  PXG_OP_STATE_WORD = 80
};

typedef struct {
  uint16_t op;   /* pxg_opcode */
  uint16_t type; /* result type of the instruction */
  int32_t arg;
  int64_t imm;
} pxg_insn;

#define PXG_MAX_PROGRAM 48
#define PXG_MAX_STACK 8

typedef struct {
  int32_t n_insns;
  int32_t result_type;
  const pxg_insn* insns;
  int32_t pool_len;     /* constant pool (string / uint128 constants) */
  int32_t reserved;
  const uint8_t* pool;
} pxg_program;

/* ---------------------------------------------------------------------------------------
 * Contexts and HBM-resident tables.
 * ------------------------------------------------------------------------------------- */
typedef struct pxg_ctx pxg_ctx;
typedef struct pxg_table pxg_table;
typedef struct pxg_agg pxg_agg;
typedef struct pxg_comm pxg_comm;

int32_t pxg_abi_version(void);
const char* pxg_last_error(void);
int32_t pxg_device_count(int32_t* count);

/* One context per device per query thread; owns a HIP stream. */
int32_t pxg_ctx_create(int32_t device, pxg_ctx** out);
int32_t pxg_ctx_destroy(pxg_ctx* ctx);
/* Blocks until all work issued through ctx is complete.  Device faults surface here. */
int32_t pxg_ctx_sync(pxg_ctx* ctx);
/* The hipStream_t the ctx issues on (for callers that record their own events). */
void* pxg_ctx_stream(pxg_ctx* ctx);
/* Kernel timing: when enabled every library kernel launch is bracketed by HIP events on the
 * ctx stream; pxg_ctx_kernel_stats returns launches and summed device milliseconds of the
 * named kernel since the last reset ("*": every kernel launched meanwhile, summed). */
int32_t pxg_ctx_set_profiling(pxg_ctx* ctx, int32_t enabled);
int32_t pxg_ctx_kernel_stats(pxg_ctx* ctx, const char* kernel_name, int64_t* launches,
                             double* total_ms);
int32_t pxg_ctx_reset_stats(pxg_ctx* ctx);
/* Restrict profiling to launches of one kernel (NULL: every kernel), so a timed region pays
 * the event bracketing only where a launch duration is wanted. */
int32_t pxg_ctx_profile_only(pxg_ctx* ctx, const char* kernel_name);

/* A table: ncols typed columns, stored as device chunks of <= 2^24 rows (STRING payload
 * < 2^31 bytes per chunk).  Appends coalesce small RowBatches through a pinned staging buffer
 * (tiny batches are the norm: src/vizier/services/agent/pem/pem_manager.cc:85-99). */
int32_t pxg_table_create(pxg_ctx* ctx, int32_t ncols, const int32_t* types, pxg_table** out);
int32_t pxg_table_destroy(pxg_table* t);
/* Append one RowBatch given as host columns (copied; the caller may free on return). */
int32_t pxg_table_append(pxg_table* t, const pxg_column_view* cols, int64_t nrows);
/* Append columns that already live in device memory (copied device-to-device). */
int32_t pxg_table_append_device(pxg_table* t, const pxg_column_view* cols, int64_t nrows);
/* Flush staging so every appended row is resident in HBM. */
int32_t pxg_table_flush(pxg_table* t);
int64_t pxg_table_num_rows(const pxg_table* t);
int32_t pxg_table_num_chunks(const pxg_table* t);
/* Device bytes of the table's column data in Arrow layout (values, offsets, payload). */
int64_t pxg_table_device_bytes(const pxg_table* t, int32_t col);
/* Copy rows [begin, end) of column col back to host (sink path): buffers from the pinned
 * result pool, released with pxg_result_free (also on error, nothing is left allocated). */
int32_t pxg_table_fetch(pxg_table* t, int32_t col, int64_t begin, int64_t end,
                        pxg_column_out* out);
/* Time-range cursor support (Table::FindRowIDFromTimeFirstGreaterThanOrEqual / ...GreaterThan,
 * src/table_store/table/table.cc:310-336): *row = the first row whose value in the
 * non-decreasing INT64/TIME64NS column col is >= value (strict = 0) or > value (strict = 1);
 * num_rows when there is none. */
int32_t pxg_table_time_bound(pxg_table* t, int32_t col, int64_t value, int32_t strict, int64_t* row);
/* Device result image (sink path; MemorySinkNode::ConsumeNextImpl,
 * src/carnot/exec/memory_sink_node.cc:75-80, keeps the row batches an operator sends it): rows
 * [starts[0], starts[n_batches]) of t as n_batches row batches (batch i = rows [starts[i],
 * starts[i+1]); eow / eos on the last one as given) in the engine's PXRB batch layout, built in
 * device memory; *bytes = its size.  Single-chunk tables (<= 2^24 rows): PXG_UNIMPLEMENTED
 * otherwise, and the caller fetches the columns instead.  pxg_pxrb_copy moves the image into a
 * host buffer of *bytes bytes (one DMA; waits); pxg_pxrb_destroy releases it. */
typedef struct pxg_pxrb pxg_pxrb;
int32_t pxg_table_pxrb_image(pxg_table* t, const int64_t* starts, int64_t n_batches, int32_t last_eow,
                             int32_t last_eos, pxg_pxrb** out, int64_t* bytes);
int32_t pxg_pxrb_copy(pxg_pxrb* img, void* dst);
int32_t pxg_pxrb_destroy(pxg_pxrb* img);

/* ---------------------------------------------------------------------------------------
 * Filter and Map over a device table (non-fused operator shapes).
 * ------------------------------------------------------------------------------------- */
/* FilterNode: evaluates pred over rows [begin,end) and writes the selected columns (in
 * `select` order) of the passing rows, order preserved, into a new device table.  Row counts
 * and sizes are known to the host on return; the column contents are written in order on the
 * ctx stream (device consumers need no sync; pxg_table_fetch synchronises).  Output columns
 * come from the ctx's buffer pool, which pxg_table_destroy refills. */
int32_t pxg_filter(pxg_table* in, const pxg_program* pred, int32_t n_select,
                   const int32_t* select, int64_t begin, int64_t end, pxg_table** out);
/* pxg_filter over rows that are the concatenation of n_splits RowBatches (split_rows[i] rows
 * each, summing to end - begin): one device pass for all of them, and out_split_rows[i]
 * receives the number of output rows that came from batch i, so the caller emits one output
 * batch per input batch exactly as FilterNode does (filter_node.cc:132-171). */
int32_t pxg_filter_split(pxg_table* in, const pxg_program* pred, int32_t n_select,
                         const int32_t* select, int64_t begin, int64_t end, int32_t n_splits,
                         const int64_t* split_rows, int64_t* out_split_rows, pxg_table** out);
/* MapNode: one output column per program (fixed-width results; a program that is a single
 * column reference of any type is passed through).  Same completion rule as pxg_filter. */
int32_t pxg_map(pxg_table* in, int32_t n_exprs, const pxg_program* exprs, int64_t begin,
                int64_t end, pxg_table** out);

/* ---------------------------------------------------------------------------------------
 * Hash group-by aggregation with device UDAs.
 * ------------------------------------------------------------------------------------- */
enum pxg_uda_kind {
  PXG_UDA_COUNT = 1,     /* CountUDA      -> INT64                                         */
  PXG_UDA_SUM = 2,       /* SumUDA        -> INT64 (INT64/BOOLEAN args) or FLOAT64          */
  PXG_UDA_MEAN = 3,      /* MeanUDA       -> FLOAT64                                        */
  PXG_UDA_MIN = 4,       /* MinUDA        -> arg type                                       */
  PXG_UDA_MAX = 5,       /* MaxUDA        -> arg type (init numeric_limits<T>::min())       */
  PXG_UDA_QUANTILES = 6, /* QuantilesUDA  -> STRING JSON {p01..p99}; 7 FLOAT64 on device    */
  PXG_UDA_MEAN_MERGE = 7,/* MeanUDA::Merge of deserialized MeanInfo states, then Finalize:
                            arg = FLOAT64 state sum, arg2 = INT64 state size -> FLOAT64
                            sum(arg) / double(sum(arg2)) (math_ops.h:586-594)              */
  PXG_UDA_MINSUM = 100   /* test UDA of agg_node_test.cc:44-72 (sum of min(a,b), init arg)  */
};

typedef struct {
  int32_t kind;        /* pxg_uda_kind */
  int32_t arg_type;    /* type of the update argument */
  pxg_program arg;     /* value expression over the input columns */
  pxg_program arg2;    /* second argument (MINSUM) */
  int32_t has_init;
  int32_t reserved;
  int64_t init_i64;    /* init argument (MINSUM: initial sum) */
} pxg_uda_spec;

typedef struct {
  int32_t n_keys;
  int32_t n_udas;
  const pxg_program* keys;  /* group key expressions: a bare column reference, or a
                               fixed-width program (e.g. bin(time_, 10s))              */
  const pxg_uda_spec* udas;
  const pxg_program* filter; /* optional predicate fused in front of the agg (NULL: none) */
  int64_t expected_groups;   /* sizing hint; the table grows on demand */
  int32_t windowed;          /* AggregateOperator.windowed */
  int32_t emit_states;       /* partial_agg && !finalize_results (plan.proto:250-257): the
                                result is the groups, then one STRING column
                                "serialized_expressions" (operators.cc:251-257) holding, per
                                group, every UDA's Serialize() bytes back to back in plan
                                order: count u64; sum i64|f64; mean {u64 size, f64 sum};
                                min/max the native value (math_ops.h:583-772).  UDAs without
                                Serialize (quantiles, minsum) are UNIMPLEMENTED, as they are
                                not splittable in the reference (udf.h:367).            */
} pxg_agg_spec;

int32_t pxg_agg_create(pxg_ctx* ctx, const pxg_agg_spec* spec, pxg_agg** out);
int32_t pxg_agg_destroy(pxg_agg* agg);
/* Update with rows [begin, end) of table (filter applied first when the spec has one). */
int32_t pxg_agg_consume(pxg_agg* agg, pxg_table* table, int64_t begin, int64_t end);
/* Finalize: resolves deferred inserts, computes quantiles, compacts groups.  Synchronises. */
int32_t pxg_agg_finalize(pxg_agg* agg, int64_t* n_groups);
/* Result columns (groups then values, AggNode output order, agg_node.cc:336-346; with
 * spec.emit_states: groups then serialized_expressions, n_cols = n_keys + 1).  For
 * QUANTILES the column is FLOAT64 with 7 values per group (p01,p10,p25,p50,p75,p90,p99,
 * group-major); the host node renders the JSON string (math_sketches.h:40-54). */
int32_t pxg_agg_result(pxg_agg* agg, pxg_column_out* cols, int32_t n_cols);
/* pxg_agg_result with skip[c] != 0 leaving value column c without buffers (type and length
 * set; the caller reads it another way, e.g. pxg_agg_quantile_lanes).  For a QUANTILES column,
 * skip[c] = 0x80 | lane_mask returns its plucked lanes instead: values = the lanes as
 * pxg_agg_quantile_lanes lays them out (lane-major, n_groups doubles per lane in mask order,
 * pluck's 0.0 for a group with a non-finite quantile), data = the n_groups finiteness bytes
 * (data_len = n_groups). */
int32_t pxg_agg_result_skip(pxg_agg* agg, pxg_column_out* cols, int32_t n_cols, const uint8_t* skip);
/* pxg_agg_finalize + pxg_agg_result_skip in one call: the finalize issues each result column's
 * device-to-host copy as soon as the column is produced (group keys while the quantile digests
 * still run), so the copies overlap the finalize.  Same columns, buffers and release
 * (pxg_result_free) as pxg_agg_result_skip. */
int32_t pxg_agg_finalize_result(pxg_agg* agg, int64_t* n_groups, pxg_column_out* cols, int32_t n_cols, const uint8_t* skip);
/* The finalized result as device column views into the agg's own result buffers (no copy),
 * for a device consumer (the engine's agg -> equijoin hand-off): valid until the agg's next
 * consume / finalize / destroy.  *bytes = the Arrow payload bytes (RowBatch::NumBytes).
 * UNIMPLEMENTED for results rendered on the host (QUANTILES, emit_states) and for the one
 * synthetic row of a group-less agg over no rows; the caller then uses pxg_agg_result. */
int32_t pxg_agg_result_device(pxg_agg* agg, pxg_column_view* cols, int32_t n_cols, int64_t* bytes);
/* The quantile lanes a post-aggregate pluck_float64 reads (MapNode over the AggNode output,
 * math_sketches.h:40-54 + the pluck UDF): the lanes set in lane_mask (bit k =
 * p01,p10,p25,p50,p75,p90,p99[k]), lane-major in lane order (the j-th selected lane of group g
 * at host_out[j * n_groups + g]) with pluck's value: 0.0 for a group whose 7 quantiles are not
 * all finite (a NaN / inf one truncates the reference's JSON, which pluck then fails to parse);
 * host_finite[g] = 1 when they are.  Host buffers hold n_groups * popcount(mask) doubles /
 * n_groups bytes. */
int32_t pxg_agg_quantile_lanes(pxg_agg* agg, int32_t uda, uint32_t lane_mask, double* host_out, uint8_t* host_finite);
void pxg_result_free(pxg_column_out* cols, int32_t n_cols);
/* Host buffers for result hand-off (no reference counterpart: replaces the per-query malloc of
 * the engine's result bytes).  Large requests come from a pool of pinned blocks reused across
 * queries (no page faults, full-speed DMA), small ones from malloc; pxg_host_free releases
 * either, and also accepts any malloc'ed pointer. */
void* pxg_host_alloc(int64_t bytes);
void pxg_host_free(void* p);
/* ClearAggState (agg_node.cc:173-180): drop all groups (windowed emit). */
int32_t pxg_agg_reset(pxg_agg* agg);
/* Number of selected (post-filter) rows consumed since the last reset. */
int32_t pxg_agg_rows_selected(pxg_agg* agg, int64_t* rows);
/* Sizes of an aggregation's device state (ExecNodeStats-style accounting, exec_node.h:41-128). */
typedef struct {
  int64_t table_capacity;   /* slots of the open-addressing group table */
  int64_t groups;           /* groups inserted since the last reset */
  int64_t rows_selected;    /* staged (post-filter) rows since the last reset */
  int64_t key_arena_bytes;  /* published group-key records */
  int64_t staging_capacity; /* staged rows the buffers hold without growing */
  int32_t fast_path_keys;   /* key count of the register-key consume kernel; 0 = generic kernel */
  int32_t big_sort_groups;  /* last finalize: big quantile groups the selection path handed to the
                               full sort path (NaN values, a gathered bin > 16384 values) */
  int32_t hc_mode;          /* 1: this run stages partition records (high-cardinality mode) */
  int32_t hc_partition_bits;/* last high-cardinality finalize: log2 of its partition count */
  int32_t hc_reruns;        /* last high-cardinality finalize: partition passes rerun because a
                               partition's distinct keys overflowed its LDS table */
} pxg_agg_stats;
int32_t pxg_agg_info(pxg_agg* agg, pxg_agg_stats* stats);

/* Partial aggregation (plan.proto:250-257).  Export serialises every group's key and UDA
 * state (quantile inputs as raw values) into n_parts device buffers partitioned by
 * hash(key) % n_parts; part_bytes[i] receives the size of part i.  Buffers are written into
 * dst (device memory, capacity dst_capacity bytes, parts laid out back to back; part i
 * starts at part_offsets[i]).  Call with dst == NULL to size.  Import merges a buffer
 * produced by export (on any device) into this agg (UDA Merge semantics). */
int32_t pxg_agg_export_partial(pxg_agg* agg, int32_t n_parts, void* dst, int64_t dst_capacity,
                               int64_t* part_offsets, int64_t* part_bytes);
int32_t pxg_agg_import_partial(pxg_agg* agg, const void* src, int64_t nbytes);
/* Import n_parts exported parts that lie in one device buffer (part i at src + part_offsets[i],
 * part_bytes[i] bytes: e.g. what one all-to-all received from every rank) in one pass. */
int32_t pxg_agg_import_partials(pxg_agg* agg, const void* src, int32_t n_parts,
                                const int64_t* part_offsets, const int64_t* part_bytes);
/* The export pxg_agg_alltoall sends: the same parts, laid out on the device (sizes, headers and
 * offsets computed by a device kernel, no host sizing pass) into a device buffer owned by the
 * aggregation (valid until its next export or destroy).  *parts receives that buffer; the parts
 * lie back to back, part i part_bytes[i] bytes (already 8-byte aligned); headers (optional,
 * n_parts * 64 bytes) receives each part's header, the first 64 bytes of the part.  The bytes
 * equal pxg_agg_export_partial's.  Exchange-v2 aggregations only (FAILED_PRECONDITION else). */
int32_t pxg_agg_export_partial_dev(pxg_agg* agg, int32_t n_parts, void** parts, int64_t* part_bytes,
                                   uint8_t* headers);

/* ---------------------------------------------------------------------------------------
 * Intra-node exchange over RCCL / xGMI (the PEM-partial -> Kelvin-finalize hop,
 * src/carnot/planner/distributed/splitter/partial_op_mgr/partial_op_mgr.cc:69-83, which the
 * reference runs over GRPCSink/GRPCSource).  One rank per GPU.
 * ------------------------------------------------------------------------------------- */
#define PXG_COMM_ID_BYTES 128
/* An RCCL unique id (PXG_COMM_ID_BYTES bytes); one rank makes it, every rank passes it on. */
int32_t pxg_comm_unique_id(uint8_t* id_out, int32_t id_bytes);
/* Communicator of `nranks` ranks over ctx's device; collective (every rank calls it). */
int32_t pxg_comm_init(pxg_ctx* ctx, int32_t rank, int32_t nranks, const uint8_t* id, int32_t id_bytes, pxg_comm** out);
int32_t pxg_comm_destroy(pxg_comm* comm);
/* A host transport behind the same communicator interface, for ranks that cannot open an RCCL
 * communicator (several ranks sharing one GPU, CPU-hosted process groups such as gloo): the
 * caller supplies only the byte mover.  pxg_agg_alltoall and pxg_agg_gather then run exactly the
 * device code of the RCCL path (device part layout, {bytes, header} records, import with the
 * received headers, gather rebase); the bytes travel through pinned host memory instead of xGMI.
 *
 * Each grouped exchange calls `fn` once with n_ops point-to-point transfers between host buffers:
 * op.send != 0 sends op.bytes from op.buf to rank op.peer, else receives op.bytes from op.peer
 * into op.buf.  The k-th op of a rank to a peer matches that peer's k-th op from the rank, as
 * grouped ncclSend / ncclRecv pairs do.  Transfers of a rank to itself and zero-byte transfers
 * are done inside libpxg and never passed.  fn returns 0 on success; anything else fails the
 * call with PXG_INTERNAL (the peers then see their own transport fail or time out).  fn runs on
 * the calling thread, inside the libpxg call. */
typedef struct {
  int32_t peer;
  int32_t send;
  void* buf;
  int64_t bytes;
} pxg_xfer;
typedef int32_t (*pxg_xfer_fn)(void* user, int32_t n_ops, const pxg_xfer* ops);
int32_t pxg_comm_init_host(pxg_ctx* ctx, int32_t rank, int32_t nranks, pxg_xfer_fn fn, void* user, pxg_comm** out);
/* Re-partition agg's state across the ranks by hash(group key): export nranks parts, exchange
 * the byte counts and the parts (grouped ncclSend/ncclRecv on the ctx stream), reset agg and
 * import what arrived.  Afterwards every group lives on exactly one rank; finalize locally.
 * A rank whose export fails (its finalize checks, or parts past the send buffer) announces -1
 * bytes to every peer; then no rank moves parts and every rank returns an error, so no peer is
 * left waiting inside the collective.
 * Collective.  bytes_sent / bytes_recv (optional) receive this rank's traffic. */
int32_t pxg_agg_alltoall(pxg_agg* agg, pxg_comm* comm, int64_t* bytes_sent, int64_t* bytes_recv);
/* Gather every rank's finalized result rows on `root` (the final rows to one
 * rank, as Kelvin's GRPCSink streams them to the query broker, grpc_sink_node.cc:305-330).  Call
 * after pxg_agg_alltoall + pxg_agg_finalize on every rank (collective).  On the root the result
 * (pxg_agg_result and friends) becomes the concatenation of all ranks' rows, its own first, then
 * the others by rank; *n_groups receives the total (0 on the other ranks, whose results are left
 * as they were).  Group-less aggregates are UNIMPLEMENTED (they merge, they do not concatenate). */
int32_t pxg_agg_gather(pxg_agg* agg, pxg_comm* comm, int32_t root, int64_t* n_groups);

/* ---------------------------------------------------------------------------------------
 * Equijoin (EquijoinNode, src/carnot/exec/equijoin_node.cc:53-470).  A hash table is built on
 * the build table's key columns (exact key equality, any duplicates kept), the probe table is
 * streamed against it, and the output is materialised as a new device table whose columns are
 * (side, column) pairs: side 0 = probe table, side 1 = build table.  Rows of a side that has no
 * match get the reference's default values (0 / false / "", AppendColumnDefaultValue).  The
 * host node maps the plan's left/right parents and JoinType onto build/probe and the two
 * emit_unmatched flags exactly as EquijoinNode::InitImpl does (equijoin_node.cc:53-116).
 * Output order is the reference's: probe rows in table order, each followed by its matching
 * build rows in build-table order (or one row with build defaults when unmatched probe rows
 * are emitted); then the unmatched build rows, grouped by key (the reference emits these in
 * hash-map order, which is unspecified).  *probe_rows (may be NULL) receives the number of
 * rows produced by probe rows, i.e. where the unmatched build rows start: the host node cuts
 * an output batch there (FlushChunkedRows at probe eos, equijoin_node.cc:388-390).
 * ------------------------------------------------------------------------------------- */
typedef struct {
  int32_t n_keys;
  int32_t emit_unmatched_probe;  /* LEFT_OUTER with probe = left, FULL_OUTER */
  int32_t emit_unmatched_build;  /* LEFT_OUTER with build = left, FULL_OUTER */
  int32_t n_out;
  const int32_t* build_keys;     /* n_keys column indices of the build table */
  const int32_t* probe_keys;     /* n_keys column indices of the probe table */
  const int32_t* out_side;       /* n_out: 0 probe, 1 build */
  const int32_t* out_col;        /* n_out: column index within that side */
} pxg_join_spec;

int32_t pxg_join(pxg_table* build, pxg_table* probe, const pxg_join_spec* spec, pxg_table** out,
                 int64_t* probe_rows);

/* ---------------------------------------------------------------------------------------
 * Synthetic http_events generator (bench/test data; SURVEY.md §8d spec, counter-based
 * splitmix64 so every row is a pure function of (seed, row) and shards are independent).
 * Host-side; writes Arrow-layout host buffers allocated by the library.
 * Columns: 0 time_ TIME64NS, 1 upid UINT128, 2 service STRING, 3 req_path STRING,
 *          4 remote_addr STRING, 5 resp_status INT64, 6 latency INT64,
 *          7 req_body_size INT64, 8 resp_body_size INT64, 9 pod STRING
 * ------------------------------------------------------------------------------------- */
#define PXG_HTTP_EVENTS_NCOLS 10
int32_t pxg_datagen_http_events(uint64_t seed, int64_t row_begin, int64_t nrows,
                                int64_t n_addr_keys, int32_t n_threads, pxg_column_out* cols);
/* The same rows generated on the device and appended to an http_events-shaped table (the 10
 * columns above), bit-identical to pxg_datagen_http_events: big bench tables are built in HBM
 * without host generation or PCIe upload.  Synchronises. */
int32_t pxg_table_append_http_events(pxg_table* t, uint64_t seed, int64_t row_begin, int64_t nrows,
                                     int64_t n_addr_keys);

/* ---------------------------------------------------------------------------------------
 * Diagnostics (tests).  Centroid-boundary chains of the quantiles t-digest emulation for n
 * group sizes d_w (device int64), computed by the per-wave speculative chain (wave = 1) or the
 * single-lane sequential chain (wave = 0); boundaries to d_starts[i * cap ...], counts to
 * d_nc[i] (-1: more than cap).  Synchronises.
 * ------------------------------------------------------------------------------------- */
int32_t pxg_digest_chains(pxg_ctx* ctx, const int64_t* d_w, int32_t n, int32_t wave, uint32_t* d_starts,
                          int32_t cap, int32_t* d_nc);
/* Diagnostics (tests).  The merged digest of one group (the multi-GPU exchange's owner side,
 * tdigest batch add restated from math_sketches.h:38 / oracle/tdigest.h merge_batch): n items in
 * part order, d_vals = raw values (arg_type bits) or centroid means (double bits), d_wt = part
 * << 48 | weight (weight 0: a raw value); the 7 quantiles to d_out7.  Synchronises. */
int32_t pxg_digest_merge(pxg_ctx* ctx, const uint64_t* d_vals, const uint64_t* d_wt, int64_t n, int32_t arg_type, double* d_out7);

#ifdef __cplusplus
}
#endif

#endif /* PXG_H_ */
