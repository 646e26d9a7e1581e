// C++ host engine: the reference's execution-graph layer with GPU nodes at the operator switch.
//
// Reference structure mirrored (names kept):
//   ExecNode NVI ........................ src/carnot/exec/exec_node.h:145-315
//   ExecutionGraph::Init / Execute ...... src/carnot/exec/exec_graph.cc:52-289
//   MemorySourceNode .................... src/carnot/exec/memory_source_node.cc:54-124
//   FilterNode / MapNode / AggNode ...... filter_node.cc:78-171, map_node.cc:47-71, agg_node.cc:88-542
//   MemorySinkNode ...................... src/carnot/exec/memory_sink_node.cc
//   udf::Registry lookup ................ src/carnot/udf/registry.cc:172-198
//   UDF / UDA signatures ................ src/carnot/funcs/builtins/math_ops.cc:52-250,
//                                         math_sketches.cc:25-28
// The GPU nodes call libpxg (include/pxg.h) only; nothing here computes a row on the CPU.
// Post-aggregation work on the G result rows (QuantilesUDA's JSON rendering,
// math_sketches.h:40-54, and pluck_float64 of it, json_ops.h:131-153) is host-side output
// formatting, as in the reference, where UDA Finalize runs on the host.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include <unistd.h>

#include "../../include/pxcarnot.h"
#include "../../include/pxg.h"
#include "json_double.h"
#include "planpb_wire.h"

namespace pxc {

// ---------------------------------------------------------------------------------------
// Status (px::Status with statuspb codes, src/common/base/status.h:150-160).
// ---------------------------------------------------------------------------------------
struct Status {
  int32_t code = PXG_OK;
  std::string msg;
  bool ok() const { return code == PXG_OK; }
  static Status OK() { return Status(); }
};

static Status Err(int32_t code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  Status s;
  s.code = code;
  s.msg = buf;
  return s;
}

static Status FromPxg(int32_t code) {
  if (code == PXG_OK) return Status::OK();
  const char* m = pxg_last_error();
  return Err(code, "%s", m ? m : "libpxg error");
}

#define PXC_RETURN_IF_ERROR(expr) \
  do {                            \
    Status s_ = (expr);           \
    if (!s_.ok()) return s_;      \
  } while (0)
#define PXG_CALL(expr) PXC_RETURN_IF_ERROR(FromPxg(expr))

static thread_local std::string g_last_error;

// Opt-in host-side stage timing (PXC_TIMING=1): one stderr line per stage of a query.
static bool TimingOn() {
  static const bool on = std::getenv("PXC_TIMING") != nullptr;
  return on;
}
struct StageClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void Mark(const char* what) {
    if (!TimingOn()) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[pxc] %-24s %9.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

// ---------------------------------------------------------------------------------------
// RowBatch (src/table_store/schema/row_batch.h:40-129): Arrow-layout host columns, shared and
// never mutated; eow / eos flags.
// ---------------------------------------------------------------------------------------
struct HostColumn {
  int32_t type = 0;
  int64_t length = 0;
  const void* values = nullptr;
  const int32_t* offsets = nullptr;
  const uint8_t* data = nullptr;
  std::shared_ptr<void> owner;  // keeps library-allocated buffers alive

  pxg_column_view View() const {
    pxg_column_view v{};
    v.type = type;
    v.length = length;
    v.values = values;
    v.offsets = offsets;
    v.data = data;
    return v;
  }
};

// Owns one pxg_column_out (released with pxg_result_free).
struct OutHolder {
  pxg_column_out c{};
  ~OutHolder() { pxg_result_free(&c, 1); }
};

static HostColumn FromOut(const pxg_column_out& c) {
  auto h = std::make_shared<OutHolder>();
  h->c = c;
  HostColumn hc;
  hc.type = c.type;
  hc.length = c.length;
  hc.values = c.values;
  hc.offsets = c.offsets;
  hc.data = c.data;
  hc.owner = h;
  return hc;
}

// A column built on the host (string / double vectors), owning its buffers.
struct OwnedColumn {
  std::vector<uint8_t> values;
  std::vector<int32_t> offsets;
  std::vector<uint8_t> data;
};

// G empty strings (one zeroed offsets array, no per-row std::string).
static HostColumn EmptyStringColumn(int64_t n) {
  // n + 1 zero offsets and a zeroed 16-byte payload pad in one host-pool block.
  const size_t ob = (static_cast<size_t>(n) + 1) * 4;
  void* b = pxg_host_alloc(static_cast<int64_t>(ob + 16));
  if (!b) throw std::bad_alloc();
  std::memset(b, 0, ob + 16);
  HostColumn hc;
  hc.type = PXG_STRING;
  hc.length = n;
  hc.offsets = static_cast<const int32_t*>(b);
  hc.data = static_cast<const uint8_t*>(b) + ob;
  hc.owner = std::shared_ptr<void>(b, [](void* q) { pxg_host_free(q); });
  return hc;
}

// An uninitialised FLOAT64 column of n values in a libpxg host-pool block (reused across queries,
// so filling it touches no fresh pages); *out receives the buffer to fill.
static HostColumn PooledDoubleColumn(int64_t n, double** out) {
  void* b = pxg_host_alloc(n * 8 + 8);
  if (!b) throw std::bad_alloc();
  HostColumn hc;
  hc.type = PXG_FLOAT64;
  hc.length = n;
  hc.values = b;
  hc.owner = std::shared_ptr<void>(b, [](void* q) { pxg_host_free(q); });
  *out = static_cast<double*>(b);
  return hc;
}


struct RowBatch {
  std::vector<HostColumn> cols;
  int64_t num_rows = 0;
  bool eow = false, eos = false;
  // A device-resident batch (the agg -> equijoin hand-off): `cols` is empty and `dev` holds one
  // device column view per output column, valid while the batch is being sent.  Only sent to
  // nodes whose AcceptsDeviceBatch() is true.
  const pxg_column_view* dev = nullptr;
  int64_t dev_bytes = 0;
  // A device result image (the equijoin -> sink hand-off, pxg_table_pxrb_image): `cols` is
  // empty and the image holds image_batches row batches (num_rows rows in all) already in the
  // PXRB batch layout.  Only sent to nodes whose AcceptsResultImage() is true.
  std::shared_ptr<pxg_pxrb> image;
  int64_t image_batches = 0;
  int64_t image_bytes = 0;
};

using RowDescriptor = std::vector<int32_t>;  // column types (schema::RowDescriptor)

// ---------------------------------------------------------------------------------------
// Device programs and the device UDF / UDA registry (compile.py is the same table).
// ---------------------------------------------------------------------------------------
struct Program {
  std::vector<pxg_insn> insns;
  std::vector<uint8_t> pool;
  int32_t result_type = 0;
  pxg_program View() const {
    pxg_program p{};
    p.n_insns = static_cast<int32_t>(insns.size());
    p.result_type = result_type;
    p.insns = insns.data();
    p.pool_len = static_cast<int32_t>(pool.size());
    p.pool = pool.empty() ? nullptr : pool.data();
    return p;
  }
  bool IsColumn() const { return insns.size() == 1 && insns[0].op == PXG_OP_COL; }
};

static pxg_insn Insn(int op, int type, int32_t arg = 0, int64_t imm = 0) {
  pxg_insn i;
  i.op = static_cast<uint16_t>(op);
  i.type = static_cast<uint16_t>(type);
  i.arg = arg;
  i.imm = imm;
  return i;
}

// Append `src` to `dst`, relocating its constant-pool references.
static void AppendProgram(const Program& src, Program* dst) {
  const int32_t base = static_cast<int32_t>(dst->pool.size());
  dst->pool.insert(dst->pool.end(), src.pool.begin(), src.pool.end());
  for (pxg_insn i : src.insns) {
    if (i.op == PXG_OP_CONST && (i.type == PXG_STRING || i.type == PXG_UINT128)) i.arg += base;
    dst->insns.push_back(i);
  }
}

struct UdfDef {
  int32_t result = 0;
  int lconv = 0, rconv = 0;  // conversion opcode applied after operand 0 / 1
  std::vector<int> ops;      // empty: relabel (x + 0)
};

enum : int32_t { B = PXG_BOOLEAN, I = PXG_INT64, U = PXG_UINT128, F = PXG_FLOAT64, S = PXG_STRING, T = PXG_TIME64NS };

// ---------------------------------------------------------------------------------------
// schemapb.RowBatchData wire codec: RowBatch::ToProto / FromProto (row_batch.cc:161-224,
// schema.proto:31-79).  One Column message per column, its data in the typed oneof
// (1 boolean, 2 int64, 3 uint128, 4 time64ns, 5 float64, 6 string); repeated scalars packed
// (proto3), UInt128 {low = 1, high = 2}; num_rows = 2, eow = 3, eos = 4.  The encoding is the
// canonical one protobuf emits (fields in number order, proto3 defaults omitted).
// ---------------------------------------------------------------------------------------
struct PbOut {
  std::string b;
  void Varint(uint64_t v) {
    while (v >= 0x80) {
      b.push_back(static_cast<char>((v & 0x7F) | 0x80));
      v >>= 7;
    }
    b.push_back(static_cast<char>(v));
  }
  void Key(uint32_t field, uint32_t wire) { Varint((static_cast<uint64_t>(field) << 3) | wire); }
  void Len(uint32_t field, const std::string& body) {
    Key(field, 2);
    Varint(body.size());
    b += body;
  }
};

static int32_t PbFieldOfType(int32_t t) {
  switch (t) {
    case B: return 1;
    case I: return 2;
    case U: return 3;
    case T: return 4;
    case F: return 5;
    case S: return 6;
    default: return 0;
  }
}

// Rows [r0, r0 + n) of one column as a schemapb.Column message body.
static std::string EncodePbColumn(const HostColumn& c, int64_t r0, int64_t n) {
  PbOut data;  // the XxxColumn message
  if (n > 0) {
    PbOut packed;
    switch (c.type) {
      case B:
        for (int64_t r = r0; r < r0 + n; ++r) packed.Varint(static_cast<const uint8_t*>(c.values)[r] ? 1 : 0);
        data.Len(1, packed.b);
        break;
      case I:
      case T:
        for (int64_t r = r0; r < r0 + n; ++r) packed.Varint(static_cast<uint64_t>(static_cast<const int64_t*>(c.values)[r]));
        data.Len(1, packed.b);
        break;
      case F:
        packed.b.assign(reinterpret_cast<const char*>(static_cast<const double*>(c.values) + r0), static_cast<size_t>(n) * 8);
        data.Len(1, packed.b);
        break;
      case U:
        for (int64_t r = r0; r < r0 + n; ++r) {
          const uint64_t* v = static_cast<const uint64_t*>(c.values) + 2 * r;
          PbOut u;
          if (v[0]) { u.Key(1, 0); u.Varint(v[0]); }
          if (v[1]) { u.Key(2, 0); u.Varint(v[1]); }
          data.Len(1, u.b);
        }
        break;
      case S:
        for (int64_t r = r0; r < r0 + n; ++r) {
          data.Key(1, 2);
          const int32_t o0 = c.offsets[r], o1 = c.offsets[r + 1];
          data.Varint(static_cast<uint64_t>(o1 - o0));
          data.b.append(reinterpret_cast<const char*>(c.data) + o0, static_cast<size_t>(o1 - o0));
        }
        break;
      default: break;
    }
  }
  PbOut col;
  col.Len(static_cast<uint32_t>(PbFieldOfType(c.type)), data.b);
  return col.b;
}

static std::string EncodeRowBatchData(const RowBatch& rb, int64_t r0, int64_t n, bool eow, bool eos) {
  PbOut m;
  for (auto& c : rb.cols) m.Len(1, EncodePbColumn(c, r0, n));
  if (n) { m.Key(2, 0); m.Varint(static_cast<uint64_t>(n)); }
  if (eow) { m.Key(3, 0); m.Varint(1); }
  if (eos) { m.Key(4, 0); m.Varint(1); }
  return m.b;
}

static Status DecodeRowBatchData(const uint8_t* p, size_t len, RowBatch* rb) {
  try {
    planpb::Reader r(p, len);
    uint32_t f, w;
    int64_t num_rows = 0;
    while (r.Next(&f, &w)) {
      if (f == 1 && w == 2) {
        planpb::Reader col = r.Sub();
        uint32_t cf, cw;
        int32_t type = 0;
        auto oc = std::make_shared<OwnedColumn>();
        int64_t rows = 0;
        while (col.Next(&cf, &cw)) {
          if (cw != 2 || cf < 1 || cf > 6) { col.Skip(cw); continue; }
          static const int32_t kTypeOfField[7] = {0, B, I, U, T, F, S};  // ProtoDataType (row_batch.cc:181-199)
          type = kTypeOfField[cf];
          oc->values.clear();
          oc->offsets.assign(1, 0);
          oc->data.clear();
          rows = 0;
          planpb::Reader d = col.Sub();
          uint32_t df, dw;
          while (d.Next(&df, &dw)) {
            if (df != 1) { d.Skip(dw); continue; }
            if (type == S) {
              const std::string v = d.String();
              oc->data.insert(oc->data.end(), v.begin(), v.end());
              oc->offsets.push_back(static_cast<int32_t>(oc->data.size()));
              ++rows;
            } else if (type == U) {
              planpb::Reader u = d.Sub();
              uint64_t lo = 0, hi = 0;
              uint32_t uf, uw;
              while (u.Next(&uf, &uw)) {
                if (uf == 1) lo = u.Varint();
                else if (uf == 2) hi = u.Varint();
                else u.Skip(uw);
              }
              const size_t at = oc->values.size();
              oc->values.resize(at + 16);
              std::memcpy(oc->values.data() + at, &lo, 8);
              std::memcpy(oc->values.data() + at + 8, &hi, 8);
              ++rows;
            } else if (type == F) {
              auto put = [&](uint64_t bits) {
                const size_t at = oc->values.size();
                oc->values.resize(at + 8);
                std::memcpy(oc->values.data() + at, &bits, 8);
                ++rows;
              };
              if (dw == 2) {
                planpb::Reader pk = d.Sub();
                while (!pk.done()) put(pk.Fixed64());
              } else {
                put(d.Fixed64());
              }
            } else {  // BOOLEAN / INT64 / TIME64NS: varints, packed or not
              std::vector<uint64_t> vs;
              d.RepeatedVarint(dw, &vs);
              for (uint64_t v : vs) {
                if (type == B) {
                  oc->values.push_back(v ? 1 : 0);
                } else {
                  const size_t at = oc->values.size();
                  oc->values.resize(at + 8);
                  std::memcpy(oc->values.data() + at, &v, 8);
                }
                ++rows;
              }
            }
          }
        }
        if (type == 0) return Err(PXG_INTERNAL, "Received unknown column data type in ProtoDataType");
        HostColumn hc;
        hc.type = type;
        hc.length = rows;
        oc->values.resize(oc->values.size() + 16);  // keeps every pointer valid for empty columns
        oc->data.resize(oc->data.size() + 16);
        hc.values = oc->values.data();
        hc.offsets = oc->offsets.data();
        hc.data = oc->data.data();
        hc.owner = oc;
        rb->cols.push_back(hc);
      } else if (f == 2 && w == 0) {
        num_rows = static_cast<int64_t>(r.Varint());
      } else if (f == 3 && w == 0) {
        rb->eow = r.Varint() != 0;
      } else if (f == 4 && w == 0) {
        rb->eos = r.Varint() != 0;
      } else {
        r.Skip(w);
      }
    }
    rb->num_rows = num_rows;
    for (auto& c : rb->cols)  // RowBatch::AddColumn (row_batch.cc:39-52)
      if (c.length != num_rows) return Err(PXG_INVALID_ARGUMENT, "column of %lld rows in a RowBatch of %lld", (long long)c.length, (long long)num_rows);
  } catch (const planpb::WireError& e) {
    return Err(PXG_INVALID_ARGUMENT, "RowBatchData: %s", e.what());
  }
  return Status::OK();
}

// Row sizes for the GRPC sink's batch split (GetRowSizes / SplitBatchSizes,
// grpc_sink_node.cc:216-273): BOOLEAN 1 B, UINT128 16 B, other fixed types 8 B, strings their
// length; batches above (1 MiB - 16 KiB) * 0.9 are cut (grpc_sink_node.h:43-50).
static std::vector<int64_t> SplitBatchSizes(const RowBatch& rb) {
  const float limit = static_cast<float>(static_cast<size_t>(1024 * 1024 - 16 * 1024)) * 0.9f;
  const int64_t desired = static_cast<int64_t>(limit);
  int64_t fixed = 0;
  bool has_str = false;
  std::vector<int64_t> str(static_cast<size_t>(rb.num_rows), 0);
  for (auto& c : rb.cols) {
    if (c.type == S) {
      has_str = true;
      for (int64_t r = 0; r < rb.num_rows; ++r) str[r] += c.offsets[r + 1] - c.offsets[r];
    } else {
      fixed += c.type == B ? 1 : c.type == U ? 16 : 8;
    }
  }
  int64_t total = fixed * rb.num_rows;
  for (int64_t v : str) total += v;
  std::vector<int64_t> out;
  if (rb.num_rows == 0 || !(static_cast<float>(total) > limit)) {
    out.push_back(rb.num_rows);
    return out;
  }
  if (has_str) {
    int64_t bytes = 0, rows = 0;
    for (int64_t r = 0; r < rb.num_rows; ++r) {
      const int64_t rowb = str[r] + fixed;
      if (rows > 0 && bytes + rowb > desired) {
        out.push_back(rows);
        bytes = rows = 0;
      }
      bytes += rowb;
      ++rows;
    }
    out.push_back(rows);
  } else {
    int64_t per = fixed ? desired / fixed : rb.num_rows;
    if (per == 0) per = 1;
    const int64_t nb = rb.num_rows / per;
    out.insert(out.end(), static_cast<size_t>(nb), per);
    if (rb.num_rows - nb * per > 0) out.push_back(rb.num_rows - nb * per);
  }
  return out;
}

class Registry {
 public:
  Registry() {
    auto reg = [&](const char* n, std::vector<int32_t> a, int32_t res, std::vector<int> ops, int l = 0, int r = 0) {
      udfs_[{n, a}] = UdfDef{res, l, r, ops};
    };
    // arithmetic (math_ops.h:33-150, math_ops.cc:57-105)
    reg("add", {I, I}, I, {PXG_OP_ADD_I}); reg("add", {F, F}, F, {PXG_OP_ADD_F});
    reg("add", {F, I}, F, {PXG_OP_ADD_F}, 0, PXG_OP_I2F); reg("add", {I, F}, F, {PXG_OP_ADD_F}, PXG_OP_I2F);
    reg("add", {T, I}, T, {PXG_OP_ADD_I}); reg("add", {I, T}, T, {PXG_OP_ADD_I});
    reg("subtract", {I, I}, I, {PXG_OP_SUB_I}); reg("subtract", {F, F}, F, {PXG_OP_SUB_F});
    reg("subtract", {F, I}, F, {PXG_OP_SUB_F}, 0, PXG_OP_I2F); reg("subtract", {I, F}, F, {PXG_OP_SUB_F}, PXG_OP_I2F);
    reg("subtract", {T, I}, T, {PXG_OP_SUB_I}); reg("subtract", {T, T}, I, {PXG_OP_SUB_I}); reg("subtract", {I, T}, I, {PXG_OP_SUB_I});
    for (auto ab : std::vector<std::pair<int32_t, int32_t>>{{I, I}, {F, I}, {I, F}, {F, F}})  // DivideUDF: double(a)/double(b)
      reg("divide", {ab.first, ab.second}, F, {PXG_OP_DIV_F}, ab.first == I ? PXG_OP_I2F : 0, ab.second == I ? PXG_OP_I2F : 0);
    reg("multiply", {I, I}, I, {PXG_OP_MUL_I}); reg("multiply", {F, F}, F, {PXG_OP_MUL_F});
    reg("multiply", {F, I}, F, {PXG_OP_MUL_F}, 0, PXG_OP_I2F); reg("multiply", {I, F}, F, {PXG_OP_MUL_F}, PXG_OP_I2F);
    for (auto ab : std::vector<std::pair<int32_t, int32_t>>{{T, I}, {T, T}, {I, T}, {I, I}}) reg("modulo", {ab.first, ab.second}, I, {PXG_OP_MOD_I});
    // logical (math_ops.h:265-315)
    reg("logicalOr", {I, I}, B, {PXG_OP_OR}); reg("logicalOr", {B, B}, B, {PXG_OP_OR});
    reg("logicalAnd", {I, I}, B, {PXG_OP_AND}); reg("logicalAnd", {B, B}, B, {PXG_OP_AND});
    reg("logicalNot", {I}, B, {PXG_OP_NOT}); reg("logicalNot", {B}, B, {PXG_OP_NOT});
    reg("negate", {I}, I, {PXG_OP_NEG_I}); reg("negate", {F}, F, {PXG_OP_NEG_F}); reg("invert", {I}, I, {PXG_OP_INV_I});
    // equality (math_ops.cc:145-175); FLOAT64 == FLOAT64 is ApproxEqualUDF
    for (int32_t t : {I, T, B}) { reg("equal", {t, t}, B, {PXG_OP_EQ_I}); reg("notEqual", {t, t}, B, {PXG_OP_NE_I}); }
    reg("equal", {S, S}, B, {PXG_OP_EQ_S}); reg("notEqual", {S, S}, B, {PXG_OP_NE_S});
    reg("equal", {U, U}, B, {PXG_OP_EQ_U}); reg("notEqual", {U, U}, B, {PXG_OP_NE_U});
    reg("equal", {B, I}, B, {PXG_OP_EQ_I}); reg("equal", {I, B}, B, {PXG_OP_EQ_I});
    reg("notEqual", {B, I}, B, {PXG_OP_NE_I}); reg("notEqual", {I, B}, B, {PXG_OP_NE_I});
    reg("equal", {I, F}, B, {PXG_OP_EQ_F}, PXG_OP_I2F); reg("equal", {F, I}, B, {PXG_OP_EQ_F}, 0, PXG_OP_I2F);
    reg("notEqual", {I, F}, B, {PXG_OP_NE_F}, PXG_OP_I2F); reg("notEqual", {F, I}, B, {PXG_OP_NE_F}, 0, PXG_OP_I2F);
    reg("equal", {F, F}, B, {PXG_OP_APPROX_EQ_F}); reg("notEqual", {F, F}, B, {PXG_OP_APPROX_NE_F});
    reg("approxEqual", {F, F}, B, {PXG_OP_APPROX_EQ_F});
    // ordering (math_ops.h:412-510)
    const std::vector<std::tuple<const char*, int, int, int>> ord = {
        {"greaterThan", PXG_OP_GT_I, PXG_OP_GT_F, PXG_OP_GT_S}, {"greaterThanEqual", PXG_OP_GE_I, PXG_OP_GE_F, PXG_OP_GE_S},
        {"lessThan", PXG_OP_LT_I, PXG_OP_LT_F, PXG_OP_LT_S}, {"lessThanEqual", PXG_OP_LE_I, PXG_OP_LE_F, PXG_OP_LE_S}};
    for (auto& o : ord) {
      reg(std::get<0>(o), {I, I}, B, {std::get<1>(o)}); reg(std::get<0>(o), {T, T}, B, {std::get<1>(o)});
      reg(std::get<0>(o), {F, F}, B, {std::get<2>(o)}); reg(std::get<0>(o), {S, S}, B, {std::get<3>(o)});
    }
    // bin (math_ops.h:512-527)
    reg("bin", {I, I}, I, {PXG_OP_BIN_I}); reg("bin", {T, T}, T, {PXG_OP_BIN_I}); reg("bin", {I, T}, I, {PXG_OP_BIN_I});
    reg("bin", {T, I}, T, {PXG_OP_BIN_I}); reg("bin", {F, I}, I, {PXG_OP_BIN_I}, PXG_OP_F2I);
    reg("time_to_int64", {T}, I, {}); reg("int64_to_time", {I}, T, {});
    // FilterNodeTest's registry-local UDF (filter_node_test.cc:41-53).
    reg("eq", {I, I}, B, {PXG_OP_EQ_I}); reg("eq", {S, S}, B, {PXG_OP_EQ_S});

    // UDAs: (name, registry types) -> (kind, arg type, output type)
    auto uda = [&](const char* n, std::vector<int32_t> a, int32_t kind, int32_t at, int32_t out) {
      udas_[{n, a}] = std::make_tuple(kind, at, out);
    };
    for (int32_t t : {F, I, B}) uda("mean", {t}, PXG_UDA_MEAN, t, F);
    uda("sum", {F}, PXG_UDA_SUM, F, F); uda("sum", {I}, PXG_UDA_SUM, I, I); uda("sum", {B}, PXG_UDA_SUM, B, I);
    for (int32_t t : {F, I, T}) { uda("max", {t}, PXG_UDA_MAX, t, t); uda("min", {t}, PXG_UDA_MIN, t, t); }
    for (int32_t t : {F, I, T, B, S, U}) uda("count", {t}, PXG_UDA_COUNT, t, I);
    uda("quantiles", {I}, PXG_UDA_QUANTILES, I, S); uda("quantiles", {F}, PXG_UDA_QUANTILES, F, S);
    // AggNodeTest's registry-local test UDAs (agg_node_test.cc:44-72, 282-289).
    uda("minsum", {I, I}, PXG_UDA_MINSUM, I, I); uda("minsum_w_init", {I, I, I}, PXG_UDA_MINSUM, I, I);
  }
  const UdfDef* GetScalarUDF(const std::string& n, const std::vector<int32_t>& t) const {
    auto it = udfs_.find({n, t});
    return it == udfs_.end() ? nullptr : &it->second;
  }
  const std::tuple<int32_t, int32_t, int32_t>* GetUDA(const std::string& n, const std::vector<int32_t>& t) const {
    auto it = udas_.find({n, t});
    return it == udas_.end() ? nullptr : &it->second;
  }

 private:
  std::map<std::pair<std::string, std::vector<int32_t>>, UdfDef> udfs_;
  std::map<std::pair<std::string, std::vector<int32_t>>, std::tuple<int32_t, int32_t, int32_t>> udas_;
};

static const Registry& GetRegistry() {
  static const Registry r;
  return r;
}

static std::string TypeName(int32_t t) {
  switch (t) {
    case B: return "BOOLEAN";
    case I: return "INT64";
    case U: return "UINT128";
    case F: return "FLOAT64";
    case S: return "STRING";
    case T: return "TIME64NS";
    default: return "UNKNOWN";
  }
}

static std::string Signature(const std::string& name, const std::vector<int32_t>& types) {
  std::string s = name + "(";
  for (size_t i = 0; i < types.size(); ++i) s += (i ? "," : "") + TypeName(types[i]);
  return s + ")";
}

// Lowers planpb.ScalarExpression trees (ScalarExpression walker, scalar_expression.h:243-346).
// env[i] is the program that computes input column i (a bare column reference, or a Map
// expression substituted into downstream operators when a chain is fused).
class ExprCompiler {
 public:
  explicit ExprCompiler(std::vector<Program> env) : env_(std::move(env)) {}
  Status Compile(const planpb::ScalarExpression& e, Program* out) const {
    Program p;
    PXC_RETURN_IF_ERROR(Emit(e, &p));
    *out = std::move(p);
    return Status::OK();
  }
  Status Const(const planpb::ScalarValue& v, Program* p) const {
    const int32_t dt = v.data_type;
    switch (dt) {
      case B: p->insns.push_back(Insn(PXG_OP_CONST, dt, 0, v.bool_value ? 1 : 0)); break;
      case I: p->insns.push_back(Insn(PXG_OP_CONST, dt, 0, v.int64_value)); break;
      case T: p->insns.push_back(Insn(PXG_OP_CONST, dt, 0, v.time64_ns_value)); break;
      case F: {
        int64_t bits;
        std::memcpy(&bits, &v.float64_value, 8);
        p->insns.push_back(Insn(PXG_OP_CONST, dt, 0, bits));
        break;
      }
      case S: {
        const int32_t off = static_cast<int32_t>(p->pool.size());
        p->pool.insert(p->pool.end(), v.string_value.begin(), v.string_value.end());
        while (p->pool.size() % 8) p->pool.push_back(0);
        p->insns.push_back(Insn(PXG_OP_CONST, dt, off, static_cast<int64_t>(v.string_value.size())));
        break;
      }
      case U: {
        const int32_t off = static_cast<int32_t>(p->pool.size());
        const uint8_t* lo = reinterpret_cast<const uint8_t*>(&v.u128_low);
        const uint8_t* hi = reinterpret_cast<const uint8_t*>(&v.u128_high);
        p->pool.insert(p->pool.end(), lo, lo + 8);
        p->pool.insert(p->pool.end(), hi, hi + 8);
        p->insns.push_back(Insn(PXG_OP_CONST, dt, off, 16));
        break;
      }
      default: return Err(PXG_UNIMPLEMENTED, "constant of type %d", dt);
    }
    p->result_type = dt;
    return Status::OK();
  }

 private:
  Status Emit(const planpb::ScalarExpression& e, Program* p) const {
    switch (e.kind) {
      case planpb::ScalarExpression::kColumn: {
        const uint64_t idx = e.column.index;
        if (idx >= env_.size()) return Err(PXG_INVALID_ARGUMENT, "column %llu out of range", (unsigned long long)idx);
        AppendProgram(env_[idx], p);
        p->result_type = env_[idx].result_type;
        return Status::OK();
      }
      case planpb::ScalarExpression::kConstant: return Const(e.constant, p);
      case planpb::ScalarExpression::kFunc: {
        const planpb::ScalarFunc& f = *e.func;
        if (!f.init_args.empty()) return Err(PXG_UNIMPLEMENTED, "scalar UDF %s with init args", f.name.c_str());
        std::vector<Program> parts(f.args.size());
        std::vector<int32_t> types;
        for (size_t i = 0; i < f.args.size(); ++i) {
          PXC_RETURN_IF_ERROR(Emit(f.args[i], &parts[i]));
          types.push_back(parts[i].result_type);
        }
        const UdfDef* d = GetRegistry().GetScalarUDF(f.name, types);
        if (!d) return Err(PXG_NOT_FOUND, "no device UDF %s", Signature(f.name, types).c_str());
        for (size_t i = 0; i < parts.size(); ++i) {
          AppendProgram(parts[i], p);
          const int conv = i == 0 ? d->lconv : d->rconv;
          if (conv) p->insns.push_back(Insn(conv, conv == PXG_OP_I2F ? F : I));
        }
        for (int op : d->ops) p->insns.push_back(Insn(op, d->result));
        if (d->ops.empty()) {  // time_to_int64 / int64_to_time: same bits, relabelled (x + 0)
          p->insns.push_back(Insn(PXG_OP_CONST, I, 0, 0));
          p->insns.push_back(Insn(PXG_OP_ADD_I, d->result));
        }
        p->result_type = d->result;
        return Status::OK();
      }
      default: return Err(PXG_INVALID_ARGUMENT, "empty scalar expression");
    }
  }
  std::vector<Program> env_;
};

static std::vector<Program> ColumnEnv(const RowDescriptor& types) {
  std::vector<Program> env(types.size());
  for (size_t i = 0; i < types.size(); ++i) {
    env[i].insns.push_back(Insn(PXG_OP_COL, types[i], static_cast<int32_t>(i)));
    env[i].result_type = types[i];
  }
  return env;
}

// ---------------------------------------------------------------------------------------
// ExecState: the device context + registry shared by one query's nodes (exec_state.h:52-180).
// ---------------------------------------------------------------------------------------
struct ExecState {
  pxg_ctx* ctx = nullptr;  // null when only lowering (pxc_explain_plan)
  // Group counts of earlier runs of the same aggregation (engine-lifetime statistics), used
  // to size the next run's hash table instead of growing it mid-consume.
  std::map<std::string, int64_t>* group_hints = nullptr;
  // Aggregation objects of earlier queries, keyed by their full spec: a query takes one,
  // resets it and gives it back at Close, so the hash table and finalize workspaces keep their
  // grown device buffers instead of being freed and reallocated per query.
  std::multimap<std::string, pxg_agg*>* agg_cache = nullptr;
  // ExecState::StopSource (exec_state.h:171-178): sources a Limit has finished with.
  std::set<uint64_t> stopped_sources;
  // Collect per-node timers and extra metrics (Carnot's `analyze`, carnot.cc:379-420).
  bool collect_exec_stats = false;
};

// ExecNodeStats (src/carnot/exec/exec_node.h:41-125): rows / bytes / batches in and out, the
// node's total time and the time spent in its children (self = total - children), extra
// metrics and info.  Row and byte counts are always kept (the sources' counts are the query's
// bytes_processed / rows_processed, exec_graph.cc:333-347); timers and extras only when the
// query collects stats.  Bytes follow RowBatch::NumBytes (row_batch.cc:67-79): fixed-width
// values by type width, STRING by the string lengths.
static int64_t RowBatchNumBytes(const RowBatch& rb);
struct ExecNodeStats {
  bool collect = false;
  int64_t bytes_input = 0, rows_input = 0, batches_input = 0;
  int64_t bytes_output = 0, rows_output = 0, batches_output = 0;
  int64_t total_ns = 0, children_ns = 0;
  std::map<std::string, double> extra_metrics;
  std::map<std::string, std::string> extra_info;
  std::chrono::steady_clock::time_point total_t0, child_t0;
  void AddInputStats(const RowBatch& rb) {
    ++batches_input;
    rows_input += rb.num_rows;
    bytes_input += RowBatchNumBytes(rb);
  }
  void AddOutputStats(const RowBatch& rb) {
    ++batches_output;
    rows_output += rb.num_rows;
    bytes_output += RowBatchNumBytes(rb);
  }
  void ResumeTotalTimer() {
    if (collect) total_t0 = std::chrono::steady_clock::now();
  }
  void StopTotalTimer() {
    if (collect) total_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - total_t0).count();
  }
  void ResumeChildTimer() {
    if (collect) child_t0 = std::chrono::steady_clock::now();
  }
  void StopChildTimer() {
    if (collect) children_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - child_t0).count();
  }
  void AddExtraMetric(const std::string& k, double v) {
    if (collect) extra_metrics[k] = v;
  }
  void AddExtraInfo(const std::string& k, const std::string& v) {
    if (collect) extra_info[k] = v;
  }
};

static int64_t RowBatchNumBytes(const RowBatch& rb) {
  if (rb.num_rows == 0) return 0;
  if (rb.dev) return rb.dev_bytes;
  int64_t b = 0;
  for (const HostColumn& c : rb.cols) {
    switch (c.type) {
      case PXG_STRING: b += c.offsets ? static_cast<int64_t>(c.offsets[c.length]) - c.offsets[0] : 0; break;
      case PXG_BOOLEAN: b += c.length; break;
      case PXG_UINT128: b += 16 * c.length; break;
      default: b += 8 * c.length; break;
    }
  }
  return b;
}

// ---------------------------------------------------------------------------------------
// ExecNode NVI (src/carnot/exec/exec_node.h:145-315).
// ---------------------------------------------------------------------------------------
class ExecNode {
 public:
  virtual ~ExecNode() = default;
  Status Init(const planpb::Operator& op, const RowDescriptor& output, const std::vector<RowDescriptor>& inputs) {
    output_ = output;
    inputs_ = inputs;
    return InitImpl(op);
  }
  Status Prepare(ExecState* s) { return PrepareImpl(s); }
  Status Open(ExecState* s) { return OpenImpl(s); }
  Status Close(ExecState* s) { return CloseImpl(s); }
  // exec_node.h:213-226: eos implies eow.
  Status ConsumeNext(ExecState* s, const RowBatch& rb, size_t parent_index) {
    if (rb.eos && !rb.eow) return Err(PXG_INTERNAL, "RowBatch has eos set without eow");
    stats_.AddInputStats(rb);
    stats_.ResumeTotalTimer();
    Status st = ConsumeNextImpl(s, rb, parent_index);
    stats_.StopTotalTimer();
    return st;
  }
  ExecNodeStats* stats() { return &stats_; }
  uint64_t plan_id = 0;  // the plan node this ExecNode runs
  void AddChild(ExecNode* child, size_t parent_index) { children_.push_back({child, parent_index}); }
  // Whether this node can observe the value of input column `col` (conservative default).
  // Lets a producer skip rendering a column no consumer reads.
  virtual bool ReadsColumnValue(size_t /*col*/) const { return true; }
  // Quantile lanes (bit k = kQuantileKeys[k]) this node plucks from input column col.
  virtual uint32_t PluckedLanes(size_t /*col*/) const { return 0x7Fu; }
  // Whether this node takes device-resident batches (RowBatch::dev) from its parents.
  virtual bool AcceptsDeviceBatch() const { return false; }
  // Whether this node takes device result images (RowBatch::image) from its parents.
  virtual bool AcceptsResultImage() const { return false; }
  const RowDescriptor& output_descriptor() const { return output_; }
  const std::vector<std::pair<ExecNode*, size_t>>& children() const { return children_; }
  virtual std::string DebugString() const = 0;

 protected:
  virtual Status InitImpl(const planpb::Operator& op) = 0;
  virtual Status PrepareImpl(ExecState*) { return Status::OK(); }
  virtual Status OpenImpl(ExecState*) { return Status::OK(); }
  virtual Status CloseImpl(ExecState*) { return Status::OK(); }
  virtual Status ConsumeNextImpl(ExecState*, const RowBatch&, size_t) { return Err(PXG_INTERNAL, "not a consumer"); }
  // exec_node.h:285-297: depth-first push to every child.
  Status SendRowBatchToChildren(ExecState* s, const RowBatch& rb) {
    stats_.ResumeChildTimer();
    for (auto& c : children_) PXC_RETURN_IF_ERROR(c.first->ConsumeNext(s, rb, c.second));
    stats_.StopChildTimer();
    stats_.AddOutputStats(rb);
    return Status::OK();
  }
  ExecNodeStats stats_;
  RowDescriptor output_;
  std::vector<RowDescriptor> inputs_;
  std::vector<std::pair<ExecNode*, size_t>> children_;
};

// Source nodes (exec_node.h:300-315): the graph pulls them until they have nothing left.
class SourceNode : public ExecNode {
 public:
  uint64_t node_id = 0;  // plan node id (LimitOperator.abortable_srcs names sources by it)
  virtual bool HasBatchesRemaining() const = 0;
  // An infinite stream (MemorySourceOperator.streaming) that sends no eow / eos per batch.
  virtual bool IsStreaming() const { return false; }
  Status GenerateNext(ExecState* s) {
    stats_.ResumeTotalTimer();
    Status st = GenerateNextImpl(s);
    stats_.StopTotalTimer();
    return st;
  }

 protected:
  virtual Status GenerateNextImpl(ExecState* s) = 0;
};

// MemorySourceNode (memory_source_node.cc:54-124) over a host table's RowBatches.
class MemorySourceNode : public SourceNode {
 public:
  MemorySourceNode(const pxc_table* t) : table_(t) {}
  std::string DebugString() const override { return "MemorySourceNode(" + std::string(table_->name) + ")"; }
  // With explicit batch flags every given batch is fed, as the reference's ExecNodeTester does
  // (src/carnot/exec/test_utils.h:319-480); otherwise the source stops at eos.
  bool HasBatchesRemaining() const override {
    if (table_->batch_flags && table_->nbatches > 0) return next_ < table_->nbatches;
    return next_ < std::max<int32_t>(table_->nbatches, 1) && !done_;
  }
  // GenerateNext: one RowBatch (column-projected) to the children.
  Status GenerateNextImpl(ExecState* s) override {
    RowBatch rb;
    const int32_t nb = table_->nbatches;
    if (nb == 0 && streaming_) {  // an infinite stream over an empty table has nothing ready
      done_ = true;
      return Status::OK();
    }
    if (nb == 0) {  // empty table: one zero-row batch with eow/eos (memory_source_node.cc:107-118)
      for (size_t c = 0; c < idxs_.size(); ++c) {
        HostColumn hc;
        hc.type = output_[c];
        static const int32_t zero_off[2] = {0, 0};
        static const uint8_t pad[16] = {0};
        hc.offsets = zero_off;
        hc.data = pad;
        hc.values = pad;
        rb.cols.push_back(hc);
      }
      rb.eow = rb.eos = true;
      done_ = true;
      return SendRowBatchToChildren(s, rb);
    }
    const int32_t b = next_++;
    for (int64_t c : idxs_) {
      const pxg_column_view& v = table_->cols[static_cast<int64_t>(b) * table_->ncols + c];
      HostColumn hc;
      hc.type = v.type;
      hc.length = v.length;
      hc.values = v.values;
      hc.offsets = v.offsets;
      hc.data = v.data;
      rb.cols.push_back(hc);
      rb.num_rows = v.length;
    }
    if (table_->batch_flags) {
      rb.eow = (table_->batch_flags[b] & 1) != 0;
      rb.eos = (table_->batch_flags[b] & 2) != 0;
    } else {
      rb.eow = rb.eos = (b == nb - 1);
    }
    if (streaming_) {  // an infinite stream sends no eow / eos; it has sent all there is
      rb.eow = rb.eos = false;
      if (next_ >= nb) done_ = true;
    }
    if (rb.eos) done_ = true;
    return SendRowBatchToChildren(s, rb);
  }

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    if (op.mem_source.has_start_time || op.mem_source.has_stop_time)
      return Err(PXG_UNIMPLEMENTED, "a time-bounded MemorySource needs a stored table (pxc_store_*)");
    streaming_ = op.mem_source.streaming;
    idxs_ = op.mem_source.column_idxs;
    if (idxs_.empty())
      for (int32_t c = 0; c < table_->ncols; ++c) idxs_.push_back(c);
    for (int64_t c : idxs_)
      if (c < 0 || c >= table_->ncols) return Err(PXG_INVALID_ARGUMENT, "source column %lld out of range", (long long)c);
    return Status::OK();
  }

 private:
  const pxc_table* table_;
  std::vector<int64_t> idxs_;
  int32_t next_ = 0;
  bool done_ = false;
  bool streaming_ = false;

 public:
  bool IsStreaming() const override { return streaming_; }
};

// Uploads a RowBatch into a fresh device table.
static Status UploadBatch(pxg_ctx* ctx, const RowBatch& rb, const RowDescriptor& types, pxg_table** out) {
  PXG_CALL(pxg_table_create(ctx, static_cast<int32_t>(types.size()), types.data(), out));
  if (rb.num_rows > 0) {
    std::vector<pxg_column_view> v;
    for (auto& c : rb.cols) v.push_back(c.View());
    PXG_CALL(pxg_table_append(*out, v.data(), rb.num_rows));
  }
  PXG_CALL(pxg_table_flush(*out));
  return Status::OK();
}

static Status FetchAll(pxg_table* t, int32_t ncols, RowBatch* rb) {
  const int64_t n = pxg_table_num_rows(t);
  rb->num_rows = n;
  for (int32_t c = 0; c < ncols; ++c) {
    pxg_column_out o{};
    PXG_CALL(pxg_table_fetch(t, c, 0, n, &o));
    rb->cols.push_back(FromOut(o));
  }
  return Status::OK();
}

// Rows [r0, r0 + n) of a host column, sharing its buffers (Arrow Slice).
static HostColumn SliceColumn(const HostColumn& c, int64_t r0, int64_t n) {
  HostColumn h = c;
  h.length = n;
  if (c.type == PXG_STRING) {
    h.offsets = c.offsets + r0;  // absolute offsets into the same payload
  } else {
    const int w = c.type == B ? 1 : c.type == U ? 16 : 8;
    h.values = static_cast<const uint8_t*>(c.values) + r0 * w;
  }
  return h;
}

// Coalescing of the small RowBatches PEM sources produce (pem_manager.cc:85-99) in front of the
// standalone device operators: batches are staged into one device table (pinned staging) and
// run together at kCoalesceRows staged rows or at eow / eos; the output is cut back into one
// batch per input batch with the input batch's eow / eos, exactly what the per-batch reference
// nodes emit (filter_node.cc:167-168, map_node.cc:67-68).
//
// Coalescing changes when a batch leaves the node, not what it holds.  Two plan shapes would see
// the difference, so there the node runs every batch as it arrives (eager): below an infinite
// stream (no eow / eos per batch, so staged rows would wait for Close), and above a Limit
// (which stops its abortable sources as soon as it has its rows, limit_node.cc:55).
class CoalescingDeviceNode : public ExecNode {
 public:
  void set_eager() { eager_ = true; }

 protected:
  static constexpr int64_t kCoalesceRows = 1 << 16;
  struct Pending {
    int64_t rows;
    bool eow, eos;
  };
  // Runs the device operator over the staged rows; fills `out` and the rows of each input batch.
  virtual Status RunStaged(ExecState* s, pxg_table* staged, int64_t n, const std::vector<int64_t>& in_rows, RowBatch* out,
                           std::vector<int64_t>* out_rows) = 0;
  Status OpenImpl(ExecState* s) override {
    if (!s->ctx) return Status::OK();
    PXG_CALL(pxg_table_create(s->ctx, static_cast<int32_t>(inputs_[0].size()), inputs_[0].data(), &staged_));
    return Status::OK();
  }
  Status CloseImpl(ExecState* s) override {
    // Batches a source sent after its eos (ExecNodeTester does) or before a stop are still
    // owed their output batches; children close after this node (topological order).
    Status st;
    if (staged_ && !pending_.empty()) st = Flush(s);
    if (staged_) pxg_table_destroy(staged_);
    staged_ = nullptr;
    return st;
  }
  Status ConsumeNextImpl(ExecState* s, const RowBatch& rb, size_t) override {
    if (rb.num_rows > 0) {
      std::vector<pxg_column_view> v;
      for (auto& c : rb.cols) v.push_back(c.View());
      PXG_CALL(pxg_table_append(staged_, v.data(), rb.num_rows));
    }
    pending_.push_back({rb.num_rows, rb.eow, rb.eos});
    staged_rows_ += rb.num_rows;
    if (!eager_ && staged_rows_ < kCoalesceRows && !rb.eow && !rb.eos) return Status::OK();
    return Flush(s);
  }

 private:
  Status Flush(ExecState* s) {
    PXG_CALL(pxg_table_flush(staged_));
    std::vector<int64_t> in_rows, out_rows;
    for (auto& p : pending_) in_rows.push_back(p.rows);
    RowBatch all;
    PXC_RETURN_IF_ERROR(RunStaged(s, staged_, staged_rows_, in_rows, &all, &out_rows));
    std::vector<Pending> pend;
    pend.swap(pending_);
    staged_rows_ = 0;
    pxg_table_destroy(staged_);
    staged_ = nullptr;
    PXG_CALL(pxg_table_create(s->ctx, static_cast<int32_t>(inputs_[0].size()), inputs_[0].data(), &staged_));
    int64_t r0 = 0;
    for (size_t i = 0; i < pend.size(); ++i) {
      RowBatch ob;
      ob.num_rows = out_rows[i];
      for (auto& c : all.cols) ob.cols.push_back(SliceColumn(c, r0, out_rows[i]));
      ob.eow = pend[i].eow;
      ob.eos = pend[i].eos;
      r0 += out_rows[i];
      PXC_RETURN_IF_ERROR(SendRowBatchToChildren(s, ob));
    }
    return Status::OK();
  }
  pxg_table* staged_ = nullptr;
  std::vector<Pending> pending_;
  int64_t staged_rows_ = 0;
  bool eager_ = false;
};

// GpuFilterNode (FilterNode, filter_node.cc:78-171): one output batch per input batch.
class GpuFilterNode : public CoalescingDeviceNode {
 public:
  std::string DebugString() const override { return "GpuFilterNode"; }
  Program pred;
  std::vector<int32_t> select;

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    ExprCompiler comp(ColumnEnv(inputs_[0]));
    PXC_RETURN_IF_ERROR(comp.Compile(op.filter.expression, &pred));
    if (pred.result_type != B) return Err(PXG_INVALID_ARGUMENT, "Predicate expression must be a boolean");
    for (auto& c : op.filter.columns) select.push_back(static_cast<int32_t>(c.index));
    if (select.empty())
      for (size_t c = 0; c < inputs_[0].size(); ++c) select.push_back(static_cast<int32_t>(c));
    return Status::OK();
  }
  Status RunStaged(ExecState*, pxg_table* staged, int64_t n, const std::vector<int64_t>& in_rows, RowBatch* out,
                   std::vector<int64_t>* out_rows) override {
    pxg_table* res = nullptr;
    const pxg_program p = pred.View();
    out_rows->assign(in_rows.size(), 0);
    int32_t code = pxg_filter_split(staged, &p, static_cast<int32_t>(select.size()), select.data(), 0, n,
                                    static_cast<int32_t>(in_rows.size()), in_rows.data(), out_rows->data(), &res);
    Status st = FromPxg(code);
    if (st.ok()) st = FetchAll(res, static_cast<int32_t>(select.size()), out);
    if (res) pxg_table_destroy(res);
    return st;
  }
};

// GpuMapNode (MapNode, map_node.cc:47-71): one output column per expression.
class GpuMapNode : public CoalescingDeviceNode {
 public:
  std::string DebugString() const override { return "GpuMapNode"; }
  std::vector<Program> exprs;

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    ExprCompiler comp(ColumnEnv(inputs_[0]));
    for (auto& e : op.map.expressions) {
      exprs.emplace_back();
      PXC_RETURN_IF_ERROR(comp.Compile(e, &exprs.back()));
    }
    return Status::OK();
  }
  Status RunStaged(ExecState*, pxg_table* staged, int64_t n, const std::vector<int64_t>& in_rows, RowBatch* out,
                   std::vector<int64_t>* out_rows) override {
    std::vector<pxg_program> pv;
    for (auto& e : exprs) pv.push_back(e.View());
    pxg_table* res = nullptr;
    int32_t code = pxg_map(staged, static_cast<int32_t>(pv.size()), pv.data(), 0, n, &res);
    Status st = FromPxg(code);
    if (st.ok()) st = FetchAll(res, static_cast<int32_t>(pv.size()), out);
    if (res) pxg_table_destroy(res);
    *out_rows = in_rows;
    return st;
  }
};

static const char* const kQuantileKeys[7] = {"p01", "p10", "p25", "p50", "p75", "p90", "p99"};

// The QuantilesUDA::Finalize JSON strings (math_sketches.h:40-54) of G groups from their 7
// doubles each, written straight into one STRING column.  Groups are split over host threads;
// every thread renders into its own buffer, then the buffers are concatenated.  Numbers are
// rendered byte-for-byte as rapidjson's Writer does (json_double.h: Grisu2 + Prettify; a NaN /
// inf value ends the object after its key, as Document::Accept stops there).
static HostColumn RenderQuantilesJson(const double* d, int64_t G) {
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({16, static_cast<int64_t>(std::thread::hardware_concurrency()), G / 2048 + 1}));
  std::vector<std::string> bufs(static_cast<size_t>(nt));
  std::vector<std::vector<int32_t>> lens(static_cast<size_t>(nt));
  auto work = [&](int64_t t) {
    const int64_t g0 = G * t / nt, g1 = G * (t + 1) / nt;
    std::string& b = bufs[static_cast<size_t>(t)];
    std::vector<int32_t>& l = lens[static_cast<size_t>(t)];
    b.reserve(static_cast<size_t>(g1 - g0) * 160);
    l.reserve(static_cast<size_t>(g1 - g0));
    for (int64_t g = g0; g < g1; ++g) {
      const size_t start = b.size();
      pxjson::AppendQuantilesJson(d + g * 7, &b);
      l.push_back(static_cast<int32_t>(b.size() - start));
    }
  };
  std::vector<std::thread> th;
  for (int64_t t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  auto o = std::make_shared<OwnedColumn>();
  o->offsets.reserve(static_cast<size_t>(G) + 1);
  o->offsets.push_back(0);
  size_t total = 0;
  for (auto& b : bufs) total += b.size();
  o->data.reserve(total + 16);
  for (int64_t t = 0; t < nt; ++t) {
    o->data.insert(o->data.end(), bufs[static_cast<size_t>(t)].begin(), bufs[static_cast<size_t>(t)].end());
    for (int32_t len : lens[static_cast<size_t>(t)]) o->offsets.push_back(o->offsets.back() + len);
  }
  o->data.resize(o->data.size() + 16, 0);
  HostColumn hc;
  hc.type = PXG_STRING;
  hc.length = G;
  hc.offsets = o->offsets.data();
  hc.data = o->data.data();
  hc.owner = o;
  return hc;
}

// GpuAggNode (AggNode, agg_node.cc:88-542).  When the graph builder fused a
// Filter / Map chain in front of it, `filter` and the substituted key / argument programs
// evaluate that chain inside the consume kernel.  Blocking: emits one batch at eos; windowed:
// one batch per eow, then ClearAggState (agg_node.cc:169-180).
// Pluck-only quantile columns fetched as their plucked lanes (pxg_agg_quantile_lanes);
// PXC_DEVICE_PLUCK=0 copies the 7 doubles per group and plucks on the host instead.
// A test switch read at each use (tests flip it between queries of one process).
static bool EnvOn(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] && e[0] != '0';
}

static bool DevicePluck() {
  static const bool on = [] {
    const char* e = std::getenv("PXC_DEVICE_PLUCK");
    return !(e && e[0] == '0');
  }();
  return on;
}

class GpuAggNode : public ExecNode {
 public:
  std::string DebugString() const override {
    return std::string(fused_ ? "GpuAggNode(fused filter/map chain)" : "GpuAggNode") + (device_input ? " <- HBM table" : "");
  }
  // Set by the graph builder for a fused chain: the agg's input columns as programs over the
  // source table, and the conjunction of the chain's predicates.
  std::vector<Program> env;
  bool has_filter = false;
  Program filter;
  bool fused_ = false;
  std::vector<uint64_t> fused_ids;  // plan ids of the Filter / Map operators fused into this node
  bool device_input = false;  // fed by a stored table through ConsumeTable
  RowDescriptor source_types;

  std::vector<Program> keys;
  struct Uda {
    int32_t kind, arg_type, out_type;
    Program arg, arg2;
    bool has_arg = false, has_arg2 = false, has_init = false;
    int64_t init = 0;
  };
  std::vector<Uda> udas;
  bool windowed = false;
  // Split aggregation (plan.proto:250-257).  emit_states (partial_agg && !finalize_results):
  // the output is the groups + serialized_expressions (operators.cc:251-257).  merge_states
  // (!partial_agg && finalize_results): the input's last column is serialized_expressions; the
  // device reads each UDA state word (PXG_OP_STATE_WORD) and merges: count/sum as SUM, min/max
  // as MIN/MAX, mean as MEAN_MERGE (UDA::Merge semantics, math_ops.h:583-772).
  bool emit_states = false, merge_states = false;
  int64_t state_col = -1;
  int64_t state_rec = 0;

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    const planpb::AggregateOperator& a = op.agg;
    if (env.empty()) env = ColumnEnv(inputs_[0]);
    if (source_types.empty()) source_types = inputs_[0];
    windowed = a.windowed;
    emit_states = a.partial_agg && !a.finalize_results;
    merge_states = !a.partial_agg && a.finalize_results;
    ExprCompiler comp(env);
    for (auto& g : a.groups) {
      if (g.index >= env.size()) return Err(PXG_INVALID_ARGUMENT, "group column %llu out of range", (unsigned long long)g.index);
      keys.push_back(env[g.index]);
    }
    if (merge_states) return InitMerge(a);
    for (auto& v : a.values) {  // AggregateExpression -> registry (registry_arg_types = init ++ args)
      std::vector<Program> args(v.args.size());
      std::vector<int32_t> types;
      for (auto& ia : v.init_args) types.push_back(ia.data_type);
      for (size_t i = 0; i < v.args.size(); ++i) {
        if (v.args[i].is_column) {
          planpb::ScalarExpression e;
          e.kind = planpb::ScalarExpression::kColumn;
          e.column = v.args[i].column;
          PXC_RETURN_IF_ERROR(comp.Compile(e, &args[i]));
        } else {
          PXC_RETURN_IF_ERROR(comp.Const(v.args[i].constant, &args[i]));
        }
        types.push_back(args[i].result_type);
      }
      auto* d = GetRegistry().GetUDA(v.name, types);
      if (!d) return Err(PXG_NOT_FOUND, "no device UDA %s", Signature(v.name, types).c_str());
      Uda u;
      u.kind = std::get<0>(*d);
      u.arg_type = std::get<1>(*d);
      u.out_type = std::get<2>(*d);
      if (!args.empty()) { u.arg = args[0]; u.has_arg = true; }
      if (args.size() > 1 && u.kind != PXG_UDA_COUNT) { u.arg2 = args[1]; u.has_arg2 = true; }
      if (!v.init_args.empty()) { u.has_init = true; u.init = v.init_args[0].int64_value; }
      if (emit_states && !(u.kind == PXG_UDA_COUNT || u.kind == PXG_UDA_SUM || u.kind == PXG_UDA_MEAN || u.kind == PXG_UDA_MIN || u.kind == PXG_UDA_MAX))
        return Err(PXG_UNIMPLEMENTED, "UDA %s has no Serialize: it does not support partial aggregation", v.name.c_str());
      udas.push_back(u);
    }
    const size_t nv = emit_states ? 1 : udas.size();
    if (output_.size() != keys.size() + nv)  // agg_node.cc:109-112, operators.cc:251-257
      return Err(PXG_INVALID_ARGUMENT, "output relation arity %zu != groups + values %zu", output_.size(), keys.size() + nv);
    return Status::OK();
  }
  // The finalize half of a split aggregate: UDAs resolved by (name, args_data_types); each
  // UDA's state is read from its offset in the serialized_expressions records.
  Status InitMerge(const planpb::AggregateOperator& a) {
    state_col = static_cast<int64_t>(env.size()) - 1;
    if (state_col < 0 || env[state_col].result_type != S || !env[state_col].IsColumn())
      return Err(PXG_INVALID_ARGUMENT, "finalize agg input must end in the serialized_expressions STRING column");
    for (auto& g : a.groups)
      if (static_cast<int64_t>(g.index) == state_col) return Err(PXG_INVALID_ARGUMENT, "serialized_expressions cannot be a group");
    const int32_t col = env[state_col].insns[0].arg;
    auto word = [col](int32_t type, int64_t off) {
      Program p;
      p.insns.push_back(Insn(PXG_OP_STATE_WORD, type, col, off));
      p.result_type = type;
      return p;
    };
    int64_t off = 0;
    for (auto& v : a.values) {
      std::vector<int32_t> types;
      for (auto& ia : v.init_args) types.push_back(ia.data_type);
      if (v.args_data_types.size() != v.args.size()) return Err(PXG_INVALID_ARGUMENT, "finalize agg %s needs args_data_types", v.name.c_str());
      for (auto t : v.args_data_types) types.push_back(t);
      auto* d = GetRegistry().GetUDA(v.name, types);
      if (!d) return Err(PXG_NOT_FOUND, "no device UDA %s", Signature(v.name, types).c_str());
      const int32_t kind = std::get<0>(*d), out = std::get<2>(*d);
      Uda u;
      u.out_type = out;
      u.has_arg = true;
      switch (kind) {
        case PXG_UDA_COUNT:  // CountUDA state: uint64 count, merged by addition
        case PXG_UDA_SUM:    // SumUDA state: the running sum (INT64 for BOOLEAN/INT64 args)
          u.kind = PXG_UDA_SUM;
          u.arg_type = out;
          u.arg = word(out, off);
          off += 8;
          break;
        case PXG_UDA_MIN:
        case PXG_UDA_MAX:
          u.kind = kind;
          u.arg_type = out;
          u.arg = word(out, off);
          off += 8;
          break;
        case PXG_UDA_MEAN:  // MeanInfo {uint64 size; double count}
          u.kind = PXG_UDA_MEAN_MERGE;
          u.arg_type = F;
          u.arg = word(F, off + 8);
          u.arg2 = word(I, off);
          u.has_arg2 = true;
          off += 16;
          break;
        default:
          return Err(PXG_UNIMPLEMENTED, "UDA %s has no Deserialize: it does not support partial aggregation", v.name.c_str());
      }
      udas.push_back(u);
    }
    state_rec = off;
    if (output_.size() != keys.size() + udas.size())
      return Err(PXG_INVALID_ARGUMENT, "output relation arity %zu != groups + values %zu", output_.size(), keys.size() + udas.size());
    return Status::OK();
  }
  Status OpenImpl(ExecState* s) override {
    if (!s->ctx) return Status::OK();
    hints_ = s->group_hints;
    if (hints_) {
      auto it = hints_->find(HintKey());
      if (it != hints_->end()) expected_groups_ = it->second;
    }
    cache_ = s->agg_cache;
    if (cache_) {
      auto it = cache_->find(SpecKey());
      if (it != cache_->end()) {
        agg_ = it->second;
        cache_->erase(it);
        PXG_CALL(pxg_agg_reset(agg_));
      }
    }
    if (!agg_) PXC_RETURN_IF_ERROR(CreateAgg(s->ctx));
    if (!device_input)
      PXG_CALL(pxg_table_create(s->ctx, static_cast<int32_t>(source_types.size()), source_types.data(), &staging_));
    return Status::OK();
  }
  Status CloseImpl(ExecState*) override {
    if (agg_ && cache_ && cache_->count(SpecKey()) == 0 && cache_->size() < kAggCacheMax) cache_->emplace(SpecKey(), agg_);
    else if (agg_) pxg_agg_destroy(agg_);
    if (staging_) pxg_table_destroy(staging_);
    agg_ = nullptr;
    staging_ = nullptr;
    return Status::OK();
  }
  Status ConsumeNextImpl(ExecState* s, const RowBatch& rb, size_t) override {
    // Tiny batches are coalesced by the table's staging before they reach HBM.
    if (rb.num_rows > 0) {
      if (merge_states) {  // every record is exactly the UDAs' Serialize() bytes
        const HostColumn& sc = rb.cols.at(static_cast<size_t>(state_col));
        for (int64_t r = 0; r < rb.num_rows; ++r)
          if (sc.offsets[r + 1] - sc.offsets[r] != state_rec)
            return Err(PXG_INVALID_ARGUMENT, "serialized_expressions of %d bytes, expected %lld", sc.offsets[r + 1] - sc.offsets[r], (long long)state_rec);
      }
      std::vector<pxg_column_view> v;
      for (auto& c : rb.cols) v.push_back(c.View());
      PXG_CALL(pxg_table_append(staging_, v.data(), rb.num_rows));
    }
    if (!(rb.eos || (windowed && rb.eow))) return Status::OK();  // agg_node.cc:169-171
    PXG_CALL(pxg_table_flush(staging_));
    PXG_CALL(pxg_agg_consume(agg_, staging_, 0, pxg_table_num_rows(staging_)));
    // New staging for the next window, ClearAggState (agg_node.cc:173-180).
    pxg_table_destroy(staging_);
    staging_ = nullptr;
    PXG_CALL(pxg_table_create(s->ctx, static_cast<int32_t>(source_types.size()), source_types.data(), &staging_));
    return Emit(s, rb.eow, rb.eos);
  }

 public:
  // Fused chain over a stored device table: rows [lo, hi) consumed in place (no staging), then
  // the one eos batch.  The programs reference the stored table's columns.
  Status ConsumeTable(ExecState* s, pxg_table* t, int64_t lo, int64_t hi) {
    StageClock clk;
    if (hi > lo) PXG_CALL(pxg_agg_consume(agg_, t, lo, hi));
    clk.Mark("agg consume (launch)");
    return Emit(s, true, true);
  }

 private:
  // Finalize, render the result batch, ClearAggState, send.
  Status Emit(ExecState* s, bool eow, bool eos) {
    StageClock clk;
    int64_t groups = 0;
    // Every consumer takes device batches (the agg -> equijoin hand-off): the result stays in HBM.
    bool dev_ok = !children_.empty() && !emit_states;
    for (auto& ch : children_) dev_ok = dev_ok && ch.first->AcceptsDeviceBatch();
    std::vector<pxg_column_out> out(keys.size() + (emit_states ? 1 : udas.size()));
    // A quantiles column no consumer reads as a string (the pluck-only C2 shape) is not copied
    // out: only the plucked lanes and a per-group finiteness flag come back (pluck on the device).
    std::vector<uint8_t> skip(out.size(), 0);
    std::vector<uint32_t> lanes(out.size(), 0);
    quantiles_raw_.clear();
    quantile_lanes_.clear();
    for (size_t c = keys.size(); c < out.size() && !emit_states; ++c) {
      if (udas[c - keys.size()].kind != PXG_UDA_QUANTILES) continue;
      bool observed = false;
      for (auto& ch : children_) {
        observed = observed || ch.first->ReadsColumnValue(c);
        lanes[c] |= ch.first->PluckedLanes(c);
      }
      // pluck-only: the column comes back as its plucked lanes (pxg.h, skip = 0x80 | lane mask)
      skip[c] = observed || !DevicePluck() ? 0 : static_cast<uint8_t>(0x80u | (lanes[c] & 0x7Fu));
    }
    bool fetched = false;
    if (dev_ok) {
      PXG_CALL(pxg_agg_finalize(agg_, &groups));
    } else {  // finalize with the result copies overlapping it
      PXG_CALL(pxg_agg_finalize_result(agg_, &groups, out.data(), static_cast<int32_t>(out.size()), skip.data()));
      fetched = true;
    }
    if (hints_) (*hints_)[HintKey()] = std::max<int64_t>(groups, 1);
    if (stats_.collect) {
      int64_t sel = 0;
      if (pxg_agg_rows_selected(agg_, &sel) == PXG_OK) stats_.AddExtraMetric("rows_aggregated", static_cast<double>(sel));
      stats_.AddExtraMetric("groups", static_cast<double>(groups));
    }
    clk.Mark("agg finalize");
    if (dev_ok) {
      std::vector<pxg_column_view> dv(keys.size() + udas.size());
      int64_t bytes = 0;
      const int32_t rc = pxg_agg_result_device(agg_, dv.data(), static_cast<int32_t>(dv.size()), &bytes);
      if (rc == PXG_OK) {
        RowBatch ob;
        ob.num_rows = groups;
        ob.eow = eow;
        ob.eos = eos;
        ob.dev = dv.data();
        ob.dev_bytes = bytes;
        clk.Mark("agg result (device views)");
        Status st = SendRowBatchToChildren(s, ob);  // consumers copy in stream order
        clk.Mark("children (device batch)");
        PXC_RETURN_IF_ERROR(st);
        PXG_CALL(pxg_agg_reset(agg_));
        return Status::OK();
      }
      if (rc != PXG_UNIMPLEMENTED) return FromPxg(rc);
    }
    if (!fetched) PXG_CALL(pxg_agg_result_skip(agg_, out.data(), static_cast<int32_t>(out.size()), skip.data()));
    const int64_t G = out.empty() ? 0 : out[0].length;
    for (size_t c = 0; c < out.size(); ++c) {
      if (!skip[c] || groups == 0) continue;
      QuantLanes ql;  // values = the lanes, data = the finiteness bytes (one owner for both)
      ql.mask = lanes[c] & 0x7Fu;
      ql.nsel = __builtin_popcount(ql.mask);
      ql.vals = FromOut(out[c]);
      ql.vals.type = F;
      ql.vals.data = nullptr;
      ql.finite = std::shared_ptr<void>(ql.vals.owner, const_cast<uint8_t*>(out[c].data));
      quantile_lanes_[c] = ql;
    }
    clk.Mark("agg result D2H");
    RowBatch ob;
    ob.num_rows = G;
    for (size_t c = 0; c < out.size(); ++c) {
      const bool q = !emit_states && c >= keys.size() && udas[c - keys.size()].kind == PXG_UDA_QUANTILES;
      if (q && skip[c]) {  // G empty strings keep the batch's relation (the lanes are owned above)
        if (groups == 0) pxg_result_free(&out[c], 1);
        ob.cols.push_back(EmptyStringColumn(out[c].length));
        continue;
      }
      HostColumn hc = FromOut(out[c]);
      if (q) {  // QuantilesUDA::Finalize JSON (math_sketches.h:40-54) from the 7 device doubles
        quantiles_raw_[c] = hc;
        ob.cols.push_back(RenderQuantilesJson(static_cast<const double*>(hc.values), hc.length));
      } else {
        ob.cols.push_back(hc);
      }
    }
    ob.eow = eow;
    ob.eos = eos;
    clk.Mark("agg render (quantile JSON)");
    PXG_CALL(pxg_agg_reset(agg_));
    clk.Mark("agg reset");
    Status st = SendRowBatchToChildren(s, ob);
    clk.Mark("children (map, sink)");
    return st;
  }

 public:
  // Raw 7-double quantile columns of the last emitted batch (post-agg pluck reads them), and
  // for pluck-only columns the plucked lanes fetched on the device instead.
  std::map<size_t, HostColumn> quantiles_raw_;
  struct QuantLanes {
    uint32_t mask = 0;
    int nsel = 0;
    HostColumn vals;               // nsel lanes of G doubles (lane-major, in bit order)
    std::shared_ptr<void> finite;  // G bytes: all 7 quantiles finite
  };
  std::map<size_t, QuantLanes> quantile_lanes_;

  // The device aggregation this node would run, handed to the caller (pxc_plan_create_agg).
  Status CreateDeviceAgg(pxg_ctx* ctx, int64_t expected_groups, pxg_agg** out) {
    expected_groups_ = expected_groups;
    PXC_RETURN_IF_ERROR(CreateAgg(ctx));
    *out = agg_;
    agg_ = nullptr;
    return Status::OK();
  }

 private:
  Status CreateAgg(pxg_ctx* ctx) {
    std::vector<pxg_program> kp;
    for (auto& k : keys) kp.push_back(k.View());
    std::vector<pxg_uda_spec> us(udas.size());
    for (size_t i = 0; i < udas.size(); ++i) {
      pxg_uda_spec& x = us[i];
      std::memset(&x, 0, sizeof(x));
      x.kind = udas[i].kind;
      x.arg_type = udas[i].arg_type;
      if (udas[i].has_arg) x.arg = udas[i].arg.View();
      if (udas[i].has_arg2) x.arg2 = udas[i].arg2.View();
      x.has_init = udas[i].has_init ? 1 : 0;
      x.init_i64 = udas[i].init;
    }
    pxg_agg_spec spec{};
    spec.n_keys = static_cast<int32_t>(kp.size());
    spec.n_udas = static_cast<int32_t>(us.size());
    spec.keys = kp.data();
    spec.udas = us.data();
    pxg_program fp = filter.View();
    spec.filter = has_filter ? &fp : nullptr;
    spec.expected_groups = expected_groups_;
    spec.windowed = windowed ? 1 : 0;
    spec.emit_states = emit_states ? 1 : 0;
    PXG_CALL(pxg_agg_create(ctx, &spec, &agg_));
    return Status::OK();
  }
  // Identity of this aggregation for the group-count statistics: source, keys, filter.
  std::string HintKey() const {
    std::string k = hint_source + "|";
    auto add = [&k](const Program& p) {
      for (auto& i : p.insns) k += std::to_string(i.op) + ":" + std::to_string(i.type) + ":" + std::to_string(i.arg) + ":" + std::to_string(i.imm) + " ";
      k += "|";
    };
    for (auto& p : keys) add(p);
    if (has_filter) add(filter);
    return k;
  }
  // Everything pxg_agg_create takes.
  std::string SpecKey() const {
    std::string k = HintKey();
    auto add = [&k](const Program& p) {
      for (auto& i : p.insns) k += std::to_string(i.op) + ":" + std::to_string(i.type) + ":" + std::to_string(i.arg) + ":" + std::to_string(i.imm) + " ";
      k.append(reinterpret_cast<const char*>(p.pool.data()), p.pool.size());
      k += "|";
    };
    for (auto& u : udas) {
      k += "U" + std::to_string(u.kind) + ":" + std::to_string(u.arg_type) + ":" + std::to_string(u.has_init) + ":" + std::to_string(u.init) + ":";
      if (u.has_arg) add(u.arg);
      if (u.has_arg2) add(u.arg2);
    }
    if (has_filter) add(filter);
    return k + (windowed ? "W" : "B") + (emit_states ? "S" : "");
  }
  static constexpr size_t kAggCacheMax = 8;
  pxg_agg* agg_ = nullptr;
  pxg_table* staging_ = nullptr;
  int64_t expected_groups_ = 0;
  std::map<std::string, int64_t>* hints_ = nullptr;
  std::multimap<std::string, pxg_agg*>* cache_ = nullptr;

 public:
  std::string hint_source;  // the source table's name (set by the graph builder)
};

// A zero-row batch of the given types (RowBatch::WithZeroRows).
static RowBatch ZeroRowBatch(const RowDescriptor& types, bool eow, bool eos) {
  static const int32_t zero_off[2] = {0, 0};
  static const uint8_t pad[16] = {0};
  RowBatch rb;
  for (int32_t t : types) {
    HostColumn hc;
    hc.type = t;
    hc.offsets = zero_off;
    hc.data = pad;
    hc.values = pad;
    rb.cols.push_back(hc);
  }
  rb.eow = eow;
  rb.eos = eos;
  return rb;
}

// pluck_float64 (PluckAsFloat64UDF, json_ops.h:131-153) of a JSON string that did not come from
// a device quantiles column: rapidjson's default parse of an object, the member's value if it
// is a number with a fraction or exponent (IsDouble), else 0.0; a parse failure gives 0.0.
static double PluckJson(const char* p, size_t n, const std::string& key) {
  size_t i = 0;
  auto ws = [&]() { while (i < n && (p[i] == ' ' || p[i] == '\t' || p[i] == '\n' || p[i] == '\r')) ++i; };
  auto str = [&](std::string* out) -> bool {
    if (i >= n || p[i] != '"') return false;
    for (++i; i < n && p[i] != '"'; ++i) {
      if (p[i] == '\\') { if (++i >= n) return false; }
      if (out) out->push_back(p[i]);
    }
    if (i >= n) return false;
    ++i;
    return true;
  };
  // skip one JSON value; *dbl / *is_double receive a number's value / kind
  std::function<bool(double*, bool*)> value = [&](double* dbl, bool* is_double) -> bool {
    ws();
    if (i >= n) return false;
    const char c = p[i];
    if (c == '"') return str(nullptr);
    if (c == '{' || c == '[') {
      const char close = c == '{' ? '}' : ']';
      ++i;
      ws();
      if (i < n && p[i] == close) { ++i; return true; }
      for (;;) {
        if (close == '}') {
          ws();
          if (!str(nullptr)) return false;
          ws();
          if (i >= n || p[i] != ':') return false;
          ++i;
        }
        if (!value(nullptr, nullptr)) return false;
        ws();
        if (i < n && p[i] == ',') { ++i; continue; }
        if (i < n && p[i] == close) { ++i; return true; }
        return false;
      }
    }
    if (!std::strncmp(p + i, "true", std::min<size_t>(4, n - i)) && n - i >= 4) { i += 4; return true; }
    if (!std::strncmp(p + i, "false", std::min<size_t>(5, n - i)) && n - i >= 5) { i += 5; return true; }
    if (!std::strncmp(p + i, "null", std::min<size_t>(4, n - i)) && n - i >= 4) { i += 4; return true; }
    const size_t s0 = i;
    bool frac = false;
    if (i < n && p[i] == '-') ++i;
    if (i >= n || !(p[i] >= '0' && p[i] <= '9')) return false;
    while (i < n && ((p[i] >= '0' && p[i] <= '9') || p[i] == '.' || p[i] == 'e' || p[i] == 'E' || p[i] == '+' || p[i] == '-')) {
      frac = frac || p[i] == '.' || p[i] == 'e' || p[i] == 'E';
      ++i;
    }
    if (dbl) *dbl = std::strtod(std::string(p + s0, i - s0).c_str(), nullptr);
    if (is_double) *is_double = frac;
    return true;
  };
  double found = 0.0;
  bool have = false;
  ws();
  if (i >= n || p[i] != '{') return 0.0;
  ++i;
  ws();
  if (i < n && p[i] == '}') return 0.0;
  for (;;) {
    ws();
    std::string k;
    if (!str(&k)) return 0.0;
    ws();
    if (i >= n || p[i] != ':') return 0.0;
    ++i;
    double d = 0;
    bool isd = false;
    if (!value(&d, &isd)) return 0.0;
    if (k == key && !have) {  // FindMember: the first member with the name
      found = isd ? d : 0.0;
      have = true;
    }
    ws();
    if (i < n && p[i] == ',') { ++i; continue; }
    if (i < n && p[i] == '}') { ++i; break; }
    return 0.0;
  }
  ws();
  return i == n ? found : 0.0;
}

// MapNode after an aggregate (map_node.cc:47-71) over the G result rows: any expression.
// pluck_float64(column, 'key') sub-expressions become extra FLOAT64 input columns (from the
// digest's own doubles when the column is a device quantiles UDA, else parsed from the JSON);
// bare column references pass through; every other expression runs as one device program
// (pxg_map) over the G rows.
class PostAggMapNode : public ExecNode {
 public:
  explicit PostAggMapNode(GpuAggNode* agg) : agg_(agg) {}
  // A quantiles column is read as a string only when some expression does more than pluck it.
  bool ReadsColumnValue(size_t col) const override { return string_reads_.count(col) > 0; }
  uint32_t PluckedLanes(size_t col) const override {
    uint32_t m = 0;
    for (auto& pk : plucks_)
      if (pk.first == static_cast<int64_t>(col))
        for (int k = 0; k < 7; ++k)
          if (pk.second == kQuantileKeys[k]) m |= 1u << k;
    return m;
  }
  std::string DebugString() const override { return "PostAggMapNode(device map over the aggregate rows)"; }

  // Rewrites one expression (pluck_float64 leaves -> extra columns) and compiles it.
  static Status Lower(const planpb::ScalarExpression& e, const RowDescriptor& in, std::vector<std::pair<int64_t, std::string>>* plucks,
                      std::set<size_t>* string_reads, planpb::ScalarExpression* out) {
    if (e.kind == planpb::ScalarExpression::kFunc && e.func->name == "pluck_float64" && e.func->args.size() == 2 &&
        e.func->args[0].kind == planpb::ScalarExpression::kColumn && e.func->args[1].kind == planpb::ScalarExpression::kConstant &&
        e.func->args[1].constant.data_type == S) {
      const uint64_t c = e.func->args[0].column.index;
      if (c >= in.size() || in[c] != S) return Err(PXG_INVALID_ARGUMENT, "pluck_float64 of a non-STRING column");
      int64_t j = -1;
      for (size_t k = 0; k < plucks->size(); ++k)
        if ((*plucks)[k].first == static_cast<int64_t>(c) && (*plucks)[k].second == e.func->args[1].constant.string_value) j = static_cast<int64_t>(k);
      if (j < 0) {
        j = static_cast<int64_t>(plucks->size());
        plucks->push_back({static_cast<int64_t>(c), e.func->args[1].constant.string_value});
      }
      out->kind = planpb::ScalarExpression::kColumn;
      out->column.index = in.size() + static_cast<uint64_t>(j);
      return Status::OK();
    }
    *out = e;
    if (e.kind == planpb::ScalarExpression::kColumn) {
      if (e.column.index < in.size() && in[e.column.index] == S) string_reads->insert(e.column.index);
      return Status::OK();
    }
    if (e.kind == planpb::ScalarExpression::kFunc) {
      out->func = std::make_shared<planpb::ScalarFunc>(*e.func);
      for (size_t a = 0; a < e.func->args.size(); ++a)
        PXC_RETURN_IF_ERROR(Lower(e.func->args[a], in, plucks, string_reads, &out->func->args[a]));
    }
    return Status::OK();
  }
  static Status OutputTypes(const planpb::Operator& op, const RowDescriptor& in, RowDescriptor* out) {
    std::vector<std::pair<int64_t, std::string>> plucks;
    std::set<size_t> reads;
    std::vector<planpb::ScalarExpression> lowered(op.map.expressions.size());
    for (size_t i = 0; i < lowered.size(); ++i) PXC_RETURN_IF_ERROR(Lower(op.map.expressions[i], in, &plucks, &reads, &lowered[i]));
    RowDescriptor env = in;
    env.insert(env.end(), plucks.size(), F);
    ExprCompiler comp(ColumnEnv(env));
    for (auto& e : lowered) {
      Program p;
      PXC_RETURN_IF_ERROR(comp.Compile(e, &p));
      out->push_back(p.result_type);
    }
    return Status::OK();
  }

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    const RowDescriptor& in = inputs_[0];
    std::vector<planpb::ScalarExpression> lowered(op.map.expressions.size());
    for (size_t i = 0; i < lowered.size(); ++i) PXC_RETURN_IF_ERROR(Lower(op.map.expressions[i], in, &plucks_, &string_reads_, &lowered[i]));
    env_types_ = in;
    env_types_.insert(env_types_.end(), plucks_.size(), F);
    ExprCompiler comp(ColumnEnv(env_types_));
    for (auto& e : lowered) {
      Program p;
      PXC_RETURN_IF_ERROR(comp.Compile(e, &p));
      if (p.IsColumn()) {
        passthrough_.push_back(p.insns[0].arg);
      } else {
        passthrough_.push_back(-1);
        device_.push_back(p);
      }
    }
    return Status::OK();
  }
  Status ConsumeNextImpl(ExecState* s, const RowBatch& rb, size_t) override {
    const int64_t G = rb.num_rows;
    std::vector<HostColumn> env = rb.cols;
    finite_.clear();
    for (auto& pk : plucks_) {
      auto it = agg_ ? agg_->quantiles_raw_.find(static_cast<size_t>(pk.first)) : decltype(agg_->quantiles_raw_.end()){};
      auto lt = agg_ ? agg_->quantile_lanes_.find(static_cast<size_t>(pk.first)) : decltype(agg_->quantile_lanes_.end()){};
      int qk = -1;
      for (int k = 0; k < 7; ++k)
        if (pk.second == kQuantileKeys[k]) qk = k;
      if (agg_ && lt != agg_->quantile_lanes_.end()) {  // plucked on the device: the lane is the column
        const auto& ql = lt->second;
        const int at = qk >= 0 && ((ql.mask >> qk) & 1u) ? __builtin_popcount(ql.mask & ((1u << qk) - 1)) : -1;
        if (at >= 0) {
          HostColumn lc = ql.vals;
          lc.length = G;
          lc.values = static_cast<const double*>(ql.vals.values) + static_cast<int64_t>(at) * G;
          env.push_back(lc);
          continue;
        }
      }
      double* v = nullptr;
      HostColumn vc = PooledDoubleColumn(G, &v);
      if (agg_ && lt != agg_->quantile_lanes_.end()) {
        for (int64_t g = 0; g < G; ++g) v[g] = 0.0;
      } else if (agg_ && it != agg_->quantiles_raw_.end()) {
        // A NaN / inf quantile truncates the reference's JSON (json_double.h), which rapidjson then
        // fails to parse: pluck_float64 returns 0.0 for every key of that group.  The per-group
        // finiteness is computed once per raw column (C2 plucks two keys of one column).
        const double* d = static_cast<const double*>(it->second.values);
        std::vector<uint8_t>& fin = finite_[pk.first];
        if (static_cast<int64_t>(fin.size()) != G) {
          fin.resize(static_cast<size_t>(G));
          // NaN / inf <=> all exponent bits set; branch-free over the 7 values so it vectorises.
          const uint64_t* bits = static_cast<const uint64_t*>(it->second.values);
          for (int64_t g = 0; g < G; ++g) {
            uint32_t bad = 0;
            for (int k = 0; k < 7; ++k) bad |= ((bits[g * 7 + k] >> 52) & 0x7FF) == 0x7FF ? 1u : 0u;
            fin[static_cast<size_t>(g)] = static_cast<uint8_t>(bad ^ 1u);
          }
        }
        for (int64_t g = 0; g < G; ++g) v[g] = (qk >= 0 && fin[static_cast<size_t>(g)]) ? d[g * 7 + qk] : 0.0;
      } else {
        const HostColumn& c = rb.cols[static_cast<size_t>(pk.first)];
        for (int64_t g = 0; g < G; ++g)
          v[g] = PluckJson(reinterpret_cast<const char*>(c.data) + c.offsets[g], static_cast<size_t>(c.offsets[g + 1] - c.offsets[g]),
                           pk.second);
      }
      env.push_back(vc);
    }
    std::vector<HostColumn> dev_out;
    if (!device_.empty() && G > 0) {
      pxg_table* in = nullptr;
      RowBatch eb;
      eb.cols = env;
      eb.num_rows = G;
      PXC_RETURN_IF_ERROR(UploadBatch(s->ctx, eb, env_types_, &in));
      std::vector<pxg_program> pv;
      for (auto& p : device_) pv.push_back(p.View());
      pxg_table* out = nullptr;
      Status st = FromPxg(pxg_map(in, static_cast<int32_t>(pv.size()), pv.data(), 0, G, &out));
      RowBatch ob;
      if (st.ok()) st = FetchAll(out, static_cast<int32_t>(pv.size()), &ob);
      if (out) pxg_table_destroy(out);
      pxg_table_destroy(in);
      PXC_RETURN_IF_ERROR(st);
      dev_out = ob.cols;
    }
    RowBatch ob;
    ob.num_rows = G;
    size_t d = 0;
    for (size_t i = 0; i < passthrough_.size(); ++i) {
      if (passthrough_[i] >= 0) {
        ob.cols.push_back(env[static_cast<size_t>(passthrough_[i])]);
      } else if (G > 0) {
        ob.cols.push_back(dev_out[d++]);
      } else {
        ob.cols.push_back(ZeroRowBatch({device_[d++].result_type}, false, false).cols[0]);
      }
    }
    ob.eow = rb.eow;
    ob.eos = rb.eos;
    return SendRowBatchToChildren(s, ob);
  }

 private:
  GpuAggNode* agg_;
  std::map<int64_t, std::vector<uint8_t>> finite_;  // per plucked raw column: group's 7 quantiles all finite
  std::vector<std::pair<int64_t, std::string>> plucks_;  // (input column, key) -> extra column
  std::set<size_t> string_reads_;
  RowDescriptor env_types_;
  std::vector<int32_t> passthrough_;  // per output: env column, or -1 for the next device program
  std::vector<Program> device_;
};

// LimitNode (limit_node.cc:55-95): forwards rows until `limit` have passed; the batch that
// reaches the limit is cut there and carries eow / eos, later batches are dropped, and the
// abortable sources are stopped (ExecState::StopSource).
class LimitNode : public ExecNode {
 public:
  std::string DebugString() const override { return "LimitNode(" + std::to_string(limit_) + ")"; }

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    limit_ = op.limit.limit;
    for (auto& c : op.limit.columns) {  // the output relation is exactly these (operators.cc:424-445)
      if (c.index >= inputs_[0].size()) return Err(PXG_INVALID_ARGUMENT, "limit column out of range");
      cols_.push_back(static_cast<size_t>(c.index));
    }
    srcs_ = op.limit.abortable_srcs;
    return Status::OK();
  }
  Status ConsumeNextImpl(ExecState* s, const RowBatch& rb, size_t) override {
    if (reached_) return Status::OK();
    const int64_t remainder = limit_ - processed_;
    RowBatch ob;
    for (size_t c : cols_) ob.cols.push_back(rb.cols[c]);
    if (remainder > rb.num_rows) {
      ob.num_rows = rb.num_rows;
      ob.eow = rb.eow;
      ob.eos = rb.eos;
      processed_ += rb.num_rows;
      return SendRowBatchToChildren(s, ob);
    }
    const int64_t keep = std::max<int64_t>(remainder, 0);
    ob.num_rows = keep;
    for (auto& c : ob.cols) c.length = keep;  // Slice(0, keep): same buffers, fewer rows
    ob.eow = ob.eos = true;
    processed_ += keep;
    reached_ = true;
    for (uint64_t id : srcs_) s->stopped_sources.insert(id);
    return SendRowBatchToChildren(s, ob);
  }

 private:
  int64_t limit_ = 0, processed_ = 0;
  bool reached_ = false;
  std::vector<size_t> cols_;
  std::vector<uint64_t> srcs_;
};

// GpuEquijoinNode (EquijoinNode, equijoin_node.cc:53-470).  InitImpl maps left/right onto
// build/probe exactly as the reference does: the probe table is the left parent when the output
// has a "time_" column taken from parent 0 (order_by_time, operators.cc:531-541,639-645;
// equijoin_node.cc:63-69), otherwise the right parent; the JoinType then decides which side's
// unmatched rows are emitted (equijoin_node.cc:71-88).  Both inputs are staged into device
// tables; once both sides reached eos the join runs once on the device (pxg_join) and its
// output goes out in rows_per_batch batches: the probe-produced rows, with a partial batch cut at
// probe eos (FlushChunkedRows, equijoin_node.cc:388-390), then the unmatched build rows
// (EmitUnmatchedBuildRows, :398-411).  The last batch carries eow/eos; a zero-row eow/eos batch
// is sent when there is no output at all (equijoin_node.cc:447-459).
class GpuEquijoinNode : public ExecNode {
 public:
  bool AcceptsDeviceBatch() const override { return true; }
  std::string DebugString() const override {
    std::ostringstream os;
    os << "GpuEquijoinNode(type=" << type_ << ", probe=" << (probe_is_left_ ? "left" : "right") << ", rows_per_batch=" << rows_per_batch_
       << ")";
    return os.str();
  }

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    if (inputs_.size() != 2) return Err(PXG_INVALID_ARGUMENT, "Join operator expects a two input relations, got %zu", inputs_.size());
    const planpb::JoinOperator& j = op.join;
    type_ = j.type;
    rows_per_batch_ = j.rows_per_batch == 0 ? 1024 : static_cast<int64_t>(j.rows_per_batch);
    for (size_t i = 0; i < j.column_names.size() && i < j.output_columns.size(); ++i) {
      if (j.column_names[i] != "time_") continue;
      probe_is_left_ = j.output_columns[i].first == 0;
      // JoinOperator::Init (operators.cc:593-603).
      if (type_ == 3) return Err(PXG_INVALID_ARGUMENT, "For time ordered joins, full outer join is not supported.");
      if (type_ == 1 && !probe_is_left_)
        return Err(PXG_INVALID_ARGUMENT, "For time ordered joins, left join is only supported when time_ comes from the left table.");
      break;
    }
    switch (type_) {
      case 0: break;
      case 1:
        emit_build_ = !probe_is_left_;
        emit_probe_ = probe_is_left_;
        break;
      case 3: emit_build_ = emit_probe_ = true; break;
      default: return Err(PXG_INTERNAL, "EquijoinNode: Unknown Join Type %d", type_);
    }
    const size_t probe_parent = probe_is_left_ ? 0 : 1;
    for (auto& c : j.equality_conditions) {
      if (c.first >= inputs_[0].size() || c.second >= inputs_[1].size()) return Err(PXG_INVALID_ARGUMENT, "join key column out of range");
      if (inputs_[0][c.first] != inputs_[1][c.second]) return Err(PXG_INVALID_ARGUMENT, "join key types differ");
      const int32_t l = static_cast<int32_t>(c.first), r = static_cast<int32_t>(c.second);
      build_keys_.push_back(probe_is_left_ ? r : l);
      probe_keys_.push_back(probe_is_left_ ? l : r);
    }
    if (build_keys_.empty()) return Err(PXG_INVALID_ARGUMENT, "join without equality conditions");
    for (auto& o : j.output_columns) {
      if (o.first > 1 || o.second >= inputs_[o.first].size()) return Err(PXG_INVALID_ARGUMENT, "join output column out of range");
      out_side_.push_back(o.first == probe_parent ? 0 : 1);
      out_col_.push_back(static_cast<int32_t>(o.second));
    }
    if (out_side_.empty()) return Err(PXG_UNIMPLEMENTED, "join with no output columns");
    return Status::OK();
  }
  Status OpenImpl(ExecState* s) override {
    if (!s->ctx) return Status::OK();
    for (int side = 0; side < 2; ++side)
      PXG_CALL(pxg_table_create(s->ctx, static_cast<int32_t>(inputs_[side].size()), inputs_[side].data(), &staged_[side]));
    return Status::OK();
  }
  Status CloseImpl(ExecState*) override {
    for (auto& t : staged_) {
      if (t) pxg_table_destroy(t);
      t = nullptr;
    }
    return Status::OK();
  }
  Status ConsumeNextImpl(ExecState* s, const RowBatch& rb, size_t parent_index) override {
    if (parent_index > 1) return Err(PXG_INTERNAL, "join parent index %zu", parent_index);
    if (eos_[parent_index]) return Err(PXG_INTERNAL, "join input %zu after eos", parent_index);
    if (rb.num_rows > 0 && rb.dev) {
      PXG_CALL(pxg_table_append_device(staged_[parent_index], rb.dev, rb.num_rows));  // HBM to HBM
    } else if (rb.num_rows > 0) {
      StageClock clk;
      std::vector<pxg_column_view> v;
      for (auto& c : rb.cols) v.push_back(c.View());
      PXG_CALL(pxg_table_append(staged_[parent_index], v.data(), rb.num_rows));
      clk.Mark("join: stage input");
    }
    if (rb.eos) eos_[parent_index] = true;
    if (!(eos_[0] && eos_[1])) return Status::OK();
    return Run(s);
  }

 private:
  Status Run(ExecState* s) {
    pxg_table* probe = staged_[probe_is_left_ ? 0 : 1];
    pxg_table* build = staged_[probe_is_left_ ? 1 : 0];
    PXG_CALL(pxg_table_flush(probe));
    PXG_CALL(pxg_table_flush(build));
    pxg_join_spec sp{};
    sp.n_keys = static_cast<int32_t>(build_keys_.size());
    sp.emit_unmatched_probe = emit_probe_;
    sp.emit_unmatched_build = emit_build_;
    sp.n_out = static_cast<int32_t>(out_side_.size());
    sp.build_keys = build_keys_.data();
    sp.probe_keys = probe_keys_.data();
    sp.out_side = out_side_.data();
    sp.out_col = out_col_.data();
    pxg_table* out = nullptr;
    int64_t nprobe = 0;
    StageClock clk;
    PXG_CALL(pxg_join(build, probe, &sp, &out, &nprobe));
    clk.Mark("join: device join");
    std::unique_ptr<pxg_table, int32_t (*)(pxg_table*)> guard(out, pxg_table_destroy);
    const int64_t n = pxg_table_num_rows(out);
    std::vector<std::pair<int64_t, int64_t>> ranges;
    for (int64_t b = 0; b < nprobe; b += rows_per_batch_) ranges.push_back({b, std::min(nprobe, b + rows_per_batch_)});
    for (int64_t b = nprobe; b < n; b += rows_per_batch_) ranges.push_back({b, std::min(n, b + rows_per_batch_)});
    if (ranges.empty()) return SendRowBatchToChildren(s, ZeroRowBatch(output_, true, true));
    // Every consumer a result sink (C5's shape) and no per-batch stats wanted: the batches are
    // laid out on the device as one PXRB image, moved to the result buffer by one DMA at
    // serialisation (PXC_NO_RESULT_IMAGE=1: tests compare with the host path below).
    bool image_ok = !s->collect_exec_stats && !children_.empty() && !EnvOn("PXC_NO_RESULT_IMAGE");
    for (auto& ch : children_) image_ok = image_ok && ch.first->AcceptsResultImage();
    if (image_ok) {
      std::vector<int64_t> starts;
      for (auto& r : ranges) starts.push_back(r.first);
      starts.push_back(ranges.back().second);
      pxg_pxrb* img = nullptr;
      int64_t bytes = 0;
      const int32_t rc = pxg_table_pxrb_image(out, starts.data(), static_cast<int64_t>(ranges.size()), 1, 1, &img, &bytes);
      if (rc == PXG_OK) {
        RowBatch ob;
        ob.num_rows = n;
        ob.eow = ob.eos = true;
        ob.image = std::shared_ptr<pxg_pxrb>(img, [](pxg_pxrb* p) { pxg_pxrb_destroy(p); });
        ob.image_batches = static_cast<int64_t>(ranges.size());
        ob.image_bytes = bytes;
        clk.Mark("join: result image");
        return SendRowBatchToChildren(s, ob);
      }
      if (rc != PXG_UNIMPLEMENTED) return FromPxg(rc);
    }
    // One device-to-host fetch per output column; the batches are slices of it (a fetch per
    // batch and column cost ~140 us each: 2634 batches of C5 took 370 ms).
    std::vector<HostColumn> full;
    for (size_t c = 0; c < out_side_.size(); ++c) {
      pxg_column_out o{};
      PXG_CALL(pxg_table_fetch(out, static_cast<int32_t>(c), 0, n, &o));
      full.push_back(FromOut(o));
    }
    clk.Mark("join: output D2H");
    for (size_t r = 0; r < ranges.size(); ++r) {
      RowBatch ob;
      ob.num_rows = ranges[r].second - ranges[r].first;
      for (auto& fc : full) ob.cols.push_back(SliceColumn(fc, ranges[r].first, ob.num_rows));
      ob.eow = ob.eos = r + 1 == ranges.size();
      PXC_RETURN_IF_ERROR(SendRowBatchToChildren(s, ob));
    }
    clk.Mark("join: output batches");
    return Status::OK();
  }

  int32_t type_ = 0;
  int64_t rows_per_batch_ = 1024;
  bool probe_is_left_ = false;
  int32_t emit_build_ = 0, emit_probe_ = 0;
  std::vector<int32_t> build_keys_, probe_keys_, out_side_, out_col_;
  pxg_table* staged_[2] = {nullptr, nullptr};
  bool eos_[2] = {false, false};
};

class SinkNode : public ExecNode {
 public:
  explicit SinkNode(std::string name) : name(std::move(name)) {}
  std::string DebugString() const override { return "SinkNode(" + name + ")"; }
  std::string name;
  std::vector<RowBatch> batches;

 protected:
  Status InitImpl(const planpb::Operator&) override { return Status::OK(); }
  Status ConsumeNextImpl(ExecState*, const RowBatch& rb, size_t) override {
    batches.push_back(rb);
    return Status::OK();
  }

 public:
  bool AcceptsResultImage() const override { return true; }
};

// GRPCSinkNode to another Carnot (grpc_sink_node.cc:276-330): every RowBatch, split above the
// request size limit with the last piece keeping eow / eos, serialised as schemapb.RowBatchData
// (the TransferResultChunkRequest payload).  The transport is the caller's: the messages are
// returned per destination GRPC source id (pxc_execute_plan_grpc).
class GrpcSinkNode : public ExecNode {
 public:
  explicit GrpcSinkNode(uint64_t dest) : dest_id(dest) {}
  std::string DebugString() const override { return "GrpcSinkNode(-> grpc source " + std::to_string(dest_id) + ")"; }
  uint64_t dest_id;
  std::vector<std::string> messages;

 protected:
  Status InitImpl(const planpb::Operator&) override { return Status::OK(); }
  Status ConsumeNextImpl(ExecState*, const RowBatch& rb, size_t) override {
    const std::vector<int64_t> sizes = SplitBatchSizes(rb);
    int64_t r0 = 0;
    for (size_t i = 0; i < sizes.size(); ++i) {
      const bool last = i + 1 == sizes.size();
      messages.push_back(EncodeRowBatchData(rb, r0, sizes[i], last && rb.eow, last && rb.eos));
      r0 += sizes[i];
    }
    return Status::OK();
  }
};

// ---------------------------------------------------------------------------------------
// HBM-resident table store (table_store::TableStore / Table, table.h:71-199).
// ---------------------------------------------------------------------------------------
struct StoredTable {
  pxg_table* t = nullptr;
  RowDescriptor types;
  std::vector<std::string> names;
  int32_t time_col = -1;  // the "time_" column, if any
  int64_t last_time = std::numeric_limits<int64_t>::min();
};
using TableStore = std::map<std::string, StoredTable>;

// UnionNode (union_node.cc).  Unordered (union_node.cc:268-289): every parent's batch is
// forwarded with its columns picked by the parent's column mapping; eow / eos are set once every
// parent has sent eos.  With a time_ output column (order_by_time, operators.cc:543) the parents'
// rows are merged by time (union_node.cc:172-258): the parent whose cursor row has the smallest
// time_ (ties: the lower parent index) supplies rows while its time stays <= the runner-up's, a
// parent without buffered rows stalls the merge until it delivers, output goes out in batches of
// rows_per_batch (default 1024) and, once every parent is at eos, as a last eow/eos batch.  A
// pending partial batch is also flushed when more than kFlushTimeout passed since the last flush
// (union_node.cc:127-146).  Rows are copied as runs (a parent's rows up to the runner-up's time)
// rather than one by one; the order is the reference's row for row.
class UnionNode : public ExecNode {
 public:
  static constexpr int64_t kDefaultRowsPerBatch = 1024;  // kDefaultUnionRowBatchSize
  static constexpr std::chrono::milliseconds kFlushTimeout{1000};  // kDefaultDataFlushTimeoutMillis
  std::string DebugString() const override { return ordered_ ? "UnionNode(ordered by time_)" : "UnionNode(unordered)"; }

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    maps_ = op.union_mappings;
    if (maps_.size() != inputs_.size()) return Err(PXG_INVALID_ARGUMENT, "Union has %zu column mappings for %zu parents", maps_.size(), inputs_.size());
    for (size_t p = 0; p < maps_.size(); ++p) {
      if (maps_[p].size() != op.union_names.size()) return Err(PXG_INVALID_ARGUMENT, "Union column mapping %zu has the wrong arity", p);
      for (size_t c = 0; c < maps_[p].size(); ++c)
        if (maps_[p][c] < 0 || static_cast<size_t>(maps_[p][c]) >= inputs_[p].size() || inputs_[p][maps_[p][c]] != output_[c])
          return Err(PXG_INVALID_ARGUMENT, "Union column mapping %zu:%zu is invalid", p, c);
    }
    eos_.assign(inputs_.size(), false);
    for (size_t c = 0; c < op.union_names.size(); ++c)
      if (op.union_names[c] == "time_") time_out_ = static_cast<int64_t>(c);
    ordered_ = time_out_ >= 0;
    if (ordered_) {
      if (output_[static_cast<size_t>(time_out_)] != PXG_TIME64NS && output_[static_cast<size_t>(time_out_)] != PXG_INT64)
        return Err(PXG_INVALID_ARGUMENT, "Union time_ column is not TIME64NS");
      rows_per_batch_ = op.union_rows_per_batch ? static_cast<int64_t>(op.union_rows_per_batch) : kDefaultRowsPerBatch;
      queue_.resize(inputs_.size());
      cursor_.assign(inputs_.size(), 0);
      ResetBuilders();
      last_flush_ = std::chrono::steady_clock::now();
    }
    return Status::OK();
  }
  Status ConsumeNextImpl(ExecState* s, const RowBatch& rb, size_t parent) override {
    if (ordered_) {
      queue_[parent].push_back(rb);
      PurgeEmpty(parent);
      PXC_RETURN_IF_ERROR(Merge(s));
      if (!sent_eos_ && built_ > 0 && std::chrono::steady_clock::now() - last_flush_ > kFlushTimeout) return Flush(s);
      return Status::OK();
    }
    if (rb.eos) eos_[parent] = true;
    RowBatch out;
    out.num_rows = rb.num_rows;
    for (int64_t i : maps_[parent]) out.cols.push_back(rb.cols[static_cast<size_t>(i)]);
    out.eow = out.eos = AllEos();
    return SendRowBatchToChildren(s, out);
  }

 private:
  struct Builder {
    int32_t type = 0;
    std::shared_ptr<OwnedColumn> col;
  };
  bool AllEos() const {
    for (bool e : eos_)
      if (!e) return false;
    return true;
  }
  void ResetBuilders() {
    builders_.assign(output_.size(), Builder{});
    for (size_t c = 0; c < output_.size(); ++c) {
      builders_[c].type = output_[c];
      builders_[c].col = std::make_shared<OwnedColumn>();
      if (output_[c] == PXG_STRING) builders_[c].col->offsets.push_back(0);
    }
    built_ = 0;
  }
  // CacheNextRowBatch (union_node.cc:240-258): drop leading zero-row batches, noting their eos.
  void PurgeEmpty(size_t p) {
    auto& q = queue_[p];
    while (!q.empty() && q.front().num_rows == 0) {
      if (q.front().eos) eos_[p] = true;
      q.pop_front();
    }
  }
  int64_t TimeAt(size_t p) const {
    const RowBatch& rb = queue_[p].front();
    return static_cast<const int64_t*>(rb.cols[static_cast<size_t>(maps_[p][static_cast<size_t>(time_out_)])].values)[cursor_[p]];
  }
  // Copies rows [r0, r1) of parent p's front batch into the output builders.
  void AppendRun(size_t p, int64_t r0, int64_t r1) {
    const RowBatch& rb = queue_[p].front();
    for (size_t c = 0; c < builders_.size(); ++c) {
      const HostColumn& in = rb.cols[static_cast<size_t>(maps_[p][c])];
      OwnedColumn& o = *builders_[c].col;
      if (in.type == PXG_STRING) {
        const int32_t a = in.offsets[r0], b = in.offsets[r1];
        const int32_t base = o.offsets.back();
        for (int64_t r = r0; r < r1; ++r) o.offsets.push_back(base + in.offsets[r + 1] - a);
        o.data.insert(o.data.end(), in.data + a, in.data + b);
      } else {
        const int w = in.type == B ? 1 : in.type == U ? 16 : 8;
        const uint8_t* v = static_cast<const uint8_t*>(in.values);
        o.values.insert(o.values.end(), v + r0 * w, v + r1 * w);
      }
    }
    built_ += r1 - r0;
  }
  Status Flush(ExecState* s) {
    const bool eos = AllEos();
    RowBatch out;
    out.num_rows = built_;
    for (auto& b : builders_) {
      HostColumn hc;
      hc.type = b.type;
      hc.length = built_;
      if (b.type == PXG_STRING) {
        b.col->data.resize(b.col->data.size() + 16, 0);
        hc.offsets = b.col->offsets.data();
        hc.data = b.col->data.data();
      } else {
        b.col->values.resize(b.col->values.size() + 16, 0);
        hc.values = b.col->values.data();
      }
      hc.owner = b.col;
      out.cols.push_back(hc);
    }
    out.eow = out.eos = eos;
    ResetBuilders();
    last_flush_ = std::chrono::steady_clock::now();
    if (eos) sent_eos_ = true;
    return SendRowBatchToChildren(s, out);
  }
  Status FlushIfFullOrEos(ExecState* s) {
    if (built_ < rows_per_batch_ && !AllEos()) return Status::OK();
    return Flush(s);
  }
  // MergeData (union_node.cc:172-238).
  Status Merge(ExecState* s) {
    while (!sent_eos_) {
      std::vector<size_t> live;
      for (size_t p = 0; p < queue_.size(); ++p) {
        if (eos_[p]) continue;
        if (queue_[p].empty()) return Status::OK();  // a parent without data stalls the merge
        live.push_back(p);
      }
      if (live.empty()) return FlushIfFullOrEos(s);
      std::sort(live.begin(), live.end(), [this](size_t a, size_t b) {
        const int64_t ta = TimeAt(a), tb = TimeAt(b);
        return ta < tb || (ta == tb && a < b);
      });
      const size_t p = live[0];
      const bool limited = live.size() > 1;
      const size_t q = limited ? live[1] : 0;
      const int64_t tq = limited ? TimeAt(q) : 0;
      while (!queue_[p].empty()) {
        const RowBatch& rb = queue_[p].front();
        const int64_t* t = static_cast<const int64_t*>(rb.cols[static_cast<size_t>(maps_[p][static_cast<size_t>(time_out_)])].values);
        const int64_t r0 = cursor_[p], n = rb.num_rows;
        const bool last = rb.eos;
        const int64_t cap = r0 + (rows_per_batch_ - built_);
        const int64_t stop = std::min(n, cap);
        int64_t r1 = r0;
        if (limited) {
          while (r1 < stop && (t[r1] < tq || (t[r1] == tq && p < q))) ++r1;
        } else {
          r1 = stop;
        }
        if (r1 > r0) AppendRun(p, r0, r1);
        cursor_[p] = r1;
        if (r1 == n) {  // `rb` is released here
          if (last) eos_[p] = true;
          queue_[p].pop_front();
          cursor_[p] = 0;
          PurgeEmpty(p);
        }
        if (r1 > r0) PXC_RETURN_IF_ERROR(FlushIfFullOrEos(s));
        if (r1 < stop) break;  // the runner-up's time is next
      }
    }
    return Status::OK();
  }

  std::vector<std::vector<int64_t>> maps_;
  std::vector<bool> eos_;
  bool ordered_ = false;
  int64_t time_out_ = -1;
  int64_t rows_per_batch_ = kDefaultRowsPerBatch;
  std::vector<std::deque<RowBatch>> queue_;
  std::vector<int64_t> cursor_;
  std::vector<Builder> builders_;
  int64_t built_ = 0;
  bool sent_eos_ = false;
  std::chrono::steady_clock::time_point last_flush_;
};

// GRPCSourceNode (grpc_source_node.cc:52-87): RowBatches received from a remote GRPCSink, in
// arrival order, as schemapb.RowBatchData messages (RowBatch::FromProto, row_batch.cc:201-224).
// The source is done once a batch with eos has been sent.
class GrpcSourceNode : public SourceNode {
 public:
  GrpcSourceNode(uint64_t id, const std::vector<std::pair<const uint8_t*, int64_t>>* msgs) : id_(id), msgs_(msgs) {}
  std::string DebugString() const override { return "GrpcSourceNode(" + std::to_string(id_) + ")"; }
  bool HasBatchesRemaining() const override { return !sent_eos_; }
  Status GenerateNextImpl(ExecState* s) override {
    if (!msgs_ || next_ >= msgs_->size())
      return Err(PXG_INVALID_ARGUMENT, "GRPC source %llu ran out of row batches before eos", (unsigned long long)id_);
    RowBatch rb;
    const auto& m = (*msgs_)[next_++];
    PXC_RETURN_IF_ERROR(DecodeRowBatchData(m.first, static_cast<size_t>(m.second), &rb));
    if (rb.cols.size() != output_.size()) return Err(PXG_INVALID_ARGUMENT, "RowBatch of %zu columns for a GRPC source of %zu", rb.cols.size(), output_.size());
    for (size_t c = 0; c < rb.cols.size(); ++c)
      if (rb.cols[c].type != output_[c]) return Err(PXG_INVALID_ARGUMENT, "RowBatch column %zu has type %d, the GRPC source declares %d", c, rb.cols[c].type, output_[c]);
    if (rb.eos && !rb.eow) return Err(PXG_INTERNAL, "Cannot have an eos without an eow");  // exec_node.h:217-220
    sent_eos_ = rb.eos;
    return SendRowBatchToChildren(s, rb);
  }

 protected:
  Status InitImpl(const planpb::Operator&) override { return Status::OK(); }

 private:
  uint64_t id_;
  const std::vector<std::pair<const uint8_t*, int64_t>>* msgs_;
  size_t next_ = 0;
  bool sent_eos_ = false;
};

// MemorySourceNode over a stored device table.  The cursor range comes from start_time /
// stop_time as in Table::Cursor (table.cc:56-95): [first row with time_ >= start, first row
// with time_ > stop).  A fused agg below consumes the range in place; otherwise the range goes
// out as RowBatches of kBatchRows rows fetched from HBM, the last one with eow/eos (an empty
// range gives one zero-row eow/eos batch, memory_source_node.cc:97-106).
class DeviceSourceNode : public SourceNode {
 public:
  static constexpr int64_t kBatchRows = 1 << 16;
  DeviceSourceNode(std::string name, const StoredTable* st) : name_(std::move(name)), st_(st) {}
  std::string DebugString() const override { return "MemorySourceNode(" + name_ + ", HBM-resident)"; }
  bool HasBatchesRemaining() const override { return !done_; }
  bool IsStreaming() const override { return ms_.streaming; }
  // RowBatch::NumBytes of the projected columns over [lo, hi): exact for the whole table
  // (string payload = device bytes - offsets), proportional for a sub-range.
  int64_t RangeBytes() const {
    const int64_t n = pxg_table_num_rows(st_->t);
    if (n <= 0 || hi_ <= lo_) return 0;
    int64_t b = 0;
    for (int64_t c : idxs_) {
      const int32_t t = st_->types[static_cast<size_t>(c)];
      int64_t cb = pxg_table_device_bytes(st_->t, static_cast<int32_t>(c));
      if (t == PXG_STRING) cb -= 4 * n;
      b += cb;
    }
    return hi_ - lo_ == n ? b : static_cast<int64_t>(static_cast<double>(b) * (hi_ - lo_) / n);
  }
  GpuAggNode* fused_agg = nullptr;
  const std::vector<int64_t>& idxs() const { return idxs_; }

  Status GenerateNextImpl(ExecState* s) override {
    if (!ranged_) {
      PXC_RETURN_IF_ERROR(Range());
      ranged_ = true;
      cur_ = lo_;
    }
    if (fused_agg) {
      done_ = true;
      // The agg reads the stored table in place: the range counts as one output batch.
      ++stats_.batches_output;
      stats_.rows_output += hi_ - lo_;
      stats_.bytes_output += RangeBytes();
      stats_.ResumeChildTimer();
      Status st = fused_agg->ConsumeTable(s, st_->t, lo_, hi_);
      stats_.StopChildTimer();
      return st;
    }
    const int64_t end = std::min(hi_, cur_ + kBatchRows);
    RowBatch rb;
    if (ms_.streaming && end <= cur_) {  // caught up: nothing ready (NextBatchReady false)
      done_ = true;
      return Status::OK();
    }
    if (end <= cur_) {
      rb = ZeroRowBatch(output_, true, true);
    } else {
      rb.num_rows = end - cur_;
      for (int64_t c : idxs_) {
        pxg_column_out o{};
        PXG_CALL(pxg_table_fetch(st_->t, static_cast<int32_t>(c), cur_, end, &o));
        rb.cols.push_back(FromOut(o));
      }
      rb.eow = rb.eos = end >= hi_ && !ms_.streaming;  // an infinite stream never ends its window
    }
    cur_ = end;
    done_ = rb.eos || (ms_.streaming && cur_ >= hi_);
    return SendRowBatchToChildren(s, rb);
  }

 protected:
  Status InitImpl(const planpb::Operator& op) override {
    const planpb::MemorySourceOperator& ms = op.mem_source;
    idxs_ = ms.column_idxs;
    if (idxs_.empty())
      for (size_t c = 0; c < st_->types.size(); ++c) idxs_.push_back(static_cast<int64_t>(c));
    for (int64_t c : idxs_)
      if (c < 0 || c >= static_cast<int64_t>(st_->types.size())) return Err(PXG_INVALID_ARGUMENT, "source column out of range");
    if ((ms.has_start_time || ms.has_stop_time) && st_->time_col < 0)
      return Err(PXG_INVALID_ARGUMENT, "table %s has no time_ column for a time-bounded source", name_.c_str());
    ms_ = ms;
    return Status::OK();
  }

 private:
  Status Range() {
    lo_ = 0;
    hi_ = pxg_table_num_rows(st_->t);
    if (ms_.has_start_time) PXG_CALL(pxg_table_time_bound(st_->t, st_->time_col, ms_.start_time, 0, &lo_));
    if (ms_.has_stop_time) PXG_CALL(pxg_table_time_bound(st_->t, st_->time_col, ms_.stop_time, 1, &hi_));
    if (hi_ < lo_) hi_ = lo_;
    return Status::OK();
  }
  std::string name_;
  const StoredTable* st_;
  planpb::MemorySourceOperator ms_;
  std::vector<int64_t> idxs_;
  int64_t lo_ = 0, hi_ = 0, cur_ = 0;
  bool ranged_ = false, done_ = false;
};

// ---------------------------------------------------------------------------------------
// ExecutionGraph (exec_graph.cc:52-289): nodes in DAG order, the operator switch picks the GPU
// node classes, and a MemorySource -> (Filter | Map)* -> Agg(blocking) chain whose
// intermediates have no other consumer is fused into one GpuAggNode (its intermediate batches
// are unobservable: a blocking agg emits only at eos, agg_node.cc:169-171).
// ---------------------------------------------------------------------------------------
class ExecutionGraph {
 public:
  Status Init(const planpb::PlanFragment& pf, int32_t ntables, const pxc_table* tables, const TableStore* store) {
    store_ = store;
    std::map<uint64_t, const planpb::Operator*> ops;
    for (auto& n : pf.nodes) ops[n.id] = &n.op;
    // Parents / children from the DAG (plan_fragment.cc:108-118); without a DAG the nodes form
    // a chain in listed order.
    std::map<uint64_t, std::vector<uint64_t>> parents, children;
    std::vector<uint64_t> ids;
    if (!pf.dag.empty()) {
      for (auto& d : pf.dag) {
        ids.push_back(d.id);
        parents[d.id] = d.sorted_parents;
        children[d.id] = d.sorted_children;
      }
    } else {
      for (size_t i = 0; i < pf.nodes.size(); ++i) {
        ids.push_back(pf.nodes[i].id);
        if (i) {
          parents[pf.nodes[i].id] = {pf.nodes[i - 1].id};
          children[pf.nodes[i - 1].id] = {pf.nodes[i].id};
        }
      }
    }
    for (uint64_t id : ids)
      if (!ops.count(id)) return Err(PXG_NOT_FOUND, "plan node %llu missing", (unsigned long long)id);
    // Topological order (Kahn, ties in listed order).
    std::vector<uint64_t> order;
    {
      std::map<uint64_t, size_t> indeg;
      for (uint64_t id : ids) indeg[id] = parents[id].size();
      std::vector<uint64_t> ready;
      for (uint64_t id : ids)
        if (indeg[id] == 0) ready.push_back(id);
      for (size_t k = 0; k < ready.size(); ++k) {
        order.push_back(ready[k]);
        for (uint64_t c : children[ready[k]])
          if (indeg.count(c) && --indeg[c] == 0) ready.push_back(c);
      }
      if (order.size() != ids.size()) return Err(PXG_INVALID_ARGUMENT, "plan DAG has a cycle");
    }
    std::map<uint64_t, ExecNode*> built;
    std::set<uint64_t> fused_away;
    for (uint64_t id : order) {
      if (fused_away.count(id)) continue;
      const planpb::Operator& op = *ops[id];
      if (op.which == 2) {
        PXC_RETURN_IF_ERROR(BuildSource(id, op, ntables, tables, ops, parents, children, &built, &fused_away));
        continue;
      }
      if (op.which == 9) {  // GRPCSourceOperator: batches from the caller's transport
        const std::vector<std::pair<const uint8_t*, int64_t>>* msgs = nullptr;
        if (grpc_inputs_) {
          auto it = grpc_inputs_->find(id);
          if (it != grpc_inputs_->end()) msgs = &it->second;
        }
        auto* src = new GrpcSourceNode(id, msgs);
        src->node_id = id;
        src->plan_id = id;
        pool_.emplace_back(src);
        for (int32_t t : op.grpc_source_types)
          if (t < B || t > T) return Err(PXG_INVALID_ARGUMENT, "GRPC source column type %d", t);
        PXC_RETURN_IF_ERROR(src->Init(op, op.grpc_source_types, {}));
        sources_.push_back(src);
        built[id] = src;
        continue;
      }
      const std::vector<uint64_t>& ps = parents[id];
      if (ps.empty()) return Err(PXG_UNIMPLEMENTED, "operator (oneof field %d) without inputs has no device node", op.which);
      std::vector<RowDescriptor> ins;
      for (uint64_t p : ps) {
        if (!built.count(p)) return Err(PXG_INTERNAL, "parent %llu not built", (unsigned long long)p);
        ins.push_back(built[p]->output_descriptor());
      }
      const RowDescriptor& cur = ins[0];
      ExecNode* node = nullptr;
      RowDescriptor out;
      switch (op.which) {
        case 6: {
          node = new GpuFilterNode();
          for (auto& c : op.filter.columns) {
            if (c.index >= cur.size()) return Err(PXG_INVALID_ARGUMENT, "filter column out of range");
            out.push_back(cur[c.index]);
          }
          if (op.filter.columns.empty()) out = cur;
          break;
        }
        case 3: {
          auto* agg = dynamic_cast<GpuAggNode*>(built[ps[0]]);
          if (agg) {
            node = new PostAggMapNode(agg);
            PXC_RETURN_IF_ERROR(PostAggMapNode::OutputTypes(op, cur, &out));
          } else {
            node = new GpuMapNode();
            ExprCompiler comp(ColumnEnv(cur));
            for (auto& e : op.map.expressions) {
              Program p;
              PXC_RETURN_IF_ERROR(comp.Compile(e, &p));
              out.push_back(p.result_type);
            }
          }
          break;
        }
        case 4: {
          node = new GpuAggNode();
          Status st;
          out = AggOutputTypes(op, ColumnEnv(cur), &st);
          PXC_RETURN_IF_ERROR(st);
          break;
        }
        case 7: {
          node = new LimitNode();
          for (auto& c : op.limit.columns) {
            if (c.index >= cur.size()) return Err(PXG_INVALID_ARGUMENT, "limit column out of range");
            out.push_back(cur[c.index]);
          }
          break;
        }
        case 8: {
          if (ins.empty() || op.union_mappings.empty()) return Err(PXG_INVALID_ARGUMENT, "Union needs parents and column mappings");
          node = new UnionNode();
          for (int64_t i : op.union_mappings[0]) {
            if (i < 0 || static_cast<size_t>(i) >= ins[0].size()) return Err(PXG_INVALID_ARGUMENT, "Union column mapping out of range");
            out.push_back(ins[0][static_cast<size_t>(i)]);
          }
          break;
        }
        case 11: {
          if (ins.size() != 2) return Err(PXG_INVALID_ARGUMENT, "Join operator expects a two input relations, got %zu", ins.size());
          node = new GpuEquijoinNode();
          for (auto& o : op.join.output_columns) {
            if (o.first > 1 || o.second >= ins[o.first].size()) return Err(PXG_INVALID_ARGUMENT, "join output column out of range");
            out.push_back(ins[o.first][o.second]);
          }
          break;
        }
        case 1000:
          if (op.grpc_sink_to_source) {
            auto* gs = new GrpcSinkNode(op.grpc_source_id);
            node = gs;
            grpc_sinks_.push_back(gs);
            out = cur;
            break;
          }
          [[fallthrough]];  // a result table sink
        case 5: {
          auto* sk = new SinkNode(op.which == 5 ? op.mem_sink.name : op.grpc_sink_table);
          node = sk;
          sinks_.push_back(sk);
          out = cur;
          break;
        }
        default: return Err(PXG_UNIMPLEMENTED, "operator (oneof field %d) has no device node", op.which);
      }
      pool_.emplace_back(node);
      node->plan_id = id;
      PXC_RETURN_IF_ERROR(node->Init(op, out, ins));
      for (size_t k = 0; k < ps.size(); ++k) built[ps[k]]->AddChild(node, k);
      built[id] = node;
      lowered_.push_back(node);
    }
    if (sources_.empty()) return Err(PXG_UNIMPLEMENTED, "plan must start with a MemorySource or GRPCSource");
    if (sinks_.empty() && grpc_sinks_.empty()) return Err(PXG_INVALID_ARGUMENT, "plan has no sink");
    MarkEagerCoalescing();
    return Status::OK();
  }

  // CoalescingDeviceNode's two eager cases: reachable from a streaming source, or with a
  // LimitNode reachable below it.
  void MarkEagerCoalescing() {
    std::set<ExecNode*> below_stream;
    std::vector<ExecNode*> stack;
    for (auto* src : sources_)
      if (src->IsStreaming()) stack.push_back(src);
    while (!stack.empty()) {
      ExecNode* n = stack.back();
      stack.pop_back();
      if (!below_stream.insert(n).second) continue;
      for (auto& c : n->children()) stack.push_back(c.first);
    }
    std::function<bool(ExecNode*, std::set<ExecNode*>*)> limit_below = [&](ExecNode* n, std::set<ExecNode*>* seen) {
      if (!seen->insert(n).second) return false;
      for (auto& c : n->children())
        if (dynamic_cast<LimitNode*>(c.first) || limit_below(c.first, seen)) return true;
      return false;
    };
    for (auto& up : pool_) {
      auto* cn = dynamic_cast<CoalescingDeviceNode*>(up.get());
      if (!cn) continue;
      std::set<ExecNode*> seen;
      if (below_stream.count(cn) || limit_below(cn, &seen)) cn->set_eager();
    }
  }

  // ExecuteSources (exec_graph.cc:177-289).
  Status Execute(ExecState* s) {
    StageClock clk;
    for (auto& n : pool_) n->stats()->collect = s->collect_exec_stats;
    for (auto& n : pool_) PXC_RETURN_IF_ERROR(n->Prepare(s));
    for (auto& n : pool_) PXC_RETURN_IF_ERROR(n->Open(s));
    clk.Mark("prepare + open");
    // Round-robin over the sources until all are exhausted (exec_graph.cc:177-289).
    Status st;
    for (bool any = true; st.ok() && any;) {
      any = false;
      for (auto* src : sources_) {
        if (!st.ok() || !src->HasBatchesRemaining() || s->stopped_sources.count(src->node_id)) continue;
        any = true;
        st = src->GenerateNext(s);
      }
    }
    clk.Mark("sources drained");
    for (auto& n : pool_) {
      Status c = n->Close(s);
      if (st.ok()) st = c;
    }
    clk.Mark("close");
    return st;
  }

  // ExecutionGraph::GetStats (exec_graph.cc:333-347) plus, per node in plan order, the
  // OperatorExecutionStats fields carnot.cc:386-420 reports under `analyze`, as JSON.
  std::string StatsJson() {
    int64_t bytes = 0, rows = 0;
    for (auto* src : sources_) {
      bytes += src->stats()->bytes_output;
      rows += src->stats()->rows_output;
    }
    std::vector<ExecNode*> nodes;
    for (auto& n : pool_) nodes.push_back(n.get());
    std::stable_sort(nodes.begin(), nodes.end(), [](ExecNode* a, ExecNode* b) { return a->plan_id < b->plan_id; });
    std::ostringstream os;
    auto q = [](const std::string& x) {
      std::string o = "\"";
      for (char c : x) {
        if (c == '"' || c == '\\') o.push_back('\\');
        if (static_cast<unsigned char>(c) >= 0x20) o.push_back(c);
      }
      return o + "\"";
    };
    os << "{\"bytes_processed\":" << bytes << ",\"rows_processed\":" << rows << ",\"nodes\":[";
    for (size_t i = 0; i < nodes.size(); ++i) {
      ExecNodeStats* st = nodes[i]->stats();
      if (st->collect) st->AddExtraMetric("batches_output", static_cast<double>(st->batches_output));
      os << (i ? "," : "") << "{\"node_id\":" << nodes[i]->plan_id << ",\"name\":" << q(nodes[i]->DebugString())
         << ",\"bytes_output\":" << st->bytes_output << ",\"records_output\":" << st->rows_output
         << ",\"batches_output\":" << st->batches_output << ",\"bytes_input\":" << st->bytes_input
         << ",\"records_input\":" << st->rows_input << ",\"batches_input\":" << st->batches_input
         << ",\"total_execution_time_ns\":" << st->total_ns << ",\"self_execution_time_ns\":" << (st->total_ns - st->children_ns);
      if (auto* a = dynamic_cast<GpuAggNode*>(nodes[i])) {
        os << ",\"fused_node_ids\":[";
        for (size_t k = 0; k < a->fused_ids.size(); ++k) os << (k ? "," : "") << a->fused_ids[k];
        os << "]";
      }
      os << ",\"extra_metrics\":{";
      size_t k = 0;
      for (auto& kv : st->extra_metrics) os << (k++ ? "," : "") << q(kv.first) << ":" << kv.second;
      os << "},\"extra_info\":{";
      k = 0;
      for (auto& kv : st->extra_info) os << (k++ ? "," : "") << q(kv.first) << ":" << q(kv.second);
      os << "}}";
    }
    os << "]}";
    return os.str();
  }

  std::string Explain() const {
    std::ostringstream os;
    for (auto* src : sources_) os << src->DebugString() << "\n";
    for (auto* n : lowered_) {
      os << "  -> " << n->DebugString() << " out=[";
      for (size_t i = 0; i < n->output_descriptor().size(); ++i) os << (i ? "," : "") << TypeName(n->output_descriptor()[i]);
      os << "]\n";
      if (auto* a = dynamic_cast<const GpuAggNode*>(n)) {
        if (a->has_filter) os << "     filter: " << ProgString(a->filter) << "\n";
        for (auto& k : a->keys) os << "     key: " << ProgString(k) << "\n";
        for (auto& u : a->udas) os << "     uda kind=" << u.kind << " arg=" << (u.has_arg ? ProgString(u.arg) : "-") << "\n";
      }
    }
    return os.str();
  }

  // The first aggregation node of the lowered graph (fused or not), or null.
  GpuAggNode* FirstAgg() const {
    for (auto* n : lowered_)
      if (auto* a = dynamic_cast<GpuAggNode*>(n)) return a;
    return nullptr;
  }

  std::vector<SinkNode*> sinks_;
  std::vector<GrpcSinkNode*> grpc_sinks_;
  // GRPCSource node id -> its RowBatchData messages in arrival order (set before Init).
  const std::map<uint64_t, std::vector<std::pair<const uint8_t*, int64_t>>>* grpc_inputs_ = nullptr;

 private:
  static std::string ProgString(const Program& p) {
    std::ostringstream os;
    for (size_t i = 0; i < p.insns.size(); ++i)
      os << (i ? " " : "") << p.insns[i].op << ":" << p.insns[i].type << ":" << p.insns[i].arg << ":" << p.insns[i].imm;
    return os.str();
  }
  // AggregateOperator output relation: groups, then values (agg_node.cc:336-346).
  static RowDescriptor AggOutputTypes(const planpb::Operator& op, const std::vector<Program>& env, Status* st) {
    RowDescriptor out;
    *st = Status::OK();
    for (auto& g : op.agg.groups) {
      if (g.index >= env.size()) {
        *st = Err(PXG_INVALID_ARGUMENT, "group column out of range");
        return out;
      }
      out.push_back(env[g.index].result_type);
    }
    if (op.agg.partial_agg && !op.agg.finalize_results) {  // operators.cc:251-257
      out.push_back(S);
      return out;
    }
    const bool merge = !op.agg.partial_agg && op.agg.finalize_results;
    for (auto& v : op.agg.values) {
      std::vector<int32_t> types;
      for (auto& ia : v.init_args) types.push_back(ia.data_type);
      if (merge) types.insert(types.end(), v.args_data_types.begin(), v.args_data_types.end());
      for (auto& a : v.args) {
        if (merge) break;
        if (a.is_column) {
          if (a.column.index >= env.size()) {
            *st = Err(PXG_INVALID_ARGUMENT, "aggregate argument column out of range");
            return out;
          }
          types.push_back(env[a.column.index].result_type);
        } else {
          types.push_back(a.constant.data_type);
        }
      }
      auto* d = GetRegistry().GetUDA(v.name, types);
      if (!d) {
        *st = Err(PXG_NOT_FOUND, "no device UDA %s", Signature(v.name, types).c_str());
        return out;
      }
      out.push_back(std::get<2>(*d));
    }
    return out;
  }

  // A MemorySource, and the fused GpuAggNode when a chain of single-consumer Filter / Map
  // nodes below it ends in a blocking Agg (the chain's intermediate batches are unobservable:
  // a blocking agg emits only at eos, agg_node.cc:169-171).
  Status BuildSource(uint64_t id, const planpb::Operator& op, int32_t ntables, const pxc_table* tables,
                     std::map<uint64_t, const planpb::Operator*>& ops, std::map<uint64_t, std::vector<uint64_t>>& parents,
                     std::map<uint64_t, std::vector<uint64_t>>& children, std::map<uint64_t, ExecNode*>* built,
                     std::set<uint64_t>* fused_away) {
    const planpb::MemorySourceOperator& ms = op.mem_source;
    const pxc_table* tab = nullptr;
    for (int32_t t = 0; t < ntables; ++t)
      if (ms.name == tables[t].name) tab = &tables[t];
    const StoredTable* stored = nullptr;
    if (!tab && store_) {
      auto it = store_->find(ms.name);
      if (it != store_->end()) stored = &it->second;
    }
    if (!tab && !stored) return Err(PXG_NOT_FOUND, "Table '%s' not found", ms.name.c_str());
    const int32_t ncols = tab ? tab->ncols : static_cast<int32_t>(stored->types.size());
    auto type_of = [&](int64_t c) { return tab ? tab->col_types[c] : stored->types[static_cast<size_t>(c)]; };
    RowDescriptor src_types;
    std::vector<int64_t> idxs = ms.column_idxs;
    if (idxs.empty())
      for (int32_t c = 0; c < ncols; ++c) idxs.push_back(c);
    for (int64_t c : idxs) {
      if (c < 0 || c >= ncols) return Err(PXG_INVALID_ARGUMENT, "source column out of range");
      src_types.push_back(type_of(c));
    }
    SourceNode* src;
    DeviceSourceNode* dsrc = nullptr;
    if (tab) {
      src = new MemorySourceNode(tab);
    } else {
      dsrc = new DeviceSourceNode(ms.name, stored);
      src = dsrc;
    }
    src->node_id = id;
    src->plan_id = id;
    pool_.emplace_back(src);
    PXC_RETURN_IF_ERROR(src->Init(op, src_types, {}));
    sources_.push_back(src);
    (*built)[id] = src;
    // An infinite stream never reaches eos, so a blocking agg below it never emits: it is not
    // fused (the source's batches go through the ordinary nodes).
    if (ms.streaming) return Status::OK();

    std::vector<uint64_t> chain;
    uint64_t agg_id = 0;
    bool found = false;
    for (uint64_t cur = id; children[cur].size() == 1;) {
      const uint64_t c = children[cur][0];
      if (parents[c].size() != 1) break;
      const planpb::Operator& cop = *ops[c];
      if (cop.which == 4) {
        if (!cop.agg.windowed) {
          agg_id = c;
          found = true;
        }
        break;
      }
      if (cop.which != 3 && cop.which != 6) break;
      chain.push_back(c);
      cur = c;
    }
    if (!found) return Status::OK();
    // Substitute the chain into programs over the source columns (for a stored table, over
    // the table's own columns: the agg then reads the device table in place).
    std::vector<Program> env = ColumnEnv(src_types);
    if (dsrc)
      for (size_t j = 0; j < env.size(); ++j) env[j].insns[0].arg = static_cast<int32_t>(idxs[j]);
    bool has_filter = false;
    Program filter;
    for (uint64_t cid : chain) {
      const planpb::Operator& cop = *ops[cid];
      ExprCompiler comp(env);
      if (cop.which == 6) {
        Program p;
        PXC_RETURN_IF_ERROR(comp.Compile(cop.filter.expression, &p));
        if (p.result_type != B) return Err(PXG_INVALID_ARGUMENT, "Predicate expression must be a boolean");
        if (!has_filter) {
          filter = p;
        } else {
          AppendProgram(p, &filter);
          filter.insns.push_back(Insn(PXG_OP_AND, B));
        }
        has_filter = true;
        std::vector<Program> ne;
        for (auto& c : cop.filter.columns) {
          if (c.index >= env.size()) return Err(PXG_INVALID_ARGUMENT, "filter column out of range");
          ne.push_back(env[c.index]);
        }
        if (!cop.filter.columns.empty()) env = ne;
      } else {
        std::vector<Program> ne(cop.map.expressions.size());
        for (size_t e = 0; e < ne.size(); ++e) PXC_RETURN_IF_ERROR(comp.Compile(cop.map.expressions[e], &ne[e]));
        env = ne;
      }
    }
    auto* agg = new GpuAggNode();
    pool_.emplace_back(agg);
    agg->plan_id = agg_id;
    for (uint64_t cid : chain) agg->fused_ids.push_back(cid);
    agg->env = env;
    agg->has_filter = has_filter;
    agg->filter = filter;
    agg->fused_ = !chain.empty();
    agg->source_types = src_types;
    agg->device_input = dsrc != nullptr;
    agg->hint_source = ms.name;
    RowDescriptor env_types;
    for (auto& p : env) env_types.push_back(p.result_type);
    Status out_ok;
    const RowDescriptor out = AggOutputTypes(*ops[agg_id], env, &out_ok);
    PXC_RETURN_IF_ERROR(out_ok);
    PXC_RETURN_IF_ERROR(agg->Init(*ops[agg_id], out, {env_types}));
    src->AddChild(agg, 0);
    if (dsrc) dsrc->fused_agg = agg;
    (*built)[agg_id] = agg;
    for (uint64_t cid : chain) fused_away->insert(cid);
    fused_away->insert(agg_id);
    lowered_.push_back(agg);
    return Status::OK();
  }

  std::vector<std::unique_ptr<ExecNode>> pool_;
  std::vector<ExecNode*> lowered_;
  std::vector<SourceNode*> sources_;
  const TableStore* store_ = nullptr;
};

// PXRB serialisation of the sinks (layout of tests/oracle_client.py::parse_pxrb).  The buffer
// is malloc'ed, sized up front and handed to the caller as is (pxc_free), so a result is
// written once: no growth copies and no second copy-out.
// PXRB STRING offsets relative to the column's first offset.
static void RebaseOffsets(uint8_t* dst, const int32_t* src, size_t count, int32_t o0) {
  if (o0 == 0) {
    std::memcpy(dst, src, 4 * count);
    return;
  }
  for (size_t i = 0; i < count; ++i) {
    const int32_t v = src[i] - o0;
    std::memcpy(dst + 4 * i, &v, 4);
  }
}

struct Writer {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  ~Writer() { pxg_host_free(p); }
  // Buffers come from libpxg's host pool (pinned, reused across queries: a 5 MB result written
  // into fresh malloc pages paid ~0.3 ms of page faults per query); released with pxc_free.
  void reserve(size_t c) {
    if (c <= cap) return;
    uint8_t* q = static_cast<uint8_t*>(pxg_host_alloc(static_cast<int64_t>(c)));
    if (!q) throw std::bad_alloc();
    if (n) std::memcpy(q, p, n);
    pxg_host_free(p);
    p = q;
    cap = c;
  }
  uint8_t* claim(size_t k) {
    if (n + k > cap) reserve(std::max(cap * 2, n + k + 4096));
    uint8_t* at = p + n;
    n += k;
    return at;
  }
  template <typename V>
  void put(V v) {
    std::memcpy(claim(sizeof(V)), &v, sizeof(V));
  }
  void bytes(const void* src, size_t k) {
    if (k) std::memcpy(claim(k), src, k);
  }
  void offsets(const int32_t* src, size_t count, int32_t o0) { RebaseOffsets(claim(4 * count), src, count, o0); }
  uint8_t* release(int64_t* len) {
    *len = static_cast<int64_t>(n);
    if (!p) p = static_cast<uint8_t*>(pxg_host_alloc(1));
    uint8_t* r = p;
    p = nullptr;
    n = cap = 0;
    return r;
  }
};

// Bytes WriteBatch will append for rb.
static size_t BatchBytes(const RowBatch& rb) {
  const size_t n = static_cast<size_t>(rb.num_rows);
  size_t b = 8 + 4 + 4;
  for (auto& c : rb.cols) {
    b += 4;
    switch (c.type) {
      case B: b += n; break;
      case U: b += n * 16; break;
      case S: b += 4 * (n + 1) + (n ? static_cast<size_t>(c.offsets[n] - c.offsets[0]) : 0); break;
      default: b += n * 8; break;
    }
  }
  return b;
}

// Writes the small header fields at once and records every column copy as a task, so the bulk
// of a result is copied by several threads (a single 64K-group batch included).
struct CopyTask {
  uint8_t* dst;
  const void* src;
  size_t bytes;  // bytes to write
  int32_t o0;    // offsets task: the first offset (src is int32_t[])
  bool offs;
};
struct TaskWriter {
  uint8_t* p;
  std::vector<CopyTask>* tasks;
  uint8_t* claim(size_t k) {
    uint8_t* at = p;
    p += k;
    return at;
  }
  template <typename V>
  void put(V v) {
    std::memcpy(claim(sizeof(V)), &v, sizeof(V));
  }
  void bytes(const void* src, size_t k) {
    if (k) tasks->push_back({claim(k), src, k, 0, false});
  }
  void offsets(const int32_t* src, size_t count, int32_t o0) { tasks->push_back({claim(4 * count), src, 4 * count, o0, true}); }
};

// Writes at a fixed position of a buffer sized up front (the parallel PXRB pass).
struct SpanWriter {
  uint8_t* p;
  uint8_t* claim(size_t k) {
    uint8_t* at = p;
    p += k;
    return at;
  }
  template <typename V>
  void put(V v) {
    std::memcpy(claim(sizeof(V)), &v, sizeof(V));
  }
  void bytes(const void* src, size_t k) {
    if (k) std::memcpy(claim(k), src, k);
  }
  void offsets(const int32_t* src, size_t count, int32_t o0) { RebaseOffsets(claim(4 * count), src, count, o0); }
};

// Persistent copy workers for the PXRB pass: a result of a few MB (C2: 4.8 MB, 0.12 ms on one
// thread) is split over threads that already exist, since starting threads per query cost more
// than the copy.  Run(n, fn) calls fn(i) for i in [0, n) on the workers and the caller.
class CopyPool {
 public:
  static CopyPool& Get() {
    // Never destroyed (workers may outlive static teardown); a forked child, which has none of
    // the parent's threads, makes its own.
    static CopyPool* p = nullptr;
    static pid_t owner = 0;
    static std::mutex m;
    std::lock_guard<std::mutex> lk(m);
    if (!p || owner != getpid()) {
      p = new CopyPool();
      owner = getpid();
    }
    return *p;
  }
  size_t workers() const { return th_.size(); }
  void Run(size_t n, const std::function<void(size_t)>& fn) {
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &fn;
    n_ = n;
    next_.store(0);
    active_ = th_.size();
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    Work(fn, n);
    lk.lock();
    done_cv_.wait(lk, [&] { return active_ == 0; });
    job_ = nullptr;
  }

 private:
  CopyPool() {
    const size_t k = std::min<size_t>(7, std::max(1u, std::thread::hardware_concurrency()) - 1);
    for (size_t i = 0; i < k; ++i)
      th_.emplace_back([this] {
        uint64_t seen = 0;
        for (;;) {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return gen_ != seen; });
          seen = gen_;
          const std::function<void(size_t)>* fn = job_;
          const size_t n = n_;
          lk.unlock();
          if (fn) Work(*fn, n);
          lk.lock();
          if (--active_ == 0) done_cv_.notify_all();
        }
      });
    for (auto& t : th_) t.detach();
  }
  void Work(const std::function<void(size_t)>& fn, size_t n) {
    for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) fn(i);
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t n_ = 0, active_ = 0;
  uint64_t gen_ = 0;
  std::atomic<size_t> next_{0};
};

template <typename W>
static void WriteBatch(W* w, const RowBatch& rb) {
  w->template put<int64_t>(rb.num_rows);
  w->template put<uint8_t>(rb.eow);
  w->template put<uint8_t>(rb.eos);
  w->template put<uint16_t>(0);
  w->template put<uint32_t>(static_cast<uint32_t>(rb.cols.size()));
  const size_t n = static_cast<size_t>(rb.num_rows);
  for (auto& c : rb.cols) {
    w->template put<int32_t>(c.type);
    switch (c.type) {
      case B: w->bytes(c.values, n); break;
      case U: w->bytes(c.values, n * 16); break;
      case S: {
        const int32_t o0 = n ? c.offsets[0] : 0;
        if (!n) {
          w->template put<int32_t>(0);
        } else {
          w->offsets(c.offsets, n + 1, o0);
        }
        if (n) w->bytes(c.data + o0, static_cast<size_t>(c.offsets[n] - o0));
        break;
      }
      default: w->bytes(c.values, n * 8); break;
    }
  }
}

}  // namespace pxc

using namespace pxc;

struct pxc_engine {
  // One engine serves concurrent callers one call at a time: the store, the group-count hints,
  // the aggregation cache and the ctx stream are shared by every query on it.
  std::mutex mu;
  pxg_ctx* ctx = nullptr;
  TableStore store;
  std::map<std::string, int64_t> group_hints;
  std::multimap<std::string, pxg_agg*> agg_cache;
  bool analyze = false;    // collect per-node timers / extras (pxc_engine_set_analyze)
  std::string last_stats;  // the last query's execution stats (pxc_engine_last_stats)
};

static int32_t Fail(const Status& s) {
  g_last_error = s.msg;
  return s.code;
}

extern "C" const char* pxc_last_error(void) { return g_last_error.c_str(); }
extern "C" void pxc_free(void* p) { pxg_host_free(p); }

// QuantilesUDA::Finalize's JSON for n groups of 7 doubles (json_double.h), as one malloc'ed
// buffer of n NUL-terminated strings (released with pxc_free).
extern "C" int32_t pxc_quantiles_json(const double* q7, int64_t n, char** out, int64_t* out_len) {
  if ((!q7 && n > 0) || n < 0 || !out || !out_len) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::string s;
  for (int64_t g = 0; g < n; ++g) {
    pxjson::AppendQuantilesJson(q7 + g * 7, &s);
    s.push_back('\0');
  }
  *out_len = static_cast<int64_t>(s.size());
  *out = static_cast<char*>(std::malloc(std::max<size_t>(s.size(), 1)));
  if (!s.empty()) std::memcpy(*out, s.data(), s.size());
  return PXG_OK;
}

extern "C" int32_t pxc_engine_create(int32_t device, pxc_engine** out) {
  if (!out) return Fail(Err(PXG_INVALID_ARGUMENT, "out is null"));
  auto* e = new pxc_engine();
  const int32_t c = pxg_ctx_create(device, &e->ctx);
  if (c != PXG_OK) {
    delete e;
    return Fail(FromPxg(c));
  }
  *out = e;
  return PXG_OK;
}

extern "C" int32_t pxc_engine_destroy(pxc_engine* e) {
  if (!e) return PXG_OK;
  for (auto& kv : e->agg_cache) pxg_agg_destroy(kv.second);
  e->agg_cache.clear();
  for (auto& kv : e->store) pxg_table_destroy(kv.second.t);
  e->store.clear();
  pxg_ctx_destroy(e->ctx);
  delete e;
  return PXG_OK;
}

using GrpcInputs = std::map<uint64_t, std::vector<std::pair<const uint8_t*, int64_t>>>;

static Status Lower(const uint8_t* plan, int64_t plan_len, int32_t ntables, const pxc_table* tables, const TableStore* store,
                    ExecutionGraph* g, const GrpcInputs* grpc_inputs = nullptr) {
  g->grpc_inputs_ = grpc_inputs;
  if (!plan || plan_len < 0) return Err(PXG_INVALID_ARGUMENT, "no plan");
  planpb::Plan p;
  try {
    p = planpb::DecodePlan(plan, static_cast<size_t>(plan_len));
  } catch (const planpb::WireError& e) {
    return Err(PXG_INVALID_ARGUMENT, "%s", e.what());
  }
  if (p.fragments.empty()) return Err(PXG_INVALID_ARGUMENT, "plan has no fragments");
  return g->Init(p.fragments[0], ntables, tables, store);
}

static int32_t Explain(const uint8_t* plan, int64_t plan_len, int32_t ntables, const pxc_table* tables, const TableStore* store,
                       char** out) {
  if (!out) return Fail(Err(PXG_INVALID_ARGUMENT, "out is null"));
  ExecutionGraph g;
  Status s = Lower(plan, plan_len, ntables, tables, store, &g);
  if (!s.ok()) return Fail(s);
  const std::string txt = g.Explain();
  *out = static_cast<char*>(std::malloc(txt.size() + 1));
  std::memcpy(*out, txt.c_str(), txt.size() + 1);
  return PXG_OK;
}

extern "C" int32_t pxc_explain_plan(const uint8_t* plan, int64_t plan_len, int32_t ntables, const pxc_table* tables, char** out) {
  return Explain(plan, plan_len, ntables, tables, nullptr, out);
}

extern "C" int32_t pxc_engine_explain_plan(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables,
                                           const pxc_table* tables, char** out) {
  if (!engine) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::lock_guard<std::mutex> lock(engine->mu);
  return Explain(plan, plan_len, ntables, tables, &engine->store, out);
}

// ---------------------------------------------------------------------------------------
// Table store ABI (TableStore::AddTable, Table::TransferRecordBatch, table.cc:174-200).
// ---------------------------------------------------------------------------------------
extern "C" int32_t pxc_store_create_table(pxc_engine* e, const char* name, int32_t ncols, const int32_t* types,
                                          const char* const* names) {
  if (!e || !name || ncols <= 0 || !types) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::lock_guard<std::mutex> lock(e->mu);
  if (e->store.count(name)) return Fail(Err(PXG_ALREADY_EXISTS, "table %s already exists", name));
  StoredTable st;
  for (int32_t c = 0; c < ncols; ++c) {
    st.types.push_back(types[c]);
    st.names.push_back(names && names[c] ? names[c] : "");
    if (st.names.back() == "time_") {
      if (types[c] != PXG_TIME64NS && types[c] != PXG_INT64) return Fail(Err(PXG_INVALID_ARGUMENT, "time_ must be TIME64NS"));
      st.time_col = c;
    }
  }
  const int32_t rc = pxg_table_create(e->ctx, ncols, types, &st.t);
  if (rc != PXG_OK) return Fail(FromPxg(rc));
  e->store.emplace(name, std::move(st));
  return PXG_OK;
}

extern "C" int32_t pxc_store_append(pxc_engine* e, const char* name, const pxg_column_view* cols, int64_t nrows) {
  if (!e || !name || (!cols && nrows > 0) || nrows < 0) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::lock_guard<std::mutex> lock(e->mu);
  auto it = e->store.find(name);
  if (it == e->store.end()) return Fail(Err(PXG_NOT_FOUND, "Table '%s' not found", name));
  StoredTable& st = it->second;
  if (nrows == 0) return PXG_OK;
  for (size_t c = 0; c < st.types.size(); ++c)
    if (cols[c].type != st.types[c] || cols[c].length != nrows)
      return Fail(Err(PXG_INVALID_ARGUMENT, "column %zu does not match the table's relation", c));
  if (st.time_col >= 0) {  // time order (the hot store's append order, table.cc:174-200)
    const int64_t* t = static_cast<const int64_t*>(cols[st.time_col].values);
    int64_t prev = st.last_time;
    for (int64_t r = 0; r < nrows; ++r) {
      if (t[r] < prev) return Fail(Err(PXG_INVALID_ARGUMENT, "time_ goes backwards at row %lld of the appended batch", (long long)r));
      prev = t[r];
    }
    st.last_time = prev;
  }
  const int32_t rc = pxg_table_append(st.t, cols, nrows);
  return rc == PXG_OK ? PXG_OK : Fail(FromPxg(rc));
}

extern "C" int32_t pxc_store_drop_table(pxc_engine* e, const char* name) {
  if (!e || !name) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::lock_guard<std::mutex> lock(e->mu);
  auto it = e->store.find(name);
  if (it == e->store.end()) return Fail(Err(PXG_NOT_FOUND, "Table '%s' not found", name));
  pxg_table_destroy(it->second.t);
  e->store.erase(it);
  return PXG_OK;
}

extern "C" int64_t pxc_store_num_rows(pxc_engine* e, const char* name) {
  if (!e || !name) return -1;
  std::lock_guard<std::mutex> lock(e->mu);
  auto it = e->store.find(name);
  if (it == e->store.end()) return -1;
  if (pxg_table_flush(it->second.t) != PXG_OK) return -1;
  return pxg_table_num_rows(it->second.t);
}

extern "C" pxg_ctx* pxc_engine_ctx(pxc_engine* e) { return e ? e->ctx : nullptr; }

extern "C" int32_t pxc_engine_set_analyze(pxc_engine* e, int32_t on) {
  if (!e) return Fail(Err(PXG_INVALID_ARGUMENT, "engine is null"));
  std::lock_guard<std::mutex> lock(e->mu);
  e->analyze = on != 0;
  return PXG_OK;
}

extern "C" int32_t pxc_engine_last_stats(pxc_engine* e, char** out, int64_t* out_len) {
  if (!e || !out || !out_len) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::lock_guard<std::mutex> lock(e->mu);
  char* p = static_cast<char*>(std::malloc(e->last_stats.size() + 1));
  std::memcpy(p, e->last_stats.c_str(), e->last_stats.size() + 1);
  *out = p;
  *out_len = static_cast<int64_t>(e->last_stats.size());
  return PXG_OK;
}

extern "C" pxg_table* pxc_store_device_table(pxc_engine* e, const char* name) {
  if (!e || !name) return nullptr;
  auto it = e->store.find(name);
  return it == e->store.end() ? nullptr : it->second.t;
}

static uint8_t* CopyOut(const std::vector<uint8_t>& b) {
  uint8_t* p = static_cast<uint8_t*>(std::malloc(std::max<size_t>(b.size(), 1)));
  if (!b.empty()) std::memcpy(p, b.data(), b.size());
  return p;
}

static int32_t ExecuteImpl(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables, const pxc_table* tables,
                           const GrpcInputs* grpc_inputs, uint8_t** out, int64_t* out_len, uint8_t** grpc_out,
                           int64_t* grpc_out_len) {
  if (!engine || !out || !out_len) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  std::lock_guard<std::mutex> lock(engine->mu);
  StageClock clk;
  ExecutionGraph g;
  Status s = Lower(plan, plan_len, ntables, tables, &engine->store, &g, grpc_inputs);
  if (!s.ok()) return Fail(s);
  if (!grpc_out && !g.grpc_sinks_.empty()) return Fail(Err(PXG_INVALID_ARGUMENT, "plan has GRPC sinks: use pxc_execute_plan_grpc"));
  clk.Mark("lower");
  ExecState st;
  st.ctx = engine->ctx;
  st.group_hints = &engine->group_hints;
  st.agg_cache = &engine->agg_cache;
  st.collect_exec_stats = engine->analyze;
  s = g.Execute(&st);
  engine->last_stats = g.StatsJson();
  if (!s.ok()) return Fail(s);
  clk.Mark("execute (total)");
  Writer w;
  size_t total = 8;
  size_t host_bytes = 0;  // bytes the host writes (device result images come by DMA)
  for (auto* sk : g.sinks_) {
    total += 8 + sk->name.size();
    for (auto& rb : sk->batches) {
      const size_t b = rb.image ? static_cast<size_t>(rb.image_bytes) : BatchBytes(rb);
      total += b;
      if (!rb.image) host_bytes += b;
    }
  }
  w.reserve(total);
  w.put<uint32_t>(0x42525850u);  // "PXRB"
  w.put<uint32_t>(static_cast<uint32_t>(g.sinks_.size()));
  // Large results are copied by up to 16 threads, one per 8 MB (a single thread copied C5's
  // 195 MB result at ~15 GB/s, 8 threads at ~65 GB/s; threads pay from ~32 MB, C2's 4.8 MB took
  // 0.12 ms on one thread and 0.23 with four).  Many batches (C5: 2634): each thread writes a contiguous range of whole batches.
  // Few large batches: the headers are written first and every column copy becomes ~1 MB
  // pieces shared by the threads.
  struct Job {
    const RowBatch* rb;
    size_t at;
  };
  std::vector<Job> jobs;
  struct ImageJob {
    pxg_pxrb* img;
    size_t at;
  };
  std::vector<ImageJob> images;
  for (auto* sk : g.sinks_) {
    w.put<uint32_t>(static_cast<uint32_t>(sk->name.size()));
    w.bytes(sk->name.data(), sk->name.size());
    size_t nb = 0;
    for (auto& rb : sk->batches) nb += rb.image ? static_cast<size_t>(rb.image_batches) : 1;
    w.put<uint32_t>(static_cast<uint32_t>(nb));
    for (auto& rb : sk->batches) {
      if (rb.image) {
        images.push_back({rb.image.get(), w.n});
        w.claim(static_cast<size_t>(rb.image_bytes));
        continue;
      }
      jobs.push_back({&rb, w.n});
      w.claim(BatchBytes(rb));
    }
  }
  // The images' DMAs run while the host writes the other batches.
  int32_t image_rc = PXG_OK;
  std::thread image_copy;
  if (!images.empty())
    image_copy = std::thread([&] {
      for (auto& im : images)
        if (image_rc == PXG_OK) image_rc = pxg_pxrb_copy(im.img, w.p + im.at);
    });
  // Up to ~1 MB: one thread.  Larger: the persistent copy workers (CopyPool), by contiguous
  // ranges of whole batches when there are many, else by ~256 KB pieces of the column copies.
  CopyPool& pool = CopyPool::Get();
  const size_t nthreads = host_bytes < (size_t(1) << 20) ? 1 : pool.workers() + 1;
  if (nthreads <= 1) {
    for (auto& j : jobs) {
      SpanWriter sw{w.p + j.at};
      WriteBatch(&sw, *j.rb);
    }
  } else if (jobs.size() >= 4 * nthreads) {
    const size_t nr = 4 * nthreads;  // contiguous ranges of ~equal bytes
    std::vector<size_t> cut(1, 0);
    for (size_t k = 0; k < nr && cut.back() < jobs.size(); ++k) {
      const size_t j0 = cut.back();
      const size_t goal = jobs[j0].at + (w.n - jobs[j0].at) / (nr - k);
      size_t j1 = j0 + 1;
      while (j1 < jobs.size() && jobs[j1].at < goal) ++j1;
      cut.push_back(j1);
    }
    pool.Run(cut.size() - 1, [&](size_t r) {
      for (size_t j = cut[r]; j < cut[r + 1]; ++j) {
        SpanWriter sw{w.p + jobs[j].at};
        WriteBatch(&sw, *jobs[j].rb);
      }
    });
  } else {
    std::vector<CopyTask> tasks;
    for (auto& j : jobs) {
      TaskWriter tw{w.p + j.at, &tasks};
      WriteBatch(&tw, *j.rb);
    }
    constexpr size_t kPiece = size_t(1) << 18;
    std::vector<CopyTask> pieces;
    for (const CopyTask& t : tasks) {
      for (size_t at = 0; at < t.bytes; at += kPiece) {
        const size_t len = std::min(kPiece, t.bytes - at);
        if (t.offs) pieces.push_back({t.dst + at, static_cast<const int32_t*>(t.src) + at / 4, len, t.o0, true});
        else pieces.push_back({t.dst + at, static_cast<const uint8_t*>(t.src) + at, len, 0, false});
      }
    }
    pool.Run(pieces.size(), [&](size_t i) {
      const CopyTask& t = pieces[i];
      if (t.offs) RebaseOffsets(t.dst, static_cast<const int32_t*>(t.src), t.bytes / 4, t.o0);
      else std::memcpy(t.dst, t.src, t.bytes);
    });
  }
  if (image_copy.joinable()) image_copy.join();
  if (image_rc != PXG_OK) return Fail(FromPxg(image_rc));
  *out = w.release(out_len);
  if (grpc_out) {  // "PXGS": per GRPC sink, its destination source id and RowBatchData messages
    Writer gw;
    gw.put<uint32_t>(0x53475850u);
    gw.put<uint32_t>(static_cast<uint32_t>(g.grpc_sinks_.size()));
    for (auto* gs : g.grpc_sinks_) {
      gw.put<uint64_t>(gs->dest_id);
      gw.put<uint32_t>(static_cast<uint32_t>(gs->messages.size()));
      for (auto& m : gs->messages) {
        gw.put<uint32_t>(static_cast<uint32_t>(m.size()));
        gw.bytes(m.data(), m.size());
      }
    }
    *grpc_out = gw.release(grpc_out_len);
  }
  clk.Mark("PXRB serialise");
  return PXG_OK;
}

extern "C" int32_t pxc_execute_plan(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables,
                                    const pxc_table* tables, uint8_t** out, int64_t* out_len) {
  return ExecuteImpl(engine, plan, plan_len, ntables, tables, nullptr, out, out_len, nullptr, nullptr);
}

extern "C" int32_t pxc_execute_plan_grpc(pxc_engine* engine, const uint8_t* plan, int64_t plan_len, int32_t ntables,
                                         const pxc_table* tables, int32_t ninputs, const pxc_grpc_input* inputs, uint8_t** out,
                                         int64_t* out_len, uint8_t** grpc_out, int64_t* grpc_out_len) {
  if (!grpc_out || !grpc_out_len || (ninputs > 0 && !inputs)) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  GrpcInputs in;
  for (int32_t i = 0; i < ninputs; ++i) {
    auto& v = in[inputs[i].grpc_source_id];
    for (int32_t m = 0; m < inputs[i].nmessages; ++m) v.push_back({inputs[i].messages[m], inputs[i].lengths[m]});
  }
  return ExecuteImpl(engine, plan, plan_len, ntables, tables, &in, out, out_len, grpc_out, grpc_out_len);
}

// The drop-in lowering of a plan's (fused) aggregation as a pxg_agg over a device table of the
// given column types: the same ExecutionGraph lowering pxc_execute_plan runs (the MemorySource
// is treated as a stored device table, so programs reference the table's own columns).  Lets a
// caller drive pxg_agg_consume / pxg_agg_finalize on an HBM-resident table directly.
extern "C" int32_t pxc_plan_create_agg(pxg_ctx* ctx, const uint8_t* plan, int64_t plan_len, const char* table_name,
                                       int32_t ncols, const int32_t* types, int64_t expected_groups, pxg_agg** out,
                                       int32_t* n_keys, int32_t* n_udas, int32_t* uda_kinds) {
  if (!ctx || !table_name || ncols <= 0 || !types || !out || !n_keys || !n_udas || !uda_kinds)
    return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  TableStore store;
  StoredTable st;
  st.types.assign(types, types + ncols);
  st.names.assign(static_cast<size_t>(ncols), "");
  store.emplace(table_name, std::move(st));
  ExecutionGraph g;
  Status s = Lower(plan, plan_len, 0, nullptr, &store, &g);
  if (!s.ok()) return Fail(s);
  GpuAggNode* a = g.FirstAgg();
  if (!a) return Fail(Err(PXG_INVALID_ARGUMENT, "plan has no aggregate"));
  if (a->udas.size() > 16) return Fail(Err(PXG_UNIMPLEMENTED, "more than 16 UDAs"));
  s = a->CreateDeviceAgg(ctx, expected_groups, out);
  if (!s.ok()) return Fail(s);
  *n_keys = static_cast<int32_t>(a->keys.size());
  *n_udas = static_cast<int32_t>(a->udas.size());
  for (size_t u = 0; u < a->udas.size(); ++u) uda_kinds[u] = a->udas[u].kind;
  return PXG_OK;
}

extern "C" int32_t pxc_rowbatch_to_proto(int32_t ncols, const pxg_column_view* cols, int64_t nrows, int32_t eow, int32_t eos,
                                         uint8_t** out, int64_t* out_len) {
  if ((ncols > 0 && !cols) || !out || !out_len || nrows < 0) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  RowBatch rb;
  rb.num_rows = nrows;
  for (int32_t c = 0; c < ncols; ++c) {
    HostColumn hc;
    hc.type = cols[c].type;
    hc.length = cols[c].length;
    hc.values = cols[c].values;
    hc.offsets = cols[c].offsets;
    hc.data = cols[c].data;
    if (PbFieldOfType(hc.type) == 0) return Fail(Err(PXG_INVALID_ARGUMENT, "column %d has type %d", c, hc.type));
    if (hc.length != nrows) return Fail(Err(PXG_INVALID_ARGUMENT, "column %d has %lld rows, batch %lld", c, (long long)hc.length, (long long)nrows));
    rb.cols.push_back(hc);
  }
  const std::string m = EncodeRowBatchData(rb, 0, nrows, eow != 0, eos != 0);
  *out_len = static_cast<int64_t>(m.size());
  *out = CopyOut(std::vector<uint8_t>(m.begin(), m.end()));
  return PXG_OK;
}

extern "C" int32_t pxc_rowbatch_from_proto(const uint8_t* msg, int64_t len, uint8_t** out, int64_t* out_len) {
  if ((!msg && len > 0) || len < 0 || !out || !out_len) return Fail(Err(PXG_INVALID_ARGUMENT, "bad arguments"));
  RowBatch rb;
  Status s = DecodeRowBatchData(msg, static_cast<size_t>(len), &rb);
  if (!s.ok()) return Fail(s);
  Writer w;
  w.put<uint32_t>(0x42525850u);
  w.put<uint32_t>(1);
  const std::string name = "rowbatch";
  w.put<uint32_t>(static_cast<uint32_t>(name.size()));
  w.bytes(name.data(), name.size());
  w.put<uint32_t>(1);
  WriteBatch(&w, rb);
  *out = w.release(out_len);
  return PXG_OK;
}
