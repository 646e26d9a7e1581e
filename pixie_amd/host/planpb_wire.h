// Decoder of the planpb wire format (the subset of src/carnot/planpb/plan.proto:30-578 on the
// Filter/Map/Agg hot path), written against the protobuf encoding rules directly: protoc and
// libprotobuf are not part of this build, and an unmodified PxL-compiled plan arrives as the
// binary px.carnot.planpb.Plan message.  Field numbers are the reference's (plan.proto,
// src/shared/types/typespb/types.proto:26-69).  Unknown fields are skipped, as protobuf does.
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace pxc {
namespace planpb {

struct WireError : std::runtime_error {
  explicit WireError(const std::string& m) : std::runtime_error("planpb decode: " + m) {}
};

// One length-delimited message being read.
class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), end_(p + n) {}
  bool done() const { return p_ >= end_; }
  // Next field header; false at the end of the message.
  bool Next(uint32_t* field, uint32_t* wire) {
    if (done()) return false;
    const uint64_t key = Varint();
    *field = static_cast<uint32_t>(key >> 3);
    *wire = static_cast<uint32_t>(key & 7);
    return true;
  }
  uint64_t Varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p_ >= end_) throw WireError("truncated varint");
      const uint8_t b = *p_++;
      v |= static_cast<uint64_t>(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    throw WireError("varint too long");
  }
  uint64_t Fixed64() {
    if (end_ - p_ < 8) throw WireError("truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p_, 8);
    p_ += 8;
    return v;
  }
  uint32_t Fixed32() {
    if (end_ - p_ < 4) throw WireError("truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p_, 4);
    p_ += 4;
    return v;
  }
  Reader Sub() {
    const uint64_t n = Varint();
    if (static_cast<uint64_t>(end_ - p_) < n) throw WireError("truncated length-delimited field");
    Reader r(p_, static_cast<size_t>(n));
    p_ += n;
    return r;
  }
  std::string String() {
    Reader r = Sub();
    return std::string(reinterpret_cast<const char*>(r.p_), static_cast<size_t>(r.end_ - r.p_));
  }
  double Double() {
    const uint64_t b = Fixed64();
    double d;
    std::memcpy(&d, &b, 8);
    return d;
  }
  void Skip(uint32_t wire) {
    switch (wire) {
      case 0: (void)Varint(); break;
      case 1: (void)Fixed64(); break;
      case 2: (void)Sub(); break;
      case 5: (void)Fixed32(); break;
      default: throw WireError("unsupported wire type " + std::to_string(wire));
    }
  }
  // A repeated varint field: packed (wire 2) or one element (wire 0).
  template <typename T>
  void RepeatedVarint(uint32_t wire, std::vector<T>* out) {
    if (wire == 2) {
      Reader r = Sub();
      while (!r.done()) out->push_back(static_cast<T>(r.Varint()));
    } else {
      out->push_back(static_cast<T>(Varint()));
    }
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
};

// px.types.UInt128 / ScalarValue (plan.proto:519-531).
struct ScalarValue {
  int32_t data_type = 0;
  int32_t which = 0;  // oneof field number (2 bool .. 7 uint128), 0 = unset
  bool bool_value = false;
  int64_t int64_value = 0;
  double float64_value = 0;
  std::string string_value;
  int64_t time64_ns_value = 0;
  uint64_t u128_low = 0, u128_high = 0;
};

struct Column {  // plan.proto:491-496
  uint64_t node = 0;
  uint64_t index = 0;
};

struct ScalarExpression;
struct ScalarFunc {  // plan.proto:533-545
  std::string name;
  std::vector<ScalarValue> init_args;
  std::vector<ScalarExpression> args;
  int64_t id = 0;
  std::vector<int32_t> args_data_types;
};

struct ScalarExpression {  // plan.proto:547-552
  enum Kind { kNone = 0, kConstant = 1, kColumn = 2, kFunc = 3 } kind = kNone;
  ScalarValue constant;
  Column column;
  std::shared_ptr<ScalarFunc> func;
};

struct AggregateExpression {  // plan.proto:553-570
  struct Arg {
    bool is_column = false;
    Column column;
    ScalarValue constant;
  };
  std::string name;
  std::vector<ScalarValue> init_args;
  std::vector<Arg> args;
  int64_t id = 0;
  std::vector<int32_t> args_data_types;
};

struct MemorySourceOperator {  // plan.proto:149-167
  std::string name;
  std::vector<int64_t> column_idxs;
  std::vector<std::string> column_names;
  std::vector<int32_t> column_types;
  bool has_start_time = false, has_stop_time = false;  // google.protobuf.Int64Value wrappers
  int64_t start_time = 0, stop_time = 0;
  bool streaming = false;
};
struct MemorySinkOperator {  // plan.proto:214-222
  std::string name;
  std::vector<int32_t> column_types;
  std::vector<std::string> column_names;
};
struct MapOperator {  // plan.proto:230-235
  std::vector<ScalarExpression> expressions;
  std::vector<std::string> column_names;
};
struct AggregateOperator {  // plan.proto:237-258
  std::vector<AggregateExpression> values;
  std::vector<Column> groups;
  std::vector<std::string> group_names;
  std::vector<std::string> value_names;
  bool windowed = false;
  bool partial_agg = false;
  bool finalize_results = false;
};
struct FilterOperator {  // plan.proto:261-266
  ScalarExpression expression;
  std::vector<Column> columns;
};

struct JoinOperator {  // plan.proto:301-336
  int32_t type = 0;  // INNER 0, LEFT_OUTER 1, FULL_OUTER 3
  std::vector<std::pair<uint64_t, uint64_t>> equality_conditions;  // (left, right) column index
  std::vector<std::pair<uint64_t, uint64_t>> output_columns;       // (parent index, column index)
  std::vector<std::string> column_names;
  uint64_t rows_per_batch = 0;
};

// OperatorType (plan.proto:58-80).
enum OperatorType : int32_t {
  OPERATOR_TYPE_UNKNOWN = 0,
  MEMORY_SOURCE_OPERATOR = 1000,
  MAP_OPERATOR = 2000,
  AGGREGATE_OPERATOR = 2100,
  FILTER_OPERATOR = 2200,
  LIMIT_OPERATOR = 2300,
  MEMORY_SINK_OPERATOR = 9000,
  GRPC_SINK_OPERATOR = 9100,
};

struct LimitOperator {  // plan.proto:269-276
  int64_t limit = 0;
  std::vector<Column> columns;
  std::vector<uint64_t> abortable_srcs;
};

struct Operator {  // plan.proto:82-110
  int32_t op_type = 0;
  int32_t which = 0;  // oneof field number
  LimitOperator limit;
  MemorySourceOperator mem_source;
  MapOperator map;
  AggregateOperator agg;
  MemorySinkOperator mem_sink;
  FilterOperator filter;
  JoinOperator join;
  std::string grpc_sink_table;  // GRPCSinkOperator.output_table.table_name
  bool grpc_sink_to_source = false;  // GRPCSinkOperator.grpc_source_id is the destination
  uint64_t grpc_source_id = 0;
  std::vector<int32_t> grpc_source_types;        // GRPCSourceOperator.column_types (plan.proto:182-187)
  std::vector<std::string> grpc_source_names;
  std::vector<std::string> union_names;              // UnionOperator (plan.proto:283-295)
  std::vector<std::vector<int64_t>> union_mappings;  // per parent: input column of each output column
  uint64_t union_rows_per_batch = 0;                 // 0: kDefaultUnionRowBatchSize (union_node.h:41)
};

struct PlanNode {
  uint64_t id = 0;
  Operator op;
};
struct DAGNode {
  uint64_t id = 0;
  std::vector<uint64_t> sorted_children;
  std::vector<uint64_t> sorted_parents;
};
struct PlanFragment {
  uint64_t id = 0;
  std::vector<DAGNode> dag;
  std::vector<PlanNode> nodes;
};
struct Plan {
  std::vector<PlanFragment> fragments;
};

// ---------------------------------------------------------------------------------------
inline void Decode(Reader r, ScalarValue* v) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    switch (f) {
      case 1: v->data_type = static_cast<int32_t>(r.Varint()); break;
      case 2: v->bool_value = r.Varint() != 0; v->which = 2; break;
      case 3: v->int64_value = static_cast<int64_t>(r.Varint()); v->which = 3; break;
      case 4: v->float64_value = r.Double(); v->which = 4; break;
      case 5: v->string_value = r.String(); v->which = 5; break;
      case 6: v->time64_ns_value = static_cast<int64_t>(r.Varint()); v->which = 6; break;
      case 7: {
        Reader u = r.Sub();
        uint32_t uf, uw;
        while (u.Next(&uf, &uw)) {
          if (uf == 1) v->u128_low = u.Varint();
          else if (uf == 2) v->u128_high = u.Varint();
          else u.Skip(uw);
        }
        v->which = 7;
        break;
      }
      default: r.Skip(w);
    }
  }
}

inline void Decode(Reader r, Column* c) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    if (f == 1) c->node = r.Varint();
    else if (f == 2) c->index = r.Varint();
    else r.Skip(w);
  }
}

inline void Decode(Reader r, ScalarExpression* e);

inline void Decode(Reader r, ScalarFunc* fn) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    switch (f) {
      case 1: fn->name = r.String(); break;
      case 2: fn->init_args.emplace_back(); Decode(r.Sub(), &fn->init_args.back()); break;
      case 3: fn->args.emplace_back(); Decode(r.Sub(), &fn->args.back()); break;
      case 4: fn->id = static_cast<int64_t>(r.Varint()); break;
      case 5: r.RepeatedVarint(w, &fn->args_data_types); break;
      default: r.Skip(w);
    }
  }
}

inline void Decode(Reader r, ScalarExpression* e) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    switch (f) {
      case 1: e->kind = ScalarExpression::kConstant; Decode(r.Sub(), &e->constant); break;
      case 2: e->kind = ScalarExpression::kColumn; Decode(r.Sub(), &e->column); break;
      case 3:
        e->kind = ScalarExpression::kFunc;
        e->func = std::make_shared<ScalarFunc>();
        Decode(r.Sub(), e->func.get());
        break;
      default: r.Skip(w);
    }
  }
}

inline void Decode(Reader r, AggregateExpression* a) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    switch (f) {
      case 3: a->name = r.String(); break;
      case 4: a->init_args.emplace_back(); Decode(r.Sub(), &a->init_args.back()); break;
      case 5: {
        a->args.emplace_back();
        Reader ar = r.Sub();
        uint32_t af, aw;
        while (ar.Next(&af, &aw)) {
          if (af == 1) Decode(ar.Sub(), &a->args.back().constant);
          else if (af == 2) { a->args.back().is_column = true; Decode(ar.Sub(), &a->args.back().column); }
          else ar.Skip(aw);
        }
        break;
      }
      case 6: a->id = static_cast<int64_t>(r.Varint()); break;
      case 7: r.RepeatedVarint(w, &a->args_data_types); break;
      default: r.Skip(w);
    }
  }
}

inline void Decode(Reader r, Operator* op) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    switch (f) {
      case 1: op->op_type = static_cast<int32_t>(r.Varint()); break;
      case 2: {
        op->which = 2;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) op->mem_source.name = s.String();
          else if (sf == 2) s.RepeatedVarint(sw, &op->mem_source.column_idxs);
          else if (sf == 3) op->mem_source.column_names.push_back(s.String());
          else if (sf == 4) s.RepeatedVarint(sw, &op->mem_source.column_types);
          else if (sf == 5 || sf == 6) {
            Reader v = s.Sub();
            uint32_t vf, vw;
            int64_t x = 0;
            while (v.Next(&vf, &vw)) {
              if (vf == 1) x = static_cast<int64_t>(v.Varint());
              else v.Skip(vw);
            }
            if (sf == 5) { op->mem_source.has_start_time = true; op->mem_source.start_time = x; }
            else { op->mem_source.has_stop_time = true; op->mem_source.stop_time = x; }
          } else if (sf == 8) op->mem_source.streaming = s.Varint() != 0;
          else s.Skip(sw);
        }
        break;
      }
      case 3: {
        op->which = 3;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) { op->map.expressions.emplace_back(); Decode(s.Sub(), &op->map.expressions.back()); }
          else if (sf == 2) op->map.column_names.push_back(s.String());
          else s.Skip(sw);
        }
        break;
      }
      case 4: {
        op->which = 4;
        Reader s = r.Sub();
        uint32_t sf, sw;
        AggregateOperator& a = op->agg;
        while (s.Next(&sf, &sw)) {
          switch (sf) {
            case 1: a.values.emplace_back(); Decode(s.Sub(), &a.values.back()); break;
            case 2: a.groups.emplace_back(); Decode(s.Sub(), &a.groups.back()); break;
            case 3: a.group_names.push_back(s.String()); break;
            case 4: a.value_names.push_back(s.String()); break;
            case 5: a.windowed = s.Varint() != 0; break;
            case 6: a.partial_agg = s.Varint() != 0; break;
            case 7: a.finalize_results = s.Varint() != 0; break;
            default: s.Skip(sw);
          }
        }
        break;
      }
      case 5: {
        op->which = 5;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) op->mem_sink.name = s.String();
          else if (sf == 2) s.RepeatedVarint(sw, &op->mem_sink.column_types);
          else if (sf == 3) op->mem_sink.column_names.push_back(s.String());
          else s.Skip(sw);
        }
        break;
      }
      case 6: {
        op->which = 6;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) Decode(s.Sub(), &op->filter.expression);
          else if (sf == 2) { op->filter.columns.emplace_back(); Decode(s.Sub(), &op->filter.columns.back()); }
          else s.Skip(sw);
        }
        break;
      }
      case 7: {  // LimitOperator
        op->which = 7;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) op->limit.limit = static_cast<int64_t>(s.Varint());
          else if (sf == 2) { op->limit.columns.emplace_back(); Decode(s.Sub(), &op->limit.columns.back()); }
          else if (sf == 3) s.RepeatedVarint(sw, &op->limit.abortable_srcs);
          else s.Skip(sw);
        }
        break;
      }
      case 11: {
        op->which = 11;
        Reader s = r.Sub();
        uint32_t sf, sw;
        JoinOperator& j = op->join;
        while (s.Next(&sf, &sw)) {
          switch (sf) {
            case 1: j.type = static_cast<int32_t>(s.Varint()); break;
            case 2:
            case 3: {
              Reader c = s.Sub();
              uint32_t cf, cw;
              std::pair<uint64_t, uint64_t> v{0, 0};
              while (c.Next(&cf, &cw)) {
                if (cf == 1) v.first = c.Varint();
                else if (cf == 2) v.second = c.Varint();
                else c.Skip(cw);
              }
              (sf == 2 ? j.equality_conditions : j.output_columns).push_back(v);
              break;
            }
            case 4: j.column_names.push_back(s.String()); break;
            case 5: j.rows_per_batch = s.Varint(); break;
            default: s.Skip(sw);
          }
        }
        break;
      }
      case 1000: {
        op->which = 1000;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 4) {
            Reader t = s.Sub();
            uint32_t tf, tw;
            while (t.Next(&tf, &tw)) {
              if (tf == 1) op->grpc_sink_table = t.String();
              else t.Skip(tw);
            }
          } else if (sf == 3) {
            op->grpc_sink_to_source = true;
            op->grpc_source_id = s.Varint();
          } else {
            s.Skip(sw);
          }
        }
        break;
      }
      case 8: {  // UnionOperator
        op->which = 8;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) {
            op->union_names.push_back(s.String());
          } else if (sf == 2) {
            Reader m = s.Sub();
            std::vector<int64_t> idx;
            uint32_t mf, mw;
            while (m.Next(&mf, &mw)) {
              if (mf == 1) m.RepeatedVarint(mw, &idx);
              else m.Skip(mw);
            }
            op->union_mappings.push_back(idx);
          } else if (sf == 3) {
            op->union_rows_per_batch = s.Varint();
          } else {
            s.Skip(sw);
          }
        }
        break;
      }
      case 9: {  // GRPCSourceOperator
        op->which = 9;
        Reader s = r.Sub();
        uint32_t sf, sw;
        while (s.Next(&sf, &sw)) {
          if (sf == 1) s.RepeatedVarint(sw, &op->grpc_source_types);
          else if (sf == 2) op->grpc_source_names.push_back(s.String());
          else s.Skip(sw);
        }
        break;
      }
      default:
        op->which = static_cast<int32_t>(f);
        r.Skip(w);
    }
  }
}

inline void Decode(Reader r, PlanFragment* pf) {
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    switch (f) {
      case 1: pf->id = r.Varint(); break;
      case 2: {
        Reader d = r.Sub();
        uint32_t df, dw;
        while (d.Next(&df, &dw)) {
          if (df != 1) { d.Skip(dw); continue; }
          pf->dag.emplace_back();
          DAGNode& n = pf->dag.back();
          Reader nr = d.Sub();
          uint32_t nf, nw;
          while (nr.Next(&nf, &nw)) {
            if (nf == 1) n.id = nr.Varint();
            else if (nf == 3) nr.RepeatedVarint(nw, &n.sorted_children);
            else if (nf == 4) nr.RepeatedVarint(nw, &n.sorted_parents);
            else nr.Skip(nw);
          }
        }
        break;
      }
      case 3: {
        pf->nodes.emplace_back();
        Reader nr = r.Sub();
        uint32_t nf, nw;
        while (nr.Next(&nf, &nw)) {
          if (nf == 1) pf->nodes.back().id = nr.Varint();
          else if (nf == 2) Decode(nr.Sub(), &pf->nodes.back().op);
          else nr.Skip(nw);
        }
        break;
      }
      default: r.Skip(w);
    }
  }
}

inline Plan DecodePlan(const uint8_t* p, size_t n) {
  Plan plan;
  Reader r(p, n);
  uint32_t f, w;
  while (r.Next(&f, &w)) {
    if (f == 2) {
      plan.fragments.emplace_back();
      Decode(r.Sub(), &plan.fragments.back());
    } else {
      r.Skip(w);
    }
  }
  return plan;
}

}  // namespace planpb
}  // namespace pxc
