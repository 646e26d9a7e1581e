// ORACLE / TEST INFRASTRUCTURE ONLY — CPU restatement of Pixie Carnot's hot path.
// Never linked into the product.  See carnot_oracle.h for the list of restated files.
//
// This is deliberately the reference's *algorithm and cost structure* (batch-at-a-time, one
// thread, per-row std::function UDF calls, per-row RowTuple with std::string copies, hash map
// of group -> buffered value columns flushed at 512 rows, per-row UDA Update), so it doubles as
// the "CPU Carnot (restated)" baseline that bench.py times.

#include "carnot_oracle.h"
#include "json_number.h"

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "json.h"
#include "tdigest.h"

namespace oracle {

// px.types.DataType (src/shared/types/typespb/types.proto:26-34).
enum DT : int32_t { UNKNOWN = 0, BOOLEAN = 1, INT64 = 2, UINT128 = 3, FLOAT64 = 4, STRING = 5, TIME64NS = 6 };

// px.statuspb.Code (src/common/base/statuspb/status.proto:27-52).
enum Code : int32_t { OK = 0, INVALID_ARGUMENT = 3, NOT_FOUND = 5, INTERNAL = 9, UNIMPLEMENTED = 10 };

struct Error : std::runtime_error {
  int32_t code;
  Error(int32_t c, const std::string& m) : std::runtime_error(m), code(c) {}
};

static DT ParseDT(const Json& j) {
  if (j.kind == Json::kString) {
    static const std::map<std::string, DT> m = {{"BOOLEAN", BOOLEAN}, {"INT64", INT64},     {"UINT128", UINT128},
                                                {"FLOAT64", FLOAT64}, {"STRING", STRING},   {"TIME64NS", TIME64NS},
                                                {"DATA_TYPE_UNKNOWN", UNKNOWN}};
    auto it = m.find(j.str);
    if (it == m.end()) throw Error(INVALID_ARGUMENT, "unknown data type " + j.str);
    return it->second;
  }
  return static_cast<DT>(j.as_i64());
}

struct U128 {
  uint64_t lo = 0, hi = 0;
  bool operator==(const U128& o) const { return lo == o.lo && hi == o.hi; }
  bool operator!=(const U128& o) const { return !(*this == o); }
};

// ColumnWrapper (src/shared/types/column_wrapper.h:108-183): a typed std::vector.
struct Col {
  DT type = UNKNOWN;
  std::vector<uint8_t> b;
  std::vector<int64_t> i;
  std::vector<double> f;
  std::vector<std::string> s;
  std::vector<U128> u;
  explicit Col(DT t) : type(t) {}
  size_t size() const {
    switch (type) {
      case BOOLEAN: return b.size();
      case INT64:
      case TIME64NS: return i.size();
      case FLOAT64: return f.size();
      case STRING: return s.size();
      case UINT128: return u.size();
      default: return 0;
    }
  }
  void reserve(size_t n) {
    switch (type) {
      case BOOLEAN: b.reserve(n); break;
      case INT64:
      case TIME64NS: i.reserve(n); break;
      case FLOAT64: f.reserve(n); break;
      case STRING: s.reserve(n); break;
      case UINT128: u.reserve(n); break;
      default: break;
    }
  }
  void clear() { b.clear(); i.clear(); f.clear(); s.clear(); u.clear(); }
  void append_from(const Col& o, size_t r) {
    switch (type) {
      case BOOLEAN: b.push_back(o.b[r]); break;
      case INT64:
      case TIME64NS: i.push_back(o.i[r]); break;
      case FLOAT64: f.push_back(o.f[r]); break;
      case STRING: s.push_back(o.s[r]); break;
      case UINT128: u.push_back(o.u[r]); break;
      default: break;
    }
  }
};
using ColPtr = std::shared_ptr<Col>;

struct RowBatch {
  std::vector<ColPtr> cols;
  int64_t num_rows = 0;
  bool eow = false, eos = false;
};

// A scalar value (ScalarValue, plan.proto:519-531).
struct Value {
  DT type = UNKNOWN;
  bool b = false;
  int64_t i = 0;
  double f = 0;
  std::string s;
  U128 u;
};

static Value ParseValue(const Json& j) {
  Value v;
  v.type = ParseDT(j["dataType"]);
  switch (v.type) {
    case BOOLEAN: v.b = j["boolValue"].as_bool(); break;
    case INT64: v.i = j["int64Value"].as_i64(); break;
    case TIME64NS: v.i = j["time64NsValue"].as_i64(); break;
    case FLOAT64: v.f = j["float64Value"].as_f64(); break;
    case STRING: v.s = j["stringValue"].as_str(); break;
    case UINT128:
      v.u.lo = j["uint128Value"]["low"].as_u64();
      v.u.hi = j["uint128Value"]["high"].as_u64();
      break;
    default: throw Error(INVALID_ARGUMENT, "bad scalar value type");
  }
  return v;
}

// EvalScalarToColumnWrapper (expression_evaluator.cc:115-134): materialise N copies.
static ColPtr ConstCol(const Value& v, size_t n) {
  auto c = std::make_shared<Col>(v.type);
  switch (v.type) {
    case BOOLEAN: c->b.assign(n, v.b); break;
    case INT64:
    case TIME64NS: c->i.assign(n, v.i); break;
    case FLOAT64: c->f.assign(n, v.f); break;
    case STRING: c->s.assign(n, v.s); break;
    case UINT128: c->u.assign(n, v.u); break;
    default: break;
  }
  return c;
}

/*********************************************************************************************
 * Scalar UDF registry (math_ops.cc:52-223, json_ops.cc:32), keyed by (name, arg types).
 *********************************************************************************************/
using UDFExec = std::function<void(const std::vector<const Col*>& args, Col* out, size_t n)>;
struct UDFDef {
  DT out;
  UDFExec exec;
};

template <DT T> struct Native;
template <> struct Native<BOOLEAN> { using type = bool; static bool get(const Col& c, size_t r) { return c.b[r] != 0; } static void put(Col* c, bool v) { c->b.push_back(v ? 1 : 0); } };
template <> struct Native<INT64> { using type = int64_t; static int64_t get(const Col& c, size_t r) { return c.i[r]; } static void put(Col* c, int64_t v) { c->i.push_back(v); } };
template <> struct Native<TIME64NS> { using type = int64_t; static int64_t get(const Col& c, size_t r) { return c.i[r]; } static void put(Col* c, int64_t v) { c->i.push_back(v); } };
template <> struct Native<FLOAT64> { using type = double; static double get(const Col& c, size_t r) { return c.f[r]; } static void put(Col* c, double v) { c->f.push_back(v); } };
// GetValueFromArrowArray<STRING> returns a std::string copy per access (arrow_adapter.h:123-131).
template <> struct Native<STRING> { using type = std::string; static std::string get(const Col& c, size_t r) { return c.s[r]; } static void put(Col* c, std::string v) { c->s.push_back(std::move(v)); } };
template <> struct Native<UINT128> { using type = U128; static U128 get(const Col& c, size_t r) { return c.u[r]; } static void put(Col* c, U128 v) { c->u.push_back(v); } };

static std::string Key(const std::string& name, const std::vector<DT>& types) {
  std::string k = name + "(";
  for (auto t : types) k += std::to_string(static_cast<int>(t)) + ",";
  return k + ")";
}

class Registry {
 public:
  static Registry& Get() {
    static Registry r;
    return r;
  }
  const UDFDef* GetUDF(const std::string& name, const std::vector<DT>& types) const {
    auto it = udfs_.find(Key(name, types));
    return it == udfs_.end() ? nullptr : &it->second;
  }

  template <DT A, DT B, DT R, typename F>
  void Bin(const std::string& name, F fn) {
    udfs_[Key(name, {A, B})] = UDFDef{R, [fn](const std::vector<const Col*>& a, Col* out, size_t n) {
                                        out->reserve(n);
                                        for (size_t r = 0; r < n; ++r)
                                          Native<R>::put(out, fn(Native<A>::get(*a[0], r), Native<B>::get(*a[1], r)));
                                      }};
  }
  template <DT A, DT R, typename F>
  void Un(const std::string& name, F fn) {
    udfs_[Key(name, {A})] = UDFDef{R, [fn](const std::vector<const Col*>& a, Col* out, size_t n) {
                                     out->reserve(n);
                                     for (size_t r = 0; r < n; ++r) Native<R>::put(out, fn(Native<A>::get(*a[0], r)));
                                   }};
  }

 private:
  std::map<std::string, UDFDef> udfs_;
  Registry();
};

// Two's-complement wrapping int64 arithmetic (the reference's signed overflow is UB; every
// supported target wraps).
static inline int64_t WAdd(int64_t a, int64_t b) { return static_cast<int64_t>(static_cast<uint64_t>(a) + static_cast<uint64_t>(b)); }
static inline int64_t WSub(int64_t a, int64_t b) { return static_cast<int64_t>(static_cast<uint64_t>(a) - static_cast<uint64_t>(b)); }
static inline int64_t WMul(int64_t a, int64_t b) { return static_cast<int64_t>(static_cast<uint64_t>(a) * static_cast<uint64_t>(b)); }
static inline int64_t SMod(int64_t a, int64_t b) { return b == 0 ? 0 : (b == -1 ? 0 : a % b); }

Registry::Registry() {
  // add / subtract / multiply (math_ops.h:33-150; math_ops.cc:57-105).
  Bin<INT64, INT64, INT64>("add", [](int64_t a, int64_t b) { return WAdd(a, b); });
  Bin<FLOAT64, FLOAT64, FLOAT64>("add", [](double a, double b) { return a + b; });
  Bin<STRING, STRING, STRING>("add", [](std::string a, std::string b) { return a + b; });
  Bin<FLOAT64, INT64, FLOAT64>("add", [](double a, int64_t b) { return a + b; });
  Bin<INT64, FLOAT64, FLOAT64>("add", [](int64_t a, double b) { return a + b; });
  Bin<TIME64NS, INT64, TIME64NS>("add", [](int64_t a, int64_t b) { return WAdd(a, b); });
  Bin<INT64, TIME64NS, TIME64NS>("add", [](int64_t a, int64_t b) { return WAdd(a, b); });
  Bin<INT64, INT64, INT64>("subtract", [](int64_t a, int64_t b) { return WSub(a, b); });
  Bin<FLOAT64, FLOAT64, FLOAT64>("subtract", [](double a, double b) { return a - b; });
  Bin<FLOAT64, INT64, FLOAT64>("subtract", [](double a, int64_t b) { return a - b; });
  Bin<INT64, FLOAT64, FLOAT64>("subtract", [](int64_t a, double b) { return a - b; });
  Bin<TIME64NS, INT64, TIME64NS>("subtract", [](int64_t a, int64_t b) { return WSub(a, b); });
  Bin<TIME64NS, TIME64NS, INT64>("subtract", [](int64_t a, int64_t b) { return WSub(a, b); });
  Bin<INT64, TIME64NS, INT64>("subtract", [](int64_t a, int64_t b) { return WSub(a, b); });
  // DivideUDF always returns double(a)/double(b) (math_ops.h:84-89).
  Bin<INT64, INT64, FLOAT64>("divide", [](int64_t a, int64_t b) { return static_cast<double>(a) / static_cast<double>(b); });
  Bin<FLOAT64, INT64, FLOAT64>("divide", [](double a, int64_t b) { return a / static_cast<double>(b); });
  Bin<INT64, FLOAT64, FLOAT64>("divide", [](int64_t a, double b) { return static_cast<double>(a) / b; });
  Bin<FLOAT64, FLOAT64, FLOAT64>("divide", [](double a, double b) { return a / b; });
  Bin<INT64, INT64, INT64>("multiply", [](int64_t a, int64_t b) { return WMul(a, b); });
  Bin<FLOAT64, FLOAT64, FLOAT64>("multiply", [](double a, double b) { return a * b; });
  Bin<FLOAT64, INT64, FLOAT64>("multiply", [](double a, int64_t b) { return a * b; });
  Bin<INT64, FLOAT64, FLOAT64>("multiply", [](int64_t a, double b) { return a * b; });
  // modulo (math_ops.cc:118-125): b1 % b2.
  Bin<TIME64NS, INT64, INT64>("modulo", SMod);
  Bin<TIME64NS, TIME64NS, INT64>("modulo", SMod);
  Bin<INT64, TIME64NS, INT64>("modulo", SMod);
  Bin<INT64, INT64, INT64>("modulo", SMod);
  // logical (math_ops.h:265-315).
  Bin<INT64, INT64, BOOLEAN>("logicalOr", [](int64_t a, int64_t b) { return a || b; });
  Bin<BOOLEAN, BOOLEAN, BOOLEAN>("logicalOr", [](bool a, bool b) { return a || b; });
  Bin<INT64, INT64, BOOLEAN>("logicalAnd", [](int64_t a, int64_t b) { return a && b; });
  Bin<BOOLEAN, BOOLEAN, BOOLEAN>("logicalAnd", [](bool a, bool b) { return a && b; });
  Un<INT64, BOOLEAN>("logicalNot", [](int64_t a) { return !a; });
  Un<BOOLEAN, BOOLEAN>("logicalNot", [](bool a) { return !a; });
  Un<INT64, INT64>("negate", [](int64_t a) { return WSub(0, a); });
  Un<FLOAT64, FLOAT64>("negate", [](double a) { return -a; });
  Un<INT64, INT64>("invert", [](int64_t a) { return ~a; });
  // equal / notEqual (math_ops.cc:145-175; math_ops.h:372-410).  FLOAT64==FLOAT64 is
  // ApproxEqualUDF (|a-b| < epsilon).
  Bin<INT64, INT64, BOOLEAN>("equal", [](int64_t a, int64_t b) { return a == b; });
  Bin<STRING, STRING, BOOLEAN>("equal", [](std::string a, std::string b) { return a == b; });
  Bin<BOOLEAN, BOOLEAN, BOOLEAN>("equal", [](bool a, bool b) { return a == b; });
  Bin<TIME64NS, TIME64NS, BOOLEAN>("equal", [](int64_t a, int64_t b) { return a == b; });
  Bin<UINT128, UINT128, BOOLEAN>("equal", [](U128 a, U128 b) { return a == b; });
  Bin<BOOLEAN, INT64, BOOLEAN>("equal", [](bool a, int64_t b) { return static_cast<int64_t>(a) == b; });
  Bin<INT64, BOOLEAN, BOOLEAN>("equal", [](int64_t a, bool b) { return a == static_cast<int64_t>(b); });
  Bin<INT64, FLOAT64, BOOLEAN>("equal", [](int64_t a, double b) { return static_cast<double>(a) == b; });
  Bin<FLOAT64, INT64, BOOLEAN>("equal", [](double a, int64_t b) { return a == static_cast<double>(b); });
  Bin<FLOAT64, FLOAT64, BOOLEAN>("equal", [](double a, double b) { return std::abs(a - b) < std::numeric_limits<double>::epsilon(); });
  Bin<INT64, INT64, BOOLEAN>("notEqual", [](int64_t a, int64_t b) { return a != b; });
  Bin<STRING, STRING, BOOLEAN>("notEqual", [](std::string a, std::string b) { return a != b; });
  Bin<BOOLEAN, BOOLEAN, BOOLEAN>("notEqual", [](bool a, bool b) { return a != b; });
  Bin<TIME64NS, TIME64NS, BOOLEAN>("notEqual", [](int64_t a, int64_t b) { return a != b; });
  Bin<UINT128, UINT128, BOOLEAN>("notEqual", [](U128 a, U128 b) { return a != b; });
  Bin<BOOLEAN, INT64, BOOLEAN>("notEqual", [](bool a, int64_t b) { return static_cast<int64_t>(a) != b; });
  Bin<INT64, BOOLEAN, BOOLEAN>("notEqual", [](int64_t a, bool b) { return a != static_cast<int64_t>(b); });
  Bin<INT64, FLOAT64, BOOLEAN>("notEqual", [](int64_t a, double b) { return static_cast<double>(a) != b; });
  Bin<FLOAT64, INT64, BOOLEAN>("notEqual", [](double a, int64_t b) { return a != static_cast<double>(b); });
  Bin<FLOAT64, FLOAT64, BOOLEAN>("notEqual", [](double a, double b) { return std::abs(a - b) > std::numeric_limits<double>::epsilon(); });
  Bin<FLOAT64, FLOAT64, BOOLEAN>("approxEqual", [](double a, double b) { return std::abs(a - b) < std::numeric_limits<double>::epsilon(); });
  // ordering comparisons (math_ops.h:412-510; math_ops.cc:177-200).
#define PXO_CMP(NAME, OP)                                                                   \
  Bin<INT64, INT64, BOOLEAN>(NAME, [](int64_t a, int64_t b) { return a OP b; });          \
  Bin<TIME64NS, TIME64NS, BOOLEAN>(NAME, [](int64_t a, int64_t b) { return a OP b; });    \
  Bin<FLOAT64, FLOAT64, BOOLEAN>(NAME, [](double a, double b) { return a OP b; });        \
  Bin<STRING, STRING, BOOLEAN>(NAME, [](std::string a, std::string b) { return a OP b; });
  PXO_CMP("greaterThan", >)
  PXO_CMP("greaterThanEqual", >=)
  PXO_CMP("lessThan", <)
  PXO_CMP("lessThanEqual", <=)
#undef PXO_CMP
  // bin (math_ops.h:512-527): a - a % b.
  Bin<INT64, INT64, INT64>("bin", [](int64_t a, int64_t b) { return WSub(a, SMod(a, b)); });
  Bin<TIME64NS, TIME64NS, TIME64NS>("bin", [](int64_t a, int64_t b) { return WSub(a, SMod(a, b)); });
  Bin<INT64, TIME64NS, INT64>("bin", [](int64_t a, int64_t b) { return WSub(a, SMod(a, b)); });
  Bin<TIME64NS, INT64, TIME64NS>("bin", [](int64_t a, int64_t b) { return WSub(a, SMod(a, b)); });
  Bin<FLOAT64, INT64, INT64>("bin", [](double a, int64_t b) {
    int64_t ia = static_cast<int64_t>(a);
    return WSub(ia, SMod(ia, b));
  });
  Un<TIME64NS, INT64>("time_to_int64", [](int64_t a) { return a; });
  Un<INT64, TIME64NS>("int64_to_time", [](int64_t a) { return a; });
  // Test-registry UDFs of FilterNodeTest (filter_node_test.cc:41-53): "eq" on INT64 / STRING.
  Bin<INT64, INT64, BOOLEAN>("eq", [](int64_t a, int64_t b) { return a == b; });
  Bin<STRING, STRING, BOOLEAN>("eq", [](std::string a, std::string b) { return a == b; });
  // pluck_float64 (json_ops.h:131-153).
  Bin<STRING, STRING, FLOAT64>("pluck_float64", [](std::string in, std::string key) {
    return oracle_pluck_float64(in.c_str(), key.c_str());
  });
}

/*********************************************************************************************
 * UDAs (math_ops.h:583-772, math_sketches.h:33-82, agg_node_test.cc:44-72 test UDAs).
 *********************************************************************************************/
// QuantilesUDA::Finalize (math_sketches.h:40-54): rapidjson Document written by
// rapidjson::Writer -- restated for the oracle in json_number.h, independently of the engine's
// pixie_amd/host/json_double.h (tests/test_json_double.py pins both against the reference's own
// known strings and rapidjson's rules, and compares them byte for byte).
std::string QuantilesJson(TDigest* d) {
  static const double kQ[7] = {0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99};
  double q[7];
  for (int k = 0; k < 7; ++k) q[k] = d->quantile(kQ[k]);
  std::string s;
  oracle_json::AppendQuantilesJson(q, &s);
  return s;
}

struct UDA {
  virtual ~UDA() = default;
  // Per-row Update from the arg columns (UDAWrapper::UpdateWrapper, udf_wrapper.h:287-310).
  virtual void Update(const std::vector<const Col*>& args, size_t r) = 0;
  virtual void Merge(const UDA& other) = 0;
  virtual void Finalize(Col* out) = 0;
  // Serialize / Deserialize (udf.h:98-100): the raw state bytes (math_ops.h:602-757).  UDAs
  // without them (QuantilesUDA, the test MinSum UDAs) are not splittable (udf.h:367).
  virtual bool SupportsPartial() const { return false; }
  virtual std::string Serialize() const { throw Error(UNIMPLEMENTED, "UDA has no Serialize"); }
  virtual void Deserialize(const char*) { throw Error(UNIMPLEMENTED, "UDA has no Deserialize"); }
};
template <typename T>
static std::string RawBytes(const T& v) { return std::string(reinterpret_cast<const char*>(&v), sizeof(v)); }
template <typename T>
static T FromRaw(const char* p) {
  T v;
  std::memcpy(&v, p, sizeof(v));
  return v;
}

template <DT A>
struct CountUDA : UDA {
  uint64_t count = 0;
  void Update(const std::vector<const Col*>&, size_t) override { ++count; }
  void Merge(const UDA& o) override { count += static_cast<const CountUDA&>(o).count; }
  void Finalize(Col* out) override { out->i.push_back(static_cast<int64_t>(count)); }
  bool SupportsPartial() const override { return true; }
  std::string Serialize() const override { return RawBytes(count); }  // math_ops.h:741-748
  void Deserialize(const char* p) override { count = FromRaw<uint64_t>(p); }
};

template <DT A>
struct MeanUDA : UDA {
  uint64_t size = 0;
  double sum = 0;  // "count" in the reference's MeanInfo
  void Update(const std::vector<const Col*>& a, size_t r) override {
    ++size;
    sum += static_cast<double>(Native<A>::get(*a[0], r));
  }
  void Merge(const UDA& o) override {
    auto& m = static_cast<const MeanUDA&>(o);
    size += m.size;
    sum += m.sum;
  }
  void Finalize(Col* out) override { out->f.push_back(sum / static_cast<double>(size)); }
  // MeanInfo {uint64 size; double count} (math_ops.h:602-609,621-624).
  bool SupportsPartial() const override { return true; }
  std::string Serialize() const override { return RawBytes(size) + RawBytes(sum); }
  void Deserialize(const char* p) override {
    size = FromRaw<uint64_t>(p);
    sum = FromRaw<double>(p + 8);
  }
};

template <DT A, DT R>
struct SumUDA : UDA {
  typename Native<R>::type sum = 0;
  void Update(const std::vector<const Col*>& a, size_t r) override {
    if constexpr (R == FLOAT64) {
      sum = sum + Native<A>::get(*a[0], r);
    } else {
      sum = WAdd(sum, static_cast<int64_t>(Native<A>::get(*a[0], r)));
    }
  }
  void Merge(const UDA& o) override {
    if constexpr (R == FLOAT64) sum = sum + static_cast<const SumUDA&>(o).sum;
    else sum = WAdd(sum, static_cast<const SumUDA&>(o).sum);
  }
  void Finalize(Col* out) override { Native<R>::put(out, sum); }
  bool SupportsPartial() const override { return true; }
  std::string Serialize() const override { return RawBytes(sum); }  // math_ops.h:639-646
  void Deserialize(const char* p) override { sum = FromRaw<typename Native<R>::type>(p); }
};

template <DT A>
struct MaxUDA : UDA {
  // MaxUDA initialises to numeric_limits<T>::min() (math_ops.h:699): for FLOAT64 that is the
  // smallest positive double.
  typename Native<A>::type v = std::numeric_limits<typename Native<A>::type>::min();
  void Update(const std::vector<const Col*>& a, size_t r) override {
    auto x = Native<A>::get(*a[0], r);
    if (v < x) v = x;
  }
  void Merge(const UDA& o) override {
    auto x = static_cast<const MaxUDA&>(o).v;
    if (x > v) v = x;
  }
  void Finalize(Col* out) override { Native<A>::put(out, v); }
  bool SupportsPartial() const override { return true; }
  std::string Serialize() const override { return RawBytes(v); }  // math_ops.h:723-730
  void Deserialize(const char* p) override { v = FromRaw<typename Native<A>::type>(p); }
};

template <DT A>
struct MinUDA : UDA {
  typename Native<A>::type v = std::numeric_limits<typename Native<A>::type>::max();
  void Update(const std::vector<const Col*>& a, size_t r) override {
    auto x = Native<A>::get(*a[0], r);
    if (v > x) v = x;
  }
  void Merge(const UDA& o) override {
    auto x = static_cast<const MinUDA&>(o).v;
    if (x < v) v = x;
  }
  void Finalize(Col* out) override { Native<A>::put(out, v); }
  bool SupportsPartial() const override { return true; }
  std::string Serialize() const override { return RawBytes(v); }  // math_ops.h:750-757
  void Deserialize(const char* p) override { v = FromRaw<typename Native<A>::type>(p); }
};

template <DT A>
struct QuantilesUDA : UDA {
  TDigest digest{1000};
  void Update(const std::vector<const Col*>& a, size_t r) override {
    digest.add(static_cast<double>(Native<A>::get(*a[0], r)));
  }
  void Merge(const UDA& o) override { digest.merge(&static_cast<const QuantilesUDA&>(o).digest); }
  void Finalize(Col* out) override { out->s.push_back(QuantilesJson(&digest)); }
};

// Test UDAs registered by AggNodeTest (agg_node_test.cc:44-72, 282-289).
struct MinSumUDA : UDA {
  int64_t sum = 0;
  void Update(const std::vector<const Col*>& a, size_t r) override {
    sum = WAdd(sum, std::min(a[0]->i[r], a[1]->i[r]));
  }
  void Merge(const UDA& o) override { sum = WAdd(sum, static_cast<const MinSumUDA&>(o).sum); }
  void Finalize(Col* out) override { out->i.push_back(sum); }
};

struct UDADef {
  DT out;
  size_t n_update_args;
  std::function<std::unique_ptr<UDA>(const std::vector<Value>& init)> make;
};

class UDARegistry {
 public:
  static UDARegistry& Get() {
    static UDARegistry r;
    return r;
  }
  const UDADef* Find(const std::string& name, const std::vector<DT>& types) const {
    auto it = defs_.find(Key(name, types));
    return it == defs_.end() ? nullptr : &it->second;
  }

 private:
  std::map<std::string, UDADef> defs_;
  template <typename T>
  void Reg(const std::string& name, std::vector<DT> types, DT out, size_t nargs) {
    defs_[Key(name, types)] = UDADef{out, nargs, [](const std::vector<Value>&) { return std::make_unique<T>(); }};
  }
  UDARegistry() {
    Reg<MeanUDA<FLOAT64>>("mean", {FLOAT64}, FLOAT64, 1);
    Reg<MeanUDA<INT64>>("mean", {INT64}, FLOAT64, 1);
    Reg<MeanUDA<BOOLEAN>>("mean", {BOOLEAN}, FLOAT64, 1);
    Reg<SumUDA<FLOAT64, FLOAT64>>("sum", {FLOAT64}, FLOAT64, 1);
    Reg<SumUDA<INT64, INT64>>("sum", {INT64}, INT64, 1);
    Reg<SumUDA<BOOLEAN, INT64>>("sum", {BOOLEAN}, INT64, 1);
    Reg<MaxUDA<FLOAT64>>("max", {FLOAT64}, FLOAT64, 1);
    Reg<MaxUDA<INT64>>("max", {INT64}, INT64, 1);
    Reg<MaxUDA<TIME64NS>>("max", {TIME64NS}, TIME64NS, 1);
    Reg<MinUDA<FLOAT64>>("min", {FLOAT64}, FLOAT64, 1);
    Reg<MinUDA<INT64>>("min", {INT64}, INT64, 1);
    Reg<MinUDA<TIME64NS>>("min", {TIME64NS}, TIME64NS, 1);
    for (DT t : {FLOAT64, INT64, TIME64NS, BOOLEAN, STRING, UINT128}) {
      defs_[Key("count", {t})] = UDADef{INT64, 1, [](const std::vector<Value>&) { return std::make_unique<CountUDA<INT64>>(); }};
    }
    Reg<QuantilesUDA<INT64>>("quantiles", {INT64}, STRING, 1);
    Reg<QuantilesUDA<FLOAT64>>("quantiles", {FLOAT64}, STRING, 1);
    Reg<MinSumUDA>("minsum", {INT64, INT64}, INT64, 2);
    defs_[Key("minsum_w_init", {INT64, INT64, INT64})] =
        UDADef{INT64, 2, [](const std::vector<Value>& init) {
                 auto u = std::make_unique<MinSumUDA>();
                 if (!init.empty()) u->sum = init[0].i;  // MinSumWithInitUDA::Init
                 return u;
               }};
  }
};

/*********************************************************************************************
 * Plan objects (plan/scalar_expression.cc:232-348, plan/operators.cc:59-395).
 *********************************************************************************************/
struct Expr {
  enum Kind { kConst, kColumn, kFunc, kAgg } kind = kConst;
  Value value;
  int64_t col_node = 0, col_index = 0;
  std::string name;
  std::vector<Value> init_args;
  std::vector<Expr> args;
  std::vector<DT> arg_types;
};

static Expr ParseColumn(const Json& j) {
  Expr e;
  e.kind = Expr::kColumn;
  e.col_node = j["node"].as_i64();
  e.col_index = j["index"].as_i64();
  return e;
}

static Expr ParseScalarExpr(const Json& j) {
  Expr e;
  if (j.has("constant")) {
    e.kind = Expr::kConst;
    e.value = ParseValue(j["constant"]);
  } else if (j.has("column")) {
    e = ParseColumn(j["column"]);
  } else if (j.has("func")) {
    const Json& f = j["func"];
    e.kind = Expr::kFunc;
    e.name = f["name"].as_str();
    for (size_t i = 0; i < f["initArgs"].size(); ++i) e.init_args.push_back(ParseValue(f["initArgs"].at(i)));
    for (size_t i = 0; i < f["args"].size(); ++i) e.args.push_back(ParseScalarExpr(f["args"].at(i)));
    for (size_t i = 0; i < f["argsDataTypes"].size(); ++i) e.arg_types.push_back(ParseDT(f["argsDataTypes"].at(i)));
  } else {
    throw Error(INVALID_ARGUMENT, "bad scalar expression");
  }
  return e;
}

static Expr ParseAggExpr(const Json& j) {
  Expr e;
  e.kind = Expr::kAgg;
  e.name = j["name"].as_str();
  for (size_t i = 0; i < j["initArgs"].size(); ++i) e.init_args.push_back(ParseValue(j["initArgs"].at(i)));
  for (size_t i = 0; i < j["args"].size(); ++i) {
    const Json& a = j["args"].at(i);
    Expr c;
    if (a.has("constant")) {
      c.kind = Expr::kConst;
      c.value = ParseValue(a["constant"]);
    } else {
      c = ParseColumn(a["column"]);
    }
    e.args.push_back(c);
  }
  for (size_t i = 0; i < j["argsDataTypes"].size(); ++i) e.arg_types.push_back(ParseDT(j["argsDataTypes"].at(i)));
  return e;
}

// Output type of an expression given the input relation (ScalarFunc::OutputDataType,
// scalar_expression.cc:278-311): computed from the children's types via the registry.
static DT ExprType(const Expr& e, const std::vector<DT>& in) {
  switch (e.kind) {
    case Expr::kConst: return e.value.type;
    case Expr::kColumn:
      if (e.col_index < 0 || static_cast<size_t>(e.col_index) >= in.size()) throw Error(INVALID_ARGUMENT, "column index out of range");
      return in[e.col_index];
    case Expr::kFunc: {
      std::vector<DT> types;
      for (auto& v : e.init_args) types.push_back(v.type);
      for (auto& a : e.args) types.push_back(ExprType(a, in));
      const UDFDef* d = Registry::Get().GetUDF(e.name, types);
      if (!d) throw Error(NOT_FOUND, "no UDF " + Key(e.name, types));
      return d->out;
    }
    case Expr::kAgg: {
      std::vector<DT> types;
      for (auto& v : e.init_args) types.push_back(v.type);
      for (auto& a : e.args) types.push_back(ExprType(a, in));
      const UDADef* d = UDARegistry::Get().Find(e.name, types);
      if (!d) throw Error(NOT_FOUND, "no UDA " + Key(e.name, types));
      return d->out;
    }
  }
  return UNKNOWN;
}

/*********************************************************************************************
 * Exec nodes (exec_node.h:133-337 NVI).
 *********************************************************************************************/
struct ExecNode {
  std::vector<ExecNode*> children;
  std::vector<size_t> child_parent_index;
  std::vector<DT> out_types;
  virtual ~ExecNode() = default;
  virtual void ConsumeNext(const RowBatch& rb, size_t parent_index) = 0;
  void Send(const RowBatch& rb) {
    if (rb.eos && !rb.eow) throw Error(INTERNAL, "eos without eow");
    for (size_t i = 0; i < children.size(); ++i) children[i]->ConsumeNext(rb, child_parent_index[i]);
  }
};

// VectorNative evaluation (expression_evaluator.cc:191-275): column leaves are copied into
// ColumnWrappers (column_wrapper.h:207-233), constants materialised, funcs via ExecBatch.
static ColPtr EvalVectorNative(const Expr& e, const RowBatch& rb) {
  switch (e.kind) {
    case Expr::kConst: return ConstCol(e.value, rb.num_rows);
    case Expr::kColumn: return std::make_shared<Col>(*rb.cols.at(e.col_index));
    case Expr::kFunc: {
      std::vector<ColPtr> kids;
      std::vector<const Col*> raw;
      std::vector<DT> types;
      for (auto& v : e.init_args) types.push_back(v.type);
      for (auto& a : e.args) {
        kids.push_back(EvalVectorNative(a, rb));
        raw.push_back(kids.back().get());
        types.push_back(kids.back()->type);
      }
      const UDFDef* d = Registry::Get().GetUDF(e.name, types);
      if (!d) throw Error(NOT_FOUND, "no UDF " + Key(e.name, types));
      auto out = std::make_shared<Col>(d->out);
      d->exec(raw, out.get(), rb.num_rows);
      return out;
    }
    default: throw Error(INVALID_ARGUMENT, "bad expression in scalar context");
  }
}

// ArrowNative evaluation (expression_evaluator.cc:277-342): column refs are shared (no copy).
static ColPtr EvalArrowNative(const Expr& e, const RowBatch& rb) {
  if (e.kind == Expr::kColumn) return rb.cols.at(e.col_index);
  if (e.kind == Expr::kConst) return ConstCol(e.value, rb.num_rows);
  std::vector<ColPtr> kids;
  std::vector<const Col*> raw;
  std::vector<DT> types;
  for (auto& v : e.init_args) types.push_back(v.type);
  for (auto& a : e.args) {
    kids.push_back(EvalArrowNative(a, rb));
    raw.push_back(kids.back().get());
    types.push_back(kids.back()->type);
  }
  const UDFDef* d = Registry::Get().GetUDF(e.name, types);
  if (!d) throw Error(NOT_FOUND, "no UDF " + Key(e.name, types));
  auto out = std::make_shared<Col>(d->out);
  d->exec(raw, out.get(), rb.num_rows);
  return out;
}

// FilterNode::ConsumeNextImpl (filter_node.cc:132-171).
struct FilterNode : ExecNode {
  Expr pred;
  std::vector<int64_t> selected;
  void ConsumeNext(const RowBatch& rb, size_t) override {
    ColPtr p = EvalVectorNative(pred, rb);
    if (p->type != BOOLEAN) throw Error(INVALID_ARGUMENT, "predicate must be boolean");
    size_t n_out = 0;
    for (size_t r = 0; r < p->b.size(); ++r) n_out += p->b[r] ? 1 : 0;
    RowBatch out;
    out.num_rows = static_cast<int64_t>(n_out);
    for (int64_t ci : selected) {
      const Col& in = *rb.cols.at(ci);
      auto c = std::make_shared<Col>(in.type);
      c->reserve(n_out);
      for (size_t r = 0; r < p->b.size(); ++r)
        if (p->b[r]) c->append_from(in, r);
      out.cols.push_back(c);
    }
    out.eow = rb.eow;
    out.eos = rb.eos;
    Send(out);
  }
};

// MapNode::ConsumeNextImpl (map_node.cc:64-71).
struct MapNode : ExecNode {
  std::vector<Expr> exprs;
  void ConsumeNext(const RowBatch& rb, size_t) override {
    RowBatch out;
    out.num_rows = rb.num_rows;
    for (auto& e : exprs) out.cols.push_back(EvalArrowNative(e, rb));
    out.eow = rb.eow;
    out.eos = rb.eos;
    Send(out);
  }
};

// RowTuple (row_tuple.h:71-188): 16 B fixed slots + strings; exact-equality semantics.
struct RowTuple {
  std::vector<DT> types;
  std::vector<std::array<uint64_t, 2>> fixed;
  std::vector<std::string> strs;
  bool operator==(const RowTuple& o) const { return fixed == o.fixed && strs == o.strs; }
};
struct RowTupleHash {
  size_t operator()(const RowTuple* rt) const {
    // Hash64 over fixed bytes then HashCombine per string (row_tuple.h:140-153); the exact hash
    // function does not affect results (output order is unspecified).
    uint64_t h = 0xcbf29ce484222325ULL;
    for (auto& f : rt->fixed) {
      h = (h ^ f[0]) * 0x100000001b3ULL;
      h = (h ^ f[1]) * 0x100000001b3ULL;
    }
    for (auto& s : rt->strs) h = (h * 31) ^ std::hash<std::string>()(s);
    return h;
  }
};
struct RowTupleEq {
  bool operator()(const RowTuple* a, const RowTuple* b) const { return *a == *b; }
};

static void ExtractIntoRowTuple(RowTuple* rt, const Col& c, size_t slot, size_t r) {
  // ExtractIntoRowTuple<DT> (row_tuple.h:246-252); strings copied into variable_values.
  switch (c.type) {
    case BOOLEAN: rt->fixed[slot] = {static_cast<uint64_t>(c.b[r] ? 1 : 0), 0}; break;
    case INT64:
    case TIME64NS: rt->fixed[slot] = {static_cast<uint64_t>(c.i[r]), 0}; break;
    case FLOAT64: {
      uint64_t bits;
      std::memcpy(&bits, &c.f[r], 8);
      rt->fixed[slot] = {bits, 0};
      break;
    }
    case UINT128: rt->fixed[slot] = {c.u[r].lo, c.u[r].hi}; break;
    case STRING: rt->strs[slot] = c.s[r]; break;
    default: break;
  }
}

static void AppendTupleValue(Col* out, const RowTuple& rt, size_t slot) {
  switch (out->type) {
    case BOOLEAN: out->b.push_back(static_cast<uint8_t>(rt.fixed[slot][0])); break;
    case INT64:
    case TIME64NS: out->i.push_back(static_cast<int64_t>(rt.fixed[slot][0])); break;
    case FLOAT64: {
      double d;
      std::memcpy(&d, &rt.fixed[slot][0], 8);
      out->f.push_back(d);
      break;
    }
    case UINT128: out->u.push_back(U128{rt.fixed[slot][0], rt.fixed[slot][1]}); break;
    case STRING: out->s.push_back(rt.strs[slot]); break;
    default: break;
  }
}

constexpr size_t kAggCompactionThreshold = 512;  // agg_node.cc:43

// AggNode (agg_node.cc:88-542).
struct AggNode : ExecNode {
  std::vector<int64_t> groups;
  std::vector<DT> group_types;
  std::vector<Expr> values;
  bool windowed = false;
  // plan.proto:250-257.  partial && !finalize: emit groups + serialized_expressions (STRING,
  // operators.cc:251-257), every UDA's Serialize() back to back in plan order.  !partial &&
  // finalize: the input is groups + serialized_expressions; each row's states are
  // Deserialize()d and Merge()d into the group's UDAs, then finalized.  Anything else: a full
  // aggregate (the reference's AggNode, which ignores both flags).
  bool partial_agg = false, finalize_results = false;
  bool EmitStates() const { return partial_agg && !finalize_results; }
  bool MergeStates() const { return !partial_agg && finalize_results; }
  int64_t state_col = -1;
  std::vector<size_t> state_off;
  size_t state_rec = 0;
  std::vector<DT> in_types;
  // CreateColumnMapping (agg_node.cc:483-507)
  std::map<int64_t, size_t> plan_to_stored;
  std::vector<int64_t> stored_to_plan;

  struct UDAInfo {
    std::unique_ptr<UDA> uda;
    const UDADef* def;
  };
  struct AggHashValue {
    std::vector<UDAInfo> udas;
    std::vector<ColPtr> agg_cols;
  };
  std::unordered_map<RowTuple*, AggHashValue*, RowTupleHash, RowTupleEq> map;
  std::vector<std::unique_ptr<RowTuple>> tuple_pool;
  std::vector<std::unique_ptr<AggHashValue>> value_pool;
  std::vector<UDAInfo> no_group_udas;
  std::vector<const UDADef*> defs;

  void Init() {
    for (auto& v : values) {
      std::vector<DT> types;
      for (auto& a : v.init_args) types.push_back(a.type);
      if (MergeStates()) {
        // The arguments name the pre-split input's columns; the plan's args_data_types give
        // the registry key (scalar_expression.cc:337-346).
        if (v.arg_types.size() != v.args.size()) throw Error(INVALID_ARGUMENT, "finalize agg needs args_data_types");
        for (auto t : v.arg_types) types.push_back(t);
      } else {
        for (auto& a : v.args) types.push_back(ExprType(a, in_types));
      }
      const UDADef* d = UDARegistry::Get().Find(v.name, types);
      if (!d) throw Error(NOT_FOUND, "no UDA " + Key(v.name, types));
      defs.push_back(d);
      if (EmitStates() || MergeStates()) {
        auto probe = d->make(v.init_args);
        if (!probe->SupportsPartial()) throw Error(UNIMPLEMENTED, "UDA " + v.name + " does not support partial aggregation");
        state_off.push_back(state_rec);
        state_rec += probe->Serialize().size();
      }
      if (MergeStates()) continue;
      for (auto& a : v.args) {
        if (a.kind == Expr::kColumn && !plan_to_stored.count(a.col_index)) {
          plan_to_stored[a.col_index] = stored_to_plan.size();
          stored_to_plan.push_back(a.col_index);
        }
      }
    }
    for (auto g : groups) group_types.push_back(in_types.at(g));
    if (MergeStates()) {
      state_col = static_cast<int64_t>(in_types.size()) - 1;
      if (state_col < 0 || in_types[state_col] != STRING || std::count(groups.begin(), groups.end(), state_col))
        throw Error(INVALID_ARGUMENT, "finalize agg input must end in the serialized_expressions STRING column");
    }
    if (groups.empty()) no_group_udas = MakeUDAs();
  }

  // Deserialize + Merge one row's states into udas (the finalize half of a split agg).
  void MergeRow(std::vector<UDAInfo>& udas, const std::string& st) {
    if (st.size() != state_rec) throw Error(INVALID_ARGUMENT, "serialized_expressions of " + std::to_string(st.size()) + " bytes, expected " + std::to_string(state_rec));
    for (size_t i = 0; i < values.size(); ++i) {
      auto tmp = defs[i]->make(values[i].init_args);
      tmp->Deserialize(st.data() + state_off[i]);
      udas[i].uda->Merge(*tmp);
    }
  }
  std::string SerializeAll(const std::vector<UDAInfo>& udas) const {
    std::string s;
    for (auto& u : udas) s += u.uda->Serialize();
    return s;
  }

  std::vector<UDAInfo> MakeUDAs() {
    std::vector<UDAInfo> v;
    for (size_t i = 0; i < values.size(); ++i) v.push_back(UDAInfo{defs[i]->make(values[i].init_args), defs[i]});
    return v;
  }

  // EvaluateAggHashValue (agg_node.cc:434-481): per UDA, ExecBatchUpdate over the buffered rows.
  void EvaluateAggHashValue(AggHashValue* val) {
    size_t n = val->agg_cols.empty() ? 0 : val->agg_cols[0]->size();
    for (size_t i = 0; i < values.size(); ++i) {
      std::vector<ColPtr> kids;
      std::vector<const Col*> raw;
      for (auto& a : values[i].args) {
        if (a.kind == Expr::kConst) kids.push_back(ConstCol(a.value, n));
        else kids.push_back(val->agg_cols[plan_to_stored[a.col_index]]);
        raw.push_back(kids.back().get());
      }
      for (size_t r = 0; r < n; ++r) val->udas[i].uda->Update(raw, r);
    }
    for (auto& c : val->agg_cols) c->clear();
  }

  void Emit(const RowBatch& rb) {
    RowBatch out;
    out.eow = rb.eow;
    out.eos = rb.eos;
    if (groups.empty()) {
      out.num_rows = 1;
      if (EmitStates()) {
        auto c = std::make_shared<Col>(STRING);
        c->s.push_back(SerializeAll(no_group_udas));
        out.cols.push_back(c);
        Send(out);
        no_group_udas = MakeUDAs();
        return;
      }
      for (size_t i = 0; i < values.size(); ++i) {
        auto c = std::make_shared<Col>(defs[i]->out);
        no_group_udas[i].uda->Finalize(c.get());
        out.cols.push_back(c);
      }
      Send(out);
      no_group_udas = MakeUDAs();  // ClearAggState
      return;
    }
    // ConvertAggHashMapToRowBatch (agg_node.cc:303-349): groups then values.
    out.num_rows = static_cast<int64_t>(map.size());
    std::vector<ColPtr> gcols, vcols;
    for (auto t : group_types) gcols.push_back(std::make_shared<Col>(t));
    if (EmitStates()) vcols.push_back(std::make_shared<Col>(STRING));
    else
      for (size_t i = 0; i < values.size(); ++i) vcols.push_back(std::make_shared<Col>(defs[i]->out));
    for (auto& kv : map) {
      for (size_t g = 0; g < groups.size(); ++g) AppendTupleValue(gcols[g].get(), *kv.first, g);
      if (!MergeStates()) EvaluateAggHashValue(kv.second);
      if (EmitStates()) vcols[0]->s.push_back(SerializeAll(kv.second->udas));
      else
        for (size_t i = 0; i < values.size(); ++i) kv.second->udas[i].uda->Finalize(vcols[i].get());
    }
    for (auto& c : gcols) out.cols.push_back(c);
    for (auto& c : vcols) out.cols.push_back(c);
    Send(out);
    map.clear();  // ClearAggState
    tuple_pool.clear();
    value_pool.clear();
  }

  void ConsumeNext(const RowBatch& rb, size_t) override {
    bool ready = rb.eos || (rb.eow && windowed);  // ReadyToEmitBatches (agg_node.cc:169-171)
    if (groups.empty()) {
      if (MergeStates()) {
        for (int64_t r = 0; r < rb.num_rows; ++r) MergeRow(no_group_udas, rb.cols.at(state_col)->s[r]);
        if (ready) Emit(rb);
        return;
      }
      // AggregateGroupByNone (agg_node.cc:182-207): ExecBatchUpdateArrow directly.
      for (size_t i = 0; i < values.size(); ++i) {
        std::vector<ColPtr> kids;
        std::vector<const Col*> raw;
        for (auto& a : values[i].args) {
          kids.push_back(a.kind == Expr::kConst ? ConstCol(a.value, rb.num_rows) : rb.cols.at(a.col_index));
          raw.push_back(kids.back().get());
        }
        for (int64_t r = 0; r < rb.num_rows; ++r) no_group_udas[i].uda->Update(raw, r);
      }
      if (ready) Emit(rb);
      return;
    }
    // ExtractRowTupleForBatch + HashRowBatch (agg_node.cc:209-271).
    std::vector<AggHashValue*> row_vals(rb.num_rows);
    for (int64_t r = 0; r < rb.num_rows; ++r) {
      auto rt = std::make_unique<RowTuple>();
      rt->types = group_types;
      rt->fixed.assign(groups.size(), {0, 0});
      rt->strs.assign(groups.size(), std::string());
      for (size_t g = 0; g < groups.size(); ++g) ExtractIntoRowTuple(rt.get(), *rb.cols.at(groups[g]), g, r);
      auto it = map.find(rt.get());
      AggHashValue* val;
      if (it == map.end()) {
        auto v = std::make_unique<AggHashValue>();
        v->udas = MakeUDAs();
        for (auto pi : stored_to_plan) v->agg_cols.push_back(std::make_shared<Col>(in_types[pi]));
        val = v.get();
        map[rt.get()] = val;
        tuple_pool.push_back(std::move(rt));
        value_pool.push_back(std::move(v));
      } else {
        val = it->second;
      }
      row_vals[r] = val;
    }
    if (MergeStates()) {
      for (int64_t r = 0; r < rb.num_rows; ++r) MergeRow(row_vals[r]->udas, rb.cols.at(state_col)->s[r]);
      if (ready) Emit(rb);
      return;
    }
    for (size_t s = 0; s < stored_to_plan.size(); ++s) {
      const Col& in = *rb.cols.at(stored_to_plan[s]);
      for (int64_t r = 0; r < rb.num_rows; ++r) row_vals[r]->agg_cols[s]->append_from(in, r);
    }
    // EvaluatePartialAggregates (agg_node.cc:273-286).
    if (!values.empty() && !stored_to_plan.empty()) {
      for (int64_t r = 0; r < rb.num_rows; ++r) {
        if (row_vals[r]->agg_cols[0]->size() > kAggCompactionThreshold) EvaluateAggHashValue(row_vals[r]);
      }
    }
    if (ready) Emit(rb);
  }
};

// LimitNode::ConsumeNextImpl (limit_node.cc:55-95): whole batches while they fit, then the
// batch that reaches the limit sliced to [0, remainder) with eow / eos, the abortable sources
// stopped (ExecState::StopSource), and every later batch dropped.
struct LimitNode : ExecNode {
  int64_t limit = 0, processed = 0;
  bool reached = false;
  std::vector<int64_t> selected;
  std::vector<uint64_t> abortable;
  std::set<uint64_t>* stopped = nullptr;
  void ConsumeNext(const RowBatch& rb, size_t) override {
    if (reached) return;
    const int64_t remainder = limit - processed;
    RowBatch out;
    if (remainder > rb.num_rows) {
      out.num_rows = rb.num_rows;
      for (int64_t ci : selected) out.cols.push_back(rb.cols.at(ci));
      processed += rb.num_rows;
      out.eow = rb.eow;
      out.eos = rb.eos;
      Send(out);
      return;
    }
    out.num_rows = remainder;
    for (int64_t ci : selected) {
      const Col& in = *rb.cols.at(ci);
      auto c = std::make_shared<Col>(in.type);
      for (int64_t r = 0; r < remainder; ++r) c->append_from(in, static_cast<size_t>(r));
      out.cols.push_back(c);
    }
    out.eow = out.eos = true;
    processed += remainder;
    reached = true;
    for (uint64_t id : abortable) stopped->insert(id);
    Send(out);
  }
};

struct SinkNode : ExecNode {
  std::string name;
  std::vector<RowBatch> batches;
  void ConsumeNext(const RowBatch& rb, size_t) override { batches.push_back(rb); }
};

struct SourceNode : ExecNode {
  uint64_t id = 0;
  std::vector<RowBatch> batches;
  bool explicit_flags = false;
  size_t next = 0;
  std::vector<int64_t> col_idxs;
  bool HasBatchesRemaining() const { return next <= batches.size() && !done; }
  bool done = false;
  void ConsumeNext(const RowBatch&, size_t) override {}
  // MemorySourceNode::GenerateNextImpl (memory_source_node.cc:92-124).
  void GenerateNext() {
    if (next >= batches.size()) {
      RowBatch z;
      z.num_rows = 0;
      for (auto t : out_types) z.cols.push_back(std::make_shared<Col>(t));
      z.eow = z.eos = true;
      done = true;
      Send(z);
      return;
    }
    RowBatch rb;
    const RowBatch& src = batches[next++];
    rb.num_rows = src.num_rows;
    for (auto ci : col_idxs) rb.cols.push_back(src.cols.at(ci));
    if (explicit_flags) {
      rb.eow = src.eow;
      rb.eos = src.eos;
      // Like ExecNodeTester, every given batch is delivered (even after an eos).
      if (next == batches.size()) done = true;
      Send(rb);
      return;
    }
    if (next == batches.size()) {
      rb.eow = rb.eos = true;
      done = true;
    }
    Send(rb);
  }
};

// EquijoinNode (equijoin_node.cc:53-470).  The probe table is the left parent when the output
// has a "time_" column taken from parent 0 (order_by_time, operators.cc:531-541,639-645 and
// equijoin_node.cc:63-69), otherwise the right parent.  Build rows are buffered per key in
// insertion order (build_buffer_), probe batches are buffered until the build side reaches
// eos, then every probe row emits its matches in build order.  Output batches hold
// rows_per_batch rows (default 1024); the pending batch is sent when the next one is started,
// a partial batch is cut when the probe side ends and after the unmatched build rows
// (FlushChunkedRows / NextOutputBatch), and the last batch carries eow/eos.
struct EquijoinNode : ExecNode {
  int type = 0;  // 0 INNER, 1 LEFT_OUTER, 3 FULL_OUTER
  std::vector<int64_t> left_keys, right_keys, build_keys, probe_keys;
  std::vector<std::pair<int64_t, int64_t>> outputs;  // (parent, column)
  std::vector<std::string> column_names;
  std::vector<DT> left_types, right_types;
  bool probe_is_left = false;
  int64_t rows_per_batch = 1024;
  bool emit_unmatched_build = false, emit_unmatched_probe = false;
  std::vector<std::string> key_order;                // build keys in first-insertion order
  std::map<std::string, std::vector<std::pair<RowBatch, size_t>>> build;  // key -> rows
  std::set<std::string> probed;
  std::vector<RowBatch> probe_buf;
  bool build_eos = false, probe_eos = false;
  // current output batch under construction
  std::vector<ColPtr> cur;
  int64_t cur_rows = 0;
  std::unique_ptr<RowBatch> pending;

  void Init() {
    for (size_t i = 0; i < column_names.size() && i < outputs.size(); ++i)
      if (column_names[i] == "time_") {
        probe_is_left = outputs[i].first == 0;
        // JoinOperator::Init (operators.cc:593-603)
        if (type == 3) throw Error(INVALID_ARGUMENT, "For time ordered joins, full outer join is not supported.");
        if (type == 1 && !probe_is_left)
          throw Error(INVALID_ARGUMENT, "For time ordered joins, left join is only supported when time_ comes from the left table.");
        break;
      }
    switch (type) {
      case 0: break;
      case 1:
        emit_unmatched_build = !probe_is_left;
        emit_unmatched_probe = probe_is_left;
        break;
      case 3: emit_unmatched_build = emit_unmatched_probe = true; break;
      default: throw Error(INTERNAL, "EquijoinNode: Unknown Join Type");
    }
    build_keys = probe_is_left ? right_keys : left_keys;
    probe_keys = probe_is_left ? left_keys : right_keys;
    if (rows_per_batch <= 0) rows_per_batch = 1024;
    NewBatch();
  }
  static std::string Key(const RowBatch& rb, const std::vector<int64_t>& keys, size_t r) {
    std::string k;
    for (int64_t c : keys) {
      const Col& col = *rb.cols.at(c);
      switch (col.type) {
        case STRING: {
          const std::string& s = col.s[r];
          uint64_t n = s.size();
          k.append(reinterpret_cast<const char*>(&n), 8);
          k += s;
          break;
        }
        case UINT128: k.append(reinterpret_cast<const char*>(&col.u[r]), 16); break;
        case FLOAT64: k.append(reinterpret_cast<const char*>(&col.f[r]), 8); break;
        case BOOLEAN: k.push_back(static_cast<char>(col.b[r])); break;
        default: k.append(reinterpret_cast<const char*>(&col.i[r]), 8); break;
      }
    }
    return k;
  }
  void NewBatch() {
    cur.clear();
    for (auto t : out_types) cur.push_back(std::make_shared<Col>(t));
    cur_rows = 0;
  }
  static void AppendDefault(Col* c) {
    switch (c->type) {
      case BOOLEAN: c->b.push_back(0); break;
      case INT64:
      case TIME64NS: c->i.push_back(0); break;
      case FLOAT64: c->f.push_back(0.0); break;
      case STRING: c->s.emplace_back(); break;
      case UINT128: c->u.push_back(U128{}); break;
      default: break;
    }
  }
  // NextOutputBatch: the pending batch goes out, the finished one becomes pending.
  void CutBatch() {
    if (cur_rows == 0) return;
    auto rb = std::make_unique<RowBatch>();
    rb->cols = cur;
    rb->num_rows = cur_rows;
    if (pending) Send(*pending);
    pending = std::move(rb);
    NewBatch();
  }
  void Emit(const RowBatch* probe_rb, size_t pr, const RowBatch* build_rb, size_t br) {
    for (size_t o = 0; o < outputs.size(); ++o) {
      const bool from_build = (outputs[o].first == 0) != probe_is_left;
      const RowBatch* src = from_build ? build_rb : probe_rb;
      const size_t row = from_build ? br : pr;
      if (src) cur[o]->append_from(*src->cols.at(outputs[o].second), row);
      else AppendDefault(cur[o].get());
    }
    if (++cur_rows == rows_per_batch) CutBatch();
  }
  void DoProbe(const RowBatch& rb) {
    if (rb.eos) probe_eos = true;
    for (size_t r = 0; r < static_cast<size_t>(rb.num_rows); ++r) {
      auto it = build.find(Key(rb, probe_keys, r));
      if (it == build.end()) {
        if (emit_unmatched_probe) Emit(&rb, r, nullptr, 0);
        continue;
      }
      probed.insert(it->first);
      for (auto& m : it->second) Emit(&rb, r, &m.first, m.second);
    }
    if (probe_eos) CutBatch();
  }
  void ConsumeNext(const RowBatch& rb, size_t parent_index) override {
    if ((parent_index == 0) == probe_is_left) {
      if (!build_eos) probe_buf.push_back(rb);
      else DoProbe(rb);
    } else {
      if (rb.eos) build_eos = true;
      for (size_t r = 0; r < static_cast<size_t>(rb.num_rows); ++r) {
        std::string k = Key(rb, build_keys, r);
        auto it = build.find(k);
        if (it == build.end()) {
          key_order.push_back(k);
          it = build.emplace(k, std::vector<std::pair<RowBatch, size_t>>()).first;
        }
        it->second.emplace_back(rb, r);
      }
      if (build_eos) {
        for (auto& b : probe_buf) DoProbe(b);
        probe_buf.clear();
      }
    }
    if (build_eos && probe_eos) {
      if (emit_unmatched_build) {
        for (auto& k : key_order) {
          if (probed.count(k)) continue;
          for (auto& m : build[k]) Emit(nullptr, 0, &m.first, m.second);
        }
        CutBatch();
      }
      if (!pending) {
        pending = std::make_unique<RowBatch>();
        pending->num_rows = 0;
        for (auto t : out_types) pending->cols.push_back(std::make_shared<Col>(t));
      }
      pending->eow = pending->eos = true;
      Send(*pending);
      pending.reset();
    }
  }
};

/*********************************************************************************************
 * Plan driver (exec_graph.cc:52-331).
 *********************************************************************************************/
struct TableIn {
  std::vector<std::string> names;
  std::vector<DT> types;
  std::vector<RowBatch> batches;
  bool explicit_flags = false;
};

struct Graph {
  std::map<uint64_t, std::unique_ptr<ExecNode>> nodes;
  std::vector<SourceNode*> sources;
  std::vector<SinkNode*> sinks;
  std::set<uint64_t> stopped;  // ExecState source_id_to_keep_running_map_ == false

  void Build(const Json& plan, const std::map<std::string, TableIn>& tables) {
    const Json& frags = plan["nodes"];
    for (size_t fi = 0; fi < frags.size(); ++fi) BuildFragment(frags.at(fi), tables);
  }

  void BuildFragment(const Json& frag, const std::map<std::string, TableIn>& tables) {
    // Topological order from the fragment DAG (plan_fragment.cc:108-118).
    std::map<uint64_t, std::vector<uint64_t>> parents;
    std::vector<uint64_t> order;
    const Json& dag_nodes = frag["dag"]["nodes"];
    std::map<uint64_t, int> indeg;
    std::map<uint64_t, std::vector<uint64_t>> kids;
    for (size_t i = 0; i < dag_nodes.size(); ++i) {
      uint64_t id = dag_nodes.at(i)["id"].as_u64();
      indeg[id];
      for (size_t p = 0; p < dag_nodes.at(i)["sortedParents"].size(); ++p) {
        uint64_t pid = dag_nodes.at(i)["sortedParents"].at(p).as_u64();
        parents[id].push_back(pid);
        indeg[id]++;
        kids[pid].push_back(id);
      }
    }
    std::vector<uint64_t> ready;
    for (auto& kv : indeg)
      if (kv.second == 0) ready.push_back(kv.first);
    while (!ready.empty()) {
      uint64_t id = ready.front();
      ready.erase(ready.begin());
      order.push_back(id);
      for (auto k : kids[id])
        if (--indeg[k] == 0) ready.push_back(k);
    }
    std::map<uint64_t, const Json*> ops;
    const Json& pn = frag["nodes"];
    for (size_t i = 0; i < pn.size(); ++i) ops[pn.at(i)["id"].as_u64()] = &pn.at(i)["op"];

    for (uint64_t id : order) {
      const Json& op = *ops.at(id);
      std::vector<DT> in;
      if (!parents[id].empty()) in = nodes.at(parents[id][0])->out_types;
      std::unique_ptr<ExecNode> node;
      if (op.has("memSourceOp")) {
        const Json& m = op["memSourceOp"];
        auto s = std::make_unique<SourceNode>();
        auto it = tables.find(m["name"].as_str());
        if (it == tables.end()) throw Error(NOT_FOUND, "Table '" + m["name"].as_str() + "' not found");
        s->batches = it->second.batches;
        s->explicit_flags = it->second.explicit_flags;
        if (m.has("startTime") || m.has("stopTime")) {
          // Table::Cursor range (table.cc:56-95, 310-336): [first row with time_ >= start,
          // first row with time_ > stop) of the time-ordered table.
          int64_t tc = -1;
          for (size_t c = 0; c < it->second.names.size(); ++c)
            if (it->second.names[c] == "time_") tc = static_cast<int64_t>(c);
          if (tc < 0) throw Error(INVALID_ARGUMENT, "table has no time_ column for a time-bounded source");
          const bool hs = m.has("startTime"), he = m.has("stopTime");
          const int64_t t0 = hs ? m["startTime"].as_i64() : 0, t1 = he ? m["stopTime"].as_i64() : 0;
          std::vector<RowBatch> kept;
          for (const RowBatch& b : s->batches) {
            const std::vector<int64_t>& tv = b.cols.at(tc)->i;
            RowBatch nb;
            for (auto& c : b.cols) nb.cols.push_back(std::make_shared<Col>(c->type));
            for (int64_t r = 0; r < b.num_rows; ++r) {
              if ((hs && tv[r] < t0) || (he && tv[r] > t1)) continue;
              for (size_t c = 0; c < b.cols.size(); ++c) nb.cols[c]->append_from(*b.cols[c], static_cast<size_t>(r));
              ++nb.num_rows;
            }
            if (nb.num_rows > 0) kept.push_back(std::move(nb));
          }
          s->batches = std::move(kept);
          s->explicit_flags = false;
        }
        for (size_t c = 0; c < m["columnIdxs"].size(); ++c) s->col_idxs.push_back(m["columnIdxs"].at(c).as_i64());
        if (s->col_idxs.empty())
          for (size_t c = 0; c < it->second.types.size(); ++c) s->col_idxs.push_back(static_cast<int64_t>(c));
        for (auto c : s->col_idxs) s->out_types.push_back(it->second.types.at(c));
        s->id = id;
        sources.push_back(s.get());
        node = std::move(s);
      } else if (op.has("filterOp")) {
        const Json& f = op["filterOp"];
        auto n = std::make_unique<FilterNode>();
        n->pred = ParseScalarExpr(f["expression"]);
        for (size_t c = 0; c < f["columns"].size(); ++c) {
          int64_t ci = f["columns"].at(c)["index"].as_i64();
          n->selected.push_back(ci);
          n->out_types.push_back(in.at(ci));
        }
        if (ExprType(n->pred, in) != BOOLEAN) throw Error(INVALID_ARGUMENT, "filter predicate must be BOOLEAN");
        node = std::move(n);
      } else if (op.has("mapOp")) {
        const Json& m = op["mapOp"];
        auto n = std::make_unique<MapNode>();
        for (size_t c = 0; c < m["expressions"].size(); ++c) {
          n->exprs.push_back(ParseScalarExpr(m["expressions"].at(c)));
          n->out_types.push_back(ExprType(n->exprs.back(), in));
        }
        node = std::move(n);
      } else if (op.has("aggOp")) {
        const Json& a = op["aggOp"];
        auto n = std::make_unique<AggNode>();
        n->in_types = in;
        n->windowed = a["windowed"].as_bool();
        n->partial_agg = a.has("partialAgg") && a["partialAgg"].as_bool();
        n->finalize_results = a.has("finalizeResults") && a["finalizeResults"].as_bool();
        for (size_t g = 0; g < a["groups"].size(); ++g) n->groups.push_back(a["groups"].at(g)["index"].as_i64());
        for (size_t v = 0; v < a["values"].size(); ++v) n->values.push_back(ParseAggExpr(a["values"].at(v)));
        n->Init();
        for (auto g : n->groups) n->out_types.push_back(in.at(g));
        if (n->EmitStates()) n->out_types.push_back(STRING);
        else
          for (auto* d : n->defs) n->out_types.push_back(d->out);
        node = std::move(n);
      } else if (op.has("joinOp")) {
        const Json& j = op["joinOp"];
        auto n = std::make_unique<EquijoinNode>();
        if (parents[id].size() != 2) throw Error(INVALID_ARGUMENT, "Join operator expects a two input relations");
        n->left_types = nodes.at(parents[id][0])->out_types;
        n->right_types = nodes.at(parents[id][1])->out_types;
        const std::string jt = j["type"].kind == Json::kString ? j["type"].as_str() : std::string();
        n->type = jt.empty() ? static_cast<int>(j["type"].as_i64()) : (jt == "INNER" ? 0 : jt == "LEFT_OUTER" ? 1 : jt == "FULL_OUTER" ? 3 : -1);
        for (size_t c = 0; c < j["equalityConditions"].size(); ++c) {
          const Json& e = j["equalityConditions"].at(c);
          n->left_keys.push_back(e["leftColumnIndex"].as_i64());
          n->right_keys.push_back(e["rightColumnIndex"].as_i64());
          if (n->left_types.at(n->left_keys.back()) != n->right_types.at(n->right_keys.back()))
            throw Error(INVALID_ARGUMENT, "join key types differ");
        }
        for (size_t c = 0; c < j["outputColumns"].size(); ++c) {
          const Json& o = j["outputColumns"].at(c);
          const int64_t pi = o["parentIndex"].as_i64(), ci = o["columnIndex"].as_i64();
          n->outputs.push_back({pi, ci});
          n->out_types.push_back((pi == 0 ? n->left_types : n->right_types).at(ci));
        }
        for (size_t c = 0; c < j["columnNames"].size(); ++c) n->column_names.push_back(j["columnNames"].at(c).as_str());
        n->rows_per_batch = j["rowsPerBatch"].as_i64();
        n->Init();
        node = std::move(n);
      } else if (op.has("limitOp")) {
        const Json& l = op["limitOp"];
        auto n = std::make_unique<LimitNode>();
        n->limit = l["limit"].as_i64();
        for (size_t c = 0; c < l["columns"].size(); ++c) {
          const int64_t ci = l["columns"].at(c)["index"].as_i64();
          n->selected.push_back(ci);
          n->out_types.push_back(in.at(ci));
        }
        for (size_t c = 0; c < l["abortableSrcs"].size(); ++c) n->abortable.push_back(l["abortableSrcs"].at(c).as_u64());
        n->stopped = &stopped;
        node = std::move(n);
      } else if (op.has("memSinkOp") || op.has("grpcSinkOp")) {
        auto n = std::make_unique<SinkNode>();
        if (op.has("memSinkOp")) n->name = op["memSinkOp"]["name"].as_str();
        else n->name = op["grpcSinkOp"]["outputTable"]["tableName"].as_str();
        n->out_types = in;
        sinks.push_back(n.get());
        node = std::move(n);
      } else {
        throw Error(UNIMPLEMENTED, "operator not supported by the restatement");
      }
      for (size_t p = 0; p < parents[id].size(); ++p) {
        nodes.at(parents[id][p])->children.push_back(node.get());
        nodes.at(parents[id][p])->child_parent_index.push_back(p);
      }
      nodes[id] = std::move(node);
    }
  }

  // ExecuteSources (exec_graph.cc:177-289): up to 10 consecutive GenerateNext per source.
  void Execute() {
    std::vector<SourceNode*> running = sources;
    while (!running.empty()) {
      std::vector<SourceNode*> still;
      for (auto* s : running) {
        for (int i = 0; i < 10 && !s->done && !stopped.count(s->id); ++i) s->GenerateNext();
        if (!s->done && !stopped.count(s->id)) still.push_back(s);
      }
      running = still;
    }
  }
};

// Given batches are re-sliced into RowBatches of batch_rows rows when batch_rows > 0 (the
// carnot_executable --rowbatch_size knob, carnot_executable.cc:46-47).  A column given with no
// buffers (values, offsets and data all null) is never read by the plan: it stays empty.
static std::map<std::string, TableIn> ImportTables(int32_t ntables, const oracle_table* tables, int64_t batch_rows = 0) {
  std::map<std::string, TableIn> out;
  for (int32_t t = 0; t < ntables; ++t) {
    const oracle_table& ot = tables[t];
    TableIn ti;
    for (int32_t c = 0; c < ot.ncols; ++c) {
      ti.names.push_back(ot.col_names ? ot.col_names[c] : std::to_string(c));
      ti.types.push_back(static_cast<DT>(ot.col_types[c]));
    }
    for (int32_t b = 0; b < ot.nbatches; ++b) {
      int64_t n = -1;
      for (int32_t c = 0; c < ot.ncols; ++c) {
        const oracle_column& oc = ot.cols[static_cast<size_t>(b) * ot.ncols + c];
        if (oc.values || oc.offsets || oc.data) n = oc.length;
      }
      if (n < 0) n = 0;
      const int64_t step = (batch_rows > 0 && !ot.batch_flags) ? batch_rows : std::max<int64_t>(n, 1);
      for (int64_t r0 = 0; r0 < n || (n == 0 && r0 == 0); r0 += step) {
        const int64_t r1 = std::min(n, r0 + step);
        RowBatch rb;
        rb.num_rows = r1 - r0;
        for (int32_t c = 0; c < ot.ncols; ++c) {
          const oracle_column& oc = ot.cols[static_cast<size_t>(b) * ot.ncols + c];
          auto col = std::make_shared<Col>(static_cast<DT>(oc.type));
          const bool present = oc.values || oc.offsets || oc.data;
          if (present) {
            switch (col->type) {
              case BOOLEAN: col->b.assign(static_cast<const uint8_t*>(oc.values) + r0, static_cast<const uint8_t*>(oc.values) + r1); break;
              case INT64:
              case TIME64NS: col->i.assign(static_cast<const int64_t*>(oc.values) + r0, static_cast<const int64_t*>(oc.values) + r1); break;
              case FLOAT64: col->f.assign(static_cast<const double*>(oc.values) + r0, static_cast<const double*>(oc.values) + r1); break;
              case UINT128: {
                const uint64_t* p = static_cast<const uint64_t*>(oc.values);
                for (int64_t r = r0; r < r1; ++r) col->u.push_back(U128{p[2 * r], p[2 * r + 1]});
                break;
              }
              case STRING:
                col->s.reserve(r1 - r0);
                for (int64_t r = r0; r < r1; ++r)
                  col->s.emplace_back(reinterpret_cast<const char*>(oc.data) + oc.offsets[r], oc.offsets[r + 1] - oc.offsets[r]);
                break;
              default: throw Error(INVALID_ARGUMENT, "bad column type");
            }
          }
          rb.cols.push_back(col);
        }
        if (ot.batch_flags) {
          rb.eow = (ot.batch_flags[b] & 1) != 0;
          rb.eos = (ot.batch_flags[b] & 2) != 0;
          ti.explicit_flags = true;
        }
        ti.batches.push_back(std::move(rb));
        if (n == 0) break;
      }
    }
    out[ot.name] = std::move(ti);
  }
  return out;
}

// PXRB serialization (parsed by tests/pxrb.py).
struct Writer {
  std::vector<uint8_t> buf;
  template <typename T>
  void put(T v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    buf.insert(buf.end(), p, p + sizeof(T));
  }
  void bytes(const void* p, size_t n) { buf.insert(buf.end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n); }
};

static void WriteBatch(Writer* w, const RowBatch& rb) {
  w->put<int64_t>(rb.num_rows);
  w->put<uint8_t>(rb.eow);
  w->put<uint8_t>(rb.eos);
  w->put<uint16_t>(0);
  w->put<uint32_t>(static_cast<uint32_t>(rb.cols.size()));
  for (auto& c : rb.cols) {
    w->put<int32_t>(c->type);
    switch (c->type) {
      case BOOLEAN: w->bytes(c->b.data(), c->b.size()); break;
      case INT64:
      case TIME64NS: w->bytes(c->i.data(), c->i.size() * 8); break;
      case FLOAT64: w->bytes(c->f.data(), c->f.size() * 8); break;
      case UINT128:
        for (auto& u : c->u) { w->put(u.lo); w->put(u.hi); }
        break;
      case STRING: {
        int32_t off = 0;
        w->put<int32_t>(0);
        for (auto& s : c->s) { off += static_cast<int32_t>(s.size()); w->put<int32_t>(off); }
        for (auto& s : c->s) w->bytes(s.data(), s.size());
        break;
      }
      default: break;
    }
  }
}

}  // namespace oracle

using namespace oracle;

static void SetErr(char* errbuf, int32_t errlen, const std::string& m) {
  if (errbuf && errlen > 0) {
    std::snprintf(errbuf, static_cast<size_t>(errlen), "%s", m.c_str());
  }
}

extern "C" int32_t oracle_execute_plan_rebatched(const char* plan_json, int32_t ntables, const oracle_table* tables,
                                                 int64_t batch_rows, double* seconds, uint8_t** out, int64_t* out_len,
                                                 char* errbuf, int32_t errlen) {
  try {
    Json plan = ParseJson(plan_json);
    auto tbl = ImportTables(ntables, tables, batch_rows);
    Graph g;
    g.Build(plan, tbl);
    auto t0 = std::chrono::steady_clock::now();
    g.Execute();
    auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    Writer w;
    w.put<uint32_t>(0x42525850u);  // "PXRB"
    w.put<uint32_t>(static_cast<uint32_t>(g.sinks.size()));
    for (auto* s : g.sinks) {
      w.put<uint32_t>(static_cast<uint32_t>(s->name.size()));
      w.bytes(s->name.data(), s->name.size());
      w.put<uint32_t>(static_cast<uint32_t>(s->batches.size()));
      for (auto& rb : s->batches) WriteBatch(&w, rb);
    }
    *out_len = static_cast<int64_t>(w.buf.size());
    *out = static_cast<uint8_t*>(std::malloc(w.buf.size()));
    std::memcpy(*out, w.buf.data(), w.buf.size());
    return OK;
  } catch (const Error& e) {
    SetErr(errbuf, errlen, e.what());
    return e.code;
  } catch (const std::exception& e) {
    SetErr(errbuf, errlen, e.what());
    return INTERNAL;
  }
}

extern "C" int32_t oracle_execute_plan(const char* plan_json, int32_t ntables, const oracle_table* tables,
                                       uint8_t** out, int64_t* out_len, char* errbuf, int32_t errlen) {
  return oracle_execute_plan_rebatched(plan_json, ntables, tables, 0, nullptr, out, out_len, errbuf, errlen);
}

extern "C" int32_t oracle_execute_plan_timed(const char* plan_json, int32_t ntables, const oracle_table* tables,
                                             double* seconds, int64_t* out_rows, char* errbuf, int32_t errlen) {
  return oracle_execute_plan_timed_rebatched(plan_json, ntables, tables, 0, seconds, out_rows, errbuf, errlen);
}

extern "C" int32_t oracle_execute_plan_timed_rebatched(const char* plan_json, int32_t ntables, const oracle_table* tables,
                                                       int64_t batch_rows, double* seconds, int64_t* out_rows, char* errbuf,
                                                       int32_t errlen) {
  try {
    Json plan = ParseJson(plan_json);
    auto tbl = ImportTables(ntables, tables, batch_rows);
    Graph g;
    g.Build(plan, tbl);
    auto t0 = std::chrono::steady_clock::now();
    g.Execute();
    auto t1 = std::chrono::steady_clock::now();
    *seconds = std::chrono::duration<double>(t1 - t0).count();
    int64_t rows = 0;
    for (auto* s : g.sinks)
      for (auto& rb : s->batches) rows += rb.num_rows;
    *out_rows = rows;
    return OK;
  } catch (const Error& e) {
    SetErr(errbuf, errlen, e.what());
    return e.code;
  } catch (const std::exception& e) {
    SetErr(errbuf, errlen, e.what());
    return INTERNAL;
  }
}

extern "C" void oracle_free(uint8_t* p) { std::free(p); }

static const double kQs[7] = {0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99};

extern "C" void oracle_tdigest_quantiles(const double* vals, int64_t n, double* out7) {
  TDigest d(1000);
  for (int64_t i = 0; i < n; ++i) d.add(vals[i]);
  for (int k = 0; k < 7; ++k) out7[k] = d.quantile(kQs[k]);
}

extern "C" void oracle_tdigest_centroids(const double* vals, int64_t n, double* means, double* weights, int64_t cap, int64_t* nc) {
  TDigest d = TDigest::FromValuesOnce(std::vector<double>(vals, vals + n), 1000);
  const auto& cs = d.processed();
  *nc = static_cast<int64_t>(cs.size()) <= cap ? static_cast<int64_t>(cs.size()) : -1;
  if (*nc < 0) return;
  for (size_t i = 0; i < cs.size(); ++i) {
    means[i] = cs[i].mean;
    weights[i] = cs[i].weight;
  }
}

extern "C" void oracle_tdigest_batch_quantiles(int32_t nparts, const int32_t* kind, const int64_t* counts, const double* data,
                                               const double* weights, double* out7) {
  std::vector<TDigest> parts;
  parts.reserve(static_cast<size_t>(nparts));
  int64_t at = 0;
  for (int32_t p = 0; p < nparts; ++p) {
    const int64_t c = counts[p];
    if (kind[p] == 0) {
      parts.push_back(TDigest::Unprocessed(std::vector<double>(data + at, data + at + c), 1000));
    } else {
      std::vector<Centroid> cs;
      for (int64_t i = 0; i < c; ++i) cs.emplace_back(data[at + i], weights[at + i]);
      parts.push_back(TDigest::FromCentroids(cs, 1000));
    }
    at += c;
  }
  std::vector<const TDigest*> batch;
  for (const auto& d : parts) batch.push_back(&d);
  TDigest out(1000);
  out.merge_batch(batch);
  static const double qs[7] = {0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99};
  for (int i = 0; i < 7; ++i) out7[i] = out.quantile(qs[i]);
}

// As oracle_tdigest_batch_quantiles, with every centroid-list part carrying its rank's true
// min / max (mins[p], maxs[p]) into the merged digest (math_sketches.h:38 merge; the carried
// reading).
extern "C" void oracle_tdigest_batch_quantiles_mm(int32_t nparts, const int32_t* kind, const int64_t* counts, const double* data,
                                                  const double* weights, const double* mins, const double* maxs, double* out7) {
  std::vector<TDigest> parts;
  parts.reserve(static_cast<size_t>(nparts));
  int64_t at = 0;
  double lo = std::numeric_limits<double>::infinity(), hi = -std::numeric_limits<double>::infinity();
  for (int32_t p = 0; p < nparts; ++p) {
    const int64_t c = counts[p];
    if (kind[p] == 0) {
      parts.push_back(TDigest::Unprocessed(std::vector<double>(data + at, data + at + c), 1000));
    } else {
      std::vector<Centroid> cs;
      for (int64_t i = 0; i < c; ++i) cs.emplace_back(data[at + i], weights[at + i]);
      parts.push_back(TDigest::FromCentroids(cs, 1000, mins[p], maxs[p]));
      if (c > 0) {
        lo = std::min(lo, mins[p]);
        hi = std::max(hi, maxs[p]);
      }
    }
    at += c;
  }
  std::vector<const TDigest*> batch;
  for (const auto& d : parts) batch.push_back(&d);
  TDigest out(1000);
  out.merge_batch(batch);
  out.carry_extremes(lo, hi);
  for (int i = 0; i < 7; ++i) out7[i] = out.quantile(kQs[i]);
}

extern "C" void oracle_tdigest_merge_quantiles(const double* a, int64_t na, const double* b, int64_t nb, double* out7) {
  TDigest d1(1000), d2(1000);
  for (int64_t i = 0; i < na; ++i) d1.add(a[i]);
  for (int64_t i = 0; i < nb; ++i) d2.add(b[i]);
  d1.merge(&d2);
  for (int k = 0; k < 7; ++k) out7[k] = d1.quantile(kQs[k]);
}

extern "C" int32_t oracle_quantiles_json(const double* vals, int64_t n, char* buf, int32_t buflen) {
  TDigest d(1000);
  for (int64_t i = 0; i < n; ++i) d.add(vals[i]);
  std::string s = QuantilesJson(&d);
  std::snprintf(buf, static_cast<size_t>(buflen), "%s", s.c_str());
  return static_cast<int32_t>(s.size());
}

// n groups of 7 doubles -> each group's QuantilesUDA::Finalize JSON followed by a NUL, back to
// back in buf (cap bytes); returns the bytes needed (nothing is written past cap).
extern "C" int64_t oracle_quantiles_json_render(const double* q7, int64_t n, char* buf, int64_t cap) {
  std::string all;
  for (int64_t g = 0; g < n; ++g) {
    oracle_json::AppendQuantilesJson(q7 + 7 * g, &all);
    all.push_back('\0');
  }
  if (buf && cap > 0) std::memcpy(buf, all.data(), static_cast<size_t>(std::min<int64_t>(cap, static_cast<int64_t>(all.size()))));
  return static_cast<int64_t>(all.size());
}

extern "C" double oracle_pluck_float64(const char* json, const char* key) {
  // PluckAsFloat64UDF::Exec (json_ops.h:131-153): parse failure / non-object / missing key /
  // null / non-double -> 0.0.  A JSON number is a "double" for rapidjson iff it has a '.' or an
  // exponent.
  try {
    Json d = ParseJson(json);
    if (d.kind != Json::kObject || !d.has(key)) return 0.0;
    const Json& v = d[key];
    if (v.kind != Json::kNumber) return 0.0;
    if (v.num.find_first_of(".eE") == std::string::npos) return 0.0;
    return std::strtod(v.num.c_str(), nullptr);
  } catch (...) {
    return 0.0;
  }
}

// Parity helper for groups whose reference t-digest depends on insertion order (> 8000 values):
// the midpoint empirical rank F(v) = (#{x < v} + #{x <= v}) / 2n of candidate quantile values
// within their group.  Rows are grouped by the exact bytes of their key columns (RowTuple
// equality, row_tuple.h:109-153); sel (optional) masks rows out.  Query q names its group by the
// same key encoding -- per key column: STRING u32 length + bytes, UINT128 16 bytes, other types
// their 8 value bytes -- at qkeys[qoffs[q], qoffs[q+1]); out[q * per_q + j] = rank of
// qv[q * per_q + j] (NaN when the group has no rows).  qcount[q] receives the group's size.
extern "C" int32_t oracle_group_ranks(const oracle_column* keys, int32_t nk, const uint8_t* sel, const double* vals, int64_t n,
                                      int32_t nq, const uint8_t* qkeys, const int64_t* qoffs, const double* qv, int32_t per_q,
                                      double* out, int64_t* qcount) {
  std::unordered_map<std::string, int32_t> want;
  for (int32_t q = 0; q < nq; ++q)
    want.emplace(std::string(reinterpret_cast<const char*>(qkeys + qoffs[q]), static_cast<size_t>(qoffs[q + 1] - qoffs[q])), q);
  std::vector<std::vector<double>> groups(static_cast<size_t>(nq));
  std::string k;
  for (int64_t r = 0; r < n; ++r) {
    if (sel && !sel[r]) continue;
    k.clear();
    for (int32_t c = 0; c < nk; ++c) {
      const oracle_column& col = keys[c];
      if (col.type == STRING) {
        const uint32_t len = static_cast<uint32_t>(col.offsets[r + 1] - col.offsets[r]);
        k.append(reinterpret_cast<const char*>(&len), 4);
        k.append(reinterpret_cast<const char*>(col.data) + col.offsets[r], len);
      } else if (col.type == BOOLEAN) {  // 1 byte per row, widened to the 8-byte query encoding
        char b[8] = {static_cast<const char*>(col.values)[r], 0, 0, 0, 0, 0, 0, 0};
        k.append(b, 8);
      } else {
        const size_t w = col.type == UINT128 ? 16 : 8;
        k.append(static_cast<const char*>(col.values) + r * w, w);
      }
    }
    auto it = want.find(k);
    if (it != want.end()) groups[static_cast<size_t>(it->second)].push_back(vals[r]);
  }
  for (int32_t q = 0; q < nq; ++q) {
    std::vector<double>& g = groups[static_cast<size_t>(q)];
    std::sort(g.begin(), g.end());
    qcount[q] = static_cast<int64_t>(g.size());
    for (int32_t j = 0; j < per_q; ++j) {
      const double v = qv[static_cast<int64_t>(q) * per_q + j];
      double r = std::numeric_limits<double>::quiet_NaN();
      if (!g.empty()) {
        const auto lo = std::lower_bound(g.begin(), g.end(), v) - g.begin();
        const auto hi = std::upper_bound(g.begin(), g.end(), v) - g.begin();
        r = (static_cast<double>(lo) + static_cast<double>(hi)) / 2.0 / static_cast<double>(g.size());
      }
      out[static_cast<int64_t>(q) * per_q + j] = r;
    }
  }
  return OK;
}
