// carnot_csv: the `carnot_executable` harness (src/carnot/carnot_executable.cc:109-300) over
// the device engine.  The reference reads a CSV whose first row holds column types
// (int64 / uint128 / float64 / boolean / string / time64ns) and whose second row holds column
// names, cuts it into RowBatches of --rowbatch_size rows, runs a query over it as table
// --table_name and writes the first output table as CSV (no header; INT64 / TIME64NS as
// integers, FLOAT64 with "%.2f", BOOLEAN as true/false, UINT128 as "high:low", STRING raw).
// The PxL compiler is not on this path, so the query arrives as a compiled binary
// px.carnot.planpb.Plan (--plan_file) instead of PxL text.
//
// Value parsing follows the reference exactly: INT64 and TIME64NS go through std::stoi (an
// `int`: values outside 32 bits are an error there as here), FLOAT64 through std::stof (a
// float, widened to double), BOOLEAN is `field == "true"`, STRING is taken as is.  The
// reference has no UINT128 case when appending values, so a uint128 column is rejected.
//
// Timing (stderr, one JSON line): `parse_s` (CSV -> RowBatches), `exec_s` (engine call:
// first GenerateNext to final emit plus PXRB serialisation), `total_s`.
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pxcarnot.h"

namespace {

// RFC 4180 fields (aria::csv::CsvParser semantics: ',' separators, '"' quoting with "" as an
// escaped quote, CR LF or LF row ends).
bool NextRow(std::istream& in, std::vector<std::string>* row) {
  row->clear();
  std::string field;
  bool quoted = false, any = false;
  int c;
  while ((c = in.get()) != EOF) {
    any = true;
    if (quoted) {
      if (c == '"') {
        if (in.peek() == '"') {
          field.push_back('"');
          in.get();
        } else {
          quoted = false;
        }
      } else {
        field.push_back(static_cast<char>(c));
      }
      continue;
    }
    if (c == '"') {
      quoted = true;
    } else if (c == ',') {
      row->push_back(field);
      field.clear();
    } else if (c == '\n') {
      row->push_back(field);
      return true;
    } else if (c == '\r') {
      if (in.peek() == '\n') in.get();
      row->push_back(field);
      return true;
    } else {
      field.push_back(static_cast<char>(c));
    }
  }
  if (any) row->push_back(field);
  return any;
}

int TypeFromHeader(const std::string& t) {
  if (t == "int64") return PXG_INT64;
  if (t == "uint128") return PXG_UINT128;
  if (t == "float64") return PXG_FLOAT64;
  if (t == "boolean") return PXG_BOOLEAN;
  if (t == "string") return PXG_STRING;
  if (t == "time64ns") return PXG_TIME64NS;
  return -1;
}

struct Col {
  int type = 0;
  std::vector<int64_t> i64;
  std::vector<double> f64;
  std::vector<uint8_t> b;
  std::vector<int32_t> off{0};
  std::string data;
};

struct Batch {
  std::vector<Col> cols;
  int64_t rows = 0;
};

template <typename T>
T Get(const uint8_t*& p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  p += sizeof(T);
  return v;
}

std::string Flag(int argc, char** argv, const char* name, const char* env, const std::string& def) {
  const std::string pre = std::string("--") + name + "=";
  for (int i = 1; i < argc; ++i)
    if (std::strncmp(argv[i], pre.c_str(), pre.size()) == 0) return argv[i] + pre.size();
  const char* e = std::getenv(env);
  return e ? e : def;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string input = Flag(argc, argv, "input_file", "INPUT_FILE", "");
  const std::string output = Flag(argc, argv, "output_file", "OUTPUT_FILE", "");
  const std::string plan_file = Flag(argc, argv, "plan_file", "PLAN_FILE", "");
  const std::string table_name = Flag(argc, argv, "table_name", "TABLE_NAME", "csv_table");
  const int64_t rb_size = std::stoll(Flag(argc, argv, "rowbatch_size", "ROWBATCH_SIZE", "100"));
  const int device = std::stoi(Flag(argc, argv, "device", "PXG_DEVICE", "0"));
  if (input.empty() || output.empty() || plan_file.empty() || rb_size <= 0) {
    std::fprintf(stderr, "usage: carnot_csv --input_file=F.csv --output_file=O.csv --plan_file=P.pb [--table_name=csv_table] "
                         "[--rowbatch_size=100] [--device=0]\n");
    return 2;
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::ifstream f(input, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", input.c_str());
    return 1;
  }
  std::vector<std::string> row, names;
  std::vector<int> types;
  if (!NextRow(f, &row)) {
    std::fprintf(stderr, "empty csv\n");
    return 1;
  }
  for (auto& t : row) {
    const int ty = TypeFromHeader(t);
    if (ty < 0) {
      std::fprintf(stderr, "Could not recognize type '%s' from header.\n", t.c_str());
      return 1;
    }
    if (ty == PXG_UINT128) {
      std::fprintf(stderr, "uint128 columns cannot be loaded from CSV (the reference appends no value for them)\n");
      return 1;
    }
    types.push_back(ty);
  }
  if (NextRow(f, &row)) names = row;
  std::vector<Batch> batches;
  try {
    while (NextRow(f, &row)) {
      if (row.size() == 1 && row[0].empty()) continue;  // blank line
      if (batches.empty() || batches.back().rows == rb_size) {
        batches.emplace_back();
        batches.back().cols.resize(types.size());
        for (size_t c = 0; c < types.size(); ++c) batches.back().cols[c].type = types[c];
      }
      Batch& b = batches.back();
      if (row.size() != types.size()) {
        std::fprintf(stderr, "row with %zu fields, header has %zu\n", row.size(), types.size());
        return 1;
      }
      for (size_t c = 0; c < types.size(); ++c) {
        Col& col = b.cols[c];
        const std::string& v = row[c];
        switch (types[c]) {
          case PXG_INT64:
          case PXG_TIME64NS: col.i64.push_back(std::stoi(v)); break;
          case PXG_FLOAT64: col.f64.push_back(static_cast<double>(std::stof(v))); break;
          case PXG_BOOLEAN: col.b.push_back(v == "true" ? 1 : 0); break;
          default:
            col.data += v;
            col.off.push_back(static_cast<int32_t>(col.data.size()));
            break;
        }
      }
      ++b.rows;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "CSV value does not parse: %s\n", e.what());
    return 1;
  }
  std::vector<pxg_column_view> views;
  for (auto& b : batches) {
    for (auto& c : b.cols) {
      pxg_column_view v{};
      v.type = c.type;
      v.length = b.rows;
      if (c.type == PXG_FLOAT64) v.values = c.f64.data();
      else if (c.type == PXG_BOOLEAN) v.values = c.b.data();
      else if (c.type == PXG_STRING) {
        c.data.append(16, '\0');
        v.offsets = c.off.data();
        v.data = reinterpret_cast<const uint8_t*>(c.data.data());
      } else v.values = c.i64.data();
      views.push_back(v);
    }
  }
  pxc_table tab{};
  tab.name = table_name.c_str();
  tab.ncols = static_cast<int32_t>(types.size());
  tab.nbatches = static_cast<int32_t>(batches.size());
  tab.col_types = types.data();
  tab.cols = views.data();
  std::ifstream pf(plan_file, std::ios::binary);
  std::stringstream ps;
  ps << pf.rdbuf();
  const std::string plan = ps.str();
  const auto t1 = std::chrono::steady_clock::now();

  pxc_engine* engine = nullptr;
  if (pxc_engine_create(device, &engine) != 0) {
    std::fprintf(stderr, "engine: %s\n", pxc_last_error());
    return 1;
  }
  uint8_t* out = nullptr;
  int64_t out_len = 0;
  const auto t2 = std::chrono::steady_clock::now();
  const int32_t rc = pxc_execute_plan(engine, reinterpret_cast<const uint8_t*>(plan.data()), static_cast<int64_t>(plan.size()), 1,
                                      &tab, &out, &out_len);
  const auto t3 = std::chrono::steady_clock::now();
  if (rc != 0) {
    std::fprintf(stderr, "Query failed to execute: %s\n", pxc_last_error());
    pxc_engine_destroy(engine);
    return 1;
  }
  // PXRB: magic, sinks; per sink: name, batches; per batch: rows, eow, eos, pad, ncols, columns.
  const uint8_t* p = out;
  const uint8_t* end = out + out_len;
  (void)Get<uint32_t>(p);
  const uint32_t nsinks = Get<uint32_t>(p);
  if (nsinks == 0) {
    std::fprintf(stderr, "Query produced no output tables.\n");
    return 1;
  }
  const uint32_t nlen = Get<uint32_t>(p);
  const std::string sink_name(reinterpret_cast<const char*>(p), nlen);
  p += nlen;
  const uint32_t nb = Get<uint32_t>(p);
  std::ofstream o(output);
  char buf[64];
  for (uint32_t bi = 0; bi < nb && p < end; ++bi) {
    const int64_t rows = Get<int64_t>(p);
    (void)Get<uint8_t>(p);
    (void)Get<uint8_t>(p);
    (void)Get<uint16_t>(p);
    const uint32_t ncols = Get<uint32_t>(p);
    std::vector<std::vector<std::string>> cells(static_cast<size_t>(rows), std::vector<std::string>(ncols));
    for (uint32_t c = 0; c < ncols; ++c) {
      const int32_t t = Get<int32_t>(p);
      for (int64_t r = 0; r < rows; ++r) {
        std::string& cell = cells[static_cast<size_t>(r)][c];
        switch (t) {
          case PXG_BOOLEAN: cell = p[r] ? "true" : "false"; break;
          case PXG_FLOAT64: {
            double v;
            std::memcpy(&v, p + 8 * r, 8);
            std::snprintf(buf, sizeof(buf), "%.2f", v);
            cell = buf;
            break;
          }
          case PXG_UINT128: {
            uint64_t lo, hi;
            std::memcpy(&lo, p + 16 * r, 8);
            std::memcpy(&hi, p + 16 * r + 8, 8);
            cell = std::to_string(hi) + ":" + std::to_string(lo);
            break;
          }
          case PXG_STRING: break;
          default: {
            int64_t v;
            std::memcpy(&v, p + 8 * r, 8);
            cell = std::to_string(v);
          }
        }
      }
      if (t == PXG_STRING) {
        const int32_t* offs = reinterpret_cast<const int32_t*>(p);
        const char* data = reinterpret_cast<const char*>(p + 4 * (rows + 1));
        for (int64_t r = 0; r < rows; ++r) cells[static_cast<size_t>(r)][c].assign(data + offs[r], static_cast<size_t>(offs[r + 1] - offs[r]));
        p += 4 * (rows + 1) + (rows ? offs[rows] : 0);
      } else {
        p += rows * (t == PXG_BOOLEAN ? 1 : t == PXG_UINT128 ? 16 : 8);
      }
    }
    for (auto& r : cells) {
      for (size_t c = 0; c < r.size(); ++c) o << (c ? "," : "") << r[c];
      o << "\n";
    }
  }
  o.close();
  pxc_free(out);
  pxc_engine_destroy(engine);
  const auto t4 = std::chrono::steady_clock::now();
  auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
  std::fprintf(stderr, "{\"output_table\": \"%s\", \"input_rows\": %" PRId64 ", \"batches\": %zu, \"parse_s\": %.6f, \"exec_s\": %.6f, \"total_s\": %.6f}\n",
               sink_name.c_str(), static_cast<int64_t>(batches.empty() ? 0 : (batches.size() - 1) * rb_size + batches.back().rows),
               batches.size(), sec(t0, t1), sec(t2, t3), sec(t0, t4));
  return 0;
}
