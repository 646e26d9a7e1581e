// ORACLE / TEST INFRASTRUCTURE ONLY — ground truth for the C2 query shape straight from the
// synthetic http_events generator, for parity at sizes the row-at-a-time restatement
// (carnot_oracle.cc) cannot hold in host memory (the 1B-row north_star table).  Test
// infrastructure: used by tests/ and bench.py's n1 parity leg only.
//
// Query: Filter(resp_status >= status_min) -> Map(latency / 1e6) ->
// Agg by (service, req_path): count, mean, quantiles.  Rows are regenerated on the host from
// the generator spec shared with the device generator (pixie_amd/csrc/pxg_datagen_spec.h; the
// two are bit-identical, tests/test_scale_parity.py), so no table is materialised: a group is
// named by its (service index, path index) draw.  Two path indices can spell the same string, so
// a path index is replaced by the first index with the same bytes: groups are exactly the
// distinct (service, req_path) byte strings (RowTuple equality, row_tuple.h:109-153).  The
// caller maps indices to key strings with oracle_http_events_tables().
//
// What is computed per group is what the reference's UDAs consume (agg_node.cc:235-286): the row
// count (CountUDA, math_ops.h:583-609), the exact integer sum of the latency column (the mean's
// numerator before the divide UDF rounds each value; MeanUDA, math_ops.h:651-695), and, for the
// groups the caller flags, every value latency/1e6 (DivideUDF, math_ops.h:84-109) in row order —
// the insertion order the reference's t-digest sees (math_sketches.h:36-54).
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../pixie_amd/csrc/pxg_datagen_spec.h"

using pxg::gen::GetTables;
using pxg::gen::kPaths;
using pxg::gen::kServices;
using pxg::gen::Tables;

namespace {
constexpr int64_t kGroups = static_cast<int64_t>(kServices) * kPaths;

// canon[k] = the smallest path index whose string equals path k's.
std::vector<int32_t> CanonicalPaths(const Tables& T) {
  std::vector<int32_t> canon(kPaths);
  for (int k = 0; k < kPaths; ++k) {
    canon[k] = k;
    const int32_t lk = T.path_off[k + 1] - T.path_off[k];
    for (int j = 0; j < k; ++j) {
      if (T.path_off[j + 1] - T.path_off[j] == lk && std::memcmp(T.path_bytes + T.path_off[j], T.path_bytes + T.path_off[k], lk) == 0) {
        canon[k] = j;
        break;
      }
    }
  }
  return canon;
}

// The draws of one row that the C2 query reads, from MakeRow's streams (pxg_datagen_spec.h):
// status first (stream 3), and for the ~12 % of rows that pass, service (1), path (2) and
// latency (4).  RowRand(seed, row, s) = SplitMix(SplitMix(seed ^ s * K) + row): the inner
// SplitMix is hoisted per stream, so a rejected row costs one SplitMix.
struct C2Draws {
  uint64_t base[5];
  explicit C2Draws(uint64_t seed) {
    for (uint64_t s = 0; s < 5; ++s) base[s] = pxg::gen::SplitMix(seed ^ (s * 0xD1B54A32D192ED03ULL));
  }
  uint64_t R(int s, int64_t row) const { return pxg::gen::SplitMix(base[s] + static_cast<uint64_t>(row)); }
};

template <typename F>
void ForRowRanges(int64_t n, int threads, F&& f) {
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) th.emplace_back([&, t] { f(t, n * t / threads, n * (t + 1) / threads); });
  for (auto& x : th) x.join();
}
}  // namespace

// The generator's key-string tables: service k = svc_bytes[svc_off[k], svc_off[k+1]), path k likewise.
// Buffers: svc_bytes >= 64*16, svc_off >= 65, path_bytes >= 1024*48, path_off >= 1025.
extern "C" void oracle_http_events_tables(char* svc_bytes, int32_t* svc_off, char* path_bytes, int32_t* path_off) {
  const Tables& T = GetTables();
  std::memcpy(svc_bytes, T.svc_bytes, sizeof(T.svc_bytes));
  std::memcpy(svc_off, T.svc_off, sizeof(T.svc_off));
  std::memcpy(path_bytes, T.path_bytes, sizeof(T.path_bytes));
  std::memcpy(path_off, T.path_off, sizeof(T.path_off));
}

// Rows [row0, row0 + n) of the seeded table.  Pass 1: counts[g] and lat_sum[g] (exact int64) for
// g = service * 1024 + canonical path over the rows passing the filter.  Pass 2 (only if collect != null):
// the values latency / 1e6 of every group with collect[g] != 0, written to vals at
// [voff[g], voff[g] + counts[g]) in row order; voff is filled here (exclusive scan over the
// flagged groups' counts) and vals must hold their total (returned).  Returns the number of
// collected values, or -1 on bad arguments.
extern "C" int64_t oracle_http_events_c2_truth(uint64_t seed, int64_t row0, int64_t n, int64_t n_pair_keys, int32_t threads,
                                               int64_t status_min, int64_t* counts, int64_t* lat_sum, const uint8_t* collect,
                                               int64_t* voff, double* vals, int64_t vals_cap) {
  if (n < 0 || !counts || !lat_sum) return -1;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  if (n_pair_keys <= 0) n_pair_keys = 10000000;
  const Tables& T = GetTables();
  const std::vector<int32_t> canon = CanonicalPaths(T);
  const C2Draws D(seed);
  auto Group = [&](int64_t r) {
    const int svc = pxg::gen::ZipfSample(T.svc_cdf, kServices, pxg::gen::U01(D.R(1, r)));
    const int path = pxg::gen::ZipfSample(T.path_cdf, kPaths, pxg::gen::U01(D.R(2, r)));
    return static_cast<int64_t>(svc) * kPaths + canon[path];
  };
  std::vector<std::vector<int64_t>> tc(threads, std::vector<int64_t>(kGroups, 0)), ts(threads, std::vector<int64_t>(kGroups, 0));
  ForRowRanges(n, threads, [&](int t, int64_t lo, int64_t hi) {
    int64_t* c = tc[t].data();
    int64_t* s = ts[t].data();
    for (int64_t r = row0 + lo; r < row0 + hi; ++r) {
      if (pxg::gen::RespStatus(pxg::gen::U01(D.R(3, r))) < status_min) continue;
      const int64_t g = Group(r);
      c[g] += 1;
      s[g] += pxg::gen::Latency(T.lat_grid, D.R(4, r));
    }
  });
  for (int64_t g = 0; g < kGroups; ++g) {
    int64_t c = 0, s = 0;
    for (int t = 0; t < threads; ++t) {
      c += tc[t][g];
      s += ts[t][g];
    }
    counts[g] = c;
    lat_sum[g] = s;
  }
  if (!collect || !voff || !vals) return 0;
  // Per-thread write positions: thread t's rows of group g follow threads 0..t-1's (row order).
  int64_t total = 0;
  std::vector<std::vector<int64_t>> pos(threads, std::vector<int64_t>(kGroups, -1));
  for (int64_t g = 0; g < kGroups; ++g) {
    voff[g] = total;
    if (!collect[g]) continue;
    for (int t = 0; t < threads; ++t) {
      pos[t][g] = total;
      total += tc[t][g];
    }
  }
  voff[kGroups] = total;
  if (total > vals_cap) return -1;
  ForRowRanges(n, threads, [&](int t, int64_t lo, int64_t hi) {
    int64_t* p = pos[t].data();
    for (int64_t r = row0 + lo; r < row0 + hi; ++r) {
      if (pxg::gen::RespStatus(pxg::gen::U01(D.R(3, r))) < status_min) continue;
      const int64_t g = Group(r);
      if (p[g] >= 0) vals[p[g]++] = static_cast<double>(pxg::gen::Latency(T.lat_grid, D.R(4, r))) / 1e6;
    }
  });
  return total;
}
