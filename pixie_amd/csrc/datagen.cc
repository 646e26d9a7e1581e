// Synthetic http_events generator (SURVEY.md §8d spec).  Bench/test data only.
//
// Columns follow the reference's http_events schema
// (src/stirling/source_connectors/socket_tracer/http_table.h:41-108,
// src/carnot/exec/test_utils.h:228-247) plus a materialised `service` and `pod` string
// (in Pixie these come from upid_to_service_name / metadata lookups, which are out of scope).
// Every value is a pure function of (seed, global row): a counter-based splitmix64 stream, so
// shards generated on different GPUs' hosts concatenate to the same 1B-row table.  The per-row
// spec lives in pxg_datagen_spec.h, shared with the device generator (pxg_datagen.hip).

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pxg.h"
#include "pxg_datagen_spec.h"
#include "pxg_errors.h"

namespace pxg {
namespace gen {

// Zipf(n, s) CDF over ranks 1..n.
static void ZipfCdf(int n, double s, double* cdf) {
  double acc = 0;
  for (int k = 1; k <= n; ++k) acc += 1.0 / std::pow(static_cast<double>(k), s);
  double run = 0;
  for (int k = 1; k <= n; ++k) {
    run += 1.0 / std::pow(static_cast<double>(k), s);
    cdf[k - 1] = run / acc;
  }
  cdf[n - 1] = 1.0;
}

// Inverse standard-normal CDF by bisection on Phi(x) = erfc(-x / sqrt 2) / 2.
static double NormInv(double p) {
  double lo = -12, hi = 12;
  for (int i = 0; i < 200; ++i) {
    const double mid = 0.5 * (lo + hi);
    if (0.5 * std::erfc(-mid / std::sqrt(2.0)) < p) lo = mid;
    else hi = mid;
  }
  return 0.5 * (lo + hi);
}

static Tables MakeTables() {
  Tables t;
  std::memset(&t, 0, sizeof(t));
  ZipfCdf(kServices, 1.1, t.svc_cdf);
  ZipfCdf(kPaths, 1.2, t.path_cdf);
  // latency: lognormal(ln 5e6, 1) inverse CDF on the grid, clamped to [1e3, 2e9]
  for (int i = 0; i <= kLatencyGrid; ++i) {
    double v;
    if (i == 0) v = 1e3;
    else if (i == kLatencyGrid) v = 2e9;
    else v = std::exp(std::log(5e6) + NormInv(static_cast<double>(i) / kLatencyGrid));
    t.lat_grid[i] = v < 1e3 ? 1e3 : (v > 2e9 ? 2e9 : v);
  }
  char buf[96];
  int at = 0;
  for (int k = 0; k < kServices; ++k) {
    const int n = std::snprintf(buf, sizeof(buf), "ns%02d/svc-%03d", k % 16, (k * 37) % 1000);
    t.svc_off[k] = at;
    std::memcpy(t.svc_bytes + at, buf, static_cast<size_t>(n));
    at += n;
  }
  t.svc_off[kServices] = at;
  static const char* kRes[] = {"users", "orders", "items", "cart", "auth", "search", "reviews", "inventory",
                               "payments", "shipping", "profile", "catalog", "metrics", "health", "events", "sessions"};
  at = 0;
  for (int k = 0; k < kPaths; ++k) {
    const uint64_t r = SplitMix(0xA5A5ULL + static_cast<uint64_t>(k));
    const char* res = kRes[r % 16];
    const int ver = 1 + static_cast<int>((r >> 8) % 3);
    const int id = static_cast<int>((r >> 16) % 100000);
    int n;
    switch ((r >> 40) % 4) {
      case 0: n = std::snprintf(buf, sizeof(buf), "/api/v%d/%s/%d", ver, res, id); break;
      case 1: n = std::snprintf(buf, sizeof(buf), "/v%d/%s/%d/detail", ver, res, id); break;
      case 2: n = std::snprintf(buf, sizeof(buf), "/api/v%d/%s?page=%d", ver, res, id % 97); break;
      default: n = std::snprintf(buf, sizeof(buf), "/internal/%s/%s/%d", res, kRes[(r >> 44) % 16], id % 1000); break;
    }
    t.path_off[k] = at;
    std::memcpy(t.path_bytes + at, buf, static_cast<size_t>(n));
    at += n;
  }
  t.path_off[kPaths] = at;
  return t;
}

const Tables& GetTables() {
  static const Tables t = MakeTables();
  return t;
}

}  // namespace gen
}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_datagen_http_events(uint64_t seed, int64_t row_begin, int64_t nrows, int64_t n_pair_keys,
                                           int32_t n_threads, pxg_column_out* cols) {
  using namespace pxg::gen;
  if (nrows < 0 || !cols) return SetError(PXG_INVALID_ARGUMENT, "datagen: bad arguments");
  if (n_pair_keys <= 0) n_pair_keys = 10000000;
  if (n_threads <= 0) n_threads = 1;
  if (n_threads > 64) n_threads = 64;
  const Tables& T = GetTables();

  const int kTypes[PXG_HTTP_EVENTS_NCOLS] = {PXG_TIME64NS, PXG_UINT128, PXG_STRING, PXG_STRING, PXG_STRING,
                                             PXG_INT64,    PXG_INT64,   PXG_INT64,  PXG_INT64,  PXG_STRING};
  for (int c = 0; c < PXG_HTTP_EVENTS_NCOLS; ++c) {
    std::memset(&cols[c], 0, sizeof(pxg_column_out));
    cols[c].type = kTypes[c];
    cols[c].length = nrows;
    size_t w = kTypes[c] == PXG_UINT128 ? 16 : 8;
    if (kTypes[c] == PXG_STRING) {
      cols[c].offsets = static_cast<int32_t*>(std::malloc(sizeof(int32_t) * (nrows + 1)));
      if (!cols[c].offsets) return SetError(PXG_RESOURCE_UNAVAILABLE, "datagen: out of host memory");
    } else {
      cols[c].values = std::malloc(w * std::max<int64_t>(nrows, 1));
      if (!cols[c].values) return SetError(PXG_RESOURCE_UNAVAILABLE, "datagen: out of host memory");
    }
  }
  const int kStrCols[4] = {2, 3, 4, 9};
  // Pass 1 (parallel): fixed columns + string lengths (into offsets[r+1]).
  std::vector<std::thread> th;
  std::vector<std::vector<int64_t>> part_bytes(n_threads, std::vector<int64_t>(4, 0));
  auto pass1 = [&](int t) {
    int64_t lo = nrows * t / n_threads, hi = nrows * (t + 1) / n_threads;
    int64_t* time_ = static_cast<int64_t*>(cols[0].values);
    uint64_t* upid = static_cast<uint64_t*>(cols[1].values);
    int64_t* status = static_cast<int64_t*>(cols[5].values);
    int64_t* lat = static_cast<int64_t*>(cols[6].values);
    int64_t* reqb = static_cast<int64_t*>(cols[7].values);
    int64_t* respb = static_cast<int64_t*>(cols[8].values);
    for (int64_t r = lo; r < hi; ++r) {
      const Row w = MakeRow(seed, row_begin + r, n_pair_keys, T.svc_cdf, T.path_cdf, T.lat_grid);
      time_[r] = w.time;
      upid[2 * r] = w.upid_lo;
      upid[2 * r + 1] = w.upid_hi;
      status[r] = w.status;
      lat[r] = w.latency;
      reqb[r] = w.req_body;
      respb[r] = w.resp_body;
      cols[2].offsets[r + 1] = T.svc_off[w.svc + 1] - T.svc_off[w.svc];
      cols[3].offsets[r + 1] = T.path_off[w.path + 1] - T.path_off[w.path];
      cols[4].offsets[r + 1] = AddrLen(w.addr_idx);
      cols[9].offsets[r + 1] = kPodLen;
      for (int s = 0; s < 4; ++s) part_bytes[t][s] += cols[kStrCols[s]].offsets[r + 1];
    }
  };
  for (int t = 0; t < n_threads; ++t) th.emplace_back(pass1, t);
  for (auto& x : th) x.join();
  th.clear();
  // Offsets: exclusive scan per thread range.
  std::vector<std::vector<int64_t>> base(n_threads, std::vector<int64_t>(4, 0));
  for (int s = 0; s < 4; ++s) {
    int64_t acc = 0;
    for (int t = 0; t < n_threads; ++t) {
      base[t][s] = acc;
      acc += part_bytes[t][s];
    }
    if (acc > INT32_MAX) return SetError(PXG_INVALID_ARGUMENT, "datagen: string column exceeds 2^31 bytes; generate in smaller batches");
    pxg_column_out& c = cols[kStrCols[s]];
    c.data_len = acc;
    c.data = static_cast<uint8_t*>(std::malloc(static_cast<size_t>(acc) + 16));
    if (!c.data) return SetError(PXG_RESOURCE_UNAVAILABLE, "datagen: out of host memory");
    std::memset(c.data + acc, 0, 16);
    c.offsets[0] = 0;
  }
  auto pass2 = [&](int t) {
    int64_t lo = nrows * t / n_threads, hi = nrows * (t + 1) / n_threads;
    int64_t run[4];
    for (int s = 0; s < 4; ++s) run[s] = base[t][s];
    for (int64_t r = lo; r < hi; ++r) {
      const Row w = MakeRow(seed, row_begin + r, n_pair_keys, T.svc_cdf, T.path_cdf, T.lat_grid);
      const int32_t sl = T.svc_off[w.svc + 1] - T.svc_off[w.svc];
      std::memcpy(cols[2].data + run[0], T.svc_bytes + T.svc_off[w.svc], static_cast<size_t>(sl));
      run[0] += sl;
      const int32_t pl = T.path_off[w.path + 1] - T.path_off[w.path];
      std::memcpy(cols[3].data + run[1], T.path_bytes + T.path_off[w.path], static_cast<size_t>(pl));
      run[1] += pl;
      run[2] += FormatAddr(w.addr_idx, reinterpret_cast<char*>(cols[4].data + run[2]));
      FormatPod(w.pod, reinterpret_cast<char*>(cols[9].data + run[3]));
      run[3] += kPodLen;
      for (int s = 0; s < 4; ++s) cols[kStrCols[s]].offsets[r + 1] = static_cast<int32_t>(run[s]);
    }
  };
  for (int t = 0; t < n_threads; ++t) th.emplace_back(pass2, t);
  for (auto& x : th) x.join();
  return PXG_OK;
}
