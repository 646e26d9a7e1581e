// Synthetic http_events generator (SURVEY.md §8d spec).  Bench/test data only.
//
// Columns follow the reference's http_events schema
// (src/stirling/source_connectors/socket_tracer/http_table.h:41-108,
// src/carnot/exec/test_utils.h:228-247) plus a materialised `service` and `pod` string
// (in Pixie these come from upid_to_service_name / metadata lookups, which are out of scope).
// Every value is a pure function of (seed, global row): a counter-based splitmix64 stream, so
// shards generated on different GPUs' hosts concatenate to the same 1B-row table.

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pxg.h"
#include "pxg_errors.h"

namespace pxg {
namespace {

inline uint64_t SplitMix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// Uniform double in [0,1) from 53 random bits.
inline double U01(uint64_t r) { return static_cast<double>(r >> 11) * (1.0 / 9007199254740992.0); }

inline uint64_t RowRand(uint64_t seed, int64_t row, uint64_t stream) {
  return SplitMix(SplitMix(seed ^ (stream * 0xD1B54A32D192ED03ULL)) + static_cast<uint64_t>(row));
}

struct Zipf {
  std::vector<double> cdf;
  Zipf(int n, double s) {
    cdf.resize(n);
    double acc = 0;
    for (int k = 1; k <= n; ++k) acc += 1.0 / std::pow(static_cast<double>(k), s);
    double run = 0;
    for (int k = 1; k <= n; ++k) {
      run += 1.0 / std::pow(static_cast<double>(k), s);
      cdf[k - 1] = run / acc;
    }
    cdf[n - 1] = 1.0;
  }
  int Sample(double u) const {
    int lo = 0, hi = static_cast<int>(cdf.size()) - 1;
    while (lo < hi) {
      int mid = (lo + hi) / 2;
      if (u < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
  }
};

struct Dict {
  std::vector<std::string> values;
};

Dict MakeServices() {
  Dict d;
  char buf[32];
  for (int k = 0; k < 64; ++k) {
    std::snprintf(buf, sizeof(buf), "ns%02d/svc-%03d", k % 16, (k * 37) % 1000);
    d.values.emplace_back(buf);
  }
  return d;
}

Dict MakePaths() {
  static const char* kRes[] = {"users", "orders", "items", "cart", "auth", "search", "reviews", "inventory",
                               "payments", "shipping", "profile", "catalog", "metrics", "health", "events", "sessions"};
  Dict d;
  char buf[96];
  for (int k = 0; k < 1024; ++k) {
    uint64_t r = SplitMix(0xA5A5ULL + static_cast<uint64_t>(k));
    const char* res = kRes[r % 16];
    int ver = 1 + static_cast<int>((r >> 8) % 3);
    int id = static_cast<int>((r >> 16) % 100000);
    switch ((r >> 40) % 4) {
      case 0: std::snprintf(buf, sizeof(buf), "/api/v%d/%s/%d", ver, res, id); break;
      case 1: std::snprintf(buf, sizeof(buf), "/v%d/%s/%d/detail", ver, res, id); break;
      case 2: std::snprintf(buf, sizeof(buf), "/api/v%d/%s?page=%d", ver, res, id % 97); break;
      default: std::snprintf(buf, sizeof(buf), "/internal/%s/%s/%d", res, kRes[(r >> 44) % 16], id % 1000); break;
    }
    d.values.emplace_back(buf);
  }
  return d;
}

// resp_status distribution: 200:0.80; 201/204/301/302: 0.02 each;
// 400/401/403/404: 0.0175 each; 500/502/503: 1/60 each.  P(>=400) = 0.12.
inline int64_t RespStatus(double u) {
  if (u < 0.80) return 200;
  if (u < 0.88) {
    static const int64_t k[4] = {201, 204, 301, 302};
    return k[static_cast<int>((u - 0.80) / 0.02) & 3];
  }
  if (u < 0.95) {
    static const int64_t k[4] = {400, 401, 403, 404};
    return k[std::min(3, static_cast<int>((u - 0.88) / 0.0175))];
  }
  static const int64_t k[3] = {500, 502, 503};
  return k[std::min(2, static_cast<int>((u - 0.95) / (0.05 / 3)))];
}

inline int64_t Latency(uint64_t r1, uint64_t r2) {
  // lognormal(mu = ln 5e6, sigma = 1.0) via Box-Muller, clamped to [1e3, 2e9] (< 2^31 so the
  // reference CSV path's stoi parses it, carnot_executable.cc:166-169).
  double u1 = (static_cast<double>(r1 >> 11) + 1.0) * (1.0 / 9007199254740993.0);
  double u2 = U01(r2);
  double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  double v = std::exp(std::log(5e6) + z);
  if (v < 1e3) v = 1e3;
  if (v > 2e9) v = 2e9;
  return static_cast<int64_t>(v);
}

void FormatAddr(uint64_t idx, char* buf, size_t n) {
  uint64_t h = SplitMix(idx * 0x9E37ULL + 17);
  std::snprintf(buf, n, "10.%u.%u.%u", static_cast<unsigned>((idx >> 16) & 0xFF), static_cast<unsigned>((idx >> 8) & 0xFF),
                static_cast<unsigned>((idx & 0xFF) ^ (h & 0x0F)));
}

void FormatPod(uint64_t pod, char* buf, size_t n) {
  std::snprintf(buf, n, "pl/pod-%04u-%05x", static_cast<unsigned>(pod), static_cast<unsigned>(SplitMix(pod + 991) & 0xFFFFF));
}

}  // namespace
}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_datagen_http_events(uint64_t seed, int64_t row_begin, int64_t nrows, int64_t n_pair_keys,
                                           int32_t n_threads, pxg_column_out* cols) {
  if (nrows < 0 || !cols) return SetError(PXG_INVALID_ARGUMENT, "datagen: bad arguments");
  if (n_pair_keys <= 0) n_pair_keys = 10000000;
  if (n_threads <= 0) n_threads = 1;
  if (n_threads > 64) n_threads = 64;
  static const Dict services = MakeServices();
  static const Dict paths = MakePaths();
  static const Zipf zsvc(64, 1.1), zpath(1024, 1.2);

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
    char buf[64];
    for (int64_t r = lo; r < hi; ++r) {
      int64_t g = row_begin + r;
      time_[r] = 1700000000000000000LL + g * 1000;
      uint64_t pair = RowRand(seed, g, 7) % static_cast<uint64_t>(n_pair_keys);
      uint64_t pod = pair % 1024;
      upid[2 * r] = SplitMix(pod ^ 0x5555ULL);  // low
      upid[2 * r + 1] = (pod << 32) | 0xABCDULL;  // high
      int svc = zsvc.Sample(U01(RowRand(seed, g, 1)));
      int path = zpath.Sample(U01(RowRand(seed, g, 2)));
      status[r] = RespStatus(U01(RowRand(seed, g, 3)));
      lat[r] = Latency(RowRand(seed, g, 4), RowRand(seed, g, 5));
      reqb[r] = static_cast<int64_t>(RowRand(seed, g, 8) % 65537);
      respb[r] = static_cast<int64_t>(RowRand(seed, g, 9) % 65537);
      cols[2].offsets[r + 1] = static_cast<int32_t>(services.values[svc].size());
      cols[3].offsets[r + 1] = static_cast<int32_t>(paths.values[path].size());
      FormatAddr(pair / 1024, buf, sizeof(buf));
      cols[4].offsets[r + 1] = static_cast<int32_t>(std::strlen(buf));
      FormatPod(pod, buf, sizeof(buf));
      cols[9].offsets[r + 1] = static_cast<int32_t>(std::strlen(buf));
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
    c.offsets[0] = 0;
  }
  auto pass2 = [&](int t) {
    int64_t lo = nrows * t / n_threads, hi = nrows * (t + 1) / n_threads;
    int64_t run[4];
    for (int s = 0; s < 4; ++s) run[s] = base[t][s];
    char buf[64];
    for (int64_t r = lo; r < hi; ++r) {
      int64_t g = row_begin + r;
      uint64_t pair = RowRand(seed, g, 7) % static_cast<uint64_t>(n_pair_keys);
      uint64_t pod = pair % 1024;
      int svc = zsvc.Sample(U01(RowRand(seed, g, 1)));
      int path = zpath.Sample(U01(RowRand(seed, g, 2)));
      const std::string& sv = services.values[svc];
      const std::string& pv = paths.values[path];
      std::memcpy(cols[2].data + run[0], sv.data(), sv.size());
      run[0] += static_cast<int64_t>(sv.size());
      std::memcpy(cols[3].data + run[1], pv.data(), pv.size());
      run[1] += static_cast<int64_t>(pv.size());
      FormatAddr(pair / 1024, buf, sizeof(buf));
      size_t la = std::strlen(buf);
      std::memcpy(cols[4].data + run[2], buf, la);
      run[2] += static_cast<int64_t>(la);
      FormatPod(pod, buf, sizeof(buf));
      size_t lp = std::strlen(buf);
      std::memcpy(cols[9].data + run[3], buf, lp);
      run[3] += static_cast<int64_t>(lp);
      for (int s = 0; s < 4; ++s) cols[kStrCols[s]].offsets[r + 1] = static_cast<int32_t>(run[s]);
    }
  };
  for (int t = 0; t < n_threads; ++t) th.emplace_back(pass2, t);
  for (auto& x : th) x.join();
  return PXG_OK;
}
