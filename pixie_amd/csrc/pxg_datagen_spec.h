// Synthetic http_events generator spec, shared by the host generator
// (datagen.cc, pxg_datagen_http_events) and the device generator (pxg_datagen.hip,
// pxg_table_append_http_events).  Every value is a pure function of (seed, global row) built from
// integer mixing and IEEE +,-,*,/ and comparisons only (no libm call on the per-row path; both
// sides compile with -ffp-contract=off), over lookup tables computed once on the host and
// uploaded unchanged -- so the host and the device produce bit-identical tables.
#pragma once

#include <cstdint>

#if defined(__HIP__)
#define PXG_HD __host__ __device__
#else
#define PXG_HD
#endif

namespace pxg {
namespace gen {

constexpr int kServices = 64;
constexpr int kPaths = 1024;
constexpr int kLatencyGrid = 4096;  // inverse-CDF intervals of the latency distribution
constexpr int kPodLen = 17;         // "pl/pod-%04u-%05x"

PXG_HD inline uint64_t SplitMix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// Uniform double in [0,1) from 53 random bits.
PXG_HD inline double U01(uint64_t r) { return static_cast<double>(r >> 11) * (1.0 / 9007199254740992.0); }

PXG_HD inline uint64_t RowRand(uint64_t seed, int64_t row, uint64_t stream) {
  return SplitMix(SplitMix(seed ^ (stream * 0xD1B54A32D192ED03ULL)) + static_cast<uint64_t>(row));
}

// Zipf sample: first k with u < cdf[k] (cdf[n-1] = 1).
PXG_HD inline int ZipfSample(const double* cdf, int n, double u) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi) / 2;
    if (u < cdf[mid]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// resp_status: 200: 0.80; 201/204/301/302: 0.02 each; 400/401/403/404: 0.0175 each;
// 500/502/503: 1/60 each.  P(>= 400) = 0.12.
PXG_HD inline int64_t RespStatus(double u) {
  if (u < 0.80) return 200;
  if (u < 0.88) {
    const int i = static_cast<int>((u - 0.80) / 0.02) & 3;
    return i == 0 ? 201 : i == 1 ? 204 : i == 2 ? 301 : 302;
  }
  if (u < 0.95) {
    int i = static_cast<int>((u - 0.88) / 0.0175);
    i = i < 3 ? i : 3;
    return i == 0 ? 400 : i == 1 ? 401 : i == 2 ? 403 : 404;
  }
  int i = static_cast<int>((u - 0.95) / (0.05 / 3));
  i = i < 2 ? i : 2;
  return i == 0 ? 500 : i == 1 ? 502 : 503;
}

// latency ns: lognormal(mu = ln 5e6, sigma = 1) by linear interpolation of its inverse CDF on a
// kLatencyGrid-interval grid (grid[0] = 1e3, grid[kLatencyGrid] = 2e9: the clamp range, < 2^31 so
// the reference CSV path's stoi parses it, carnot_executable.cc:166-169).
PXG_HD inline int64_t Latency(const double* grid, uint64_t r) {
  const double x = U01(r) * kLatencyGrid;
  int i = static_cast<int>(x);
  i = i < kLatencyGrid - 1 ? i : kLatencyGrid - 1;
  const double f = x - static_cast<double>(i);
  const double d = grid[i + 1] - grid[i];
  const double v = grid[i] + f * d;
  return static_cast<int64_t>(v < 1e3 ? 1e3 : (v > 2e9 ? 2e9 : v));
}

PXG_HD inline int DecDigits(uint32_t v) { return v >= 100 ? 3 : (v >= 10 ? 2 : 1); }

PXG_HD inline char* PutDec(uint32_t v, char* p) {
  const int n = DecDigits(v);
  for (int i = n - 1; i >= 0; --i) {
    p[i] = static_cast<char>('0' + v % 10);
    v /= 10;
  }
  return p + n;
}

// remote_addr of address index idx: "10.%u.%u.%u".
PXG_HD inline void AddrOctets(uint64_t idx, uint32_t* a, uint32_t* b, uint32_t* c) {
  const uint64_t h = SplitMix(idx * 0x9E37ULL + 17);
  *a = static_cast<uint32_t>((idx >> 16) & 0xFF);
  *b = static_cast<uint32_t>((idx >> 8) & 0xFF);
  *c = static_cast<uint32_t>((idx & 0xFF) ^ (h & 0x0F));
}
PXG_HD inline int AddrLen(uint64_t idx) {
  uint32_t a, b, c;
  AddrOctets(idx, &a, &b, &c);
  return 5 + DecDigits(a) + DecDigits(b) + DecDigits(c);
}
PXG_HD inline int FormatAddr(uint64_t idx, char* p) {
  uint32_t a, b, c;
  AddrOctets(idx, &a, &b, &c);
  char* q = p;
  *q++ = '1';
  *q++ = '0';
  *q++ = '.';
  q = PutDec(a, q);
  *q++ = '.';
  q = PutDec(b, q);
  *q++ = '.';
  q = PutDec(c, q);
  return static_cast<int>(q - p);
}

// pod name: "pl/pod-%04u-%05x" (pod < 1024).
PXG_HD inline void FormatPod(uint64_t pod, char* p) {
  const char* pre = "pl/pod-";
  for (int i = 0; i < 7; ++i) p[i] = pre[i];
  uint32_t v = static_cast<uint32_t>(pod);
  for (int i = 10; i >= 7; --i) {
    p[i] = static_cast<char>('0' + v % 10);
    v /= 10;
  }
  p[11] = '-';
  uint32_t h = static_cast<uint32_t>(SplitMix(pod + 991) & 0xFFFFF);
  for (int i = 16; i >= 12; --i) {
    const uint32_t d = h & 0xF;
    p[i] = static_cast<char>(d < 10 ? '0' + d : 'a' + d - 10);
    h >>= 4;
  }
}

// The per-row draws of one row.
struct Row {
  int64_t time;
  uint64_t upid_lo, upid_hi;
  int svc, path;
  uint64_t pair, pod, addr_idx;
  int64_t status, latency, req_body, resp_body;
};

PXG_HD inline Row MakeRow(uint64_t seed, int64_t g, int64_t n_pair_keys, const double* svc_cdf, const double* path_cdf,
                          const double* lat_grid) {
  Row w;
  w.time = 1700000000000000000LL + g * 1000;
  w.pair = RowRand(seed, g, 7) % static_cast<uint64_t>(n_pair_keys);
  w.pod = w.pair % 1024;
  w.addr_idx = w.pair / 1024;
  w.upid_lo = SplitMix(w.pod ^ 0x5555ULL);
  w.upid_hi = (w.pod << 32) | 0xABCDULL;
  w.svc = ZipfSample(svc_cdf, kServices, U01(RowRand(seed, g, 1)));
  w.path = ZipfSample(path_cdf, kPaths, U01(RowRand(seed, g, 2)));
  w.status = RespStatus(U01(RowRand(seed, g, 3)));
  w.latency = Latency(lat_grid, RowRand(seed, g, 4));
  w.req_body = static_cast<int64_t>(RowRand(seed, g, 8) % 65537);
  w.resp_body = static_cast<int64_t>(RowRand(seed, g, 9) % 65537);
  return w;
}

// Host-computed lookup tables (uploaded to the device as they are).
struct Tables {
  double svc_cdf[kServices];
  double path_cdf[kPaths];
  double lat_grid[kLatencyGrid + 1];
  char svc_bytes[kServices * 16];
  int32_t svc_off[kServices + 1];
  char path_bytes[kPaths * 48];
  int32_t path_off[kPaths + 1];
};

// Defined in datagen.cc.
const Tables& GetTables();

}  // namespace gen
}  // namespace pxg
