// Device emulation of QuantilesUDA's t-digest (math_sketches.h:33-82 over third-party
// pixie-io/tdigest @85e0f700, compression 1000) for one group whose W values are sorted.
//
// For W <= 8*ceil(delta) the reference never processes before Finalize, so its digest is ONE
// process() over the sorted multiset with unit weights.  With unit weights wSoFar before
// element i is exactly i, so the centroid boundaries depend only on W:
//   s_0 = 0, wLimit_0 = W * Q(1);  s_{j+1} = max(s_j + 1, floor(wLimit_j)),
//   wLimit_{j+1} = W * Q(L(s_{j+1} / W) + 1)
// with L = integratedLocation, Q = integratedQ.  Q(L(x)+1) has the closed form
//   ((2x-1) cos(pi/d) + sqrt(1-(2x-1)^2) sin(pi/d) + 1) / 2      (d = delta, clamp to 1)
// which is evaluated first; whenever floor() could be decided differently by rounding (within
// 1e-9 of an integer, or near the clamp) the reference's own asin/sin expression is used.
// Each centroid mean is the reference's incremental update m += (v - m) / w in sorted order,
// and quantile() follows tdigest's cumulative-midpoint interpolation including its min/max
// tails.  For W >= ~1273 rounding-free singletons end; for W <= 1200 every centroid is a
// singleton (W * pi / (2 d) < 2) and the chain is skipped.
// Compile with -ffp-contract=off: the reference host build does not fuse multiply-adds.
#pragma once

#include "pxg_device.h"

namespace pxg {

constexpr double kDelta = 1000.0;
constexpr double kPi = 3.14159265358979323846;
constexpr double kDblMin = 2.2250738585072014e-308;   // numeric_limits<double>::min()
constexpr double kDblMax = 1.7976931348623157e+308;
constexpr int kSingletonMaxW = 1200;

__device__ __constant__ const double kQuantileQ[7] = {0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99};

__device__ __forceinline__ double StdMin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double StdMax(double a, double b) { return (a < b) ? b : a; }

__device__ __forceinline__ double WeightedAverageSorted(double x1, double w1, double x2, double w2) {
  const double x = (x1 * w1 + x2 * w2) / (w1 + w2);
  return StdMax(x1, StdMin(x, x2));
}
__device__ __forceinline__ double WeightedAverage(double x1, double w1, double x2, double w2) {
  return (x1 <= x2) ? WeightedAverageSorted(x1, w1, x2, w2) : WeightedAverageSorted(x2, w2, x1, w1);
}

__device__ __forceinline__ double IntegratedQ(double k) {
  return (sin(StdMin(k, kDelta) * kPi / kDelta - kPi / 2) + 1) / 2;
}
__device__ __forceinline__ double IntegratedLocation(double q) { return kDelta * (asin(2.0 * q - 1.0) + kPi / 2) / kPi; }

// wLimit after a boundary at index b (W total unit weights).  x = b / W is formed as
// b * (1/W) on the fast path: that moves wl by ~W * 1e-16, far inside the 1e-9 margin that
// sends a near-integer wl to the reference's own expression (which divides exactly).
__device__ __forceinline__ double NextLimit(int64_t b, double W, double invW) {
  const double kCos = 0.99999506519785548;   // cos(pi/1000)
  const double kSin = 0.0031415874858795635; // sin(pi/1000)
  const double x = static_cast<double>(static_cast<int32_t>(b)) * invW;
  const double t = 2.0 * x - 1.0;
  bool exact = t >= kCos - 1e-9;
  double wl = 0;
  if (!exact) {
    const double s = sqrt(fmax(0.0, (1.0 - t) * (1.0 + t)));
    wl = W * ((t * kCos + s * kSin + 1.0) * 0.5);
    const double r = rint(wl);
    if (fabs(wl - r) < 1e-9 * fmax(1.0, wl)) exact = true;
  }
  if (exact) wl = W * IntegratedQ(IntegratedLocation(static_cast<double>(b) / W) + 1.0);
  return wl;
}

// Generic quantile over centroids given accessors start(j) (j in [0,nc), start(0)=0),
// mean(j); W total weight.
template <typename StartF, typename MeanF>
__device__ double DigestQuantile(double q, int64_t nc, int64_t W, StartF start, MeanF mean) {
  if (nc <= 0) return __longlong_as_double(0x7FF8000000000000LL);
  if (nc == 1) return mean(0);
  const double Wd = static_cast<double>(W);
  const double index = q * Wd;
  auto weight = [&](int64_t j) -> double {
    return static_cast<double>((j + 1 < nc ? start(j + 1) : W) - start(j));
  };
  auto cum = [&](int64_t j) -> double {
    return j < nc ? static_cast<double>(start(j)) + weight(j) / 2.0 : Wd;
  };
  const double w0 = weight(0);
  const double mn = StdMin(kDblMax, mean(0));
  const double mx = StdMax(kDblMin, mean(nc - 1));
  if (index <= w0 / 2.0) return mn + 2.0 * index / w0 * (mean(0) - mn);
  int64_t lo = 0, hi = nc;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cum(mid) < index) lo = mid + 1;
    else hi = mid;
  }
  if (lo < nc) {
    const double z1 = index - cum(lo - 1);
    const double z2 = cum(lo) - index;
    return WeightedAverage(mean(lo - 1), z2, mean(lo), z1);
  }
  const double wl = weight(nc - 1);
  const double z1 = index - Wd - wl / 2.0;
  const double z2 = wl / 2 - z1;
  return WeightedAverage(mean(nc - 1), z1, mx, z2);
}

// tdigest::quantile() of a processed digest whose min_ / max_ are given explicitly (a merged
// digest: the merge tracks them from the merged lists' ends, not from its own first / last
// centroid), same interpolation as DigestQuantile.
template <typename StartF, typename MeanF>
__device__ double DigestQuantileMM(double q, int64_t nc, int64_t W, StartF start, MeanF mean, double mn, double mx) {
  if (nc <= 0) return __longlong_as_double(0x7FF8000000000000LL);
  if (nc == 1) return mean(0);
  const double Wd = static_cast<double>(W);
  const double index = q * Wd;
  auto weight = [&](int64_t j) -> double {
    return static_cast<double>((j + 1 < nc ? start(j + 1) : W) - start(j));
  };
  auto cum = [&](int64_t j) -> double {
    return j < nc ? static_cast<double>(start(j)) + weight(j) / 2.0 : Wd;
  };
  const double w0 = weight(0);
  if (index <= w0 / 2.0) return mn + 2.0 * index / w0 * (mean(0) - mn);
  int64_t lo = 0, hi = nc;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cum(mid) < index) lo = mid + 1;
    else hi = mid;
  }
  if (lo < nc) {
    const double z1 = index - cum(lo - 1);
    const double z2 = cum(lo) - index;
    return WeightedAverage(mean(lo - 1), z2, mean(lo), z1);
  }
  const double wl = weight(nc - 1);
  const double z1 = index - Wd - wl / 2.0;
  const double z2 = wl / 2 - z1;
  return WeightedAverage(mean(nc - 1), z1, mx, z2);
}

// Singleton digest (W <= kSingletonMaxW): centroid j = value j.
template <typename ValF>
__device__ __forceinline__ double SingletonQuantile(double q, int64_t W, ValF val) {
  return DigestQuantile(q, W, W, [](int64_t j) { return j; }, val);
}

// One step of the boundary chain: the centroid after the one starting at b starts at
// max(b + 1, floor(wLimit(b))) (W when wLimit reaches W; b = 0 uses the initial limit
// W * Q(1)).  A result >= W ends the chain.
__device__ __forceinline__ int32_t ChainNext(int32_t b, double Wd, double invW, int32_t W32) {
  const double wl = b == 0 ? Wd * IntegratedQ(1.0) : NextLimit(b, Wd, invW);
  const double f = floor(wl);
  const int32_t nb = f >= Wd ? W32 : static_cast<int32_t>(f);
  return nb < b + 1 ? b + 1 : nb;
}

// Build the centroid boundaries for W unit weights.  Single thread.  Returns the centroid
// count, or -1 if more than max_c centroids would be needed.
__device__ inline int64_t DigestBoundaries(int64_t W, uint32_t* starts, int64_t max_c) {
  if (W <= 0) return 0;
  int64_t nc = 0;
  starts[nc++] = 0;
  const double Wd = static_cast<double>(W);
  const double invW = 1.0 / Wd;
  const int32_t W32 = static_cast<int32_t>(W);  // W < 2^31 (staged rows are < 2^32 per agg)
  int32_t b = 0;
  while (true) {
    const int32_t nb = ChainNext(b, Wd, invW, W32);
    if (nb >= W32) break;
    if (nc >= max_c) return -1;
    starts[nc++] = static_cast<uint32_t>(nb);
    b = nb;
  }
  return nc;
}

// The same chain computed by one wave, ~10 steps per round instead of one: lane 0 evaluates
// the step at the current boundary b; the k + 2 lanes of group k (k = 1..9) evaluate it at the
// k + 2 integers just below the loss-free k-step prediction W * Q(L(b / W) + k) (+1 for
// rounding), the window that holds the k-th next boundary, since each step's floor loses less
// than one unit.  The round then follows the chain through the evaluated points (scalar
// ballot + readlane per step) as far as it stays inside the windows.  Every boundary comes
// from ChainNext at exactly the previous boundary, so the chain is bit-identical to
// DigestBoundaries; the windows only decide how many steps a round advances.  Wave-uniform
// control; `starts` written by the lanes holding the new boundaries.
constexpr int kSpecGroups = 10;
__device__ __forceinline__ void SpecLaneRole(int lane, int& k, int& d) {
  k = 0;
  d = 0;
  if (lane == 0) return;
  int base = 1;
  k = 1;
  while (lane >= base + k + 2) {
    base += k + 2;
    ++k;
  }
  d = lane - base;
}

template <bool kStats = false>
__device__ __forceinline__ int64_t DigestBoundariesWave(int64_t W, uint32_t* starts, int64_t max_c, uint64_t* stats = nullptr) {
  uint64_t st_eval = 0, st_res = 0, st_it = 0, st_exact = 0, t0 = 0, t1 = 0;
  const int lane = threadIdx.x & 63;
  if (W <= 0) return 0;
  if (lane == 0) starts[0] = 0;
  const double Wd = static_cast<double>(W);
  const double invW = 1.0 / Wd;
  const int32_t W32 = static_cast<int32_t>(W);
  const int32_t Wu = __builtin_amdgcn_readfirstlane(W32);  // wave-uniform (scalar compares)
  int k, d;
  SpecLaneRole(lane, k, d);
  const double ck = cos(static_cast<double>(k) * (kPi / kDelta));
  const double sk = sin(static_cast<double>(k) * (kPi / kDelta));
  int64_t nc = 1;
  int32_t b = 0;
  while (true) {
    if (kStats) t0 = __builtin_readcyclecounter();
    int32_t top = b;
    if (k > 0) {
      const double t = 2.0 * (static_cast<double>(b) * invW) - 1.0;
      top = W32;
      if (t <= ck) {  // else the k-step rotation passes the end of the scale
        const double s = sqrt(fmax(0.0, (1.0 - t) * (1.0 + t)));
        const double p = Wd * ((t * ck + s * sk + 1.0) * 0.5);
        top = p >= Wd ? W32 : static_cast<int32_t>(floor(p)) + 1;
      }
      if (top < b + k) top = b + k;
    }
    const int32_t x = top - d;
    const bool ok = x >= b + k && x < W32;
    const int32_t fx = ok ? ChainNext(x, Wd, invW, W32) : -1;
    if (kStats) {
      const double tt = 2.0 * (static_cast<double>(x) * invW) - 1.0;
      const double ss = sqrt(fmax(0.0, (1.0 - tt) * (1.0 + tt)));
      const double wl = Wd * ((tt * 0.99999506519785548 + ss * 0.0031415874858795635 + 1.0) * 0.5);
      const bool ex = ok && x > 0 && (tt >= 0.99999506519785548 - 1e-9 || fabs(wl - rint(wl)) < 1e-9 * fmax(1.0, wl));
      st_exact += __ballot(ex) ? 1 : 0;
      t1 = __builtin_readcyclecounter();
      st_eval += t1 - t0;
      ++st_it;
    }
    // Follow the chain with scalar arithmetic, branch-free: the next boundary after cur sits
    // in group kk's window at offset top_kk - cur, i.e. in lane base_kk + top_kk - cur (a
    // uniform index, so a plain readlane); the new boundaries are collected into lanes 0..
    int32_t cur = b, mine = 0;
    int cnt = 0;
    bool live = true, done = false;
    int base = 1;
#pragma unroll
    for (int kk = 0; kk < kSpecGroups; ++kk) {
      int32_t nx;
      if (kk == 0) {
        nx = __builtin_amdgcn_readlane(fx, 0);
      } else {
        const int32_t off = __builtin_amdgcn_readlane(top, base) - cur;
        const bool inwin = off >= 0 && off < kk + 2;
        live = live && inwin;
        nx = __builtin_amdgcn_readlane(fx, base + (inwin ? off : 0));
        base += kk + 2;
      }
      const bool fin = live && nx >= Wu;
      done = done || fin;
      live = live && !fin;
      if (live && lane == cnt) mine = nx;
      cnt += live ? 1 : 0;
      cur = live ? nx : cur;
    }
    if (nc + cnt > max_c) return -1;
    if (lane < cnt) starts[nc + lane] = static_cast<uint32_t>(mine);
    nc += cnt;
    b = cur;
    if (kStats) st_res += __builtin_readcyclecounter() - t1;
    if (done) break;
  }
  if (kStats && (threadIdx.x & 63) == 0) {
    stats[0] = st_eval;
    stats[1] = st_res;
    stats[2] = st_it;
    stats[3] = st_exact;
  }
  return nc;
}

// Incremental centroid mean over sorted values [s, e) (Centroid::add with unit weights).
template <typename ValF>
__device__ __forceinline__ double CentroidMean(ValF val, int64_t s, int64_t e) {
  double m = val(s);
  double w = 1.0;
  for (int64_t t = s + 1; t < e; ++t) {
    w += 1.0;
    m += 1.0 * (val(t) - m) / w;
  }
  return m;
}

}  // namespace pxg
