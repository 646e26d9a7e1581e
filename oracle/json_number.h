// ORACLE / TEST INFRASTRUCTURE ONLY.  The oracle's own restatement of the number writer behind
// QuantilesUDA::Finalize (src/carnot/funcs/builtins/math_sketches.h:40-54: a rapidjson::Document
// written by rapidjson::Writer<StringBuffer>).  rapidjson is not vendored in the reference; it is
// pinned at Tencent/rapidjson@f56928de85d56add3ca6ae7cf7f119a42ee1585b
// (bazel/repository_locations.bzl:153-157).  Writer::Double calls internal::dtoa(v, buf, 324):
//   * +-0 -> "0.0" / "-0.0"; a negative value gets '-' and is written as its magnitude;
//   * Grisu2 (Loitsch, "Printing floating-point numbers quickly and accurately", PLDI 2010) over
//     64-bit "DiyFp" numbers: the value's boundaries m- / m+ normalised to a common exponent, a
//     cached power c_k = 10^(-348 + 8i) that brings the exponent of m+ into [-60, -32], the
//     products rounded half-up on bit 63 of the low word, m- + 1 ulp and m+ - 1 ulp, then digit
//     generation (integral part digit by digit while the remainder exceeds delta, then
//     fractional digits) and the GrisuRound walk towards the scaled value;
//   * Prettify with maxDecimalPlaces = 324: for K digits d and exponent k (v = d * 10^k, kk =
//     K + k): 0 <= k && kk <= 21 -> digits, zeros, ".0"; 0 < kk <= 21 -> a point inside the
//     digits; -6 < kk <= 0 -> "0." and zeros; one digit -> "de<kk-1>"; else "d.ddde<kk-1>" with
//     the exponent as '-'? plus its decimal digits (no '+', no padding);
//   * NaN / inf: Writer::Double fails (default write flags) and Document::Accept stops, so the
//     object ends right after the key's ':'.
//
// This file is written independently of pixie_amd/host/json_double.h (the product's renderer):
// the cached powers are computed here at first use with exact multi-precision arithmetic
// (10^k rounded to 64 significant bits, half-up), not read from a generated table, and the
// digit generation and Prettify are separate code.  tests/test_json_double.py compares the two
// renderers byte for byte over ~10^6 doubles.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace oracle_json {

struct Fp {  // f * 2^e
  uint64_t f;
  int e;
};

inline Fp FpMul(const Fp& a, const Fp& b) {
  const uint64_t a_hi = a.f >> 32, a_lo = a.f & 0xFFFFFFFFu, b_hi = b.f >> 32, b_lo = b.f & 0xFFFFFFFFu;
  // Schoolbook 32 x 32 partial products, then the upper 64 bits rounded on bit 63 of the lower.
  const uint64_t hh = a_hi * b_hi, hl = a_hi * b_lo, lh = a_lo * b_hi, ll = a_lo * b_lo;
  const uint64_t mid = (ll >> 32) + (hl & 0xFFFFFFFFu) + (lh & 0xFFFFFFFFu);
  uint64_t hi = hh + (hl >> 32) + (lh >> 32) + (mid >> 32);
  const uint64_t lo = (mid << 32) | (ll & 0xFFFFFFFFu);
  if (lo >> 63) ++hi;
  return Fp{hi, a.e + b.e + 64};
}

// ---- cached powers: 10^q (q = -348 + 8i, i < 87) as (64-bit significand, binary exponent) ----
// Little-endian base-2^32 natural numbers, just enough for 10^348 and 2^k / 10^348.
using Big = std::vector<uint32_t>;

inline void BigMulSmall(Big& x, uint32_t m) {
  uint64_t carry = 0;
  for (auto& w : x) {
    const uint64_t t = static_cast<uint64_t>(w) * m + carry;
    w = static_cast<uint32_t>(t);
    carry = t >> 32;
  }
  if (carry) x.push_back(static_cast<uint32_t>(carry));
}
inline uint32_t BigDivSmall(Big& x, uint32_t d) {  // x /= d, returns the remainder
  uint64_t rem = 0;
  for (size_t i = x.size(); i-- > 0;) {
    const uint64_t t = (rem << 32) | x[i];
    x[i] = static_cast<uint32_t>(t / d);
    rem = t % d;
  }
  while (!x.empty() && x.back() == 0) x.pop_back();
  return static_cast<uint32_t>(rem);
}
inline int BigBits(const Big& x) {
  if (x.empty()) return 0;
  int b = 32 * static_cast<int>(x.size() - 1);
  for (uint32_t t = x.back(); t; t >>= 1) ++b;
  return b;
}
inline bool BigBit(const Big& x, int i) { return (x[static_cast<size_t>(i) / 32] >> (i % 32)) & 1u; }
inline uint64_t BigTop64(const Big& x, int* shift) {  // top 64 bits, half-up on the next bit
  const int nb = BigBits(x);
  *shift = nb - 64;
  uint64_t f = 0;
  for (int i = 0; i < 64; ++i) f = (f << 1) | ((nb - 1 - i >= 0 && BigBit(x, nb - 1 - i)) ? 1u : 0u);  // (short x: zeros below)
  if (nb > 64 && BigBit(x, nb - 65)) ++f;  // (10^q is never a tie: its low bits are not all zero)
  return f;
}

struct Power {
  uint64_t f;
  int e;
};
inline Power ExactPower10(int q) {
  if (q >= 0) {
    Big x{1};
    for (int i = 0; i < q; ++i) BigMulSmall(x, 10);
    int sh = 0;
    uint64_t f = BigTop64(x, &sh);
    if (f == 0) {  // the rounding carried out of 64 bits (does not happen for powers of ten)
      f = uint64_t(1) << 63;
      ++sh;
    }
    return Power{f, sh};
  }
  // 10^q = 2^-s * (2^s / 10^-q): floor division by 10 repeated -q times is the exact floor of
  // 2^s / 10^-q; s leaves 66+ quotient bits, and the dropped remainder only makes the rounding
  // bit's sticky part non-zero (never a tie).
  const int s = 64 + 4 * (-q) + 8;
  Big x(static_cast<size_t>(s / 32 + 1), 0u);
  x[static_cast<size_t>(s / 32)] = 1u << (s % 32);
  for (int i = 0; i < -q; ++i) BigDivSmall(x, 10);
  int sh = 0;
  const uint64_t f = BigTop64(x, &sh);
  return Power{f, sh - s};
}

inline const std::vector<Power>& CachedPowers() {
  static const std::vector<Power> table = [] {
    std::vector<Power> t;
    for (int i = 0; i < 87; ++i) t.push_back(ExactPower10(-348 + 8 * i));
    return t;
  }();
  return table;
}

// GetCachedPower: the cached power whose product with a number of binary exponent e lands the
// exponent in Grisu2's window; K receives minus its decimal exponent.
inline Fp CachedPowerFor(int e, int* K) {
  const double dk = (-61 - e) * 0.30102999566398114 + 347;
  int k = static_cast<int>(dk);
  if (dk - k > 0.0) ++k;
  const unsigned idx = static_cast<unsigned>((k >> 3) + 1);
  *K = 348 - static_cast<int>(idx * 8);
  const Power& p = CachedPowers()[idx];
  return Fp{p.f, p.e};
}

// ---- Grisu2 ----
inline void Round(std::string& digits, uint64_t delta, uint64_t rest, uint64_t ten_kappa, uint64_t wp_w) {
  while (rest < wp_w && delta - rest >= ten_kappa && (rest + ten_kappa < wp_w || wp_w - rest > rest + ten_kappa - wp_w)) {
    digits.back() = static_cast<char>(digits.back() - 1);
    rest += ten_kappa;
  }
}

inline int DecimalDigits(uint32_t v) {
  int n = 1;
  while (v >= 10) {
    v /= 10;
    ++n;
  }
  return n;
}

inline uint64_t Pow10u(int i) {
  uint64_t r = 1;
  while (i-- > 0) r *= 10;
  return r;
}

// Digits of the shortest-in-Grisu2 representation of (Mp - delta, Mp], W the scaled value.
inline void Digits(const Fp& W, const Fp& Mp, uint64_t delta, std::string& digits, int* K) {
  const int sh = -Mp.e;  // the scaled numbers have a fixed point at bit sh
  const uint64_t one = uint64_t(1) << sh;
  const uint64_t wp_w = Mp.f - W.f;
  uint32_t integral = static_cast<uint32_t>(Mp.f >> sh);
  uint64_t frac = Mp.f & (one - 1);
  int kappa = DecimalDigits(integral);
  while (kappa > 0) {
    const uint32_t div = static_cast<uint32_t>(Pow10u(kappa - 1));
    const uint32_t d = integral / div;
    integral %= div;
    if (d != 0 || !digits.empty()) digits.push_back(static_cast<char>('0' + d));
    --kappa;
    const uint64_t rest = (static_cast<uint64_t>(integral) << sh) + frac;
    if (rest <= delta) {
      *K += kappa;
      Round(digits, delta, rest, Pow10u(kappa) << sh, wp_w);
      return;
    }
  }
  for (;;) {
    frac *= 10;
    delta *= 10;
    const char d = static_cast<char>(frac >> sh);
    if (d != 0 || !digits.empty()) digits.push_back(static_cast<char>('0' + d));
    frac &= one - 1;
    --kappa;
    if (frac < delta) {
      *K += kappa;
      const int idx = -kappa;
      Round(digits, delta, frac, one, wp_w * (idx < 20 ? Pow10u(idx) : 0));
      return;
    }
  }
}

// A positive finite double -> (digits, K) with value ~ digits * 10^K.
inline void Grisu(double v, std::string& digits, int* K) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  const int be = static_cast<int>((u >> 52) & 0x7FF);
  const uint64_t frac = u & ((uint64_t(1) << 52) - 1);
  Fp x = be ? Fp{frac | (uint64_t(1) << 52), be - 1075} : Fp{frac, -1074};
  // Upper boundary (2f + 1) / 2, normalised so that bit 63 is set.
  Fp plus{(x.f << 1) + 1, x.e - 1};
  while (!(plus.f & (uint64_t(1) << 53))) {
    plus.f <<= 1;
    --plus.e;
  }
  plus.f <<= 10;
  plus.e -= 10;
  // Lower boundary: closer below a power of two (f is the hidden bit alone).
  Fp minus = (x.f == (uint64_t(1) << 52)) ? Fp{(x.f << 2) - 1, x.e - 2} : Fp{(x.f << 1) - 1, x.e - 1};
  minus.f <<= (minus.e - plus.e);
  minus.e = plus.e;
  // The value itself, normalised.
  Fp w = x;
  while (!(w.f & (uint64_t(1) << 63))) {
    w.f <<= 1;
    --w.e;
  }
  const Fp c = CachedPowerFor(plus.e, K);
  const Fp W = FpMul(w, c);
  Fp Wp = FpMul(plus, c);
  Fp Wm = FpMul(minus, c);
  Wm.f += 1;
  Wp.f -= 1;
  digits.clear();
  Digits(W, Wp, Wp.f - Wm.f, digits, K);
}

inline void Exponent(int e, std::string& out) {
  if (e < 0) {
    out.push_back('-');
    e = -e;
  }
  out += std::to_string(e);
}

// internal::dtoa(value, buffer, 324) for a finite value, appended to out.
inline void AppendNumber(double v, std::string& out) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  if ((u << 1) == 0) {
    out += (u >> 63) ? "-0.0" : "0.0";
    return;
  }
  if (u >> 63) {
    out.push_back('-');
    v = -v;
  }
  std::string d;
  int k = 0;
  Grisu(v, d, &k);
  const int len = static_cast<int>(d.size());
  const int kk = len + k;
  if (k >= 0 && kk <= 21) {
    out += d;
    out.append(static_cast<size_t>(kk - len), '0');
    out += ".0";
  } else if (kk > 0 && kk <= 21) {
    out.append(d, 0, static_cast<size_t>(kk));
    out.push_back('.');
    out.append(d, static_cast<size_t>(kk), std::string::npos);
  } else if (kk > -6 && kk <= 0) {
    out += "0.";
    out.append(static_cast<size_t>(-kk), '0');
    out += d;
  } else if (len == 1) {
    out += d;
    out.push_back('e');
    Exponent(kk - 1, out);
  } else {
    out.push_back(d[0]);
    out.push_back('.');
    out.append(d, 1, std::string::npos);
    out.push_back('e');
    Exponent(kk - 1, out);
  }
}

inline bool Finite(double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  return ((u >> 52) & 0x7FF) != 0x7FF;
}

// The document QuantilesUDA::Finalize writes: {"p01":..,...,"p99":..}, cut after the key of the
// first non-finite value.
inline void AppendQuantilesJson(const double* q, std::string* out) {
  static const char* const kKeys[7] = {"p01", "p10", "p25", "p50", "p75", "p90", "p99"};
  out->push_back('{');
  for (int i = 0; i < 7; ++i) {
    if (i > 0) out->push_back(',');
    *out += '"';
    *out += kKeys[i];
    *out += "\":";
    if (!Finite(q[i])) return;
    AppendNumber(q[i], *out);
  }
  out->push_back('}');
}

}  // namespace oracle_json
