// JSON number rendering exactly as the reference's QuantilesUDA::Finalize produces it
// (src/carnot/funcs/builtins/math_sketches.h:40-54: a rapidjson::Document written with
// rapidjson::Writer<StringBuffer>).  rapidjson is a third-party dependency pinned at
// Tencent/rapidjson@f56928de85d56add3ca6ae7cf7f119a42ee1585b (bazel/repository_locations.bzl:
// 153-157) and is not vendored in the reference; this header restates its published number
// writer:
//   * Writer::WriteDouble -> internal::dtoa(value, buffer, maxDecimalPlaces = 324):
//     0 and -0 -> "0.0" / "-0.0"; otherwise a sign, Grisu2 digits, then Prettify.
//   * Grisu2 (Loitsch 2010) with 64-bit DiyFp arithmetic, the 87 cached powers
//     10^(-348 + 8i) (tools/gen_grisu_powers.py), DigitGen and GrisuRound.
//   * Prettify: fixed notation for decimal exponents in (-6, 21] with ".0" on integral values,
//     otherwise d[.ddd]e[-]X (no '+', no zero padding).
//   * NaN / +-inf: WriteDouble returns false with the default write flags, so
//     Document::Accept stops right after the key and its ':' -- the rendered object is
//     truncated there (e.g. `{"p01":` for an empty digest).
// Shared by the engine (carnot_host.cc) and the test oracle (oracle/carnot_oracle.cc).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>

namespace pxjson {

struct DiyFp {
  uint64_t f;
  int e;
};

inline DiyFp Mul(DiyFp a, DiyFp b) {  // 64x64 -> upper 64 bits, rounded by bit 63 of the low half
  const unsigned __int128 p = static_cast<unsigned __int128>(a.f) * b.f;
  uint64_t h = static_cast<uint64_t>(p >> 64);
  const uint64_t l = static_cast<uint64_t>(p);
  if (l & (uint64_t(1) << 63)) ++h;
  return DiyFp{h, a.e + b.e + 64};
}

inline DiyFp Normalize(DiyFp x) {
  while (!(x.f & (uint64_t(1) << 63))) {
    x.f <<= 1;
    x.e--;
  }
  return x;
}

constexpr uint64_t kHiddenBit = uint64_t(1) << 52;
constexpr uint64_t kSignificandMask = kHiddenBit - 1;

inline DiyFp FromDouble(double d) {
  uint64_t u;
  std::memcpy(&u, &d, 8);
  const int biased_e = static_cast<int>((u >> 52) & 0x7FF);
  const uint64_t significand = u & kSignificandMask;
  if (biased_e != 0) return DiyFp{significand + kHiddenBit, biased_e - 1075};
  return DiyFp{significand, -1074};
}

inline void NormalizedBoundaries(DiyFp v, DiyFp* minus, DiyFp* plus) {
  DiyFp pl{(v.f << 1) + 1, v.e - 1};
  while (!(pl.f & (kHiddenBit << 1))) {
    pl.f <<= 1;
    pl.e--;
  }
  pl.f <<= 10;  // 64 - 52 - 2
  pl.e -= 10;
  DiyFp mi = (v.f == kHiddenBit) ? DiyFp{(v.f << 2) - 1, v.e - 2} : DiyFp{(v.f << 1) - 1, v.e - 1};
  mi.f <<= mi.e - pl.e;
  mi.e = pl.e;
  *plus = pl;
  *minus = mi;
}

static const uint64_t kPow10F[87] = {
    0xfa8fd5a0081c0288ULL, 0xbaaee17fa23ebf76ULL, 0x8b16fb203055ac76ULL,
    0xcf42894a5dce35eaULL, 0x9a6bb0aa55653b2dULL, 0xe61acf033d1a45dfULL,
    0xab70fe17c79ac6caULL, 0xff77b1fcbebcdc4fULL, 0xbe5691ef416bd60cULL,
    0x8dd01fad907ffc3cULL, 0xd3515c2831559a83ULL, 0x9d71ac8fada6c9b5ULL,
    0xea9c227723ee8bcbULL, 0xaecc49914078536dULL, 0x823c12795db6ce57ULL,
    0xc21094364dfb5637ULL, 0x9096ea6f3848984fULL, 0xd77485cb25823ac7ULL,
    0xa086cfcd97bf97f4ULL, 0xef340a98172aace5ULL, 0xb23867fb2a35b28eULL,
    0x84c8d4dfd2c63f3bULL, 0xc5dd44271ad3cdbaULL, 0x936b9fcebb25c996ULL,
    0xdbac6c247d62a584ULL, 0xa3ab66580d5fdaf6ULL, 0xf3e2f893dec3f126ULL,
    0xb5b5ada8aaff80b8ULL, 0x87625f056c7c4a8bULL, 0xc9bcff6034c13053ULL,
    0x964e858c91ba2655ULL, 0xdff9772470297ebdULL, 0xa6dfbd9fb8e5b88fULL,
    0xf8a95fcf88747d94ULL, 0xb94470938fa89bcfULL, 0x8a08f0f8bf0f156bULL,
    0xcdb02555653131b6ULL, 0x993fe2c6d07b7facULL, 0xe45c10c42a2b3b06ULL,
    0xaa242499697392d3ULL, 0xfd87b5f28300ca0eULL, 0xbce5086492111aebULL,
    0x8cbccc096f5088ccULL, 0xd1b71758e219652cULL, 0x9c40000000000000ULL,
    0xe8d4a51000000000ULL, 0xad78ebc5ac620000ULL, 0x813f3978f8940984ULL,
    0xc097ce7bc90715b3ULL, 0x8f7e32ce7bea5c70ULL, 0xd5d238a4abe98068ULL,
    0x9f4f2726179a2245ULL, 0xed63a231d4c4fb27ULL, 0xb0de65388cc8ada8ULL,
    0x83c7088e1aab65dbULL, 0xc45d1df942711d9aULL, 0x924d692ca61be758ULL,
    0xda01ee641a708deaULL, 0xa26da3999aef774aULL, 0xf209787bb47d6b85ULL,
    0xb454e4a179dd1877ULL, 0x865b86925b9bc5c2ULL, 0xc83553c5c8965d3dULL,
    0x952ab45cfa97a0b3ULL, 0xde469fbd99a05fe3ULL, 0xa59bc234db398c25ULL,
    0xf6c69a72a3989f5cULL, 0xb7dcbf5354e9beceULL, 0x88fcf317f22241e2ULL,
    0xcc20ce9bd35c78a5ULL, 0x98165af37b2153dfULL, 0xe2a0b5dc971f303aULL,
    0xa8d9d1535ce3b396ULL, 0xfb9b7cd9a4a7443cULL, 0xbb764c4ca7a44410ULL,
    0x8bab8eefb6409c1aULL, 0xd01fef10a657842cULL, 0x9b10a4e5e9913129ULL,
    0xe7109bfba19c0c9dULL, 0xac2820d9623bf429ULL, 0x80444b5e7aa7cf85ULL,
    0xbf21e44003acdd2dULL, 0x8e679c2f5e44ff8fULL, 0xd433179d9c8cb841ULL,
    0x9e19db92b4e31ba9ULL, 0xeb96bf6ebadf77d9ULL, 0xaf87023b9bf0ee6bULL,
};
static const int16_t kPow10E[87] = {
    -1220, -1193, -1166, -1140, -1113, -1087, -1060, -1034, -1007, -980, -954, -927,
    -901, -874, -847, -821, -794, -768, -741, -715, -688, -661, -635, -608,
    -582, -555, -529, -502, -475, -449, -422, -396, -369, -343, -316, -289,
    -263, -236, -210, -183, -157, -130, -103, -77, -50, -24, 3, 30,
    56, 83, 109, 136, 162, 189, 216, 242, 269, 295, 322, 348,
    375, 402, 428, 455, 481, 508, 534, 561, 588, 614, 641, 667,
    694, 720, 747, 774, 800, 827, 853, 880, 907, 933, 960, 986,
    1013, 1039, 1066,
};

inline DiyFp GetCachedPower(int e, int* K) {
  const double dk = (-61 - e) * 0.30102999566398114 + 347;
  int k = static_cast<int>(dk);
  if (dk - k > 0.0) k++;
  const unsigned index = static_cast<unsigned>((k >> 3) + 1);
  *K = -(-348 + static_cast<int>(index << 3));
  return DiyFp{kPow10F[index], kPow10E[index]};
}

inline void GrisuRound(char* buffer, int len, uint64_t delta, uint64_t rest, uint64_t ten_kappa, uint64_t wp_w) {
  while (rest < wp_w && delta - rest >= ten_kappa && (rest + ten_kappa < wp_w || wp_w - rest > rest + ten_kappa - wp_w)) {
    buffer[len - 1]--;
    rest += ten_kappa;
  }
}

inline int CountDecimalDigit32(uint32_t n) {
  if (n < 10) return 1;
  if (n < 100) return 2;
  if (n < 1000) return 3;
  if (n < 10000) return 4;
  if (n < 100000) return 5;
  if (n < 1000000) return 6;
  if (n < 10000000) return 7;
  if (n < 100000000) return 8;
  return 9;
}

inline void DigitGen(DiyFp W, DiyFp Mp, uint64_t delta, char* buffer, int* len, int* K) {
  // 10^0 .. 10^19 (uint64): the fractional loop's rounding scales wp_w by 10^-kappa for up to 19
  // fractional digits (rapidjson: `index < 20 ? kPow10[index] : 0`).  An earlier version of this
  // header had 10 uint32 entries and `index < 9`, which skipped GrisuRound after the 9th fractional
  // digit and left e.g. 2419999.9999999997 where rapidjson writes 2419999.9999999995; the oracle's
  // separate restatement (oracle/json_number.h) exposed it.
  static const uint64_t kPow10[] = {1ULL,
                                    10ULL,
                                    100ULL,
                                    1000ULL,
                                    10000ULL,
                                    100000ULL,
                                    1000000ULL,
                                    10000000ULL,
                                    100000000ULL,
                                    1000000000ULL,
                                    10000000000ULL,
                                    100000000000ULL,
                                    1000000000000ULL,
                                    10000000000000ULL,
                                    100000000000000ULL,
                                    1000000000000000ULL,
                                    10000000000000000ULL,
                                    100000000000000000ULL,
                                    1000000000000000000ULL,
                                    10000000000000000000ULL};
  const DiyFp one{uint64_t(1) << -Mp.e, Mp.e};
  const uint64_t wp_w = Mp.f - W.f;
  uint32_t p1 = static_cast<uint32_t>(Mp.f >> -one.e);
  uint64_t p2 = Mp.f & (one.f - 1);
  int kappa = CountDecimalDigit32(p1);
  *len = 0;
  while (kappa > 0) {
    const uint32_t div = static_cast<uint32_t>(kPow10[kappa - 1]);
    const uint32_t d = p1 / div;
    p1 %= div;
    if (d || *len) buffer[(*len)++] = static_cast<char>('0' + d);
    kappa--;
    const uint64_t tmp = (static_cast<uint64_t>(p1) << -one.e) + p2;
    if (tmp <= delta) {
      *K += kappa;
      GrisuRound(buffer, *len, delta, tmp, kPow10[kappa] << -one.e, wp_w);
      return;
    }
  }
  for (;;) {
    p2 *= 10;
    delta *= 10;
    const char d = static_cast<char>(p2 >> -one.e);
    if (d || *len) buffer[(*len)++] = static_cast<char>('0' + d);
    p2 &= one.f - 1;
    kappa--;
    if (p2 < delta) {
      *K += kappa;
      const int index = -kappa;
      GrisuRound(buffer, *len, delta, p2, one.f, wp_w * (index < 20 ? kPow10[index] : 0));
      return;
    }
  }
}

inline void Grisu2(double value, char* buffer, int* length, int* K) {
  const DiyFp v = FromDouble(value);
  DiyFp w_m, w_p;
  NormalizedBoundaries(v, &w_m, &w_p);
  const DiyFp c_mk = GetCachedPower(w_p.e, K);
  const DiyFp W = Mul(Normalize(v), c_mk);
  DiyFp Wp = Mul(w_p, c_mk);
  DiyFp Wm = Mul(w_m, c_mk);
  Wm.f++;
  Wp.f--;
  DigitGen(W, Wp, Wp.f - Wm.f, buffer, length, K);
}

inline char* WriteExponent(int K, char* buffer) {
  if (K < 0) {
    *buffer++ = '-';
    K = -K;
  }
  if (K >= 100) {
    *buffer++ = static_cast<char>('0' + K / 100);
    K %= 100;
    *buffer++ = static_cast<char>('0' + K / 10);
    *buffer++ = static_cast<char>('0' + K % 10);
  } else if (K >= 10) {
    *buffer++ = static_cast<char>('0' + K / 10);
    *buffer++ = static_cast<char>('0' + K % 10);
  } else {
    *buffer++ = static_cast<char>('0' + K);
  }
  return buffer;
}

// Prettify with maxDecimalPlaces = 324 (Writer's default), so no truncation branch is taken.
inline char* Prettify(char* buffer, int length, int k) {
  const int kk = length + k;  // 10^(kk-1) <= v < 10^kk
  if (0 <= k && kk <= 21) {   // 1234e7 -> 12340000000.0
    for (int i = length; i < kk; i++) buffer[i] = '0';
    buffer[kk] = '.';
    buffer[kk + 1] = '0';
    return &buffer[kk + 2];
  }
  if (0 < kk && kk <= 21) {  // 1234e-2 -> 12.34
    std::memmove(&buffer[kk + 1], &buffer[kk], static_cast<size_t>(length - kk));
    buffer[kk] = '.';
    return &buffer[length + 1];
  }
  if (-6 < kk && kk <= 0) {  // 1234e-6 -> 0.001234
    const int offset = 2 - kk;
    std::memmove(&buffer[offset], &buffer[0], static_cast<size_t>(length));
    buffer[0] = '0';
    buffer[1] = '.';
    for (int i = 2; i < offset; i++) buffer[i] = '0';
    return &buffer[length + offset];
  }
  if (length == 1) {  // 1e30
    buffer[1] = 'e';
    return WriteExponent(kk - 1, &buffer[2]);
  }
  std::memmove(&buffer[2], &buffer[1], static_cast<size_t>(length - 1));  // 1234e30 -> 1.234e33
  buffer[1] = '.';
  buffer[length + 1] = 'e';
  return WriteExponent(kk - 1, &buffer[length + 2]);
}

inline bool IsNanOrInf(double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  return ((u >> 52) & 0x7FF) == 0x7FF;
}

// internal::dtoa: writes a finite double into buf (>= 32 bytes), returns the end.
inline char* Dtoa(double value, char* buffer) {
  uint64_t u;
  std::memcpy(&u, &value, 8);
  if ((u & ~(uint64_t(1) << 63)) == 0) {  // +-0
    if (u >> 63) *buffer++ = '-';
    buffer[0] = '0';
    buffer[1] = '.';
    buffer[2] = '0';
    return &buffer[3];
  }
  if (value < 0) {
    *buffer++ = '-';
    value = -value;
  }
  int length, K;
  Grisu2(value, buffer, &length, &K);
  return Prettify(buffer, length, K);
}

// Appends QuantilesUDA::Finalize's JSON for the 7 quantiles q[0..6] to out.
inline void AppendQuantilesJson(const double* q, std::string* out) {
  static const char* const kKeys[7] = {"p01", "p10", "p25", "p50", "p75", "p90", "p99"};
  out->push_back('{');
  char buf[40];
  for (int k = 0; k < 7; ++k) {
    if (k) out->push_back(',');
    out->push_back('"');
    out->append(kKeys[k], 3);
    out->append("\":", 2);
    if (IsNanOrInf(q[k])) return;  // Writer::Double fails: Accept stops, the object stays open
    out->append(buf, static_cast<size_t>(Dtoa(q[k], buf) - buf));
  }
  out->push_back('}');
}

}  // namespace pxjson
