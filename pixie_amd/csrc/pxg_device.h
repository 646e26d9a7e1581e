// Device-side data layout and helpers shared by the libpxg kernels (gfx950 / CDNA4, wave64).
//
// HBM layout of a table: columns are Arrow-layout arrays grouped in chunks of
// <= 2^24 rows; STRING = int32 offsets relative to the chunk's payload + payload bytes padded
// by 16 B so that 8-byte word loads past the end stay in bounds.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pxg.h"

namespace pxg {

constexpr int kMaxCols = 16;
constexpr int kMaxKeys = 4;
constexpr int kMaxUdas = 16;
constexpr int kMaxVals = 16;  // distinct staged value streams (a split-agg merge of 9 UDAs reads 11)
constexpr int kChunkShift = 24;
constexpr int64_t kChunkRows = int64_t(1) << kChunkShift;
constexpr int kWave = 64;

struct DevCol {
  const uint8_t* values;   // fixed width
  const int32_t* offsets;  // STRING
  const uint8_t* data;     // STRING payload (+16 B pad)
};

struct DevChunk {
  int64_t nrows;
  int64_t row_base;
  DevCol cols[kMaxCols];
};

// A decoded program (pxg_program) in device memory, with a pre-classified fast shape.
enum ProgShape : int32_t {
  kShapeGeneric = 0,
  kShapeCol = 1,          // single column reference
  kShapeColOpConst = 2,   // COL [conv] CONST OP  (conv in {none, I2F, B2I})
};

struct DevInsn {
  uint16_t op;
  uint16_t type;
  int32_t arg;
  int64_t imm;
};

struct DevProgram {
  int32_t n;
  int32_t result_type;
  int32_t shape;
  int32_t col;       // shape col
  int32_t conv;      // shape conversion opcode (0 = none)
  int32_t binop;     // shape binary opcode
  int64_t cimm;      // shape constant bits
  const uint8_t* pool;
  DevInsn insns[PXG_MAX_PROGRAM];
};

struct Val {
  uint64_t a;  // fixed value bits / string pointer / u128 low
  uint64_t b;  // string length / u128 high
};

__device__ __forceinline__ double AsF(uint64_t x) { return __longlong_as_double(static_cast<long long>(x)); }
__device__ __forceinline__ uint64_t FBits(double d) { return static_cast<uint64_t>(__double_as_longlong(d)); }

// ---------------------------------------------------------------------------------------
// Hashing.  Any hash works for correctness (group output is unordered, test_utils.h:439-447);
// equality is always checked on the exact bytes (row_tuple.h:109-133).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t Fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// Unaligned 8-byte little-endian load built from aligned 8-byte loads (buffers are padded).
__device__ __forceinline__ uint64_t LoadWordU(const uint8_t* p) {
  uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~uintptr_t(7));
  unsigned sh = static_cast<unsigned>(a & 7) * 8;
  uint64_t lo = w[0];
  if (sh == 0) return lo;
  uint64_t hi = w[1];
  return (lo >> sh) | (hi << (64 - sh));
}

__device__ __forceinline__ uint64_t TailMask(uint32_t nbytes) {
  return nbytes >= 8 ? ~0ULL : ((1ULL << (nbytes * 8)) - 1);
}

__device__ __forceinline__ uint64_t HashBytes(const uint8_t* p, uint32_t len, uint64_t h) {
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w = LoadWordU(p + i);
    h = (h ^ w) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29;
  }
  if (i < len) {
    uint64_t w = LoadWordU(p + i) & TailMask(len - i);
    h = (h ^ w) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29;
  }
  return Fmix64(h ^ (static_cast<uint64_t>(len) * 0xC2B2AE3D27D4EB4FULL));
}

__device__ __forceinline__ bool BytesEqual(const uint8_t* a, const uint8_t* b, uint32_t len) {
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8)
    if (LoadWordU(a + i) != LoadWordU(b + i)) return false;
  if (i < len) {
    uint64_t m = TailMask(len - i);
    if ((LoadWordU(a + i) & m) != (LoadWordU(b + i) & m)) return false;
  }
  return true;
}

// Lexicographic byte compare (std::string operator<): returns <0, 0, >0.
__device__ __forceinline__ int BytesCompare(const uint8_t* a, uint32_t la, const uint8_t* b, uint32_t lb) {
  uint32_t n = la < lb ? la : lb;
  for (uint32_t i = 0; i < n; i += 8) {
    uint32_t rem = n - i;
    uint64_t m = TailMask(rem);
    uint64_t x = LoadWordU(a + i) & m, y = LoadWordU(b + i) & m;
    if (x != y) {
      // first differing byte decides (little-endian words)
      uint64_t d = x ^ y;
      int byte = __ffsll(static_cast<long long>(d)) - 1;
      byte >>= 3;
      uint8_t xa = static_cast<uint8_t>(x >> (byte * 8)), ya = static_cast<uint8_t>(y >> (byte * 8));
      return xa < ya ? -1 : 1;
    }
  }
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

// Order-preserving map of double bits onto signed int64 (for min/max/sort); -0.0 < +0.0.
__device__ __forceinline__ int64_t OrderedFromDouble(uint64_t bits) {
  int64_t s = static_cast<int64_t>(bits);
  return s ^ ((s >> 63) & 0x7FFFFFFFFFFFFFFFLL);
}
__device__ __forceinline__ uint64_t DoubleFromOrdered(int64_t o) {
  return static_cast<uint64_t>(o ^ ((o >> 63) & 0x7FFFFFFFFFFFFFFFLL));
}
// Unsigned sort key for doubles (ascending).
__device__ __forceinline__ uint64_t SortKeyF(uint64_t bits) {
  return bits ^ ((bits >> 63) ? ~0ULL : 0x8000000000000000ULL);
}
__device__ __forceinline__ uint64_t FromSortKeyF(uint64_t k) {
  return k ^ ((k >> 63) ? 0x8000000000000000ULL : ~0ULL);
}

// ---------------------------------------------------------------------------------------
// Column access.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ Val LoadCol(const DevCol& c, int type, int64_t r) {
  Val v;
  switch (type) {
    case PXG_BOOLEAN: v.a = c.values[r]; v.b = 0; break;
    case PXG_UINT128: {
      const uint64_t* p = reinterpret_cast<const uint64_t*>(c.values) + 2 * r;
      v.a = p[0];
      v.b = p[1];
      break;
    }
    case PXG_STRING: {
      int32_t o0 = c.offsets[r], o1 = c.offsets[r + 1];
      v.a = reinterpret_cast<uint64_t>(c.data + o0);
      v.b = static_cast<uint64_t>(o1 - o0);
      break;
    }
    default: v.a = reinterpret_cast<const uint64_t*>(c.values)[r]; v.b = 0; break;
  }
  return v;
}

__device__ __forceinline__ int64_t SModI(int64_t a, int64_t b) { return (b == 0 || b == -1) ? 0 : a % b; }

__host__ __device__ __forceinline__ bool IsStrOp(int op) { return op >= PXG_OP_EQ_S && op <= PXG_OP_GE_S; }

// Binary op on two fixed-width slots; result bits (bool = 0/1).
__device__ __forceinline__ uint64_t BinOp(int op, uint64_t x, uint64_t y) {
  int64_t a = static_cast<int64_t>(x), b = static_cast<int64_t>(y);
  double fa = AsF(x), fb = AsF(y);
  switch (op) {
    case PXG_OP_ADD_I: return x + y;
    case PXG_OP_SUB_I: return x - y;
    case PXG_OP_MUL_I: return x * y;
    case PXG_OP_MOD_I: return static_cast<uint64_t>(SModI(a, b));
    case PXG_OP_BIN_I: return x - static_cast<uint64_t>(SModI(a, b));
    case PXG_OP_ADD_F: return FBits(fa + fb);
    case PXG_OP_SUB_F: return FBits(fa - fb);
    case PXG_OP_MUL_F: return FBits(fa * fb);
    case PXG_OP_DIV_F: return FBits(fa / fb);
    case PXG_OP_EQ_I: return a == b;
    case PXG_OP_NE_I: return a != b;
    case PXG_OP_LT_I: return a < b;
    case PXG_OP_LE_I: return a <= b;
    case PXG_OP_GT_I: return a > b;
    case PXG_OP_GE_I: return a >= b;
    case PXG_OP_EQ_F: return fa == fb;
    case PXG_OP_NE_F: return fa != fb;
    case PXG_OP_LT_F: return fa < fb;
    case PXG_OP_LE_F: return fa <= fb;
    case PXG_OP_GT_F: return fa > fb;
    case PXG_OP_GE_F: return fa >= fb;
    case PXG_OP_APPROX_EQ_F: return fabs(fa - fb) < 2.220446049250313e-16;
    case PXG_OP_APPROX_NE_F: return fabs(fa - fb) > 2.220446049250313e-16;
    case PXG_OP_AND: return (x != 0) && (y != 0);
    case PXG_OP_OR: return (x != 0) || (y != 0);
    default: return 0;
  }
}

__device__ __forceinline__ uint64_t Conv(int op, uint64_t x) {
  switch (op) {
    case PXG_OP_I2F: return FBits(static_cast<double>(static_cast<int64_t>(x)));
    case PXG_OP_B2I: return x != 0;
    case PXG_OP_I2B: return x != 0;
    case PXG_OP_F2I: return static_cast<uint64_t>(static_cast<int64_t>(AsF(x)));
    default: return x;
  }
}

__device__ __forceinline__ uint64_t StrOp(int op, const Val& x, const Val& y) {
  const uint8_t* pa = reinterpret_cast<const uint8_t*>(x.a);
  const uint8_t* pb = reinterpret_cast<const uint8_t*>(y.a);
  uint32_t la = static_cast<uint32_t>(x.b), lb = static_cast<uint32_t>(y.b);
  if (op == PXG_OP_EQ_S) return la == lb && BytesEqual(pa, pb, la);
  if (op == PXG_OP_NE_S) return !(la == lb && BytesEqual(pa, pb, la));
  int c = BytesCompare(pa, la, pb, lb);
  switch (op) {
    case PXG_OP_LT_S: return c < 0;
    case PXG_OP_LE_S: return c <= 0;
    case PXG_OP_GT_S: return c > 0;
    default: return c >= 0;
  }
}

// The two fast shapes alone (no interpreter stack: kernels that only take these shapes keep
// their register budget small).  Fixed-width columns only.
__device__ __forceinline__ uint64_t EvalShape(const DevProgram* __restrict__ p, const DevChunk& ch, int64_t r,
                                              const int32_t* __restrict__ col_types) {
  const Val v = LoadCol(ch.cols[p->col], col_types[p->col], r);
  if (p->shape == kShapeCol) return v.a;
  const uint64_t x = p->conv ? Conv(p->conv, v.a) : v.a;
  return BinOp(p->binop, x, static_cast<uint64_t>(p->cimm));
}

// A fast shape applied to an already loaded value of its (fixed-width) column.
__device__ __forceinline__ uint64_t ApplyShape(const DevProgram* __restrict__ p, uint64_t v) {
  if (p->shape == kShapeCol) return v;
  const uint64_t x = p->conv ? Conv(p->conv, v) : v;
  return BinOp(p->binop, x, static_cast<uint64_t>(p->cimm));
}

// A `col op const` integer comparison (no conversion) on an 8-byte signed column as a range test:
// BinOp(op, x, c) == (lo <= x <= hi) != neg.  Lets a filter loop issue all its loads before any
// compare, with no per-row dispatch on the op.
__device__ __forceinline__ bool FilterRange(const DevProgram* __restrict__ p, int col_type, int64_t* lo, int64_t* hi, bool* neg) {
  if (p->shape != kShapeColOpConst || p->conv != 0 || (col_type != PXG_INT64 && col_type != PXG_TIME64NS)) return false;
  const int64_t c = p->cimm;
  *lo = INT64_MIN;
  *hi = INT64_MAX;
  *neg = false;
  switch (p->binop) {
    case PXG_OP_EQ_I: *lo = c; *hi = c; return true;
    case PXG_OP_NE_I: *lo = c; *hi = c; *neg = true; return true;
    case PXG_OP_GE_I: *lo = c; return true;
    case PXG_OP_LE_I: *hi = c; return true;
    case PXG_OP_GT_I:
      if (c == INT64_MAX) *neg = true;  // empty: the full range negated
      else *lo = c + 1;
      return true;
    case PXG_OP_LT_I:
      if (c == INT64_MIN) *neg = true;
      else *hi = c - 1;
      return true;
    default: return false;
  }
}

// Whether rows of a fast shape's column can be read two at a time with 16-byte loads: an 8-byte
// column whose values start 16-byte aligned (the pair loads then start at even rows).
__device__ __forceinline__ bool PairLoadable(const DevProgram* __restrict__ p, const DevChunk& ch,
                                             const int32_t* __restrict__ col_types) {
  const int t = col_types[p->col];
  return (t == PXG_INT64 || t == PXG_FLOAT64 || t == PXG_TIME64NS) &&
         (reinterpret_cast<uintptr_t>(ch.cols[p->col].values) & 15) == 0;
}

// Evaluate a program on row r of chunk ch.  Uniform control flow across the wave (every lane
// runs the same program); the generic path keeps its stack in private memory.
__device__ inline Val EvalProgram(const DevProgram* __restrict__ p, const DevChunk& ch, int64_t r,
                                  const int32_t* __restrict__ col_types) {
  const int shape = p->shape;
  if (shape == kShapeCol) {
    return LoadCol(ch.cols[p->col], col_types[p->col], r);
  }
  if (shape == kShapeColOpConst) {
    Val v = LoadCol(ch.cols[p->col], col_types[p->col], r);
    uint64_t x = p->conv ? Conv(p->conv, v.a) : v.a;
    Val o;
    o.a = BinOp(p->binop, x, static_cast<uint64_t>(p->cimm));
    o.b = 0;
    return o;
  }
  Val st[PXG_MAX_STACK];
  int sp = 0;
  const int n = p->n;
  for (int pc = 0; pc < n; ++pc) {
    const DevInsn in = p->insns[pc];
    switch (in.op) {
      case PXG_OP_COL: st[sp++] = LoadCol(ch.cols[in.arg], col_types[in.arg], r); break;
      case PXG_OP_CONST:
        if (in.type == PXG_STRING) {
          st[sp].a = reinterpret_cast<uint64_t>(p->pool + in.arg);
          st[sp].b = static_cast<uint64_t>(in.imm);
        } else if (in.type == PXG_UINT128) {
          const uint64_t* q = reinterpret_cast<const uint64_t*>(p->pool + in.arg);
          st[sp].a = q[0];
          st[sp].b = q[1];
        } else {
          st[sp].a = static_cast<uint64_t>(in.imm);
          st[sp].b = 0;
        }
        ++sp;
        break;
      case PXG_OP_I2F:
      case PXG_OP_B2I:
      case PXG_OP_I2B:
      case PXG_OP_F2I: st[sp - 1].a = Conv(in.op, st[sp - 1].a); break;
      case PXG_OP_NEG_I: st[sp - 1].a = 0 - st[sp - 1].a; break;
      case PXG_OP_INV_I: st[sp - 1].a = ~st[sp - 1].a; break;
      case PXG_OP_NEG_F: st[sp - 1].a = st[sp - 1].a ^ 0x8000000000000000ULL; break;
      case PXG_OP_NOT: st[sp - 1].a = st[sp - 1].a == 0; break;
      case PXG_OP_STATE_WORD: {  // UDA::Deserialize of one state word (udf.h:98-100)
        const DevCol& c = ch.cols[in.arg];
        const int32_t o0 = c.offsets[r], o1 = c.offsets[r + 1];
        uint64_t w = 0;
        if (static_cast<int64_t>(o1 - o0) >= in.imm + 8) __builtin_memcpy(&w, c.data + o0 + in.imm, 8);
        st[sp].a = w;
        st[sp].b = 0;
        ++sp;
        break;
      }
      case PXG_OP_EQ_U: --sp; st[sp - 1].a = (st[sp - 1].a == st[sp].a) && (st[sp - 1].b == st[sp].b); st[sp - 1].b = 0; break;
      case PXG_OP_NE_U: --sp; st[sp - 1].a = !((st[sp - 1].a == st[sp].a) && (st[sp - 1].b == st[sp].b)); st[sp - 1].b = 0; break;
      default:
        --sp;
        if (IsStrOp(in.op)) {
          st[sp - 1].a = StrOp(in.op, st[sp - 1], st[sp]);
        } else {
          st[sp - 1].a = BinOp(in.op, st[sp - 1].a, st[sp].a);
        }
        st[sp - 1].b = 0;
        break;
    }
  }
  return st[0];
}

// Copy len bytes with unaligned 16 / 8 / 4-byte moves (gfx950 serves them in hardware); the last
// move overlaps the previous one and ends exactly at len, so nothing outside [dst, dst + len) is
// written and nothing outside [src, src + len) is read, and there is no byte-by-byte tail.
__device__ __forceinline__ void CopyBytesOverlap(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t len) {
  if (len >= 16) {
    uint32_t k = 0;
    for (; k + 16 < len; k += 16) {
      ulonglong2 x;
      __builtin_memcpy(&x, src + k, 16);
      __builtin_memcpy(dst + k, &x, 16);
    }
    ulonglong2 x;
    __builtin_memcpy(&x, src + len - 16, 16);
    __builtin_memcpy(dst + len - 16, &x, 16);
  } else if (len >= 8) {
    uint64_t a, b;
    __builtin_memcpy(&a, src, 8);
    __builtin_memcpy(&b, src + len - 8, 8);
    __builtin_memcpy(dst, &a, 8);
    __builtin_memcpy(dst + len - 8, &b, 8);
  } else if (len >= 4) {
    uint32_t a, b;
    __builtin_memcpy(&a, src, 4);
    __builtin_memcpy(&b, src + len - 4, 4);
    __builtin_memcpy(dst, &a, 4);
    __builtin_memcpy(dst + len - 4, &b, 4);
  } else {
    for (uint32_t k = 0; k < len; ++k) dst[k] = src[k];
  }
}

// Wave-local LDS ordering for lanes of one wave exchanging data through LDS.
__device__ __forceinline__ void WaveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XCD-aware remap of a linear block id (bijective for any grid size): blocks that the
// dispatcher places on one XCD (b % 8 equal) get consecutive logical ids so neighbouring
// tiles share an L2 (cdna_hip_programming.md §5.5 T1).
__device__ __forceinline__ uint32_t XcdRemap(uint32_t orig, uint32_t nwg) {
  uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

}  // namespace pxg
