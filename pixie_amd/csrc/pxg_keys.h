// Group-key helpers shared by the agg kernels: key extraction from a row or from the key
// arena, hashing and exact equality (RowTuple semantics, src/carnot/exec/row_tuple.h:109-153:
// fixed values compare by bits, strings by bytes).
#pragma once

#include "pxg_agg.h"

namespace pxg {

struct KeySet {
  Val v[kMaxKeys];
};

__device__ __forceinline__ void LoadKeysRow(const AggPlanDev* __restrict__ plan, const DevChunk& ch, int64_t r, KeySet& k) {
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i)
    if (i < plan->n_keys) k.v[i] = EvalProgram(&plan->keys[i], ch, r, plan->col_types);
}

// Arena record: per key, STRING = [len word][ceil(len/8) byte words]; UINT128 = 2 words;
// other fixed types = 1 word.
__device__ __forceinline__ void LoadKeysArena(const AggPlanDev* __restrict__ plan, const uint64_t* rec, KeySet& k) {
  int w = 0;
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    if (i >= plan->n_keys) break;
    const int t = plan->key_types[i];
    if (t == PXG_STRING) {
      uint64_t len = rec[w];
      k.v[i].a = reinterpret_cast<uint64_t>(rec + w + 1);
      k.v[i].b = len;
      w += 1 + static_cast<int>((len + 7) >> 3);
    } else if (t == PXG_UINT128) {
      k.v[i].a = rec[w];
      k.v[i].b = rec[w + 1];
      w += 2;
    } else {
      k.v[i].a = rec[w];
      k.v[i].b = 0;
      w += 1;
    }
  }
}

__device__ __forceinline__ uint32_t KeyRecordWords(const AggPlanDev* __restrict__ plan, const KeySet& k) {
  uint32_t w = 0;
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    if (i >= plan->n_keys) break;
    const int t = plan->key_types[i];
    if (t == PXG_STRING) w += 1 + static_cast<uint32_t>((k.v[i].b + 7) >> 3);
    else if (t == PXG_UINT128) w += 2;
    else w += 1;
  }
  return w;
}

__device__ __forceinline__ void WriteKeyRecord(const AggPlanDev* __restrict__ plan, const KeySet& k, uint64_t* rec) {
  int w = 0;
  for (int i = 0; i < kMaxKeys; ++i) {
    if (i >= plan->n_keys) break;
    const int t = plan->key_types[i];
    if (t == PXG_STRING) {
      const uint32_t len = static_cast<uint32_t>(k.v[i].b);
      const uint8_t* src = reinterpret_cast<const uint8_t*>(k.v[i].a);
      rec[w] = len;
      const uint32_t nw = (len + 7) >> 3;
      for (uint32_t j = 0; j < nw; ++j) {
        uint32_t rem = len - j * 8;
        rec[w + 1 + j] = LoadWordU(src + j * 8) & TailMask(rem);
      }
      w += 1 + static_cast<int>(nw);
    } else if (t == PXG_UINT128) {
      rec[w] = k.v[i].a;
      rec[w + 1] = k.v[i].b;
      w += 2;
    } else {
      rec[w] = k.v[i].a;
      w += 1;
    }
  }
}

__device__ __forceinline__ uint64_t HashKeys(const AggPlanDev* __restrict__ plan, const KeySet& k) {
  uint64_t h = 0x243F6A8885A308D3ULL;
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    if (i >= plan->n_keys) break;
    const int t = plan->key_types[i];
    uint64_t hk;
    if (t == PXG_STRING) {
      hk = HashBytes(reinterpret_cast<const uint8_t*>(k.v[i].a), static_cast<uint32_t>(k.v[i].b), 0x13198A2E03707344ULL);
    } else if (t == PXG_UINT128) {
      hk = Fmix64(k.v[i].a ^ Fmix64(k.v[i].b + 0xA4093822299F31D0ULL));
    } else {
      hk = Fmix64(k.v[i].a + 0x082EFA98EC4E6C89ULL);
    }
    h = Fmix64(h * 0x9E3779B97F4A7C15ULL + hk);
  }
  return h;
}

__device__ __forceinline__ bool KeysEqual(const AggPlanDev* __restrict__ plan, const KeySet& x, const KeySet& y) {
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    if (i >= plan->n_keys) break;
    const int t = plan->key_types[i];
    if (t == PXG_STRING) {
      if (x.v[i].b != y.v[i].b) return false;
      if (!BytesEqual(reinterpret_cast<const uint8_t*>(x.v[i].a), reinterpret_cast<const uint8_t*>(y.v[i].a),
                      static_cast<uint32_t>(x.v[i].b)))
        return false;
    } else if (t == PXG_UINT128) {
      if (x.v[i].a != y.v[i].a || x.v[i].b != y.v[i].b) return false;
    } else {
      if (x.v[i].a != y.v[i].a) return false;
    }
  }
  return true;
}

}  // namespace pxg
