// Stable LSD radix sort of (u32 key, u64 value) records by dense key (pxg_finalize.hip).
#pragma once

#include "pxg_internal.h"

namespace pxg {

// Radix sort pass state: tile x digit counts / offsets and the global digit totals.
struct RadixPassWs {
  DevBuf hist, ghist, part;  // hist: tile-major digit counts; part: per range of tiles
};

struct RadixWs {
  DevBuf key[2], val[2], scan;  // scan: scratch for the caller's own scans
  RadixPassWs rs;
};

// Sorts n records by DenseKey(keys[i]) = rank ? (keys[i] < cap ? rank[keys[i]] : G) : keys[i],
// a value in [0, G], keeping input order among equal keys.  On return *skeys holds the sorted
// dense keys and *svals the values in the same order (both inside ws).  n < 2^32.
int32_t RadixSortPairs(Ctx* ctx, const uint32_t* keys, const uint32_t* rank, uint32_t cap, uint32_t G, const uint64_t* vals,
                       uint64_t n, RadixWs& ws, const uint32_t** skeys, const uint64_t** svals);

// Sorts n records stably by bits [shift0, shift0 + nbits) of keys[i], moving nvals u64 value
// streams with them (vals[v][i]).  Ping-pong buffers kb / vb are grown as needed; on return
// stream v sorted is at *svals + v * n.
int32_t RadixSortBits(Ctx* ctx, const uint32_t* keys, int shift0, int nbits, const uint64_t* const* vals, int nvals, uint64_t n,
                      DevBuf kb[2], DevBuf vb[2], RadixPassWs& ws, const uint32_t** skeys, const uint64_t** svals);

// gstart[k] = first index of dense key k in the sorted keys, gstart[G] = count of keys < G.
// Keys that never occur keep whatever gstart held (callers size groups from dense ids only).
int32_t GroupStarts(Ctx* ctx, const uint32_t* skeys, uint64_t n, uint32_t G, uint32_t* gstart);

}  // namespace pxg
