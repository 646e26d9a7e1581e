// Grouping of staged records (pxg_group.hip): stable LSD radix sort of (u32 key, u64 value)
// records by dense key, and the fused split of the largest groups.
#pragma once

#include "pxg_internal.h"

namespace pxg {

constexpr int kRadixBits = 8;
constexpr uint32_t kFsMaxU = 255;     // designated groups of the fused split (one bucket each)
constexpr uint32_t kFsMinRows = 4096;  // designate a group whose sampled estimate reaches this

struct ValPtrs {
  uint64_t* p[kMaxVals];
};
struct ConstValPtrs {
  const uint64_t* p[kMaxVals];
};

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

// Sorts n records by DenseKey (rank map as in RadixSortPairs; without one, bits [shift0,
// shift0 + fixed_bits) of the keys) into the ping-pong buffers kbuf / vbuf, nvals value streams
// riding along; *skeys / *svals name the sorted streams.
int32_t RadixSortStreams(Ctx* ctx, const uint32_t* keys, const uint32_t* rank, uint32_t cap, uint32_t G, ConstValPtrs vin, int nvals,
                         uint64_t n, uint32_t* kbuf[2], ValPtrs vbuf[2], RadixPassWs& ws, const uint32_t** skeys, ConstValPtrs* svals,
                         int shift0 = 0, int fixed_bits = 0);

// Dense group ids in slot order: rank[slot] (exclusive scan of occupancy), gslot[id] = slot,
// *d_ngroups = the occupied count.
int32_t DenseIdsBySlot(Ctx* ctx, const unsigned long long* slots, uint32_t cap, uint32_t* rank, uint32_t* gslot, uint32_t* d_ngroups,
                       void* scan_tmp);

// Fused split, step 1: a 1/128 sample of the staged slots designates the largest groups (at most
// kFsMaxU, each sampled at >= kFsMinRows / 128); ids: the rest [0, Gr) then the designated
// [Gr, G), both in slot order (rank[slot], gslot[id]); *d_ftotal = designated << 32 | occupied.
int32_t DesignateLargeGroups(Ctx* ctx, const unsigned long long* slots, uint32_t cap, const uint32_t* st_slot, uint64_t n, uint32_t G,
                             DevBuf& split_cnt, DevBuf& split_flags, uint32_t* rank, uint32_t* gslot, uint32_t* d_ngroups, void* scan_tmp,
                             uint64_t** d_ftotal);
// Step 2: the 9-bit first pass.  Designated records' values go straight to their final place in
// vfin; rest records (key = rest id, values) to kout_rest / vrest at [0, n_rest), sorted by their
// low digit.  Enqueues n_rest (u32 at pinned + 104) and *d_ftotal (u64 at pinned + 112) to
// pinned memory and records ctx->ev_split before the scatter; *base_out: the bucket bases.
int32_t FusedSplitPass(Ctx* ctx, const uint32_t* st_slot, uint64_t n, const uint32_t* rank, uint32_t cap, uint32_t G, const uint64_t* d_ftotal,
                       ConstValPtrs vin, int nvs, DevBuf& split_hist, DevBuf& split_tot, DevBuf& fs_keys, RadixPassWs& rs, uint32_t* kout_rest,
                       ValPtrs vrest, ValPtrs vfin, const uint32_t** base_out);
// The designated groups' starts (device, j <= nd: group Gr + j starts at [j]; [nd] = n) out of
// FusedSplitPass's *base_out; final as soon as FusedSplitPass's scatter has run.
const uint32_t* FusedSplitDesignatedStarts(const uint32_t* base);
// Step 3 (after the rest's group starts): gstart of the designated groups and gstart[G].
int32_t FusedSplitGstart(Ctx* ctx, const uint32_t* base, const uint64_t* d_ftotal, uint32_t G, uint32_t* gstart);
// Whether a finalize of n staged records takes the fused split (PXG_FSPLIT=0 / 1: tests force it).
bool FusedSplitOn(uint64_t n);

}  // namespace pxg
