// Equijoin on device tables (EquijoinNode, src/carnot/exec/equijoin_node.cc:53-470).
//
// Build: every build row is inserted into an open-addressing table keyed by its join key
// (slot word = tag | first row's ref, written by CAS only; key equality is exact bytes against
// that representative row, RowTuple semantics, row_tuple.h:109-153), and records its slot.
// Occupied slots get dense key ids (flag scan); a stable radix sort of the build refs by dense
// id turns build_buffer_ (equijoin_node.cc:200-264) into CSR form: the rows of key d are
// sorted_refs[kstart[d], kstart[d+1]) in build-row order, the order the reference appends them.
// Probe: each probe row finds its key (read-only) and contributes that key's row count (or one
// row with default build values when unmatched probe rows are emitted); an exclusive scan of
// the counts places every probe row's output, in probe-row order, and the (probe ref, build
// ref) pairs are written from the CSR ranges.  Unmatched build rows (EmitUnmatchedBuildRows,
// equijoin_node.cc:398-411) follow in dense-key order (the reference's order is hash-map order,
// unspecified).  Columns are then gathered per output column; STRING columns by length, scan,
// byte copy.  Row refs are (chunk << 24) | local row; kNullRef marks the missing side.
#include <algorithm>

#include "pxg_internal.h"
#include "pxg_scan.h"
#include "pxg_sort.h"

namespace pxg {

constexpr uint32_t kNullRef = 0xFFFFFFFFu;
constexpr int kJoinMaxKeys = 4;

struct JoinKeyDev {
  int32_t n;
  int32_t type[kJoinMaxKeys];
  int32_t col[kJoinMaxKeys];
};

struct JoinTableDev {
  unsigned long long* slots;  // tag << 33 | ref of the key's first build row (0 = empty)
  const uint32_t* rank;       // slot -> dense key id (valid for occupied slots)
  const uint32_t* kstart;     // dense key id -> first index in sorted_refs; kstart[G] = build rows
  const uint64_t* sorted_refs;
  uint32_t* probed;           // per dense key: a probe row matched it
  uint32_t mask;
};

__device__ __forceinline__ int64_t RefRow(uint32_t ref) { return static_cast<int64_t>(ref & (kChunkRows - 1)); }
__device__ __forceinline__ uint32_t RefChunk(uint32_t ref) { return ref >> kChunkShift; }

__device__ __forceinline__ uint64_t JoinHash(const JoinKeyDev& k, const DevChunk& ch, int64_t r) {
  uint64_t h = 0x243F6A8885A308D3ULL;
  for (int i = 0; i < k.n; ++i) {
    const Val v = LoadCol(ch.cols[k.col[i]], k.type[i], r);
    uint64_t hk;
    if (k.type[i] == PXG_STRING) hk = HashBytes(reinterpret_cast<const uint8_t*>(v.a), static_cast<uint32_t>(v.b), 0x13198A2E03707344ULL);
    else if (k.type[i] == PXG_UINT128) hk = Fmix64(v.a ^ Fmix64(v.b + 0xA4093822299F31D0ULL));
    else hk = Fmix64(v.a + 0x082EFA98EC4E6C89ULL);
    h = Fmix64(h * 0x9E3779B97F4A7C15ULL + hk);
  }
  return h;
}

__device__ __forceinline__ bool JoinKeysEqual(const JoinKeyDev& ka, const DevChunk& ca, int64_t ra, const JoinKeyDev& kb,
                                              const DevChunk& cb, int64_t rb) {
  for (int i = 0; i < ka.n; ++i) {
    const Val x = LoadCol(ca.cols[ka.col[i]], ka.type[i], ra);
    const Val y = LoadCol(cb.cols[kb.col[i]], kb.type[i], rb);
    if (ka.type[i] == PXG_STRING) {
      if (x.b != y.b || !BytesEqual(reinterpret_cast<const uint8_t*>(x.a), reinterpret_cast<const uint8_t*>(y.a), static_cast<uint32_t>(x.b)))
        return false;
    } else if (ka.type[i] == PXG_UINT128) {
      if (x.a != y.a || x.b != y.b) return false;
    } else if (x.a != y.a) {
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ uint32_t JoinTag(uint64_t h) { return static_cast<uint32_t>((h >> 33) | 1u) & 0x7FFFFFFFu; }

// One build chunk: insert every row, recording its slot and ref (global row order).
// Rows that find no slot are counted in *overflow.
__global__ void JoinBuildKernel(JoinKeyDev key, const DevChunk* __restrict__ bchunks, uint32_t chunk, unsigned long long* __restrict__ slots,
                                uint32_t mask, uint32_t* __restrict__ bslot, uint64_t* __restrict__ bref, unsigned int* __restrict__ overflow) {
  const DevChunk& ch = bchunks[chunk];
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < ch.nrows;
       r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t h = JoinHash(key, ch, r);
    const uint32_t tag = JoinTag(h);
    const uint32_t ref = (chunk << kChunkShift) | static_cast<uint32_t>(r);
    uint32_t pos = static_cast<uint32_t>(h) & mask;
    bool placed = false;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
      unsigned long long w = __hip_atomic_load(&slots[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0) {
        unsigned long long expected = 0;
        const unsigned long long desired = (static_cast<unsigned long long>(tag) << 33) | ref;
        if (__hip_atomic_compare_exchange_strong(&slots[pos], &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          placed = true;
        } else {
          w = expected;
        }
      }
      if (!placed && static_cast<uint32_t>(w >> 33) == tag) {
        const uint32_t rep = static_cast<uint32_t>(w);
        placed = JoinKeysEqual(key, ch, r, key, bchunks[RefChunk(rep)], RefRow(rep));
      }
      if (placed) break;
      pos = (pos + 1) & mask;
    }
    const int64_t g = ch.row_base + r;
    bslot[g] = placed ? pos : 0xFFFFFFFFu;  // unplaced rows sort last (dense id G)
    bref[g] = ref;
    if (!placed) atomicAdd(overflow, 1u);
  }
}

__global__ void JoinSlotFlagsKernel(const unsigned long long* __restrict__ slots, uint32_t cap, uint32_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) flags[i] = slots[i] != 0 ? 1u : 0u;
}

// Probe lookup: dense id of the row's key or kNullRef.
__device__ __forceinline__ uint32_t JoinLookup(const JoinKeyDev& pkey, const DevChunk& pch, int64_t r, const JoinKeyDev& bkey,
                                               const DevChunk* __restrict__ bchunks, const JoinTableDev& tab) {
  const uint64_t h = JoinHash(pkey, pch, r);
  const uint32_t tag = JoinTag(h);
  uint32_t pos = static_cast<uint32_t>(h) & tab.mask;
  for (uint32_t probe = 0; probe <= tab.mask; ++probe) {
    const unsigned long long w = tab.slots[pos];
    if (w == 0) return kNullRef;
    if (static_cast<uint32_t>(w >> 33) == tag) {
      const uint32_t rep = static_cast<uint32_t>(w);
      if (JoinKeysEqual(pkey, pch, r, bkey, bchunks[RefChunk(rep)], RefRow(rep))) return tab.rank[pos];
    }
    pos = (pos + 1) & tab.mask;
  }
  return kNullRef;
}

// Output rows per probe row (global probe row index): row count of the matching key, or 1 for
// an unmatched row that is emitted, else 0.
__global__ void JoinProbeCountKernel(JoinKeyDev pkey, const DevChunk* __restrict__ pchunks, uint32_t chunk, JoinKeyDev bkey,
                                     const DevChunk* __restrict__ bchunks, JoinTableDev tab, int emit_unmatched,
                                     uint32_t* __restrict__ key_of, uint32_t* __restrict__ cnt) {
  const DevChunk& ch = pchunks[chunk];
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < ch.nrows;
       r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t d = JoinLookup(pkey, ch, r, bkey, bchunks, tab);
    const int64_t g = ch.row_base + r;
    key_of[g] = d;
    if (d != kNullRef) {
      cnt[g] = tab.kstart[d + 1] - tab.kstart[d];
      if (!tab.probed[d]) tab.probed[d] = 1u;  // benign race: every writer stores 1
    } else {
      cnt[g] = emit_unmatched ? 1u : 0u;
    }
  }
}

__global__ void JoinProbeWriteKernel(const DevChunk* __restrict__ pchunks, uint32_t chunk, JoinTableDev tab,
                                     const uint32_t* __restrict__ key_of, const uint32_t* __restrict__ off,
                                     const uint32_t* __restrict__ cnt, uint32_t* __restrict__ pref, uint32_t* __restrict__ bref) {
  const DevChunk& ch = pchunks[chunk];
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < ch.nrows;
       r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t g = ch.row_base + r;
    const uint32_t n = cnt[g];
    if (n == 0) continue;
    const uint32_t o = off[g];
    const uint32_t me = (chunk << kChunkShift) | static_cast<uint32_t>(r);
    const uint32_t d = key_of[g];
    if (d == kNullRef) {
      pref[o] = me;
      bref[o] = kNullRef;
      continue;
    }
    const uint64_t* src = tab.sorted_refs + tab.kstart[d];
    for (uint32_t j = 0; j < n; ++j) {
      pref[o + j] = me;
      bref[o + j] = static_cast<uint32_t>(src[j]);
    }
  }
}

// Unmatched build rows: per dense key never probed, its row count.
__global__ void JoinUnprobedCountKernel(JoinTableDev tab, uint32_t G, uint32_t* __restrict__ cnt) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= G) return;
  cnt[d] = tab.probed[d] ? 0u : tab.kstart[d + 1] - tab.kstart[d];
}

__global__ void JoinUnprobedWriteKernel(JoinTableDev tab, uint32_t G, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                        uint64_t base, uint32_t* __restrict__ pref, uint32_t* __restrict__ bref) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= G || cnt[d] == 0) return;
  const uint64_t o = base + off[d];
  const uint64_t* src = tab.sorted_refs + tab.kstart[d];
  for (uint32_t j = 0; j < cnt[d]; ++j) {
    pref[o + j] = kNullRef;
    bref[o + j] = static_cast<uint32_t>(src[j]);
  }
}

// Column gathers.  A missing side gives the type's default value (0, false, "").
__global__ void JoinGatherFixedKernel(const DevChunk* __restrict__ chunks, int col, int width, const uint32_t* __restrict__ ref,
                                      uint64_t n, uint8_t* __restrict__ out) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t r = ref[i];
    uint8_t* dst = out + i * width;
    if (r == kNullRef) {
      for (int b = 0; b < width; ++b) dst[b] = 0;
      continue;
    }
    const uint8_t* src = chunks[RefChunk(r)].cols[col].values + RefRow(r) * width;
    if (width == 8) *reinterpret_cast<uint64_t*>(dst) = *reinterpret_cast<const uint64_t*>(src);
    else if (width == 16) {
      reinterpret_cast<uint64_t*>(dst)[0] = reinterpret_cast<const uint64_t*>(src)[0];
      reinterpret_cast<uint64_t*>(dst)[1] = reinterpret_cast<const uint64_t*>(src)[1];
    } else {
      for (int b = 0; b < width; ++b) dst[b] = src[b];
    }
  }
}

__global__ void JoinStringLenKernel(const DevChunk* __restrict__ chunks, int col, const uint32_t* __restrict__ ref, uint64_t n,
                                    uint32_t* __restrict__ len) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t r = ref[i];
    if (r == kNullRef) {
      len[i] = 0;
      continue;
    }
    const int32_t* o = chunks[RefChunk(r)].cols[col].offsets;
    len[i] = static_cast<uint32_t>(o[RefRow(r) + 1] - o[RefRow(r)]);
  }
}

__global__ void JoinStringCopyKernel(const DevChunk* __restrict__ chunks, int col, const uint32_t* __restrict__ ref, uint64_t n,
                                     const uint32_t* __restrict__ offs, uint8_t* __restrict__ data) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t r = ref[i];
    if (r == kNullRef) continue;
    const DevCol& c = chunks[RefChunk(r)].cols[col];
    const int32_t o0 = c.offsets[RefRow(r)];
    const uint32_t l = offs[i + 1] - offs[i];
    const uint8_t* src = c.data + o0;
    uint8_t* dst = data + offs[i];
    for (uint32_t b = 0; b < l; ++b) dst[b] = src[b];
  }
}

// ---------------------------------------------------------------------------------------
// Host orchestration.
// ---------------------------------------------------------------------------------------
static int GridFor64(uint64_t n, int block, int cap) {
  uint64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > static_cast<uint64_t>(cap)) g = cap;
  return static_cast<int>(g);
}

static int32_t JoinImpl(Table& B, Table& P, const pxg_join_spec& sp, pxg_table** out, int64_t* probe_rows) {
  Ctx* ctx = B.ctx;
  PXG_RETURN_IF_ERROR(B.EnsureDeviceDescriptors());
  PXG_RETURN_IF_ERROR(P.EnsureDeviceDescriptors());
  JoinKeyDev bk{}, pk{};
  bk.n = pk.n = sp.n_keys;
  for (int i = 0; i < sp.n_keys; ++i) {
    bk.col[i] = sp.build_keys[i];
    pk.col[i] = sp.probe_keys[i];
    bk.type[i] = B.types[bk.col[i]];
    pk.type[i] = P.types[pk.col[i]];
  }
  const uint64_t nb = static_cast<uint64_t>(B.nrows), np = static_cast<uint64_t>(P.nrows);
  if (nb >= kNullRef || np >= kNullRef) return SetError(PXG_UNIMPLEMENTED, "join sides are limited to 2^32 - 1 rows");
  uint32_t cap = 1024;
  while (cap < 2 * nb + 1) cap <<= 1;
  const DevChunk* bch = B.d_chunks.as<const DevChunk>();
  const DevChunk* pch = P.d_chunks.as<const DevChunk>();
  const int gcap = ctx->num_cus * 8;
  DevBuf slots, rank, meta, bslot, brefs, kstart, probed, key_of, cnt, off, ucnt, uoff, pref, bref;
  RadixWs rws;
  // Temporaries come from the ctx buffer pool and go back to it (a hipFree synchronises the
  // device; C5's join paid ~3 ms of them).
  struct PoolBack {
    Ctx* ctx;
    std::vector<DevBuf*> bufs;
    ~PoolBack() {
      for (DevBuf* b : bufs) PoolRelease(ctx, *b);
    }
  } back{ctx, {&slots, &rank, &meta, &bslot, &brefs, &kstart, &probed, &key_of, &cnt, &off, &ucnt, &uoff, &pref, &bref, &rws.key[0],
               &rws.key[1], &rws.val[0], &rws.val[1], &rws.scan, &rws.rs.hist, &rws.rs.ghist, &rws.rs.part}};
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, slots, static_cast<size_t>(cap) * 8));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, rank, static_cast<size_t>(cap) * 4 + 16));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, meta, 64));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, bslot, nb * 4 + 16));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, brefs, nb * 8 + 16));
  PXG_RETURN_IF_ERROR(rws.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(std::max<uint64_t>(np, cap) + 1)) + 64));
  uint32_t* d_meta = meta.as<uint32_t>();  // [0] overflow, [1] G, [2] probe output rows, [3] build output rows
  PXG_HIP(hipMemsetAsync(slots.p, 0, static_cast<size_t>(cap) * 8, ctx->stream));
  PXG_HIP(hipMemsetAsync(meta.p, 0, 64, ctx->stream));
  // 1. Build: insert, dense key ids, CSR by stable sort.
  for (size_t c = 0; c < B.chunks.size(); ++c)
    PXG_RETURN_IF_ERROR(Launch(ctx, "join_build", JoinBuildKernel, dim3(GridFor64(B.chunks[c]->nrows, 256, gcap)), dim3(256), 0, bk, bch,
                               static_cast<uint32_t>(c), slots.as<unsigned long long>(), cap - 1, bslot.as<uint32_t>(),
                               brefs.as<uint64_t>(), reinterpret_cast<unsigned int*>(d_meta)));
  PXG_RETURN_IF_ERROR(Launch(ctx, "join_slot_flags", JoinSlotFlagsKernel, dim3(GridFor64(cap, 256, 1 << 30)), dim3(256), 0,
                             slots.as<const unsigned long long>(), cap, rank.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, rank.as<const uint32_t>(), rank.as<uint32_t>(), cap, d_meta + 1, rws.scan.p));
  uint32_t hmeta[2] = {0, 0};
  PXG_HIP(hipMemcpyAsync(hmeta, d_meta, 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  if (hmeta[0]) return SetError(PXG_INTERNAL, "join build table overflow (%u rows)", hmeta[0]);
  const uint32_t G = hmeta[1];
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, kstart, (static_cast<size_t>(G) + 1) * 4 + 16));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, probed, static_cast<size_t>(G) * 4 + 16));
  PXG_HIP(hipMemsetAsync(probed.p, 0, static_cast<size_t>(G) * 4 + 16, ctx->stream));
  JoinTableDev tab;
  tab.slots = slots.as<unsigned long long>();
  tab.rank = rank.as<const uint32_t>();
  tab.kstart = kstart.as<const uint32_t>();
  tab.sorted_refs = nullptr;
  tab.probed = probed.as<uint32_t>();
  tab.mask = cap - 1;
  if (nb > 0) {
    const uint32_t* skeys = nullptr;
    const uint64_t* svals = nullptr;
    PXG_RETURN_IF_ERROR(RadixSortPairs(ctx, bslot.as<const uint32_t>(), rank.as<const uint32_t>(), cap, G, brefs.as<const uint64_t>(), nb, rws,
                                       &skeys, &svals));
    PXG_RETURN_IF_ERROR(GroupStarts(ctx, skeys, nb, G, kstart.as<uint32_t>()));
    tab.sorted_refs = svals;
  }
  // 2. Probe: counts, scan, (probe ref, build ref) pairs.
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, key_of, np * 4 + 16));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, cnt, np * 4 + 16));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, off, np * 4 + 16));
  for (size_t c = 0; c < P.chunks.size(); ++c)
    PXG_RETURN_IF_ERROR(Launch(ctx, "join_probe_count", JoinProbeCountKernel, dim3(GridFor64(P.chunks[c]->nrows, 256, gcap)), dim3(256), 0,
                               pk, pch, static_cast<uint32_t>(c), bk, bch, tab, sp.emit_unmatched_probe, key_of.as<uint32_t>(),
                               cnt.as<uint32_t>()));
  if (np > 0) PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, cnt.as<const uint32_t>(), off.as<uint32_t>(), static_cast<int64_t>(np), d_meta + 2, rws.scan.p));
  if (sp.emit_unmatched_build && G > 0) {
    PXG_RETURN_IF_ERROR(PoolAlloc(ctx, ucnt, static_cast<size_t>(G) * 4 + 16));
    PXG_RETURN_IF_ERROR(PoolAlloc(ctx, uoff, static_cast<size_t>(G) * 4 + 16));
    PXG_RETURN_IF_ERROR(Launch(ctx, "join_unprobed_count", JoinUnprobedCountKernel, dim3(GridFor64(G, 256, 1 << 30)), dim3(256), 0, tab, G,
                               ucnt.as<uint32_t>()));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, ucnt.as<const uint32_t>(), uoff.as<uint32_t>(), G, d_meta + 3, rws.scan.p));
  }
  uint32_t hcount[2] = {0, 0};
  PXG_HIP(hipMemcpyAsync(hcount, d_meta + 2, 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  const uint32_t n_probe_out = hcount[0], n_build_out = hcount[1];
  const uint64_t n_out = static_cast<uint64_t>(n_probe_out) + n_build_out;
  if (n_out >= kNullRef) return SetError(PXG_UNIMPLEMENTED, "join output exceeds 2^32 - 1 rows");
  if (probe_rows) *probe_rows = n_probe_out;
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, pref, n_out * 4 + 16));
  PXG_RETURN_IF_ERROR(PoolAlloc(ctx, bref, n_out * 4 + 16));
  for (size_t c = 0; c < P.chunks.size() && n_probe_out > 0; ++c)
    PXG_RETURN_IF_ERROR(Launch(ctx, "join_probe_write", JoinProbeWriteKernel, dim3(GridFor64(P.chunks[c]->nrows, 256, gcap)), dim3(256), 0,
                               pch, static_cast<uint32_t>(c), tab, key_of.as<const uint32_t>(), off.as<const uint32_t>(),
                               cnt.as<const uint32_t>(), pref.as<uint32_t>(), bref.as<uint32_t>()));
  if (n_build_out > 0)
    PXG_RETURN_IF_ERROR(Launch(ctx, "join_unprobed_write", JoinUnprobedWriteKernel, dim3(GridFor64(G, 256, 1 << 30)), dim3(256), 0, tab, G,
                               ucnt.as<const uint32_t>(), uoff.as<const uint32_t>(), static_cast<uint64_t>(n_probe_out),
                               pref.as<uint32_t>(), bref.as<uint32_t>()));
  PXG_RETURN_IF_ERROR(rws.scan.Ensure(ScanScratchBytes(static_cast<int64_t>(n_out + 1)) + 64));
  void* scratch = rws.scan.p;
  // Output table.
  std::vector<int32_t> otypes(sp.n_out);
  for (int i = 0; i < sp.n_out; ++i) otypes[i] = sp.out_side[i] == 0 ? P.types[sp.out_col[i]] : B.types[sp.out_col[i]];
  PXG_RETURN_IF_ERROR(NewTable(ctx, sp.n_out, otypes.data(), out));
  if (n_out == 0) return PXG_OK;
  // Output columns in pooled buffers: string lengths and their scans first, every payload size
  // read back with one synchronisation, then the gathers.  A result that fits one chunk adopts
  // the buffers as its chunk (no copy); a larger one is appended chunk by chunk.
  std::vector<DevBuf> bufs(3 * static_cast<size_t>(sp.n_out));
  struct PoolBackVec {
    Ctx* ctx;
    std::vector<DevBuf>& v;
    ~PoolBackVec() {
      for (DevBuf& b : v) PoolRelease(ctx, b);
    }
  } back_out{ctx, bufs};
  std::vector<pxg_column_view> views(sp.n_out);
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps);
  if (static_cast<size_t>(sp.n_out) * 4 > Ctx::kPinnedBytes - Ctx::kPinnedOps) return SetError(PXG_UNIMPLEMENTED, "too many join outputs");
  int n_str = 0;
  for (int i = 0; i < sp.n_out; ++i) {
    if (otypes[i] != PXG_STRING) continue;
    const bool probe_side = sp.out_side[i] == 0;
    DevBuf& o = bufs[3 * i + 1];
    PXG_RETURN_IF_ERROR(PoolAlloc(ctx, o, (n_out + 1) * 4 + 16));
    PXG_RETURN_IF_ERROR(Launch(ctx, "join_gather", JoinStringLenKernel, dim3(GridFor64(n_out, 256, gcap)), dim3(256), 0, probe_side ? pch : bch,
                               sp.out_col[i], probe_side ? pref.as<const uint32_t>() : bref.as<const uint32_t>(), n_out, o.as<uint32_t>()));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, o.as<const uint32_t>(), o.as<uint32_t>(), static_cast<int64_t>(n_out), o.as<uint32_t>() + n_out,
                                         scratch));
    PXG_HIP(hipMemcpyAsync(pin + i, o.as<uint32_t>() + n_out, 4, hipMemcpyDeviceToHost, ctx->stream));
    ++n_str;
  }
  if (n_str > 0) PXG_HIP(hipStreamSynchronize(ctx->stream));
  bool one_chunk = static_cast<int64_t>(n_out) <= kChunkRows;
  for (int i = 0; i < sp.n_out; ++i) {
    const bool probe_side = sp.out_side[i] == 0;
    const DevChunk* ch = probe_side ? pch : bch;
    const uint32_t* ref = probe_side ? pref.as<const uint32_t>() : bref.as<const uint32_t>();
    const int col = sp.out_col[i];
    const int t = otypes[i];
    pxg_column_view& v = views[i];
    std::memset(&v, 0, sizeof(v));
    v.type = t;
    v.length = static_cast<int64_t>(n_out);
    if (t == PXG_STRING) {
      DevBuf& o = bufs[3 * i + 1];
      DevBuf& d = bufs[3 * i + 2];
      const uint32_t bytes = pin[i];
      one_chunk = one_chunk && bytes < (uint32_t(1) << 31) - 64;
      PXG_RETURN_IF_ERROR(PoolAlloc(ctx, d, static_cast<size_t>(bytes) + 16));
      PXG_RETURN_IF_ERROR(Launch(ctx, "join_gather", JoinStringCopyKernel, dim3(GridFor64(n_out, 256, gcap)), dim3(256), 0, ch, col, ref, n_out,
                                 o.as<const uint32_t>(), d.as<uint8_t>()));
      v.offsets = o.as<const int32_t>();
      v.data = d.as<const uint8_t>();
    } else {
      const int w = TypeWidth(t);
      DevBuf& val = bufs[3 * i];
      PXG_RETURN_IF_ERROR(PoolAlloc(ctx, val, n_out * w + 16));
      PXG_RETURN_IF_ERROR(Launch(ctx, "join_gather", JoinGatherFixedKernel, dim3(GridFor64(n_out, 256, gcap)), dim3(256), 0, ch, col, w, ref,
                                 n_out, val.as<uint8_t>()));
      v.values = val.p;
    }
  }
  Table& ot = (*out)->impl;
  if (one_chunk) {
    auto c = std::make_unique<Chunk>();
    c->row_base = 0;
    c->nrows = static_cast<int64_t>(n_out);
    c->rows_cap = c->nrows;
    c->sealed = true;
    c->cols.resize(static_cast<size_t>(sp.n_out));
    for (int i = 0; i < sp.n_out; ++i) {
      ChunkCol& cc = c->cols[i];
      if (otypes[i] == PXG_STRING) {
        cc.offsets = std::move(bufs[3 * i + 1]);
        cc.data = std::move(bufs[3 * i + 2]);
        cc.data_len = pin[i];
      } else {
        cc.values = std::move(bufs[3 * i]);
      }
    }
    ot.chunks.push_back(std::move(c));
    ot.nrows = static_cast<int64_t>(n_out);
    ot.version++;
    return PXG_OK;  // contents complete in stream order (consumers on the ctx stream need no sync)
  }
  const int32_t rc = ot.AppendRows(views.data(), static_cast<int64_t>(n_out), hipMemcpyDeviceToDevice);
  if (rc != PXG_OK) return rc;
  PXG_RETURN_IF_ERROR(ot.FlushStage());
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}

}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_join(pxg_table* build, pxg_table* probe, const pxg_join_spec* spec, pxg_table** out, int64_t* probe_rows) {
  if (!build || !probe || !spec || !out) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  *out = nullptr;
  if (probe_rows) *probe_rows = 0;
  Table& B = build->impl;
  Table& P = probe->impl;
  if (B.ctx != P.ctx) return SetError(PXG_INVALID_ARGUMENT, "join tables belong to different contexts");
  if (spec->n_keys < 1 || spec->n_keys > kJoinMaxKeys) return SetError(PXG_UNIMPLEMENTED, "1..%d equality conditions supported", kJoinMaxKeys);
  for (int i = 0; i < spec->n_keys; ++i) {
    const int b = spec->build_keys[i], p = spec->probe_keys[i];
    if (b < 0 || b >= B.ncols || p < 0 || p >= P.ncols) return SetError(PXG_INVALID_ARGUMENT, "join key column out of range");
    if (B.types[b] != P.types[p]) return SetError(PXG_INVALID_ARGUMENT, "join key %d: build type %d != probe type %d", i, B.types[b], P.types[p]);
    if (B.types[b] == PXG_BOOLEAN) return SetError(PXG_UNIMPLEMENTED, "BOOLEAN join keys");
  }
  if (spec->n_out < 0 || spec->n_out > kMaxCols) return SetError(PXG_UNIMPLEMENTED, "at most %d output columns", kMaxCols);
  for (int i = 0; i < spec->n_out; ++i) {
    const Table& T = spec->out_side[i] == 0 ? P : B;
    if (spec->out_side[i] < 0 || spec->out_side[i] > 1 || spec->out_col[i] < 0 || spec->out_col[i] >= T.ncols)
      return SetError(PXG_INVALID_ARGUMENT, "join output column %d out of range", i);
  }
  PXG_RETURN_IF_ERROR(B.FlushStage());
  PXG_RETURN_IF_ERROR(P.FlushStage());
  const int32_t rc = JoinImpl(B, P, *spec, out, probe_rows);
  if (rc != PXG_OK && *out) {
    pxg_table_destroy(*out);
    *out = nullptr;
  }
  return rc;
}
