// Standalone FilterNode / MapNode over device tables (operator shapes the fused agg path does
// not cover).
//
// FilterNode::ConsumeNextImpl (filter_node.cc:132-171): evaluate the predicate, then compact
// every selected column, preserving row order (filter_node.cc:88-92).  On the device this is
// ballot compaction: pass 1 streams the predicate's columns and writes one 64-row ballot word
// per wave iteration plus one count per 4096-row tile; a small scan turns the tile counts into
// output bases; pass 2 re-reads the ballot words, ranks every selected row inside its tile
// (LDS prefix of the tile's ballot popcounts + the lane's popcount below it) and gathers every
// selected column in one launch.  STRING columns: the gather writes lengths and source rows,
// one scan makes the offsets, and a word-wise copy moves the payload (8-byte unaligned loads and
// stores, gfx950 serves them in hardware).
//
// MapNode::ConsumeNextImpl (map_node.cc:64-71): one output column per expression; column
// references pass through (device-to-device copies).
//
// No per-call hipMalloc: programs, ballot words, tile counts, scan scratch and string source
// rows live in the ctx's grow-only ops workspace, output columns come from the ctx buffer pool
// (refilled by pxg_table_destroy).  A filter synchronises twice per call whatever the chunk
// count (selected counts; string payload sizes), a map once (passed-through string extents).
#include <algorithm>

#include "pxg_internal.h"
#include "pxg_program.h"
#include "pxg_scan.h"

namespace pxg {

constexpr int kOpsBlock = 256;
constexpr int kOpsTileRows = 4096;                      // rows per workgroup tile
constexpr int kOpsMasksPerTile = kOpsTileRows / 64;     // 64 ballot words
constexpr int kOpsMasksPerWave = kOpsMasksPerTile / 4;  // 16 per wave

// Device programs of one call, uploaded once into the ctx workspace.
static int32_t UploadPrograms(Ctx* ctx, const pxg_program* progs, int n, const Table& t, const DevProgram** d_progs,
                              const int32_t** d_types) {
  std::vector<DevProgram> dp(static_cast<size_t>(std::max(n, 1)));
  std::vector<uint8_t> pool;
  std::vector<size_t> offs(static_cast<size_t>(std::max(n, 1)));
  for (int i = 0; i < n; ++i) PXG_RETURN_IF_ERROR(CompileProgram(progs[i], t.types.data(), t.ncols, &dp[i], &pool, &offs[i]));
  const size_t prog_bytes = dp.size() * sizeof(DevProgram);
  const size_t types_off = (prog_bytes + 255) & ~size_t(255);
  const size_t pool_off = types_off + kMaxCols * 4 + 256;
  OpsWorkspace& w = ctx->ops;
  PXG_RETURN_IF_ERROR(w.prog.Ensure(pool_off + pool.size() + 16));
  uint8_t* base = w.prog.as<uint8_t>();
  for (int i = 0; i < n; ++i) dp[i].pool = base + pool_off + offs[i];
  std::vector<uint8_t> host(pool_off + pool.size(), 0);
  std::memcpy(host.data(), dp.data(), prog_bytes);
  for (int k = 0; k < t.ncols; ++k) std::memcpy(host.data() + types_off + 4 * k, &t.types[k], 4);
  if (!pool.empty()) std::memcpy(host.data() + pool_off, pool.data(), pool.size());
  PXG_HIP(hipMemcpyAsync(base, host.data(), host.size(), hipMemcpyHostToDevice, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));  // `host` is pageable and goes out of scope
  *d_progs = reinterpret_cast<const DevProgram*>(base);
  *d_types = reinterpret_cast<const int32_t*>(base + types_off);
  return PXG_OK;
}

// Pass 1: ballot words of the predicate and per-tile selected counts.
__global__ void __launch_bounds__(kOpsBlock) FilterMaskKernel(const DevProgram* __restrict__ prog, const DevChunk* __restrict__ chunks,
                                                              int chunk, const int32_t* __restrict__ types, int64_t lo, int64_t n,
                                                              unsigned long long* __restrict__ masks, uint32_t* __restrict__ tile_cnt) {
  __shared__ uint32_t s_cnt[kOpsBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const DevChunk& ch = chunks[chunk];
  const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * kOpsTileRows;
  uint32_t cnt = 0;
  if (prog->shape == kShapeCol || prog->shape == kShapeColOpConst) {
    // Fast shapes (col, col op const over a fixed-width column): the wave's 16 loads are issued
    // together, then evaluated.
    const DevCol& col = ch.cols[prog->col];
    const int ty = types[prog->col];
    uint64_t raw[kOpsMasksPerWave];
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave; ++k) {
      const int64_t r = tile0 + (static_cast<int64_t>(wid) * kOpsMasksPerWave + k) * 64 + lane;
      raw[k] = r < n ? LoadCol(col, ty, lo + r).a : 0ULL;
    }
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave; ++k) {
      const int64_t r = tile0 + (static_cast<int64_t>(wid) * kOpsMasksPerWave + k) * 64 + lane;
      uint64_t v = raw[k];
      if (prog->shape == kShapeColOpConst) {
        if (prog->conv) v = Conv(prog->conv, v);
        v = BinOp(prog->binop, v, static_cast<uint64_t>(prog->cimm));
      }
      const unsigned long long m = __ballot(r < n && v != 0);
      cnt += static_cast<uint32_t>(__popcll(m));
      const int64_t mi = static_cast<int64_t>(blockIdx.x) * kOpsMasksPerTile + wid * kOpsMasksPerWave + k;
      if (lane == 0) masks[mi] = m;
    }
  } else {
    for (int k = 0; k < kOpsMasksPerWave; ++k) {
      const int64_t r = tile0 + (static_cast<int64_t>(wid) * kOpsMasksPerWave + k) * 64 + lane;
      const bool pass = r < n && EvalProgram(prog, ch, lo + r, types).a != 0;
      const unsigned long long m = __ballot(pass);
      cnt += static_cast<uint32_t>(__popcll(m));
      const int64_t mi = static_cast<int64_t>(blockIdx.x) * kOpsMasksPerTile + wid * kOpsMasksPerWave + k;
      if (lane == 0) masks[mi] = m;
    }
  }
  if (lane == 0) s_cnt[wid] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

struct GatherCols {
  int32_t n;
  int32_t width[kMaxCols];  // bytes per value; 0 = STRING
  const uint8_t* src[kMaxCols];       // fixed values
  const int32_t* src_off[kMaxCols];   // STRING offsets
  uint8_t* dst[kMaxCols];             // fixed output values
  uint32_t* dst_len[kMaxCols];        // STRING: length of output row (scanned to offsets later)
  uint32_t* dst_src[kMaxCols];        // STRING: source payload byte offset of output row
};

// Pass 2: rank every selected row (tile base + prefix of the tile's ballot popcounts + the
// lane's bits below it) and gather every selected column.
__global__ void __launch_bounds__(kOpsBlock) FilterGatherKernel(const unsigned long long* __restrict__ masks,
                                                                const uint32_t* __restrict__ tile_base, int64_t lo, int64_t n,
                                                                GatherCols gc) {
  __shared__ uint32_t s_pre[kOpsMasksPerTile];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  const int64_t mask0 = static_cast<int64_t>(blockIdx.x) * kOpsMasksPerTile;
  if (threadIdx.x < kOpsMasksPerTile) {  // one wave: exclusive prefix of the 64 popcounts
    const uint32_t c = static_cast<uint32_t>(__popcll(masks[mask0 + threadIdx.x]));
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    s_pre[threadIdx.x] = x - c;
  }
  __syncthreads();
  const uint32_t base = tile_base[blockIdx.x];
  // Every selected row of the wave's 16 ballot words is placed first; then each column's loads
  // for all of them are issued together (16 in flight per lane) before the stores.
  uint32_t sel = 0, pos[kOpsMasksPerWave];
#pragma unroll
  for (int k = 0; k < kOpsMasksPerWave; ++k) {
    const int mi = wid * kOpsMasksPerWave + k;
    const unsigned long long m = masks[mask0 + mi];
    sel |= static_cast<uint32_t>((m >> lane) & 1ULL) << k;
    pos[k] = base + s_pre[mi] + static_cast<uint32_t>(__popcll(m & lanemask_lt));
  }
  if (!sel) return;
  const int64_t r0 = lo + static_cast<int64_t>(blockIdx.x) * kOpsTileRows + wid * kOpsMasksPerWave * 64 + lane;
  for (int c = 0; c < gc.n; ++c) {
    const int w = gc.width[c];
    if (w == 8) {
      const uint64_t* src = reinterpret_cast<const uint64_t*>(gc.src[c]) + r0;
      uint64_t* dst = reinterpret_cast<uint64_t*>(gc.dst[c]);
      uint64_t v[kOpsMasksPerWave];
#pragma unroll
      for (int k = 0; k < kOpsMasksPerWave; ++k) v[k] = (sel >> k) & 1 ? src[k * 64] : 0ULL;
#pragma unroll
      for (int k = 0; k < kOpsMasksPerWave; ++k)
        if ((sel >> k) & 1) dst[pos[k]] = v[k];
    } else if (w == 0) {
      const int32_t* off = gc.src_off[c] + r0;
      int32_t a[kOpsMasksPerWave], b[kOpsMasksPerWave];
#pragma unroll
      for (int k = 0; k < kOpsMasksPerWave; ++k) {
        a[k] = (sel >> k) & 1 ? off[k * 64] : 0;
        b[k] = (sel >> k) & 1 ? off[k * 64 + 1] : 0;
      }
#pragma unroll
      for (int k = 0; k < kOpsMasksPerWave; ++k)
        if ((sel >> k) & 1) {
          gc.dst_len[c][pos[k]] = static_cast<uint32_t>(b[k] - a[k]);
          gc.dst_src[c][pos[k]] = static_cast<uint32_t>(a[k]);
        }
    } else {
      for (int k = 0; k < kOpsMasksPerWave; ++k) {
        if (!((sel >> k) & 1)) continue;
        const int64_t r = r0 + k * 64;
        if (w == 16) reinterpret_cast<ulonglong2*>(gc.dst[c])[pos[k]] = reinterpret_cast<const ulonglong2*>(gc.src[c])[r];
        else gc.dst[c][pos[k]] = gc.src[c][r];
      }
    }
  }
  (void)n;
}

// String payload gather: output row i gets len = doff[i + 1] - doff[i] bytes from source byte
// offset src[i] (recorded by the gather pass, so no dependent offset load here).  Copies are
// unaligned 16 / 8 / 4-byte moves (gfx950 serves them in hardware); the last move of a string
// overlaps the previous one and ends exactly at len, so a thread never writes outside its own
// string and there is no byte-by-byte tail.  All loads of a string are issued before its stores.
template <int W>
struct Word;
template <>
struct Word<16> { using T = ulonglong2; };
template <>
struct Word<8> { using T = uint64_t; };
template <>
struct Word<4> { using T = uint32_t; };
template <int W>
__device__ __forceinline__ typename Word<W>::T LoadU(const uint8_t* p) {
  typename Word<W>::T x;
  __builtin_memcpy(&x, p, W);
  return x;
}
template <int W>
__device__ __forceinline__ void StoreU(uint8_t* p, typename Word<W>::T x) { __builtin_memcpy(p, &x, W); }

__global__ void StrGatherKernel(const uint8_t* __restrict__ sdata, const uint32_t* __restrict__ src, const uint32_t* __restrict__ doff,
                                uint8_t* __restrict__ ddata, int64_t m) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t o0 = doff[i];
  const uint32_t len = doff[i + 1] - o0;
  const uint8_t* s = sdata + src[i];
  uint8_t* d = ddata + o0;
  if (len >= 16) {
    if (len <= 48) {  // the common case: at most three 16-byte moves, loads first
      const ulonglong2 a = LoadU<16>(s), c = LoadU<16>(s + len - 16);
      const ulonglong2 b = len > 32 ? LoadU<16>(s + 16) : a;
      StoreU<16>(d, a);
      if (len > 32) StoreU<16>(d + 16, b);
      StoreU<16>(d + len - 16, c);
    } else {
      uint32_t k = 0;
      for (; k + 16 < len; k += 16) StoreU<16>(d + k, LoadU<16>(s + k));
      StoreU<16>(d + len - 16, LoadU<16>(s + len - 16));
    }
  } else if (len >= 8) {
    const uint64_t a = LoadU<8>(s), b = LoadU<8>(s + len - 8);
    StoreU<8>(d, a);
    StoreU<8>(d + len - 8, b);
  } else if (len >= 4) {
    const uint32_t a = LoadU<4>(s), b = LoadU<4>(s + len - 4);
    StoreU<4>(d, a);
    StoreU<4>(d + len - 4, b);
  } else {
    for (uint32_t k = 0; k < len; ++k) d[k] = s[k];
  }
}

__global__ void MapEvalKernel(const DevProgram* __restrict__ prog, const DevChunk* __restrict__ chunks, int chunk,
                              const int32_t* __restrict__ types, int64_t lo, int64_t n, uint8_t* __restrict__ out, int width) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Val v = EvalProgram(prog, chunks[chunk], lo + i, types);
  if (width == 1) out[i] = static_cast<uint8_t>(v.a != 0);
  else if (width == 16) { reinterpret_cast<uint64_t*>(out)[2 * i] = v.a; reinterpret_cast<uint64_t*>(out)[2 * i + 1] = v.b; }
  else reinterpret_cast<uint64_t*>(out)[i] = v.a;
}

__global__ void RebaseKernel(int32_t* __restrict__ dst, const int32_t* __restrict__ src, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i] - src[0];
}

// Filter rows [begin, end) of t into a new table; per_split (optional) receives the selected
// rows of each of n_splits consecutive input row ranges (split_rows[i] rows each).  Three
// phases over all chunks at once, so a call synchronises twice (selected counts; string
// payload sizes) however many chunks the table has: masks + tile scans, then the gathers and
// string length scans, then the payload copies.  Output columns come from the ctx pool.
static int32_t FilterImpl(Table& t, const pxg_program& pred, int32_t n_select, const int32_t* select, int64_t begin, int64_t end,
                          int32_t n_splits, const int64_t* split_rows, int64_t* per_split, pxg_table** out) {
  Ctx* ctx = t.ctx;
  PXG_RETURN_IF_ERROR(t.EnsureDeviceDescriptors());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "bad row range");
  if (pred.result_type != PXG_BOOLEAN) return SetError(PXG_INVALID_ARGUMENT, "Predicate expression must be a boolean");
  std::vector<int32_t> otypes;
  int n_str = 0;
  for (int i = 0; i < n_select; ++i) {
    if (select[i] < 0 || select[i] >= t.ncols) return SetError(PXG_INVALID_ARGUMENT, "selected column %d out of range", select[i]);
    otypes.push_back(t.types[select[i]]);
    n_str += t.types[select[i]] == PXG_STRING ? 1 : 0;
  }
  if (n_splits > 0) {
    int64_t tot = 0;
    for (int i = 0; i < n_splits; ++i) tot += split_rows[i];
    if (tot != end - begin) return SetError(PXG_INVALID_ARGUMENT, "split rows add up to %lld, range has %lld", (long long)tot, (long long)(end - begin));
  }
  struct Part {
    size_t c;
    int64_t lo, n, ntiles, mask0, tile0;
    uint32_t m = 0;
    uint64_t gsrc0 = 0;  // per string column: m source rows at gsrc0 + s_str * m
  };
  std::vector<Part> parts;
  int64_t nmasks = 0, ntile_words = 0;
  for (size_t c = 0; c < t.chunks.size(); ++c) {
    const Chunk& ch = *t.chunks[c];
    const int64_t lo = std::max(begin, ch.row_base) - ch.row_base;
    const int64_t hi = std::min(end, ch.row_base + ch.nrows) - ch.row_base;
    if (lo >= hi) continue;
    Part p;
    p.c = c;
    p.lo = lo;
    p.n = hi - lo;
    p.ntiles = (p.n + kOpsTileRows - 1) / kOpsTileRows;
    p.mask0 = nmasks;
    p.tile0 = ntile_words;
    nmasks += p.ntiles * kOpsMasksPerTile;
    ntile_words += p.ntiles + 1;
    parts.push_back(p);
  }
  const size_t pin_cap = (Ctx::kPinnedBytes - Ctx::kPinnedOps) / 4;
  if (parts.size() * static_cast<size_t>(std::max(n_str, 1)) > pin_cap)
    return SetError(PXG_UNIMPLEMENTED, "filter over %zu chunks", parts.size());
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps);
  const DevProgram* d_prog = nullptr;
  const int32_t* d_types = nullptr;
  PXG_RETURN_IF_ERROR(UploadPrograms(ctx, &pred, 1, t, &d_prog, &d_types));
  pxg_table* ot = nullptr;
  PXG_RETURN_IF_ERROR(NewTable(ctx, static_cast<int32_t>(otypes.size()), otypes.data(), &ot));
  std::unique_ptr<pxg_table, int32_t (*)(pxg_table*)> guard(ot, pxg_table_destroy);
  Table& o = ot->impl;
  OpsWorkspace& w = ctx->ops;
  int64_t max_tiles = 1;
  for (const Part& p : parts) max_tiles = std::max(max_tiles, p.ntiles);
  PXG_RETURN_IF_ERROR(w.masks.Ensure(static_cast<size_t>(nmasks) * 8 + 64));
  PXG_RETURN_IF_ERROR(w.tiles.Ensure(static_cast<size_t>(ntile_words) * 4 + 64));
  PXG_RETURN_IF_ERROR(w.scan.Ensure(ScanScratchBytes(max_tiles + 1) + 64));
  // Phase A: ballot words, tile counts -> tile bases and the chunk's selected count.
  for (size_t i = 0; i < parts.size(); ++i) {
    const Part& p = parts[i];
    uint32_t* tiles = w.tiles.as<uint32_t>() + p.tile0;
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_mask", FilterMaskKernel, dim3(static_cast<unsigned>(p.ntiles)), dim3(kOpsBlock), 0, d_prog,
                               t.d_chunks.as<const DevChunk>(), static_cast<int>(p.c), d_types, p.lo, p.n,
                               w.masks.as<unsigned long long>() + p.mask0, tiles));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, tiles, tiles, p.ntiles, tiles + p.ntiles, w.scan.p));
    PXG_HIP(hipMemcpyAsync(pin + i, tiles + p.ntiles, 4, hipMemcpyDeviceToHost, ctx->stream));
  }
  std::vector<unsigned long long> host_masks;
  if (n_splits > 0) {  // ballot words back to the host: per-split counts by popcount
    host_masks.resize(static_cast<size_t>(nmasks));
    PXG_HIP(hipMemcpyAsync(host_masks.data(), w.masks.p, static_cast<size_t>(nmasks) * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  uint64_t gsrc_words = 0;
  for (size_t i = 0; i < parts.size(); ++i) {
    parts[i].m = pin[i];
    parts[i].gsrc0 = gsrc_words;
    gsrc_words += static_cast<uint64_t>(parts[i].m) * n_str;
  }
  if (n_splits > 0) {
    for (const Part& p : parts) {
      const Chunk& ch = *t.chunks[p.c];
      // split i covers input rows [s0, s1) of [begin, end); this chunk covers [cb, cb + n)
      const int64_t cb = ch.row_base + p.lo - begin;
      int64_t s0 = 0;
      for (int i = 0; i < n_splits; ++i) {
        const int64_t s1 = s0 + split_rows[i];
        const int64_t a = std::max(s0, cb) - cb, b = std::min(s1, cb + p.n) - cb;
        for (int64_t r = a; r < b;) {
          const int64_t wi = r >> 6;
          const int64_t e = std::min(b, (wi + 1) << 6);
          unsigned long long mk = host_masks[static_cast<size_t>(p.mask0 + wi)] >> (r & 63);
          const int64_t bits = e - r;
          if (bits < 64) mk &= (1ULL << bits) - 1;
          per_split[i] += __builtin_popcountll(mk);
          r = e;
        }
        s0 = s1;
      }
    }
  }
  // Phase B: output chunks, the gathers, string lengths -> offsets.
  PXG_RETURN_IF_ERROR(w.gsrc.Ensure(gsrc_words * 4 + 64));
  std::vector<GatherCols> gcs(parts.size());
  for (size_t i = 0; i < parts.size(); ++i) {
    const Part& p = parts[i];
    const Chunk& ch = *t.chunks[p.c];
    const uint32_t m = p.m;
    auto oc = std::make_unique<Chunk>();
    oc->row_base = o.nrows;
    oc->nrows = m;
    oc->rows_cap = m;
    oc->sealed = true;
    oc->cols.resize(static_cast<size_t>(n_select));
    GatherCols& gc = gcs[i];
    std::memset(&gc, 0, sizeof(gc));
    gc.n = n_select;
    int si = 0;
    for (int s = 0; s < n_select; ++s) {
      const int ci = select[s];
      const int ty = t.types[ci];
      ChunkCol& dc = oc->cols[static_cast<size_t>(s)];
      if (ty != PXG_STRING) {
        const int wd = TypeWidth(ty);
        gc.width[s] = wd;
        PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.values, static_cast<size_t>(m) * wd + 16));
        gc.src[s] = ch.cols[ci].values.as<const uint8_t>();
        gc.dst[s] = dc.values.as<uint8_t>();
      } else {
        gc.width[s] = 0;
        PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.offsets, (static_cast<size_t>(m) + 1) * 4 + 16));
        gc.src_off[s] = ch.cols[ci].offsets.as<const int32_t>();
        gc.dst_len[s] = dc.offsets.as<uint32_t>();
        gc.dst_src[s] = w.gsrc.as<uint32_t>() + p.gsrc0 + static_cast<uint64_t>(si) * m;
        ++si;
      }
    }
    if (m > 0 && n_select > 0)
      PXG_RETURN_IF_ERROR(Launch(ctx, "filter_gather", FilterGatherKernel, dim3(static_cast<unsigned>(p.ntiles)), dim3(kOpsBlock), 0,
                                 static_cast<const unsigned long long*>(w.masks.as<unsigned long long>() + p.mask0),
                                 static_cast<const uint32_t*>(w.tiles.as<uint32_t>() + p.tile0), p.lo, p.n, gc));
    si = 0;
    for (int s = 0; s < n_select; ++s) {
      if (gc.width[s] != 0) continue;
      uint32_t* doff = gc.dst_len[s];
      PXG_RETURN_IF_ERROR(w.scan2.Ensure(ScanScratchBytes(static_cast<int64_t>(m) + 1) + 64));
      PXG_HIP(hipMemsetAsync(doff + m, 0, 4, ctx->stream));
      PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, doff, doff, static_cast<int64_t>(m) + 1, nullptr, w.scan2.p));
      PXG_HIP(hipMemcpyAsync(pin + i * n_str + si, doff + m, 4, hipMemcpyDeviceToHost, ctx->stream));
      ++si;
    }
    o.nrows += m;
    o.chunks.push_back(std::move(oc));
  }
  // Phase C: string payloads.
  if (n_str > 0) {
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    for (size_t i = 0; i < parts.size(); ++i) {
      const Part& p = parts[i];
      const Chunk& ch = *t.chunks[p.c];
      Chunk& oc = *o.chunks[i];
      int si = 0;
      for (int s = 0; s < n_select; ++s) {
        if (gcs[i].width[s] != 0) continue;
        const int ci = select[s];
        ChunkCol& dc = oc.cols[static_cast<size_t>(s)];
        const uint32_t bytes = pin[i * n_str + si];
        PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.data, static_cast<size_t>(bytes) + 16));
        dc.data_len = bytes;
        if (p.m > 0)
          PXG_RETURN_IF_ERROR(Launch(ctx, "str_gather", StrGatherKernel, dim3(GridFor(p.m, 256, 1 << 30)), dim3(256), 0,
                                     ch.cols[ci].data.as<const uint8_t>(), static_cast<const uint32_t*>(gcs[i].dst_src[s]), static_cast<const uint32_t*>(gcs[i].dst_len[s]),
                                     dc.data.as<uint8_t>(), static_cast<int64_t>(p.m)));
        ++si;
      }
    }
  }
  ++o.version;
  *out = guard.release();
  return PXG_OK;
}

}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_filter(pxg_table* inp, const pxg_program* pred, int32_t n_select, const int32_t* select, int64_t begin,
                              int64_t end, pxg_table** out) {
  if (!inp || !pred || !out || n_select < 0 || (n_select > 0 && !select)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  return FilterImpl(inp->impl, *pred, n_select, select, begin, end, 0, nullptr, nullptr, out);
}

extern "C" int32_t pxg_filter_split(pxg_table* inp, const pxg_program* pred, int32_t n_select, const int32_t* select, int64_t begin,
                                    int64_t end, int32_t n_splits, const int64_t* split_rows, int64_t* out_split_rows,
                                    pxg_table** out) {
  if (!inp || !pred || !out || n_select < 0 || (n_select > 0 && !select) || n_splits < 0 ||
      (n_splits > 0 && (!split_rows || !out_split_rows)))
    return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  for (int i = 0; i < n_splits; ++i) out_split_rows[i] = 0;
  return FilterImpl(inp->impl, *pred, n_select, select, begin, end, n_splits, split_rows, out_split_rows, out);
}

extern "C" int32_t pxg_map(pxg_table* inp, int32_t n_exprs, const pxg_program* exprs, int64_t begin, int64_t end, pxg_table** out) {
  if (!inp || !out || n_exprs < 0 || (n_exprs > 0 && !exprs)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Table& t = inp->impl;
  Ctx* ctx = t.ctx;
  PXG_RETURN_IF_ERROR(t.EnsureDeviceDescriptors());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "bad row range");
  std::vector<int32_t> otypes;
  int n_str_pass = 0;
  for (int e = 0; e < n_exprs; ++e) {
    const pxg_program& p = exprs[e];
    const bool passthrough = p.n_insns == 1 && p.insns && p.insns[0].op == PXG_OP_COL;
    if (p.result_type == PXG_STRING && !passthrough)
      return SetError(PXG_UNIMPLEMENTED, "STRING-producing scalar UDFs are not implemented on device");
    otypes.push_back(p.result_type);
    n_str_pass += p.result_type == PXG_STRING ? 1 : 0;
  }
  const DevProgram* d_progs = nullptr;
  const int32_t* d_types = nullptr;
  PXG_RETURN_IF_ERROR(UploadPrograms(ctx, exprs, n_exprs, t, &d_progs, &d_types));
  pxg_table* ot = nullptr;
  PXG_RETURN_IF_ERROR(NewTable(ctx, static_cast<int32_t>(otypes.size()), otypes.data(), &ot));
  std::unique_ptr<pxg_table, int32_t (*)(pxg_table*)> guard(ot, pxg_table_destroy);
  Table& o = ot->impl;
  struct Part {
    size_t c;
    int64_t lo, n;
  };
  std::vector<Part> parts;
  for (size_t c = 0; c < t.chunks.size(); ++c) {
    const Chunk& ch = *t.chunks[c];
    const int64_t lo = std::max(begin, ch.row_base) - ch.row_base;
    const int64_t hi = std::min(end, ch.row_base + ch.nrows) - ch.row_base;
    if (lo < hi) parts.push_back({c, lo, hi - lo});
  }
  // Passed-through STRING columns: every chunk's first / last offset in one readback.
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps);
  if (n_str_pass > 0) {
    if (parts.size() * n_str_pass * 2 > (Ctx::kPinnedBytes - Ctx::kPinnedOps) / 4)
      return SetError(PXG_UNIMPLEMENTED, "map over %zu chunks", parts.size());
    size_t k = 0;
    for (const Part& p : parts) {
      const Chunk& ch = *t.chunks[p.c];
      for (int e = 0; e < n_exprs; ++e) {
        if (exprs[e].result_type != PXG_STRING) continue;
        const int32_t* so = ch.cols[exprs[e].insns[0].arg].offsets.as<int32_t>();
        PXG_HIP(hipMemcpyAsync(pin + k, so + p.lo, 4, hipMemcpyDeviceToHost, ctx->stream));
        PXG_HIP(hipMemcpyAsync(pin + k + 1, so + p.lo + p.n, 4, hipMemcpyDeviceToHost, ctx->stream));
        k += 2;
      }
    }
    PXG_HIP(hipStreamSynchronize(ctx->stream));
  }
  size_t k = 0;
  for (const Part& p : parts) {
    const Chunk& ch = *t.chunks[p.c];
    const int64_t lo = p.lo, n = p.n;
    auto oc = std::make_unique<Chunk>();
    oc->row_base = o.nrows;
    oc->nrows = n;
    oc->rows_cap = n;
    oc->sealed = true;
    oc->cols.resize(static_cast<size_t>(n_exprs));
    for (int e = 0; e < n_exprs; ++e) {
      const pxg_program& pr = exprs[e];
      ChunkCol& dc = oc->cols[static_cast<size_t>(e)];
      const int ty = pr.result_type;
      if (pr.n_insns == 1 && pr.insns[0].op == PXG_OP_COL) {
        const ChunkCol& sc = ch.cols[pr.insns[0].arg];
        if (ty == PXG_STRING) {
          const uint32_t o0 = pin[k], o1 = pin[k + 1];
          k += 2;
          PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.offsets, (n + 1) * 4 + 16));
          PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.data, static_cast<size_t>(o1 - o0) + 16));
          dc.data_len = o1 - o0;
          PXG_RETURN_IF_ERROR(Launch(ctx, "map_rebase", RebaseKernel, dim3(GridFor(n + 1, 256, 1 << 30)), dim3(256), 0,
                                     dc.offsets.as<int32_t>(), sc.offsets.as<const int32_t>() + lo, n + 1));
          if (o1 > o0)
            PXG_HIP(hipMemcpyAsync(dc.data.p, sc.data.as<uint8_t>() + o0, o1 - o0, hipMemcpyDeviceToDevice, ctx->stream));
        } else {
          const int w = TypeWidth(ty);
          PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.values, n * w + 16));
          PXG_HIP(hipMemcpyAsync(dc.values.p, sc.values.as<uint8_t>() + lo * w, n * w, hipMemcpyDeviceToDevice, ctx->stream));
        }
        continue;
      }
      const int w = TypeWidth(ty);
      PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.values, n * w + 16));
      PXG_RETURN_IF_ERROR(Launch(ctx, "map_eval", MapEvalKernel, dim3(GridFor(n, 256, 1 << 30)), dim3(256), 0, d_progs + e,
                                 t.d_chunks.as<const DevChunk>(), static_cast<int>(p.c), d_types, lo, n, dc.values.as<uint8_t>(), w));
    }
    o.nrows += n;
    o.chunks.push_back(std::move(oc));
  }
  ++o.version;
  *out = guard.release();
  return PXG_OK;
}
