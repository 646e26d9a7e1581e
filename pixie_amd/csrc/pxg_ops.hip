// Standalone FilterNode / MapNode over device tables (operator shapes the fused agg path does
// not cover).
//
// FilterNode::ConsumeNextImpl (filter_node.cc:132-171): evaluate the predicate, then compact
// every selected column, preserving row order (filter_node.cc:88-92).  On the device this is
// ballot compaction in three launches over every chunk of the call at once (up to kFBatch
// chunks per launch, their descriptors passed by value):
//   count: streams the predicate's columns, writes one 64-row ballot word per wave iteration,
//          and per 4096-row tile the selected rows and each selected STRING column's selected
//          payload bytes;
//   scan:  one workgroup per (chunk, quantity) turns the tile figures into exclusive bases and
//          chunk totals (one readback: the output sizes);
//   write: re-reads the ballot words, ranks every selected row inside its tile (prefix of the
//          tile's ballot popcounts + the lane's bits below it), gathers the fixed-width columns,
//          and for each STRING column scans the tile's selected lengths in LDS, writes the end
//          offsets and moves the payload (unaligned 16 / 8 / 4-byte moves).
// One synchronisation per call (the output sizes), whatever the chunk count.
//
// MapNode::ConsumeNextImpl (map_node.cc:64-71): one output column per expression; column
// references pass through (device-to-device copies).
//
// No per-call hipMalloc: programs, ballot words and tile figures live in the ctx's grow-only ops
// workspace, output columns come from the ctx buffer pool (refilled by pxg_table_destroy).
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
                              const int32_t** d_types, int32_t* shape0 = nullptr) {
  std::vector<DevProgram> dp(static_cast<size_t>(std::max(n, 1)));
  std::vector<uint8_t> pool;
  std::vector<size_t> offs(static_cast<size_t>(std::max(n, 1)));
  for (int i = 0; i < n; ++i) PXG_RETURN_IF_ERROR(CompileProgram(progs[i], t.types.data(), t.ncols, &dp[i], &pool, &offs[i]));
  if (shape0) *shape0 = n > 0 ? dp[0].shape : kShapeGeneric;
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

// One string's payload: len bytes from s to d as unaligned 16 / 8 / 4-byte moves; the last move
// overlaps the previous one and ends exactly at len, so nothing outside the string is written.
__device__ __forceinline__ void CopyString(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, uint32_t len) {
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

// The chunks of one launch (by value: no upload, no synchronisation for descriptors).
constexpr int kFBatch = 8;
struct FPart {
  int32_t c;       // input chunk
  int32_t ntiles;
  int64_t lo, n;   // chunk rows [lo, lo + n)
  int64_t tile0;   // global index of the part's first tile (ballot words at tile * 64)
};
struct FOut {      // a part's output chunk, per selected column
  uint8_t* val[kMaxCols];
  int32_t* off[kMaxCols];
  uint8_t* data[kMaxCols];
};
struct FSel {
  int32_t n, n_str;
  int32_t col[kMaxCols];    // input column of each selected column
  int32_t width[kMaxCols];  // bytes per value; 0 = STRING
  int32_t sidx[kMaxCols];   // STRING: its ordinal among the selected STRING columns
};
struct FBatch {
  int32_t n;        // parts in this launch
  int64_t t_begin;  // global tile of blockIdx.x == 0
  FPart part[kFBatch];
};
struct FOutBatch {
  FOut out[kFBatch];
};

// A launch's descriptors.  They reach the kernels through global memory, written by a one-
// workgroup copy kernel that takes them by value: indexing a by-value kernel argument with a
// run-time chunk / column index makes the compiler copy the whole argument into per-thread
// scratch (measured: the write pass took 2.5 ms instead of ~0.4).
struct FDesc {
  FBatch fb;
  FSel sel;
  FOutBatch fo;
};
static_assert(sizeof(FDesc) % 8 == 0 && sizeof(FDesc) <= 3840, "FDesc travels as a kernel argument");

__global__ void __launch_bounds__(256) FDescCopyKernel(FDesc d, uint64_t* __restrict__ dst) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(&d);
  for (uint32_t i = threadIdx.x; i < sizeof(FDesc) / 8; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ int FindPart(const FBatch& b, int64_t tile) {
  int p = 0;
  while (p + 1 < b.n && tile >= b.part[p + 1].tile0) ++p;
  return p;
}

// Count: ballot words of the predicate and per tile the selected rows (fig[tile]).
// kFast: the predicate is a column or column-op-constant over a fixed-width column (no program
// interpreter, whose value stack would give every wave a scratch allocation).
template <bool kFast>
__global__ void __launch_bounds__(kOpsBlock) FilterCountKernel(const DevProgram* __restrict__ prog, const DevChunk* __restrict__ chunks,
                                                               const int32_t* __restrict__ types, const FDesc* __restrict__ fd,
                                                               unsigned long long* __restrict__ masks, uint32_t* __restrict__ fig, int64_t T) {
  const FBatch& fb = fd->fb;
  __shared__ uint32_t s_cnt[1][kOpsBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t tile = fb.t_begin + blockIdx.x;
  const FPart& pt = fb.part[FindPart(fb, tile)];
  const DevChunk& ch = chunks[pt.c];
  const int64_t t0 = (tile - pt.tile0) * kOpsTileRows;  // part-relative first row
  const int64_t n = pt.n, lo = pt.lo;
  unsigned long long m[kOpsMasksPerWave];
  const int pty = kFast ? types[prog->col] : 0;
  const bool pairs = kFast && (pty == PXG_INT64 || pty == PXG_FLOAT64 || pty == PXG_TIME64NS) && ((lo & 1) == 0);
  if (pairs) {
    // 16-byte loads, two rows per lane (8 loads in flight per lane); the even / odd rows'
    // ballots are interleaved into the 64-row words.
    const uint64_t* col = reinterpret_cast<const uint64_t*>(ch.cols[prog->col].values) + lo;
    ulonglong2 raw[kOpsMasksPerWave / 2];
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave / 2; ++k) {
      const int64_t r = t0 + static_cast<int64_t>(wid) * kOpsMasksPerWave * 64 + k * 128 + 2 * lane;
      raw[k] = r < n ? *reinterpret_cast<const ulonglong2*>(col + r) : make_ulonglong2(0, 0);
    }
    auto spread = [](uint64_t x) {  // bit i -> bit 2i (x < 2^32)
      x = (x | (x << 16)) & 0x0000FFFF0000FFFFULL;
      x = (x | (x << 8)) & 0x00FF00FF00FF00FFULL;
      x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0FULL;
      x = (x | (x << 2)) & 0x3333333333333333ULL;
      x = (x | (x << 1)) & 0x5555555555555555ULL;
      return x;
    };
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave / 2; ++k) {
      const int64_t r = t0 + static_cast<int64_t>(wid) * kOpsMasksPerWave * 64 + k * 128 + 2 * lane;
      uint64_t v0 = raw[k].x, v1 = raw[k].y;
      if (prog->shape == kShapeColOpConst) {
        if (prog->conv) {
          v0 = Conv(prog->conv, v0);
          v1 = Conv(prog->conv, v1);
        }
        v0 = BinOp(prog->binop, v0, static_cast<uint64_t>(prog->cimm));
        v1 = BinOp(prog->binop, v1, static_cast<uint64_t>(prog->cimm));
      }
      const unsigned long long me = __ballot(r < n && v0 != 0);
      const unsigned long long mo = __ballot(r + 1 < n && v1 != 0);
      m[2 * k] = spread(me & 0xFFFFFFFFULL) | (spread(mo & 0xFFFFFFFFULL) << 1);
      m[2 * k + 1] = spread(me >> 32) | (spread(mo >> 32) << 1);
    }
  } else if constexpr (kFast) {
    // Fast shapes (col, col op const over a fixed-width column): the wave's 16 loads are issued
    // together, then evaluated.
    const DevCol& col = ch.cols[prog->col];
    const int ty = types[prog->col];
    uint64_t raw[kOpsMasksPerWave];
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave; ++k) {
      const int64_t r = t0 + (static_cast<int64_t>(wid) * kOpsMasksPerWave + k) * 64 + lane;
      raw[k] = r < n ? LoadCol(col, ty, lo + r).a : 0ULL;
    }
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave; ++k) {
      const int64_t r = t0 + (static_cast<int64_t>(wid) * kOpsMasksPerWave + k) * 64 + lane;
      uint64_t v = raw[k];
      if (prog->shape == kShapeColOpConst) {
        if (prog->conv) v = Conv(prog->conv, v);
        v = BinOp(prog->binop, v, static_cast<uint64_t>(prog->cimm));
      }
      m[k] = __ballot(r < n && v != 0);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOpsMasksPerWave; ++k) {
      const int64_t r = t0 + (static_cast<int64_t>(wid) * kOpsMasksPerWave + k) * 64 + lane;
      m[k] = __ballot(r < n && EvalProgram(prog, ch, lo + r, types).a != 0);
    }
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < kOpsMasksPerWave; ++k) {
    cnt += static_cast<uint32_t>(__popcll(m[k]));
    if (lane == 0) masks[tile * kOpsMasksPerTile + wid * kOpsMasksPerWave + k] = m[k];
  }
  if (lane == 0) s_cnt[0][wid] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) fig[tile] = s_cnt[0][0] + s_cnt[0][1] + s_cnt[0][2] + s_cnt[0][3];
}

// Scan: workgroup (p, q) turns quantity q's tile figures of part p into exclusive bases (in
// place) and writes the part's total to totals[(part0 + p) * (1 + n_str) + q].  A part has at
// most kChunkRows / kOpsTileRows = 4096 tiles: 16 per thread.
constexpr int kFScanPer = 16;
static_assert(kOpsBlock * kFScanPer * kOpsTileRows >= kChunkRows, "a part's tiles must fit one scan workgroup");
__global__ void __launch_bounds__(kOpsBlock) FilterScanKernel(const FDesc* __restrict__ fd, int part0, int nq, uint32_t* __restrict__ fig,
                                                              int64_t T, uint32_t* __restrict__ totals, uint32_t* __restrict__ maxes) {
  __shared__ uint32_t s_part[kOpsBlock];
  __shared__ uint32_t s_max[kOpsBlock / 64];
  const FPart& pt = fd->fb.part[blockIdx.x];
  const int q = blockIdx.y;
  uint32_t* f = fig + q * T + pt.tile0;
  const int nt = pt.ntiles;
  const int i0 = threadIdx.x * kFScanPer;
  uint32_t v[kFScanPer];
  uint32_t sum = 0, mx = 0;
#pragma unroll
  for (int j = 0; j < kFScanPer; ++j) {
    v[j] = i0 + j < nt ? f[i0 + j] : 0u;
    sum += v[j];
    mx = max(mx, v[j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, o, 64)));
  if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = mx;
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < kOpsBlock; o <<= 1) {  // inclusive Hillis-Steele scan of the partials
    const uint32_t y = threadIdx.x >= o ? s_part[threadIdx.x - o] : 0u;
    __syncthreads();
    s_part[threadIdx.x] += y;
    __syncthreads();
  }
  uint32_t run = s_part[threadIdx.x] - sum;
#pragma unroll
  for (int j = 0; j < kFScanPer; ++j) {
    if (i0 + j < nt) f[i0 + j] = run;
    run += v[j];
  }
  if (threadIdx.x == kOpsBlock - 1) totals[(part0 + blockIdx.x) * nq + q] = s_part[kOpsBlock - 1];
  if (threadIdx.x == 0 && q == 0) maxes[part0 + blockIdx.x] = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
}

// Decoupled look-back status words (one per tile and STRING column): bits 62-63 the state
// (0 not ready, 1 the tile's own byte count, 2 the inclusive prefix within its chunk).
constexpr uint64_t kLbAgg = uint64_t(1) << 62, kLbIncl = uint64_t(2) << 62, kLbVal = (uint64_t(1) << 62) - 1;

// Write: the tile's selected rows in output order.  The ballot words give every selected row its
// rank (prefix of the tile's ballot popcounts + the lane's bits below it) and an LDS table maps
// rank -> tile row; then thread t handles ranks t, t + 256, ..., so every column's gather, store
// and string copy runs on dense lanes (at 12% selectivity a per-row loop leaves 7 of 8 lanes
// idle).  Row bases come from the scan pass.  STRING columns: the tile sums its selected lengths,
// finds its byte base by decoupled look-back over the preceding tiles of its chunk (tiles are
// taken in launch order from a counter, so every tile it waits for is already running), then a
// block scan per round of 256 ranks places each payload and writes the end offsets.
// The first kFLdsStr STRING columns keep every selected row's {start, length} in dynamic LDS
// (lds_cap entries per column: the largest tile count of the call, from the scan) between the
// byte count and the payload copy, so the offsets are read once.
constexpr int kFLdsStr = 2;
__global__ void __launch_bounds__(kOpsBlock) FilterWriteKernel(const DevChunk* __restrict__ chunks, const FDesc* __restrict__ fd,
                                                               const unsigned long long* __restrict__ masks, const uint32_t* __restrict__ fig,
                                                               int64_t T, unsigned int* __restrict__ tile_ctr, uint64_t* __restrict__ lb,
                                                               uint32_t lds_cap) {
  extern __shared__ uint32_t s_dyn[];  // [kFLdsStr][lds_cap] starts, then [kFLdsStr][lds_cap] lengths
  __shared__ uint32_t s_pre[kOpsMasksPerTile];
  __shared__ uint16_t s_row[kOpsTileRows];
  __shared__ uint32_t s_wave[kOpsBlock / 64];
  __shared__ uint32_t s_tot;
  __shared__ uint64_t s_agg[kMaxCols], s_base[kMaxCols];
  __shared__ int64_t s_tile;
  const FBatch& fb = fd->fb;
  const FSel& sel = fd->sel;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ULL << lane) - 1;
  if (threadIdx.x == 0) s_tile = fb.t_begin + static_cast<int64_t>(atomicAdd(tile_ctr, 1u));
  __syncthreads();
  const int64_t tile = s_tile;
  const int p = FindPart(fb, tile);
  const FPart& pt = fb.part[p];
  const FOut& out = fd->fo.out[p];
  const DevChunk& ch = chunks[pt.c];
  const int64_t mask0 = tile * kOpsMasksPerTile;
  if (threadIdx.x < kOpsMasksPerTile) {  // one wave: exclusive prefix of the 64 popcounts
    const uint32_t c = static_cast<uint32_t>(__popcll(masks[mask0 + threadIdx.x]));
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    s_pre[threadIdx.x] = x - c;
    if (threadIdx.x == kOpsMasksPerTile - 1) s_tot = x;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kOpsMasksPerWave; ++k) {
    const int mi = wid * kOpsMasksPerWave + k;
    const unsigned long long m = masks[mask0 + mi];
    if ((m >> lane) & 1ULL) s_row[s_pre[mi] + __popcll(m & lanemask_lt)] = static_cast<uint16_t>(mi * 64 + lane);
  }
  __syncthreads();
  const uint32_t tile_sel = s_tot;
  const uint32_t base = fig[tile];
  const int64_t row0 = pt.lo + (tile - pt.tile0) * kOpsTileRows;
  const int64_t first = pt.tile0;  // the chunk's first tile: its bytes start at 0
  // 1. Every STRING column's selected payload bytes, published at once (the look-back comes
  //    after the fixed-width gathers, so the predecessors have had time to publish too).
  for (int c = 0; c < sel.n; ++c) {
    if (sel.width[c] != 0) continue;
    const int32_t* off = ch.cols[sel.col[c]].offsets + row0;
    const int si = sel.sidx[c];
    uint32_t* s_st = s_dyn + static_cast<uint32_t>(si) * lds_cap;
    uint32_t* s_ln = s_dyn + static_cast<uint32_t>(kFLdsStr + si) * lds_cap;
    const bool keep = si < kFLdsStr && tile_sel <= lds_cap;
    uint32_t bytes = 0;
    for (uint32_t i = threadIdx.x; i < tile_sel; i += kOpsBlock) {
      const uint32_t r = s_row[i];
      const int32_t a = off[r];
      const uint32_t len = static_cast<uint32_t>(off[r + 1] - a);
      bytes += len;
      if (keep) {
        s_st[i] = static_cast<uint32_t>(a);
        s_ln[i] = len;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o, 64);
    if (lane == 0) s_wave[wid] = bytes;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t agg = static_cast<uint64_t>(s_wave[0]) + s_wave[1] + s_wave[2] + s_wave[3];
      s_agg[sel.sidx[c]] = agg;
      __hip_atomic_store(&lb[static_cast<int64_t>(sel.sidx[c]) * T + tile], (tile == first ? kLbIncl : kLbAgg) | agg, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  // 2. Fixed-width columns.
  for (int c = 0; c < sel.n; ++c) {
    const int w = sel.width[c];
    const DevCol& sc = ch.cols[sel.col[c]];
    if (w == 8) {
      const uint64_t* src = reinterpret_cast<const uint64_t*>(sc.values) + row0;
      uint64_t* dst = reinterpret_cast<uint64_t*>(out.val[c]) + base;
      for (uint32_t i = threadIdx.x; i < tile_sel; i += kOpsBlock) dst[i] = src[s_row[i]];
    } else if (w == 16) {
      const ulonglong2* src = reinterpret_cast<const ulonglong2*>(sc.values) + row0;
      ulonglong2* dst = reinterpret_cast<ulonglong2*>(out.val[c]) + base;
      for (uint32_t i = threadIdx.x; i < tile_sel; i += kOpsBlock) dst[i] = src[s_row[i]];
    } else if (w != 0) {
      const uint8_t* src = sc.values + row0;
      uint8_t* dst = out.val[c] + base;
      for (uint32_t i = threadIdx.x; i < tile_sel; i += kOpsBlock) dst[i] = src[s_row[i]];
    }
  }
  // 3. Byte bases by look-back (the first wave, one STRING column after the other).
  if (wid == 0) {
    for (int q = 0; q < sel.n_str; ++q) {
      uint64_t* st = lb + static_cast<int64_t>(q) * T;
      uint64_t excl = 0;
      if (tile != first) {
        int64_t j = tile - 1;
        while (true) {
          const int64_t idx = j - lane;
          const uint64_t wv = idx >= first ? __hip_atomic_load(&st[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
          const uint64_t flag = wv >> 62;
          const unsigned long long incl = __ballot(flag == 2);
          const unsigned long long zero = __ballot(flag == 0);
          const int fi = incl ? __ffsll(static_cast<long long>(incl)) - 1 : 64;
          const unsigned long long need = fi == 64 ? ~0ULL : ((2ULL << fi) - 1);
          if (zero & need) continue;  // a predecessor has not published yet: read the window again
          uint64_t v = lane <= fi ? (wv & kLbVal) : 0;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
          excl += v;
          if (fi < 64) break;
          j -= 64;
        }
        if (lane == 0) __hip_atomic_store(&st[tile], kLbIncl | (excl + s_agg[q]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) s_base[q] = excl;
    }
  }
  __syncthreads();
  // 4. STRING payloads: a block scan per round of 256 ranks, carried across rounds.
  for (int c = 0; c < sel.n; ++c) {
    if (sel.width[c] != 0) continue;
    const DevCol& sc = ch.cols[sel.col[c]];
    const int32_t* off = sc.offsets + row0;
    int32_t* doff = out.off[c] + base + 1;
    uint8_t* ddata = out.data[c];
    uint32_t carry = static_cast<uint32_t>(s_base[sel.sidx[c]]);
    const int si = sel.sidx[c];
    const uint32_t* s_st = s_dyn + static_cast<uint32_t>(si) * lds_cap;
    const uint32_t* s_ln = s_dyn + static_cast<uint32_t>(kFLdsStr + si) * lds_cap;
    const bool kept = si < kFLdsStr && tile_sel <= lds_cap;
    for (uint32_t r0 = 0; r0 < tile_sel; r0 += kOpsBlock) {  // block-uniform rounds
      const uint32_t i = r0 + threadIdx.x;
      const bool on = i < tile_sel;
      int32_t a = 0;
      uint32_t len = 0;
      if (on) {
        if (kept) {
          a = static_cast<int32_t>(s_st[i]);
          len = s_ln[i];
        } else {
          const uint32_t r = s_row[i];
          a = off[r];
          len = static_cast<uint32_t>(off[r + 1] - a);
        }
      }
      uint32_t x = len;  // inclusive wave scan, then the waves before this one
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      __syncthreads();  // the previous round has read s_wave
      if (lane == 63) s_wave[wid] = x;
      __syncthreads();
      uint32_t before = 0, round = 0;
#pragma unroll
      for (int v = 0; v < kOpsBlock / 64; ++v) {
        before += v < wid ? s_wave[v] : 0u;
        round += s_wave[v];
      }
      const uint32_t end = carry + before + x;
      if (on) {
        doff[i] = static_cast<int32_t>(end);
        CopyString(sc.data + a, ddata + end - len, len);
      }
      carry += round;
    }
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
// rows of each of n_splits consecutive input row ranges (split_rows[i] rows each).  One output
// chunk per input chunk; output columns come from the ctx pool.
static int32_t FilterImpl(Table& t, const pxg_program& pred, int32_t n_select, const int32_t* select, int64_t begin, int64_t end,
                          int32_t n_splits, const int64_t* split_rows, int64_t* per_split, pxg_table** out) {
  Ctx* ctx = t.ctx;
  PXG_RETURN_IF_ERROR(t.EnsureDeviceDescriptors());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "bad row range");
  if (pred.result_type != PXG_BOOLEAN) return SetError(PXG_INVALID_ARGUMENT, "Predicate expression must be a boolean");
  if (n_select > kMaxCols) return SetError(PXG_UNIMPLEMENTED, "at most %d selected columns", kMaxCols);
  std::vector<int32_t> otypes;
  FSel fs;
  std::memset(&fs, 0, sizeof(fs));
  fs.n = n_select;
  for (int i = 0; i < n_select; ++i) {
    if (select[i] < 0 || select[i] >= t.ncols) return SetError(PXG_INVALID_ARGUMENT, "selected column %d out of range", select[i]);
    const int ty = t.types[select[i]];
    otypes.push_back(ty);
    fs.col[i] = select[i];
    fs.width[i] = ty == PXG_STRING ? 0 : TypeWidth(ty);
    fs.sidx[i] = ty == PXG_STRING ? fs.n_str++ : -1;
  }
  const int nq = 1;  // the scan pass: selected rows only (string bytes by look-back in the write)
  if (n_splits > 0) {
    int64_t tot = 0;
    for (int i = 0; i < n_splits; ++i) tot += split_rows[i];
    if (tot != end - begin) return SetError(PXG_INVALID_ARGUMENT, "split rows add up to %lld, range has %lld", (long long)tot, (long long)(end - begin));
  }
  std::vector<FPart> parts;
  int64_t T = 0;
  for (size_t c = 0; c < t.chunks.size(); ++c) {
    const Chunk& ch = *t.chunks[c];
    const int64_t lo = std::max(begin, ch.row_base) - ch.row_base;
    const int64_t hi = std::min(end, ch.row_base + ch.nrows) - ch.row_base;
    if (lo >= hi) continue;
    FPart p;
    p.c = static_cast<int32_t>(c);
    p.lo = lo;
    p.n = hi - lo;
    p.ntiles = static_cast<int32_t>((p.n + kOpsTileRows - 1) / kOpsTileRows);
    p.tile0 = T;
    T += p.ntiles;
    parts.push_back(p);
  }
  const size_t pin_cap = (Ctx::kPinnedBytes - Ctx::kPinnedOps) / 4;
  // pinned: [0, P) selected rows, then per (part, STRING column) the input byte range (2 words)
  // and the output bytes (2 words, the look-back's u64 inclusive prefix)
  if (parts.size() * (2 + 4 * static_cast<size_t>(fs.n_str)) + 2 > pin_cap) return SetError(PXG_UNIMPLEMENTED, "filter over %zu chunks", parts.size());
  uint32_t* pin = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps);
  pxg_table* ot = nullptr;
  PXG_RETURN_IF_ERROR(NewTable(ctx, static_cast<int32_t>(otypes.size()), otypes.data(), &ot));
  std::unique_ptr<pxg_table, int32_t (*)(pxg_table*)> guard(ot, pxg_table_destroy);
  Table& o = ot->impl;
  if (parts.empty()) {
    *out = guard.release();
    return PXG_OK;
  }
  const DevProgram* d_prog = nullptr;
  const int32_t* d_types = nullptr;
  int32_t shape = kShapeGeneric;
  PXG_RETURN_IF_ERROR(UploadPrograms(ctx, &pred, 1, t, &d_prog, &d_types, &shape));
  const bool fast = shape == kShapeCol || shape == kShapeColOpConst;
  OpsWorkspace& w = ctx->ops;
  PXG_RETURN_IF_ERROR(w.masks.Ensure(static_cast<size_t>(T) * kOpsMasksPerTile * 8 + 64));
  PXG_RETURN_IF_ERROR(w.tiles.Ensure(static_cast<size_t>(T) * nq * 4 + parts.size() * (nq + 1) * 4 + 64));
  uint32_t* fig = w.tiles.as<uint32_t>();
  uint32_t* totals = fig + T * nq;
  uint32_t* maxes = totals + parts.size() * nq;  // the largest tile count of each part
  // Chunks per launch (tests: PXG_FILTER_BATCH=1..8 forces launch boundaries at small sizes).
  const char* fbe = std::getenv("PXG_FILTER_BATCH");
  const size_t nbatch = fbe && std::atoi(fbe) >= 1 && std::atoi(fbe) <= kFBatch ? static_cast<size_t>(std::atoi(fbe)) : kFBatch;
  auto batch_of = [&](size_t b0) {
    FBatch fb;
    std::memset(&fb, 0, sizeof(fb));
    fb.n = static_cast<int32_t>(std::min<size_t>(nbatch, parts.size() - b0));
    fb.t_begin = parts[b0].tile0;
    for (int i = 0; i < fb.n; ++i) fb.part[i] = parts[b0 + i];
    return fb;
  };
  auto batch_tiles = [&](const FBatch& fb) { return fb.part[fb.n - 1].tile0 + fb.part[fb.n - 1].ntiles - fb.t_begin; };
  // Count + scan of every batch, then one readback of the output sizes.
  // The descriptors' device copy (stream order: a launch's copy runs after the previous launch).
  PXG_RETURN_IF_ERROR(w.gsrc.Ensure(sizeof(FDesc) + 64));
  const FDesc* d_desc = w.gsrc.as<const FDesc>();
  FDesc desc;
  std::memset(&desc, 0, sizeof(desc));
  desc.sel = fs;
  for (size_t b0 = 0; b0 < parts.size(); b0 += nbatch) {
    const FBatch fb = batch_of(b0);
    desc.fb = fb;
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_desc", FDescCopyKernel, dim3(1), dim3(256), 0, desc, w.gsrc.as<uint64_t>()));
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_count", fast ? FilterCountKernel<true> : FilterCountKernel<false>,
                               dim3(static_cast<unsigned>(batch_tiles(fb))), dim3(kOpsBlock), 0, d_prog, t.d_chunks.as<const DevChunk>(),
                               d_types, d_desc, w.masks.as<unsigned long long>(), fig, T));
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_scan", FilterScanKernel, dim3(static_cast<unsigned>(fb.n), static_cast<unsigned>(nq)), dim3(kOpsBlock),
                               0, d_desc, static_cast<int>(b0), nq, fig, T, totals, maxes));
  }
  // totals then maxes (adjacent on the device)
  PXG_HIP(hipMemcpyAsync(pin, totals, parts.size() * (nq + 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
  // Each STRING column's input byte range of each part: the worst-case output payload (the write
  // pass finds the exact size by look-back, read back at the end).
  int32_t* pin_rng = reinterpret_cast<int32_t*>(pin + parts.size() * (nq + 1));
  for (size_t i = 0; i < parts.size(); ++i)
    for (int sidx = 0, s2 = 0; s2 < n_select; ++s2) {
      if (fs.width[s2] != 0) continue;
      const int32_t* so = t.chunks[parts[i].c]->cols[select[s2]].offsets.as<const int32_t>();
      PXG_HIP(hipMemcpyAsync(pin_rng + 2 * (i * fs.n_str + sidx), so + parts[i].lo, 4, hipMemcpyDeviceToHost, ctx->stream));
      PXG_HIP(hipMemcpyAsync(pin_rng + 2 * (i * fs.n_str + sidx) + 1, so + parts[i].lo + parts[i].n, 4, hipMemcpyDeviceToHost, ctx->stream));
      ++sidx;
    }
  std::vector<unsigned long long> host_masks;
  if (n_splits > 0) {  // ballot words back to the host: per-split counts by popcount
    host_masks.resize(static_cast<size_t>(T) * kOpsMasksPerTile);
    PXG_HIP(hipMemcpyAsync(host_masks.data(), w.masks.p, host_masks.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  if (n_splits > 0) {
    for (const FPart& p : parts) {
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
          unsigned long long mk = host_masks[static_cast<size_t>(p.tile0 * kOpsMasksPerTile + wi)] >> (r & 63);
          const int64_t bits = e - r;
          if (bits < 64) mk &= (1ULL << bits) - 1;
          per_split[i] += __builtin_popcountll(mk);
          r = e;
        }
        s0 = s1;
      }
    }
  }
  // Output chunks, then the write launches.
  std::vector<FOut> outs(parts.size());
  for (size_t i = 0; i < parts.size(); ++i) {
    const uint32_t m = pin[i * nq];
    auto oc = std::make_unique<Chunk>();
    oc->row_base = o.nrows;
    oc->nrows = m;
    oc->rows_cap = m;
    oc->sealed = true;
    oc->cols.resize(static_cast<size_t>(n_select));
    FOut& fo = outs[i];
    std::memset(&fo, 0, sizeof(fo));
    for (int s = 0; s < n_select; ++s) {
      ChunkCol& dc = oc->cols[static_cast<size_t>(s)];
      if (fs.width[s] != 0) {
        PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.values, static_cast<size_t>(m) * fs.width[s] + 16));
        fo.val[s] = dc.values.as<uint8_t>();
      } else {
        const int32_t* rg = pin_rng + 2 * (i * fs.n_str + fs.sidx[s]);
        const size_t worst = static_cast<size_t>(rg[1] - rg[0]);
        PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.offsets, (static_cast<size_t>(m) + 1) * 4 + 16));
        PXG_RETURN_IF_ERROR(PoolAlloc(ctx, dc.data, (m > 0 ? worst : 0) + 16));
        PXG_HIP(hipMemsetAsync(dc.offsets.p, 0, 4, ctx->stream));  // offsets[0]; the write stores end offsets
        fo.off[s] = dc.offsets.as<int32_t>();
        fo.data[s] = dc.data.as<uint8_t>();
      }
    }
    o.nrows += m;
    o.chunks.push_back(std::move(oc));
  }
  uint32_t max_sel = 0;
  for (size_t i = 0; i < parts.size(); ++i) max_sel = std::max(max_sel, pin[parts.size() * nq + i]);
  const size_t lds_bytes = fs.n_str > 0 ? static_cast<size_t>(2 * kFLdsStr) * max_sel * 4 : 0;
  uint64_t* lb = nullptr;
  unsigned int* tile_ctr = nullptr;
  if (n_select > 0) {
    PXG_RETURN_IF_ERROR(w.scan.Ensure(static_cast<size_t>(T) * std::max(fs.n_str, 1) * 8 + 64));
    PXG_RETURN_IF_ERROR(w.scan2.Ensure(((parts.size() + nbatch - 1) / nbatch) * 4 + 64));
    lb = w.scan.as<uint64_t>();
    tile_ctr = w.scan2.as<unsigned int>();
    if (fs.n_str > 0) PXG_HIP(hipMemsetAsync(lb, 0, static_cast<size_t>(T) * fs.n_str * 8, ctx->stream));
    PXG_HIP(hipMemsetAsync(tile_ctr, 0, ((parts.size() + nbatch - 1) / nbatch) * 4, ctx->stream));
  }
  for (size_t b0 = 0; b0 < parts.size() && n_select > 0; b0 += nbatch) {
    const FBatch fb = batch_of(b0);
    desc.fb = fb;
    std::memset(&desc.fo, 0, sizeof(desc.fo));
    for (int i = 0; i < fb.n; ++i) desc.fo.out[i] = outs[b0 + i];
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_desc", FDescCopyKernel, dim3(1), dim3(256), 0, desc, w.gsrc.as<uint64_t>()));
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_write", FilterWriteKernel, dim3(static_cast<unsigned>(batch_tiles(fb))), dim3(kOpsBlock), lds_bytes,
                               t.d_chunks.as<const DevChunk>(), d_desc, static_cast<const unsigned long long*>(w.masks.as<unsigned long long>()),
                               static_cast<const uint32_t*>(fig), T, tile_ctr + b0 / nbatch, lb, max_sel));
  }
  if (fs.n_str > 0 && n_select > 0) {  // exact payload sizes: each part's last inclusive prefix
    uint64_t* pin_out = reinterpret_cast<uint64_t*>((reinterpret_cast<uintptr_t>(pin_rng + 2 * parts.size() * fs.n_str) + 7) & ~uintptr_t(7));
    for (size_t i = 0; i < parts.size(); ++i)
      for (int sidx = 0; sidx < fs.n_str; ++sidx)
        PXG_HIP(hipMemcpyAsync(pin_out + i * fs.n_str + sidx, lb + static_cast<int64_t>(sidx) * T + parts[i].tile0 + parts[i].ntiles - 1, 8,
                               hipMemcpyDeviceToHost, ctx->stream));
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    for (size_t i = 0; i < parts.size(); ++i)
      for (int s2 = 0; s2 < n_select; ++s2)
        if (fs.width[s2] == 0) o.chunks[i]->cols[static_cast<size_t>(s2)].data_len = static_cast<int64_t>(pin_out[i * fs.n_str + fs.sidx[s2]] & kLbVal);
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
