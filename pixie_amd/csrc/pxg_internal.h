// Host-side internals of libpxg: context, device buffers, kernel timing, tables.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pxg.h"
#include "pxg_device.h"
#include "pxg_errors.h"

#define PXG_HIP(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return ::pxg::SetError(PXG_INTERNAL, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                             __FILE__, __LINE__);                                               \
  } while (0)

#define PXG_RETURN_IF_ERROR(expr) \
  do {                            \
    int32_t s_ = (expr);          \
    if (s_ != PXG_OK) return s_;  \
  } while (0)

namespace pxg {

// Boolean environment switch (set and not "0"); read at each use, so tests can flip it.
inline bool EnvFlag(const char* name) {
  const char* e = std::getenv(name);
  return e != nullptr && e[0] != 0 && !(e[0] == '0' && e[1] == 0);
}

// Device allocation that frees itself; capacity-tracked for growth.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { Free(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
    return *this;
  }
  ~DevBuf() { Free(); }
  void Free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  int32_t Alloc(size_t n) {
    Free();
    if (n == 0) n = 16;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
      p = nullptr;
      return SetError(PXG_RESOURCE_UNAVAILABLE, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    }
    bytes = n;
    return PXG_OK;
  }
  // Ensure capacity >= n, preserving the first `keep` bytes (stream-ordered copy).
  int32_t Reserve(size_t n, size_t keep, hipStream_t s) {
    if (n <= bytes) return PXG_OK;
    size_t cap = bytes ? bytes : 256;
    while (cap < n) cap *= 2;
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, cap);
    if (e != hipSuccess) return SetError(PXG_RESOURCE_UNAVAILABLE, "hipMalloc(%zu) failed: %s", cap, hipGetErrorString(e));
    if (keep && p) {
      e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return SetError(PXG_INTERNAL, "hipMemcpyAsync failed: %s", hipGetErrorString(e));
      e = hipStreamSynchronize(s);
      if (e != hipSuccess) return SetError(PXG_INTERNAL, "sync failed: %s", hipGetErrorString(e));
    }
    Free();
    p = q;
    bytes = cap;
    return PXG_OK;
  }
  // Capacity >= n without power-of-two rounding (the caller picks the growth policy).
  int32_t ReserveExact(size_t n, size_t keep, hipStream_t s) {
    if (n <= bytes) return PXG_OK;
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, n);
    if (e != hipSuccess) return SetError(PXG_RESOURCE_UNAVAILABLE, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    if (keep && p) {
      e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return SetError(PXG_INTERNAL, "hipMemcpyAsync failed: %s", hipGetErrorString(e));
      e = hipStreamSynchronize(s);
      if (e != hipSuccess) return SetError(PXG_INTERNAL, "sync failed: %s", hipGetErrorString(e));
    }
    Free();
    p = q;
    bytes = n;
    return PXG_OK;
  }
  // Grow-only scratch: capacity >= n, contents not preserved.
  int32_t Ensure(size_t n) { return Reserve(n, 0, nullptr); }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

struct KernelStat {
  int64_t launches = 0;
  double total_ms = 0;
};

struct PendingTiming {
  std::string name;
  hipEvent_t start, stop;
};

// Grow-only workspace of the standalone Filter / Map operators (pxg_ops.hip).
struct OpsWorkspace {
  DevBuf prog, masks, tiles, scan, scan2, gsrc;
};

// Per-context cache of device buffers released by destroyed operator output tables, so the
// standalone Filter / Map do not hipMalloc (and their tables' destruction does not hipFree,
// which synchronises the device) on every call.  Reuse is ordered by the ctx stream: every
// kernel that reads a released buffer was issued on that stream before the next user's.
struct BufPool {
  std::multimap<size_t, void*> free;
  size_t cached = 0;
  size_t cap = size_t(16) << 30;
};

struct Ctx {
  int device = 0;
  OpsWorkspace ops;
  BufPool pool;
  hipStream_t stream = nullptr;
  // Side stream for latency-bound work that overlaps the main stream (fork/join by events).
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // Second side stream: the big-group quantile merges overlap the mid digests and the key output.
  hipStream_t side2 = nullptr;
  hipEvent_t ev_fork2 = nullptr, ev_join2 = nullptr;
  hipEvent_t ev_meta = nullptr;  // finalize: the big-group metadata readback has landed
  hipEvent_t ev_chain = nullptr; // finalize: the digest boundary chains are done (side stream)
  hipEvent_t ev_split = nullptr; // finalize: the staging split's bucket totals have landed (pinned)
  hipEvent_t ev_early = nullptr; // finalize: the fused split's designated groups are final (main stream)
  hipEvent_t ev_pub = nullptr;   // consume: the publish read-back is on the host (main stream)
  bool profiling = false;
  std::string profile_only;  // non-empty: only launches of this kernel name are timed
  std::map<std::string, KernelStat> stats;
  std::vector<PendingTiming> pending;
  std::vector<hipEvent_t> free_events;
  int num_cus = 256;
  // Pinned scratch for counters read back by the host (async D2H, no staging copy):
  // [0, 64) consume publish, [64, 104) finalize class counts, [104, 128) finalize split
  // totals, [128, 256) finalize totals (HC / export phases reuse [192, 256)), [256, 264) the
  // device result image's size (pxg_pxrb.hip),
  // [kPinnedOps, kPinnedBytes) standalone Filter / Map per-chunk counts.
  void* pinned = nullptr;
  static constexpr size_t kPinnedOps = 4096, kPinnedBytes = 65536;
  // Finalize: t-digest boundary chains of every mid-class group size (a pure function of the
  // size; pxg_finalize.hip EnsureMidChains), built on first use.
  DevBuf mid_chains;
  // Tile status words of the single-pass look-back scans (pxg_scan.hip), one array per stream
  // (main, side, side 2), zeroed when allocated: a word left by another process in recycled
  // device memory must never carry a live epoch.
  DevBuf scan_status[3];

  hipEvent_t GetEvent();
  int32_t ResolveTimings();
};

// Buffer pool (BufPool): a cached buffer of at least `bytes` (and at most twice that), else a
// new one; Release hands a DevBuf's memory to the pool (b is left empty).
int32_t PoolAlloc(Ctx* ctx, DevBuf& b, size_t bytes);
void PoolRelease(Ctx* ctx, DevBuf& b);
void PoolClear(Ctx* ctx);

// Opt-in host-side stage timing of the library (PXG_TIMING=1): one stderr line per stage.
struct HostClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  static bool On() {
    static const bool on = std::getenv("PXG_TIMING") != nullptr;
    return on;
  }
  void Mark(const char* what) {
    if (!On()) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[pxg] %-28s %9.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};


// Launch helper: optional event bracketing on the launch stream (stats resolved lazily).
template <typename... KArgs, typename... Args>
inline int32_t LaunchOn(Ctx* ctx, hipStream_t stream, const char* name, void (*kernel)(KArgs...), dim3 grid, dim3 block,
                        size_t shmem, Args&&... args) {
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return PXG_OK;
  hipEvent_t s0 = nullptr, s1 = nullptr;
  // profile_only selects the launches whose name starts with it ("agg_consume" also times
  // "agg_consume_prefix", the probe-record prefix launch).
  const bool timed = ctx->profiling && (ctx->profile_only.empty() || std::strncmp(name, ctx->profile_only.c_str(), ctx->profile_only.size()) == 0);
  if (timed) {
    s0 = ctx->GetEvent();
    s1 = ctx->GetEvent();
    (void)hipEventRecord(s0, stream);
  }
  hipLaunchKernelGGL(kernel, grid, block, shmem, stream, std::forward<Args>(args)...);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return SetError(PXG_INTERNAL, "launch %s failed: %s", name, hipGetErrorString(e));
  if (timed) {
    (void)hipEventRecord(s1, stream);
    ctx->pending.push_back(PendingTiming{name, s0, s1});
  }
  return PXG_OK;
}

template <typename... KArgs, typename... Args>
inline int32_t Launch(Ctx* ctx, const char* name, void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t shmem,
                      Args&&... args) {
  return LaunchOn(ctx, ctx->stream, name, kernel, grid, block, shmem, std::forward<Args>(args)...);
}

// Fork the side stream off the main stream / join it back.
inline int32_t ForkSide(Ctx* ctx) {
  if (hipEventRecord(ctx->ev_fork, ctx->stream) != hipSuccess || hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0) != hipSuccess)
    return SetError(PXG_INTERNAL, "side stream fork failed");
  return PXG_OK;
}
inline int32_t JoinSide(Ctx* ctx) {
  if (hipEventRecord(ctx->ev_join, ctx->side) != hipSuccess || hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0) != hipSuccess)
    return SetError(PXG_INTERNAL, "side stream join failed");
  return PXG_OK;
}

inline int32_t ForkSide2(Ctx* ctx) {
  if (hipEventRecord(ctx->ev_fork2, ctx->stream) != hipSuccess || hipStreamWaitEvent(ctx->side2, ctx->ev_fork2, 0) != hipSuccess)
    return SetError(PXG_INTERNAL, "side stream 2 fork failed");
  return PXG_OK;
}
inline int32_t JoinSide2(Ctx* ctx) {
  if (hipEventRecord(ctx->ev_join2, ctx->side2) != hipSuccess || hipStreamWaitEvent(ctx->stream, ctx->ev_join2, 0) != hipSuccess)
    return SetError(PXG_INTERNAL, "side stream 2 join failed");
  return PXG_OK;
}

inline int GridFor(int64_t items, int per_block, int cap) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

// ---------------------------------------------------------------------------------------
// Tables.
// ---------------------------------------------------------------------------------------
struct ChunkCol {
  DevBuf values;   // fixed-width
  DevBuf offsets;  // STRING (int32, nrows_cap + 1)
  DevBuf data;     // STRING payload
  int64_t data_len = 0;
};

struct Chunk {
  int64_t nrows = 0;
  int64_t rows_cap = 0;
  int64_t row_base = 0;
  std::vector<ChunkCol> cols;
  bool sealed = false;
};

int TypeWidth(int type);

struct Table {
  Ctx* ctx = nullptr;
  int32_t ncols = 0;
  std::vector<int32_t> types;
  std::vector<std::unique_ptr<Chunk>> chunks;
  int64_t nrows = 0;
  // Pinned host staging for coalescing small RowBatches.
  struct Stage {
    std::vector<std::vector<uint8_t>> fixed;   // per col
    std::vector<std::vector<int32_t>> offsets; // per col (STRING), starts with 0
    std::vector<std::vector<uint8_t>> data;    // per col (STRING)
    int64_t rows = 0;
    int64_t bytes = 0;
  } stage;
  // Device copy of the chunk descriptors (rebuilt when chunks change).
  DevBuf d_chunks;
  DevBuf d_types;
  int64_t d_chunks_version = -1;
  int64_t version = 0;

  int32_t FlushStage();
  int32_t AppendRows(const pxg_column_view* cols, int64_t nrows, hipMemcpyKind kind);
  int32_t EnsureDeviceDescriptors();
  DevChunk Descriptor(size_t i) const;
};

}  // namespace pxg

struct pxg_table;
namespace pxg {
int32_t NewTable(Ctx* ctx, int32_t ncols, const int32_t* types, pxg_table** out);
// Host buffers of pxg_column_out results (pxg_result_free releases them): large ones are pinned
// pool blocks, reused across results.
void* ResultAlloc(size_t n);
void ResultFree(void* p);
// Device -> host copy on `stream` (stream-ordered): into a block of the pinned result pool (up
// to kCopyKernelMaxBytes) by a copy kernel, otherwise hipMemcpyAsync.
constexpr size_t kCopyKernelMaxBytes = size_t(8) << 20;
int32_t CopyD2H(Ctx* ctx, hipStream_t stream, void* host, const void* dev, size_t n);
// Several small device values (each <= 64 bytes, 4-byte aligned sizes and addresses) into the
// ctx's pinned scratch at byte offsets dst_off, by one kernel launch: a hipMemcpyAsync per value
// cost ~5 us of stream time each (round 6 C2 trace: 9 such copies per step).
struct SmallCopy {
  const void* src;
  uint32_t dst_off;
  uint32_t bytes;
};
constexpr int kMaxSmallCopies = 8;
int32_t ReadbackSmall(Ctx* ctx, hipStream_t stream, const SmallCopy* items, int n);
// Zero up to four device ranges (4-byte aligned, sizes multiples of 4) in one launch.
int32_t ZeroRanges(Ctx* ctx, hipStream_t stream, void* const* ptrs, const size_t* bytes, int n);
}

struct pxg_ctx {
  pxg::Ctx impl;
};
struct pxg_table {
  pxg::Table impl;
};
