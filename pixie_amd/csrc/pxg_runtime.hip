// libpxg runtime: contexts, kernel timing, HBM-resident tables (RowBatch coalescing), fetch.
//
// Table ↔ reference: table_store::Table keeps hot/cold RowBatches per table
// (src/table_store/table/table.h:71-199) and MemorySourceNode hands them to the graph one
// batch at a time (src/carnot/exec/memory_source_node.cc:92-124).  Here a table is the
// HBM-resident image of those batches, coalesced into <= 2^24-row chunks so the operators see
// a few large Arrow-layout arrays instead of thousands of 100-row batches.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "pxg_internal.h"
#include "pxg_scan.h"

namespace pxg {

int TypeWidth(int type) {
  switch (type) {
    case PXG_BOOLEAN: return 1;
    case PXG_UINT128: return 16;
    case PXG_STRING: return 0;
    default: return 8;
  }
}

int32_t PoolAlloc(Ctx* ctx, DevBuf& b, size_t bytes) {
  PoolRelease(ctx, b);
  if (bytes == 0) bytes = 16;
  BufPool& pool = ctx->pool;
  auto it = pool.free.lower_bound(bytes);
  if (it != pool.free.end() && it->first <= 2 * bytes + (size_t(1) << 20)) {
    b.p = it->second;
    b.bytes = it->first;
    pool.cached -= it->first;
    pool.free.erase(it);
    return PXG_OK;
  }
  // New buffers are rounded up (1 MiB granules past 1 MiB) so later requests of similar size reuse them.
  const size_t gran = bytes > (size_t(1) << 20) ? (size_t(1) << 20) : 4096;
  const size_t n = (bytes + gran - 1) / gran * gran;
  hipError_t e = hipMalloc(&b.p, n);
  if (e != hipSuccess) {
    PoolClear(ctx);
    e = hipMalloc(&b.p, n);
  }
  if (e != hipSuccess) {
    b.p = nullptr;
    return SetError(PXG_RESOURCE_UNAVAILABLE, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
  }
  b.bytes = n;
  return PXG_OK;
}

void PoolRelease(Ctx* ctx, DevBuf& b) {
  if (!b.p) return;
  BufPool& pool = ctx->pool;
  pool.free.emplace(b.bytes, b.p);
  pool.cached += b.bytes;
  b.p = nullptr;
  b.bytes = 0;
  while (pool.cached > pool.cap && !pool.free.empty()) {  // evict the largest
    auto last = std::prev(pool.free.end());
    (void)hipFree(last->second);
    pool.cached -= last->first;
    pool.free.erase(last);
  }
}

void PoolClear(Ctx* ctx) {
  for (auto& kv : ctx->pool.free) (void)hipFree(kv.second);
  ctx->pool.free.clear();
  ctx->pool.cached = 0;
}

hipEvent_t Ctx::GetEvent() {
  if (!free_events.empty()) {
    hipEvent_t e = free_events.back();
    free_events.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

int32_t Ctx::ResolveTimings() {
  for (auto& p : pending) {
    hipError_t e = hipEventSynchronize(p.stop);
    if (e != hipSuccess) return SetError(PXG_INTERNAL, "event sync failed: %s", hipGetErrorString(e));
    float ms = 0;
    hipEventElapsedTime(&ms, p.start, p.stop);
    auto& st = stats[p.name];
    st.launches += 1;
    st.total_ms += ms;
    free_events.push_back(p.start);
    free_events.push_back(p.stop);
  }
  pending.clear();
  return PXG_OK;
}

// ---------------------------------------------------------------------------------------
// Tables
// ---------------------------------------------------------------------------------------
__global__ void RebaseOffsetsKernel(int32_t* __restrict__ dst, const int32_t* __restrict__ src, int64_t n, int32_t sub,
                                    int32_t add) {
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i] - sub + add;
}

DevChunk Table::Descriptor(size_t i) const {
  DevChunk d;
  std::memset(&d, 0, sizeof(d));
  const Chunk& c = *chunks[i];
  d.nrows = c.nrows;
  d.row_base = c.row_base;
  for (int k = 0; k < ncols && k < kMaxCols; ++k) {
    d.cols[k].values = c.cols[k].values.as<uint8_t>();
    d.cols[k].offsets = c.cols[k].offsets.as<int32_t>();
    d.cols[k].data = c.cols[k].data.as<uint8_t>();
  }
  return d;
}

int32_t Table::EnsureDeviceDescriptors() {
  PXG_RETURN_IF_ERROR(FlushStage());
  if (d_chunks_version == version) return PXG_OK;
  std::vector<DevChunk> h(std::max<size_t>(chunks.size(), 1));
  for (size_t i = 0; i < chunks.size(); ++i) h[i] = Descriptor(i);
  if (d_chunks.bytes < h.size() * sizeof(DevChunk)) PXG_RETURN_IF_ERROR(PoolAlloc(ctx, d_chunks, h.size() * sizeof(DevChunk) * 2));
  PXG_HIP(hipMemcpyAsync(d_chunks.p, h.data(), h.size() * sizeof(DevChunk), hipMemcpyHostToDevice, ctx->stream));
  if (!d_types.p) {
    std::vector<int32_t> t(kMaxCols, 0);
    for (int k = 0; k < ncols; ++k) t[k] = types[k];
    PXG_RETURN_IF_ERROR(PoolAlloc(ctx, d_types, kMaxCols * sizeof(int32_t)));
    PXG_HIP(hipMemcpyAsync(d_types.p, t.data(), kMaxCols * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  }
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  d_chunks_version = version;
  return PXG_OK;
}

static constexpr int64_t kStageRows = 1 << 20;
static constexpr int64_t kStageBytes = 64 << 20;
static constexpr int64_t kMaxChunkData = (int64_t(1) << 31) - 64;

// One int32 from device memory, ordered after the work already issued on the ctx stream (the
// stream is non-blocking: a plain hipMemcpy on the null stream would not wait for it).
static int32_t ReadDeviceI32(Ctx* ctx, const int32_t* p, int32_t* out) {
  PXG_HIP(hipMemcpyAsync(out, p, 4, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}

// Append rows [0, n) of `cols` (host or device pointers per `kind`) into the table's chunks.
int32_t Table::AppendRows(const pxg_column_view* cols, int64_t n, hipMemcpyKind kind) {
  const bool from_host = (kind == hipMemcpyHostToDevice);
  int64_t done = 0;
  while (done < n) {
    Chunk* ch = chunks.empty() ? nullptr : chunks.back().get();
    if (!ch || ch->sealed || ch->nrows >= kChunkRows) {
      auto c = std::make_unique<Chunk>();
      c->row_base = nrows;
      c->cols.resize(ncols);
      chunks.push_back(std::move(c));
      ch = chunks.back().get();
    }
    int64_t take = std::min<int64_t>(n - done, kChunkRows - ch->nrows);
    // String payload bounds: shrink `take` so every string column stays < 2^31 bytes.
    for (int k = 0; k < ncols; ++k) {
      if (types[k] != PXG_STRING) continue;
      const int32_t* off = cols[k].offsets;
      int32_t o_first, o_last;
      if (from_host) {
        o_first = off[done];
        o_last = off[done + take];
      } else {
        PXG_RETURN_IF_ERROR(ReadDeviceI32(ctx, off + done, &o_first));
        PXG_RETURN_IF_ERROR(ReadDeviceI32(ctx, off + done + take, &o_last));
      }
      int64_t bytes = static_cast<int64_t>(o_last) - o_first;
      while (ch->cols[k].data_len + bytes > kMaxChunkData && take > 1) {
        take /= 2;
        if (from_host) {
          o_last = off[done + take];
        } else {
          PXG_RETURN_IF_ERROR(ReadDeviceI32(ctx, off + done + take, &o_last));
        }
        bytes = static_cast<int64_t>(o_last) - o_first;
      }
      if (ch->cols[k].data_len + bytes > kMaxChunkData) {
        if (ch->nrows == 0) return SetError(PXG_INVALID_ARGUMENT, "single string value exceeds 2^31 bytes");
        ch->sealed = true;
        take = 0;
        break;
      }
    }
    if (take == 0) continue;  // sealed; next iteration opens a new chunk
    const int64_t r0 = ch->nrows, r1 = ch->nrows + take;
    // Chunk capacity in rows: exact on the first append, then doubling up to kChunkRows (a
    // power-of-two byte rounding would waste up to 2x HBM on a full chunk: 1B-row tables).
    const int64_t cap_rows = r0 == 0 ? r1 : std::max<int64_t>(r1, std::min<int64_t>(kChunkRows, 2 * r0));
    for (int k = 0; k < ncols; ++k) {
      ChunkCol& cc = ch->cols[k];
      const int t = types[k];
      if (t != PXG_STRING) {
        const size_t w = TypeWidth(t);
        if (cc.values.bytes < static_cast<size_t>(r1) * w + 16)
          PXG_RETURN_IF_ERROR(cc.values.ReserveExact(static_cast<size_t>(cap_rows) * w + 16, static_cast<size_t>(r0) * w, ctx->stream));
        const uint8_t* src = static_cast<const uint8_t*>(cols[k].values) + static_cast<size_t>(done) * w;
        PXG_HIP(hipMemcpyAsync(cc.values.as<uint8_t>() + static_cast<size_t>(r0) * w, src, static_cast<size_t>(take) * w, kind,
                               ctx->stream));
        continue;
      }
      const int32_t* off = cols[k].offsets;
      int32_t o_first, o_last;
      if (from_host) {
        o_first = off[done];
        o_last = off[done + take];
      } else {
        PXG_RETURN_IF_ERROR(ReadDeviceI32(ctx, off + done, &o_first));
        PXG_RETURN_IF_ERROR(ReadDeviceI32(ctx, off + done + take, &o_last));
      }
      const int64_t bytes = static_cast<int64_t>(o_last) - o_first;
      if (o_first < 0 || bytes < 0)
        return SetError(PXG_INVALID_ARGUMENT, "column %d: string offsets %d (row %lld) .. %d (row %lld) are not monotone", k, o_first,
                        static_cast<long long>(done), o_last, static_cast<long long>(done + take));
      if (cc.offsets.bytes < static_cast<size_t>(r1 + 1) * 4 + 16)
        PXG_RETURN_IF_ERROR(cc.offsets.ReserveExact(static_cast<size_t>(cap_rows + 1) * 4 + 16, static_cast<size_t>(r0 + 1) * 4, ctx->stream));
      const size_t need = static_cast<size_t>(cc.data_len + bytes) + 16;
      if (cc.data.bytes < need) {
        const size_t grow = r0 == 0 ? need : std::max(need, std::min(2 * cc.data.bytes, static_cast<size_t>(kMaxChunkData) + 16));
        PXG_RETURN_IF_ERROR(cc.data.ReserveExact(grow, static_cast<size_t>(cc.data_len), ctx->stream));
      }
      PXG_HIP(hipMemcpyAsync(cc.data.as<uint8_t>() + cc.data_len, cols[k].data + o_first, static_cast<size_t>(bytes), kind, ctx->stream));
      const int32_t add = static_cast<int32_t>(cc.data_len);
      if (from_host) {
        std::vector<int32_t> tmp(static_cast<size_t>(take) + 1);
        for (int64_t i = 0; i <= take; ++i) tmp[i] = off[done + i] - o_first + add;
        PXG_HIP(hipMemcpyAsync(cc.offsets.as<int32_t>() + r0, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        PXG_HIP(hipStreamSynchronize(ctx->stream));  // tmp goes out of scope
      } else {
        PXG_RETURN_IF_ERROR(Launch(ctx, "rebase_offsets", RebaseOffsetsKernel, dim3(GridFor(take + 1, 256, 1 << 30)), dim3(256), 0,
                                   cc.offsets.as<int32_t>() + r0, off + done, take + 1, o_first, add));
      }
      cc.data_len += bytes;
    }
    ch->nrows = r1;
    nrows += take;
    done += take;
    ++version;
  }
  if (!from_host) PXG_HIP(hipStreamSynchronize(ctx->stream));
  else PXG_HIP(hipStreamSynchronize(ctx->stream));
  return PXG_OK;
}

int32_t Table::FlushStage() {
  if (stage.rows == 0) return PXG_OK;
  std::vector<pxg_column_view> v(ncols);
  for (int k = 0; k < ncols; ++k) {
    std::memset(&v[k], 0, sizeof(v[k]));
    v[k].type = types[k];
    v[k].length = stage.rows;
    if (types[k] == PXG_STRING) {
      v[k].offsets = stage.offsets[k].data();
      v[k].data = stage.data[k].data();
    } else {
      v[k].values = stage.fixed[k].data();
    }
  }
  int64_t rows = stage.rows;
  stage.rows = 0;
  stage.bytes = 0;
  int32_t s = AppendRows(v.data(), rows, hipMemcpyHostToDevice);
  for (int k = 0; k < ncols; ++k) {
    stage.fixed[k].clear();
    stage.data[k].clear();
    stage.offsets[k].assign(1, 0);
  }
  return s;
}

}  // namespace pxg

using namespace pxg;

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" int32_t pxg_abi_version(void) { return PXG_ABI_VERSION; }
extern "C" const char* pxg_last_error(void) { return LastErrorRef().c_str(); }

extern "C" int32_t pxg_device_count(int32_t* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return SetError(PXG_RESOURCE_UNAVAILABLE, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = n;
  return PXG_OK;
}

// Side stream 2 carries the finalize's critical chain (the big groups' selection path, which
// waits on the sort and on nothing the other streams produce later): at the highest stream
// priority its kernels take CUs first and the small / mid digests fill in around them.
// PXG_SIDE2_PRIO=0: default priority (A/B).
static hipError_t CreateSide2(hipStream_t* s) {
  const char* e = std::getenv("PXG_SIDE2_PRIO");
  if (e && std::atoi(e) == 0) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

extern "C" int32_t pxg_ctx_create(int32_t device, pxg_ctx** out) {
  if (!out) return SetError(PXG_INVALID_ARGUMENT, "out is null");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return SetError(PXG_RESOURCE_UNAVAILABLE, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= n) return SetError(PXG_INVALID_ARGUMENT, "device %d out of range [0,%d)", device, n);
  auto* c = new pxg_ctx();
  c->impl.device = device;
  e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete c;
    return SetError(PXG_INTERNAL, "hipSetDevice: %s", hipGetErrorString(e));
  }
  e = hipStreamCreateWithFlags(&c->impl.stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return SetError(PXG_INTERNAL, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  if (hipStreamCreateWithFlags(&c->impl.side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_join, hipEventDisableTiming) != hipSuccess ||
      CreateSide2(&c->impl.side2) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_fork2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_join2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_meta, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_chain, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_split, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_early, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->impl.ev_pub, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return SetError(PXG_INTERNAL, "side stream / event creation failed");
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->impl.num_cus = prop.multiProcessorCount;
  if (hipHostMalloc(&c->impl.pinned, Ctx::kPinnedBytes, hipHostMallocDefault) != hipSuccess) {
    delete c;
    return SetError(PXG_RESOURCE_UNAVAILABLE, "pinned host scratch allocation failed");
  }
  *out = c;
  return PXG_OK;
}

extern "C" int32_t pxg_ctx_destroy(pxg_ctx* ctx) {
  if (!ctx) return PXG_OK;
  hipStreamSynchronize(ctx->impl.stream);
  PoolClear(&ctx->impl);
  ctx->impl.ResolveTimings();
  for (auto e : ctx->impl.free_events) hipEventDestroy(e);
  if (ctx->impl.pinned) hipHostFree(ctx->impl.pinned);
  hipStreamSynchronize(ctx->impl.side);
  hipEventDestroy(ctx->impl.ev_fork);
  hipEventDestroy(ctx->impl.ev_join);
  hipStreamDestroy(ctx->impl.side);
  hipStreamSynchronize(ctx->impl.side2);
  hipEventDestroy(ctx->impl.ev_fork2);
  hipEventDestroy(ctx->impl.ev_join2);
  hipEventDestroy(ctx->impl.ev_meta);
  hipEventDestroy(ctx->impl.ev_chain);
  hipEventDestroy(ctx->impl.ev_split);
  hipEventDestroy(ctx->impl.ev_early);
  hipEventDestroy(ctx->impl.ev_pub);
  hipStreamDestroy(ctx->impl.side2);
  hipStreamDestroy(ctx->impl.stream);
  delete ctx;
  return PXG_OK;
}

extern "C" int32_t pxg_ctx_sync(pxg_ctx* ctx) {
  if (!ctx) return SetError(PXG_INVALID_ARGUMENT, "ctx is null");
  PXG_HIP(hipStreamSynchronize(ctx->impl.stream));
  return PXG_OK;
}

extern "C" void* pxg_ctx_stream(pxg_ctx* ctx) { return ctx ? static_cast<void*>(ctx->impl.stream) : nullptr; }

extern "C" int32_t pxg_ctx_set_profiling(pxg_ctx* ctx, int32_t enabled) {
  if (!ctx) return SetError(PXG_INVALID_ARGUMENT, "ctx is null");
  ctx->impl.profiling = enabled != 0;
  return PXG_OK;
}

extern "C" int32_t pxg_ctx_profile_only(pxg_ctx* ctx, const char* kernel_name) {
  if (!ctx) return SetError(PXG_INVALID_ARGUMENT, "ctx is null");
  ctx->impl.profile_only = kernel_name ? kernel_name : "";
  return PXG_OK;
}

extern "C" int32_t pxg_ctx_kernel_stats(pxg_ctx* ctx, const char* name, int64_t* launches, double* total_ms) {
  if (!ctx || !name) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  PXG_RETURN_IF_ERROR(ctx->impl.ResolveTimings());
  if (name[0] == '*' && name[1] == 0) {  // every kernel launched while profiling was on
    int64_t l = 0;
    double ms = 0;
    for (const auto& kv : ctx->impl.stats) {
      l += kv.second.launches;
      ms += kv.second.total_ms;
    }
    if (launches) *launches = l;
    if (total_ms) *total_ms = ms;
    return PXG_OK;
  }
  auto it = ctx->impl.stats.find(name);
  if (launches) *launches = it == ctx->impl.stats.end() ? 0 : it->second.launches;
  if (total_ms) *total_ms = it == ctx->impl.stats.end() ? 0 : it->second.total_ms;
  return PXG_OK;
}

extern "C" int32_t pxg_ctx_reset_stats(pxg_ctx* ctx) {
  if (!ctx) return SetError(PXG_INVALID_ARGUMENT, "ctx is null");
  PXG_RETURN_IF_ERROR(ctx->impl.ResolveTimings());
  ctx->impl.stats.clear();
  return PXG_OK;
}

namespace pxg {
int32_t NewTable(Ctx* ctx, int32_t ncols, const int32_t* types, pxg_table** out) {
  if (!ctx || !out || ncols < 0 || (ncols > 0 && !types)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  if (ncols > kMaxCols) return SetError(PXG_UNIMPLEMENTED, "tables are limited to %d columns", kMaxCols);
  for (int k = 0; k < ncols; ++k)
    if (types[k] < PXG_BOOLEAN || types[k] > PXG_TIME64NS) return SetError(PXG_INVALID_ARGUMENT, "bad column type %d", types[k]);
  auto* t = new pxg_table();
  t->impl.ctx = ctx;
  t->impl.ncols = ncols;
  t->impl.types.assign(types, types + ncols);
  t->impl.stage.fixed.resize(ncols);
  t->impl.stage.data.resize(ncols);
  t->impl.stage.offsets.assign(ncols, std::vector<int32_t>(1, 0));
  *out = t;
  return PXG_OK;
}
}  // namespace pxg

extern "C" int32_t pxg_table_create(pxg_ctx* ctx, int32_t ncols, const int32_t* types, pxg_table** out) {
  if (!ctx) return SetError(PXG_INVALID_ARGUMENT, "ctx is null");
  return NewTable(&ctx->impl, ncols, types, out);
}

extern "C" int32_t pxg_table_destroy(pxg_table* t) {
  if (!t) return PXG_OK;
  // Column buffers go to the ctx pool (no device-wide sync); what is left is freed.
  Ctx* ctx = t->impl.ctx;
  for (auto& ch : t->impl.chunks) {
    for (auto& col : ch->cols) {
      PoolRelease(ctx, col.values);
      PoolRelease(ctx, col.offsets);
      PoolRelease(ctx, col.data);
    }
  }
  PoolRelease(ctx, t->impl.d_chunks);
  PoolRelease(ctx, t->impl.d_types);
  delete t;
  return PXG_OK;
}

static int32_t CheckViews(const Table& t, const pxg_column_view* cols, int64_t nrows) {
  if (nrows < 0) return SetError(PXG_INVALID_ARGUMENT, "negative row count");
  if (nrows > 0 && !cols) return SetError(PXG_INVALID_ARGUMENT, "cols is null");
  for (int k = 0; k < t.ncols && nrows > 0; ++k) {
    // RowBatch::AddColumn checks (src/table_store/schema/row_batch.cc:39-52).
    if (cols[k].type != t.types[k]) return SetError(PXG_INVALID_ARGUMENT, "column %d type %d != schema %d", k, cols[k].type, t.types[k]);
    if (cols[k].length != nrows) return SetError(PXG_INVALID_ARGUMENT, "column %d length %lld != %lld", k, (long long)cols[k].length, (long long)nrows);
    if (t.types[k] == PXG_STRING ? (!cols[k].offsets || !cols[k].data) : !cols[k].values)
      return SetError(PXG_INVALID_ARGUMENT, "column %d missing buffers", k);
  }
  return PXG_OK;
}

extern "C" int32_t pxg_table_append(pxg_table* tp, const pxg_column_view* cols, int64_t nrows) {
  if (!tp) return SetError(PXG_INVALID_ARGUMENT, "table is null");
  Table& t = tp->impl;
  PXG_RETURN_IF_ERROR(CheckViews(t, cols, nrows));
  if (nrows == 0) return PXG_OK;
  if (nrows >= kStageRows / 4) {
    PXG_RETURN_IF_ERROR(t.FlushStage());
    return t.AppendRows(cols, nrows, hipMemcpyHostToDevice);
  }
  // Coalesce into the host staging buffer.
  for (int k = 0; k < t.ncols; ++k) {
    if (t.types[k] == PXG_STRING) {
      auto& off = t.stage.offsets[k];
      auto& dat = t.stage.data[k];
      int32_t base = static_cast<int32_t>(dat.size());
      int32_t o0 = cols[k].offsets[0];
      int64_t bytes = cols[k].offsets[nrows] - o0;
      dat.insert(dat.end(), cols[k].data + o0, cols[k].data + o0 + bytes);
      for (int64_t i = 1; i <= nrows; ++i) off.push_back(cols[k].offsets[i] - o0 + base);
      t.stage.bytes += bytes;
    } else {
      size_t w = TypeWidth(t.types[k]);
      const uint8_t* s = static_cast<const uint8_t*>(cols[k].values);
      t.stage.fixed[k].insert(t.stage.fixed[k].end(), s, s + nrows * w);
      t.stage.bytes += nrows * static_cast<int64_t>(w);
    }
  }
  t.stage.rows += nrows;
  if (t.stage.rows >= kStageRows || t.stage.bytes >= kStageBytes) return t.FlushStage();
  return PXG_OK;
}

extern "C" int32_t pxg_table_append_device(pxg_table* tp, const pxg_column_view* cols, int64_t nrows) {
  if (!tp) return SetError(PXG_INVALID_ARGUMENT, "table is null");
  Table& t = tp->impl;
  PXG_RETURN_IF_ERROR(CheckViews(t, cols, nrows));
  if (nrows == 0) return PXG_OK;
  PXG_RETURN_IF_ERROR(t.FlushStage());
  return t.AppendRows(cols, nrows, hipMemcpyDeviceToDevice);
}

extern "C" int32_t pxg_table_flush(pxg_table* t) {
  if (!t) return SetError(PXG_INVALID_ARGUMENT, "table is null");
  PXG_RETURN_IF_ERROR(t->impl.FlushStage());
  PXG_HIP(hipStreamSynchronize(t->impl.ctx->stream));
  return PXG_OK;
}

extern "C" int64_t pxg_table_num_rows(const pxg_table* t) { return t ? t->impl.nrows + t->impl.stage.rows : 0; }
extern "C" int32_t pxg_table_num_chunks(const pxg_table* t) { return t ? static_cast<int32_t>(t->impl.chunks.size()) : 0; }

extern "C" int64_t pxg_table_device_bytes(const pxg_table* tp, int32_t col) {
  if (!tp || col < 0 || col >= tp->impl.ncols) return -1;
  const Table& t = tp->impl;
  int64_t b = 0;
  for (auto& c : t.chunks) {
    if (t.types[col] == PXG_STRING) b += 4 * c->nrows + c->cols[col].data_len;
    else b += TypeWidth(t.types[col]) * c->nrows;
  }
  return b;
}

// dst[i] = src[i] - sub + add: a chunk's STRING offsets rebased onto the fetched payload.
__global__ void OffsetsRebaseKernel(const int32_t* __restrict__ src, int64_t count, int32_t sub, int64_t add, int32_t* __restrict__ dst) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < count) dst[i] = static_cast<int32_t>(src[i] - sub + add);
}

// Rows [begin, end) of one column into host buffers of the pinned result pool: every copy is an
// async DMA on the ctx stream (a pageable hipMemcpy per chunk ran at ~3 GB/s: C5's 162 MB join
// output took 64 ms), STRING offsets are rebased on the device, and one synchronisation ends it.
static int32_t TableFetch(pxg_table* tp, int32_t col, int64_t begin, int64_t end, pxg_column_out* out) {
  Table& t = tp->impl;
  PXG_RETURN_IF_ERROR(t.FlushStage());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "bad row range");
  std::memset(out, 0, sizeof(*out));
  const int type = t.types[col];
  out->type = type;
  out->length = end - begin;
  const int64_t n = end - begin;
  hipStream_t st = t.ctx->stream;
  struct Piece {
    const Chunk* c;
    int64_t l0, l1, at;  // chunk rows [l0, l1) land at output row `at`
  };
  std::vector<Piece> pieces;
  for (auto& cp : t.chunks) {
    const int64_t lo = std::max(begin, cp->row_base), hi = std::min(end, cp->row_base + cp->nrows);
    if (lo < hi) pieces.push_back({cp.get(), lo - cp->row_base, hi - cp->row_base, lo - begin});
  }
  if (type != PXG_STRING) {
    const size_t w = TypeWidth(type);
    out->values = ResultAlloc(std::max<size_t>(n * w, 1));
    if (!out->values) return SetError(PXG_RESOURCE_UNAVAILABLE, "host result allocation failed");
    for (auto& pc : pieces)
      PXG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(out->values) + pc.at * w, pc.c->cols[col].values.as<uint8_t>() + pc.l0 * w,
                             (pc.l1 - pc.l0) * w, hipMemcpyDeviceToHost, st));
    PXG_HIP(hipStreamSynchronize(st));
    return PXG_OK;
  }
  out->offsets = static_cast<int32_t*>(ResultAlloc((n + 1) * 4));
  if (!out->offsets) return SetError(PXG_RESOURCE_UNAVAILABLE, "host result allocation failed");
  out->offsets[0] = 0;
  // Each piece's first / last offsets (payload range), one synchronisation for all of them.
  std::vector<int32_t> bounds(2 * pieces.size() + 2);
  int32_t* pb = static_cast<int32_t*>(ResultAlloc(bounds.size() * 4));
  if (!pb) return SetError(PXG_RESOURCE_UNAVAILABLE, "host result allocation failed");
  struct PinGuard {
    void* p;
    ~PinGuard() { ResultFree(p); }
  } pg{pb};
  for (size_t i = 0; i < pieces.size(); ++i) {
    const int32_t* off = pieces[i].c->cols[col].offsets.as<const int32_t>();
    PXG_HIP(hipMemcpyAsync(pb + 2 * i, off + pieces[i].l0, 4, hipMemcpyDeviceToHost, st));
    PXG_HIP(hipMemcpyAsync(pb + 2 * i + 1, off + pieces[i].l1, 4, hipMemcpyDeviceToHost, st));
  }
  PXG_HIP(hipStreamSynchronize(st));
  int64_t total = 0;
  std::vector<int64_t> base(pieces.size());
  for (size_t i = 0; i < pieces.size(); ++i) {
    base[i] = total;
    total += pb[2 * i + 1] - pb[2 * i];
  }
  if (total >= (int64_t(1) << 31)) return SetError(PXG_UNIMPLEMENTED, "fetched STRING payload exceeds 2 GiB");
  out->data = static_cast<uint8_t*>(ResultAlloc(static_cast<size_t>(total) + 16));
  if (!out->data) return SetError(PXG_RESOURCE_UNAVAILABLE, "host result allocation failed");
  out->data_len = total;
  DevBuf reb;
  if (n > 0) PXG_RETURN_IF_ERROR(reb.Alloc(static_cast<size_t>(n + 1) * 4));
  for (size_t i = 0; i < pieces.size(); ++i) {
    const Piece& pc = pieces[i];
    const int64_t cnt = pc.l1 - pc.l0;  // offsets l0+1 .. l1 land at rows at+1 .. at+cnt
    PXG_RETURN_IF_ERROR(Launch(t.ctx, "offsets_rebase", OffsetsRebaseKernel, dim3(GridFor(cnt, 256, 1 << 30)), dim3(256), 0,
                               pc.c->cols[col].offsets.as<const int32_t>() + pc.l0 + 1, cnt, pb[2 * i], base[i],
                               reb.as<int32_t>() + pc.at + 1));
    if (pb[2 * i + 1] > pb[2 * i])
      PXG_HIP(hipMemcpyAsync(out->data + base[i], pc.c->cols[col].data.as<uint8_t>() + pb[2 * i], pb[2 * i + 1] - pb[2 * i],
                             hipMemcpyDeviceToHost, st));
  }
  if (n > 0) PXG_HIP(hipMemcpyAsync(out->offsets + 1, reb.as<int32_t>() + 1, static_cast<size_t>(n) * 4, hipMemcpyDeviceToHost, st));
  PXG_HIP(hipStreamSynchronize(st));
  return PXG_OK;
}

extern "C" int32_t pxg_table_fetch(pxg_table* tp, int32_t col, int64_t begin, int64_t end, pxg_column_out* out) {
  if (!tp || !out || col < 0 || col >= tp->impl.ncols) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  const int32_t rc = TableFetch(tp, col, begin, end, out);
  if (rc != PXG_OK) {
    (void)hipStreamSynchronize(tp->impl.ctx->stream);  // no copy may still target the buffers
    pxg_result_free(out, 1);
  }
  return rc;
}

// First row whose value in a non-decreasing INT64 / TIME64NS column is >= value (strict = 0) or
// > value (strict = 1): one thread, a binary search over the chunks by row_base, then over the
// rows of the chunk (~log2(rows) dependent loads).
__global__ void TimeBoundKernel(const DevChunk* __restrict__ chunks, int nchunks, int col, int64_t value, int strict,
                                int64_t nrows, int64_t* __restrict__ out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t lo = 0, hi = nrows;
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    int cl = 0, ch = nchunks - 1;
    while (cl < ch) {
      const int cm = (cl + ch + 1) / 2;
      if (chunks[cm].row_base <= mid) cl = cm;
      else ch = cm - 1;
    }
    const DevChunk& c = chunks[cl];
    const int64_t v = reinterpret_cast<const int64_t*>(c.cols[col].values)[mid - c.row_base];
    if (strict ? v > value : v >= value) hi = mid;
    else lo = mid + 1;
  }
  *out = lo;
}

extern "C" int32_t pxg_table_time_bound(pxg_table* tp, int32_t col, int64_t value, int32_t strict, int64_t* row) {
  if (!tp || !row || col < 0 || col >= tp->impl.ncols) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Table& t = tp->impl;
  if (t.types[col] != PXG_INT64 && t.types[col] != PXG_TIME64NS) return SetError(PXG_INVALID_ARGUMENT, "time bound needs an INT64/TIME64NS column");
  PXG_RETURN_IF_ERROR(t.FlushStage());
  *row = 0;
  if (t.nrows == 0) return PXG_OK;
  PXG_RETURN_IF_ERROR(t.EnsureDeviceDescriptors());
  DevBuf res;
  PXG_RETURN_IF_ERROR(res.Alloc(16));
  PXG_RETURN_IF_ERROR(Launch(t.ctx, "table_time_bound", TimeBoundKernel, dim3(1), dim3(64), 0, t.d_chunks.as<const DevChunk>(),
                             static_cast<int>(t.chunks.size()), col, value, strict ? 1 : 0, t.nrows, res.as<int64_t>()));
  PXG_HIP(hipMemcpyAsync(row, res.p, 8, hipMemcpyDeviceToHost, t.ctx->stream));
  PXG_HIP(hipStreamSynchronize(t.ctx->stream));
  return PXG_OK;
}

namespace pxg {
// Host buffers of large results come from a pool of pinned blocks (power-of-two classes), so a
// result copy is a DMA into memory that is already resident: no page faults on fresh pages and
// no bounce through the runtime's staging buffers.  pxg_result_free hands them back.
namespace {
constexpr size_t kPinnedMinBytes = size_t(1) << 16;
constexpr size_t kPinnedKeepBytes = size_t(1) << 32;  // retained free blocks (a C5 query cycles ~1 GB of them)
std::mutex g_pin_mu;
std::map<void*, size_t> g_pin_live;                      // block -> class bytes
std::map<size_t, std::vector<void*>> g_pin_free;
size_t g_pin_kept = 0;
}  // namespace

void* ResultAlloc(size_t n) {
  if (n < kPinnedMinBytes) return std::malloc(std::max<size_t>(n, 1));
  size_t c = kPinnedMinBytes;
  while (c < n) c <<= 1;
  std::lock_guard<std::mutex> lock(g_pin_mu);
  auto& fl = g_pin_free[c];
  void* p = nullptr;
  if (!fl.empty()) {
    p = fl.back();
    fl.pop_back();
    g_pin_kept -= c;
  } else {
    HostClock clk;
    if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) return std::malloc(n);
    if (HostClock::On()) {
      char what[64];
      std::snprintf(what, sizeof(what), "pinned alloc %zu KiB", c >> 10);
      clk.Mark(what);
    }
  }
  g_pin_live[p] = c;
  return p;
}

// Is [p, p + n) inside one live block of the pinned pool?
static bool PinnedPoolHolds(const void* p, size_t n) {
  std::lock_guard<std::mutex> lock(g_pin_mu);
  auto it = g_pin_live.upper_bound(const_cast<void*>(p));
  if (it == g_pin_live.begin()) return false;
  --it;
  const uint8_t* b = static_cast<const uint8_t*>(it->first);
  const uint8_t* q = static_cast<const uint8_t*>(p);
  return q >= b && q + n <= b + it->second;
}

// Device -> pinned-pool host copy by a kernel storing into the mapped host block (16-byte vector
// stores, then the byte tail).
__global__ void CopyToHostKernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, size_t n) {
  const size_t tid = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const bool aligned = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
  size_t done = 0;
  if (aligned) {
    const size_t n16 = n >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (size_t i = tid; i < n16; i += stride) d4[i] = s4[i];
    done = n16 << 4;
  }
  for (size_t i = done + tid; i < n; i += stride) dst[i] = src[i];
}

int32_t CopyD2H(Ctx* ctx, hipStream_t stream, void* host, const void* dev, size_t n) {
  if (n == 0) return PXG_OK;
  // Result-sized copies into the pinned pool go by kernel: a hipMemcpyAsync into a recycled pool
  // block was measured to block the issuing thread for ~7-10 ms once (the second query of an
  // engine), a kernel launch never blocks it.  Large copies keep the DMA engines.
  if (n <= kCopyKernelMaxBytes && PinnedPoolHolds(host, n)) {
    const int grid = static_cast<int>(std::min<size_t>(1024, std::max<size_t>(1, (n + 16 * 256 - 1) / (16 * 256))));
    return LaunchOn(ctx, stream, "copy_to_host", CopyToHostKernel, dim3(grid), dim3(256), 0, static_cast<uint8_t*>(host),
                    static_cast<const uint8_t*>(dev), n);
  }
  PXG_HIP(hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, stream));
  return PXG_OK;
}

struct SmallCopies {
  const uint32_t* src[kMaxSmallCopies];
  uint32_t dst_off[kMaxSmallCopies];
  uint32_t words[kMaxSmallCopies];
  int n;
};
// Thread t: item t / 16, word t % 16 (64 bytes per item at most).
__global__ void __launch_bounds__(128) SmallReadbackKernel(SmallCopies c, uint8_t* __restrict__ host) {
  const int i = threadIdx.x >> 4, w = threadIdx.x & 15;
  if (i < c.n && static_cast<uint32_t>(w) < c.words[i]) reinterpret_cast<uint32_t*>(host + c.dst_off[i])[w] = c.src[i][w];
}

int32_t ReadbackSmall(Ctx* ctx, hipStream_t stream, const SmallCopy* items, int n) {
  if (n <= 0) return PXG_OK;
  if (n > kMaxSmallCopies) return SetError(PXG_INTERNAL, "%d small copies in one readback", n);
  SmallCopies c;
  std::memset(&c, 0, sizeof(c));
  c.n = n;
  for (int i = 0; i < n; ++i) {
    if (items[i].bytes > 64 || (items[i].bytes & 3) || (items[i].dst_off & 3) || (reinterpret_cast<uintptr_t>(items[i].src) & 3) ||
        items[i].dst_off + items[i].bytes > Ctx::kPinnedBytes)
      return SetError(PXG_INTERNAL, "small readback item %d: %u bytes at %u", i, items[i].bytes, items[i].dst_off);
    c.src[i] = static_cast<const uint32_t*>(items[i].src);
    c.dst_off[i] = items[i].dst_off;
    c.words[i] = items[i].bytes / 4;
  }
  return LaunchOn(ctx, stream, "copy_to_host", SmallReadbackKernel, dim3(1), dim3(128), 0, c, static_cast<uint8_t*>(ctx->pinned));
}

struct ZeroSpec {
  uint4* p[4];
  uint64_t n16[4];  // 16-byte units
  uint32_t* tail[4];
  uint32_t tail_words[4];
  int n;
};
__global__ void __launch_bounds__(256) ZeroRangesKernel(ZeroSpec z) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint4 zero = make_uint4(0, 0, 0, 0);
  for (int r = 0; r < z.n; ++r) {
    for (uint64_t i = tid; i < z.n16[r]; i += stride) z.p[r][i] = zero;
    if (tid < z.tail_words[r]) z.tail[r][tid] = 0;
  }
}

int32_t ZeroRanges(Ctx* ctx, hipStream_t stream, void* const* ptrs, const size_t* bytes, int n) {
  if (n <= 0) return PXG_OK;
  if (n > 4) return SetError(PXG_INTERNAL, "%d zero ranges in one launch", n);
  ZeroSpec z;
  std::memset(&z, 0, sizeof(z));
  z.n = n;
  uint64_t most = 1;
  for (int r = 0; r < n; ++r) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptrs[r]);
    if ((a & 3) || (bytes[r] & 3)) return SetError(PXG_INTERNAL, "zero range %d not 4-byte aligned", r);
    // 16-byte body from the first 16-byte boundary; the 4-byte words before it and after it as tail.
    const uintptr_t b16 = (a + 15) & ~uintptr_t(15);
    const size_t head = std::min<size_t>(bytes[r], b16 - a);
    const size_t body = ((bytes[r] - head) / 16) * 16;
    z.p[r] = reinterpret_cast<uint4*>(b16);
    z.n16[r] = body / 16;
    // head and trailing words: at most 3 + 3 words, written as one tail list would need two
    // ranges; instead a range with an unaligned head is zeroed word by word entirely.
    if (head != 0) {
      z.n16[r] = 0;
      z.tail[r] = reinterpret_cast<uint32_t*>(a);
      z.tail_words[r] = static_cast<uint32_t>(bytes[r] / 4);
      if (bytes[r] / 4 > 256u * 1024u) return SetError(PXG_INTERNAL, "unaligned zero range of %zu bytes", bytes[r]);
    } else {
      z.tail[r] = reinterpret_cast<uint32_t*>(b16 + body);
      z.tail_words[r] = static_cast<uint32_t>((bytes[r] - body) / 4);
    }
    most = std::max<uint64_t>(most, std::max<uint64_t>(z.n16[r], z.tail_words[r]));
  }
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(2048, (most + 255) / 256));
  return LaunchOn(ctx, stream, "zero_ranges", ZeroRangesKernel, dim3(std::max(1u, grid)), dim3(256), 0, z);
}

void ResultFree(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lock(g_pin_mu);
    auto it = g_pin_live.find(p);
    if (it != g_pin_live.end()) {
      const size_t c = it->second;
      g_pin_live.erase(it);
      if (g_pin_kept + c <= kPinnedKeepBytes) {
        g_pin_free[c].push_back(p);
        g_pin_kept += c;
      } else {
        (void)hipHostFree(p);
      }
      return;
    }
  }
  std::free(p);
}
}  // namespace pxg

extern "C" void* pxg_host_alloc(int64_t bytes) { return pxg::ResultAlloc(bytes > 0 ? static_cast<size_t>(bytes) : 1); }
extern "C" void pxg_host_free(void* p) { pxg::ResultFree(p); }

extern "C" void pxg_result_free(pxg_column_out* cols, int32_t n) {
  if (!cols) return;
  for (int32_t i = 0; i < n; ++i) {
    pxg::ResultFree(cols[i].values);
    pxg::ResultFree(cols[i].offsets);
    pxg::ResultFree(cols[i].data);
    cols[i].values = nullptr;
    cols[i].offsets = nullptr;
    cols[i].data = nullptr;
  }
}
