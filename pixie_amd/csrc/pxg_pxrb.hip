// Device-side result serialisation: rows of a device table cut into row batches and written in
// the engine's PXRB batch layout (pixie_amd/host/carnot_host.cc WriteBatch; parsed by
// tests/oracle_client.py::parse_pxrb) as one image in HBM, then moved to the caller's host
// buffer with one DMA.
//
// Reference: MemorySinkNode::ConsumeNextImpl (src/carnot/exec/memory_sink_node.cc:75-80) keeps
// every RowBatch it receives; an equijoin's output reaches it as rows_per_batch batches
// (equijoin_node.cc:153-477).  The host path fetched each output column, sliced it into those
// batches and copied every slice into the result buffer (C5: 195 MB, 2634 batches: a column
// fetch, 2634 batch objects and a 16-thread host copy).  Here the slices are laid out on the
// device, so the only host-bound traffic is the DMA of the finished image.
//
// Batch layout (little endian): int64 rows, u8 eow, u8 eos, u16 0, u32 ncols; per column: int32
// type, then BOOLEAN 1 B / row, UINT128 16 B / row, STRING int32 offsets (rows + 1, relative to
// the batch's first) and the payload bytes, otherwise 8 B / row.
#include "pxg_internal.h"
#include "pxg_scan.h"

#include <algorithm>
#include <vector>

namespace pxg {
namespace {

constexpr int kPxrbHeader = 16;

struct PxrbTypes {
  int32_t n;
  int32_t t[kMaxCols];
};

__device__ __forceinline__ uint64_t ColBytes(const DevCol& c, int type, int64_t r0, int64_t n) {
  switch (type) {
    case PXG_BOOLEAN: return static_cast<uint64_t>(n);
    case PXG_UINT128: return 16ull * n;
    case PXG_STRING: return 4ull * (n + 1) + static_cast<uint64_t>(n ? c.offsets[r0 + n] - c.offsets[r0] : 0);
    default: return 8ull * n;
  }
}

// sizes[b] = bytes of batch b (rows [starts[b], starts[b+1]) of the chunk).
__global__ void PxrbSizesKernel(DevChunk ch, PxrbTypes ty, const int64_t* __restrict__ starts, int64_t nb, uint64_t* __restrict__ sizes) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const int64_t r0 = starts[b] - ch.row_base, n = starts[b + 1] - starts[b];
  uint64_t s = kPxrbHeader;
  for (int c = 0; c < ty.n; ++c) s += 4 + ColBytes(ch.cols[c], ty.t[c], r0, n);
  sizes[b] = s;
}

__device__ __forceinline__ void PutLE(uint8_t* dst, uint64_t v, int bytes, int lane) {
  if (lane < bytes) dst[lane] = static_cast<uint8_t>(v >> (8 * lane));
}

// One workgroup per (batch, column): the column's type word and data at its place in the
// batch (the places of the columns before it are recomputed: <= 16 columns).  Column 0's
// workgroup writes the batch header.  Byte-granular stores: a batch's fields start at arbitrary
// byte offsets, and consecutive lanes still write consecutive bytes.
__global__ void __launch_bounds__(256) PxrbWriteKernel(DevChunk ch, PxrbTypes ty, const int64_t* __restrict__ starts, int64_t nb,
                                                       const uint64_t* __restrict__ boff, int last_eow, int last_eos,
                                                       uint8_t* __restrict__ img) {
  const int64_t b = blockIdx.x / ty.n;
  const int c = static_cast<int>(blockIdx.x % ty.n);
  if (b >= nb) return;
  const int t = threadIdx.x;
  const int64_t r0 = starts[b] - ch.row_base, n = starts[b + 1] - starts[b];
  uint8_t* base = img + boff[b];
  if (c == 0) {
    const bool last = b == nb - 1;
    PutLE(base, static_cast<uint64_t>(n), 8, t);
    if (t == 8) base[8] = last && last_eow ? 1 : 0;
    if (t == 9) base[9] = last && last_eos ? 1 : 0;
    if (t == 10 || t == 11) base[t] = 0;
    if (t >= 12 && t < 16) base[t] = static_cast<uint8_t>(static_cast<uint32_t>(ty.n) >> (8 * (t - 12)));
  }
  uint64_t pos = kPxrbHeader;
  for (int k = 0; k < c; ++k) pos += 4 + ColBytes(ch.cols[k], ty.t[k], r0, n);
  uint8_t* dst = base + pos;
  const int type = ty.t[c];
  PutLE(dst, static_cast<uint32_t>(type), 4, t);
  dst += 4;
  const DevCol& col = ch.cols[c];
  if (type == PXG_STRING) {
    const int32_t* off = col.offsets + r0;
    const int32_t o0 = off[0];
    for (int64_t i = t; i <= n; i += blockDim.x) {
      const uint32_t v = static_cast<uint32_t>(off[i] - o0);
      uint8_t* d = dst + 4 * i;
      d[0] = static_cast<uint8_t>(v);
      d[1] = static_cast<uint8_t>(v >> 8);
      d[2] = static_cast<uint8_t>(v >> 16);
      d[3] = static_cast<uint8_t>(v >> 24);
    }
    if (n == 0) return;
    const uint8_t* src = col.data + o0;
    const int64_t len = off[n] - o0;
    dst += 4 * (n + 1);
    for (int64_t j = t; j < len; j += blockDim.x) dst[j] = src[j];
    return;
  }
  const int w = type == PXG_BOOLEAN ? 1 : type == PXG_UINT128 ? 16 : 8;
  const uint8_t* src = col.values + r0 * w;
  const int64_t len = n * w;
  for (int64_t j = t; j < len; j += blockDim.x) dst[j] = src[j];
}

}  // namespace
}  // namespace pxg

using namespace pxg;

struct pxg_pxrb {
  Ctx* ctx = nullptr;
  DevBuf img;
  int64_t bytes = 0;
};

extern "C" int32_t pxg_table_pxrb_image(pxg_table* tp, const int64_t* starts, int64_t n_batches, int32_t last_eow, int32_t last_eos,
                                        pxg_pxrb** out, int64_t* bytes) {
  if (!tp || !out || !bytes || n_batches <= 0 || !starts) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  *out = nullptr;
  *bytes = 0;
  Table& t = tp->impl;
  PXG_RETURN_IF_ERROR(t.FlushStage());
  for (int64_t b = 0; b < n_batches; ++b)
    if (starts[b] > starts[b + 1] || starts[b] < 0) return SetError(PXG_INVALID_ARGUMENT, "batch starts must be non-decreasing");
  if (starts[n_batches] > t.nrows) return SetError(PXG_INVALID_ARGUMENT, "batch rows past the table's %lld rows", (long long)t.nrows);
  // Every batch inside one chunk: the image path takes single-chunk tables (<= 2^24 rows);
  // callers fall back to fetching the columns otherwise.
  if (t.chunks.size() != 1) return SetError(PXG_UNIMPLEMENTED, "device result image of a %zu-chunk table", t.chunks.size());
  if (t.ncols > kMaxCols) return SetError(PXG_UNIMPLEMENTED, "device result image of %d columns", t.ncols);
  Ctx* ctx = t.ctx;
  PxrbTypes ty;
  ty.n = t.ncols;
  for (int c = 0; c < t.ncols; ++c) ty.t[c] = t.types[c];
  const DevChunk ch = t.Descriptor(0);
  DevBuf d_starts, sizes, scan;
  PXG_RETURN_IF_ERROR(d_starts.Alloc(static_cast<size_t>(n_batches + 1) * 8));
  PXG_RETURN_IF_ERROR(sizes.Alloc(static_cast<size_t>(n_batches + 1) * 8));
  PXG_RETURN_IF_ERROR(scan.Alloc(ScanScratchBytes(n_batches) + 64));
  PXG_HIP(hipMemcpyAsync(d_starts.p, starts, static_cast<size_t>(n_batches + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  PXG_RETURN_IF_ERROR(Launch(ctx, "pxrb_sizes", PxrbSizesKernel, dim3(GridFor(n_batches, 256, 1 << 30)), dim3(256), 0, ch, ty,
                             d_starts.as<const int64_t>(), n_batches, sizes.as<uint64_t>()));
  uint64_t* boff = sizes.as<uint64_t>();
  PXG_RETURN_IF_ERROR(ScanExclusiveU64(ctx, boff, boff, n_batches, boff + n_batches, scan.p));
  uint64_t* pin = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(ctx->pinned) + 256);
  PXG_HIP(hipMemcpyAsync(pin, boff + n_batches, 8, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  const uint64_t total = *pin;
  auto* img = new pxg_pxrb();
  img->ctx = ctx;
  img->bytes = static_cast<int64_t>(total);
  const int32_t rc = PoolAlloc(ctx, img->img, total + 16);
  if (rc != PXG_OK) {
    delete img;
    return rc;
  }
  const int64_t blocks = n_batches * t.ncols;
  if (blocks >= (int64_t(1) << 31)) {
    PoolRelease(ctx, img->img);
    delete img;
    return SetError(PXG_UNIMPLEMENTED, "device result image of %lld batch columns", (long long)blocks);
  }
  const int32_t lrc = Launch(ctx, "pxrb_write", PxrbWriteKernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, ch, ty,
                             d_starts.as<const int64_t>(), n_batches, static_cast<const uint64_t*>(boff), last_eow ? 1 : 0,
                             last_eos ? 1 : 0, img->img.as<uint8_t>());
  // The scratch buffers are freed below: the launch must have finished with them.
  const hipError_t se = hipStreamSynchronize(ctx->stream);
  if (lrc != PXG_OK || se != hipSuccess) {
    PoolRelease(ctx, img->img);
    delete img;
    return lrc != PXG_OK ? lrc : SetError(PXG_INTERNAL, "pxrb image: %s", hipGetErrorString(se));
  }
  *out = img;
  *bytes = img->bytes;
  return PXG_OK;
}

extern "C" int32_t pxg_pxrb_copy(pxg_pxrb* img, void* dst) {
  if (!img || (!dst && img->bytes > 0)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  if (img->bytes == 0) return PXG_OK;
  PXG_HIP(hipMemcpyAsync(dst, img->img.p, static_cast<size_t>(img->bytes), hipMemcpyDeviceToHost, img->ctx->stream));
  PXG_HIP(hipStreamSynchronize(img->ctx->stream));
  return PXG_OK;
}

extern "C" int32_t pxg_pxrb_destroy(pxg_pxrb* img) {
  if (!img) return PXG_OK;
  PoolRelease(img->ctx, img->img);
  delete img;
  return PXG_OK;
}
