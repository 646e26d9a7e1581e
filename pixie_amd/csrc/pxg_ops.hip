// Standalone FilterNode / MapNode over device tables (operator shapes the fused agg path
// does not cover).  FilterNode::ConsumeNextImpl (filter_node.cc:132-171): evaluate the
// predicate, then compact every selected column preserving row order (filter_node.cc:88-92).
// MapNode::ConsumeNextImpl (map_node.cc:64-71): one output column per expression; column
// references are passed through.
#include <algorithm>

#include "pxg_internal.h"
#include "pxg_program.h"
#include "pxg_scan.h"

namespace pxg {

struct ProgBuf {
  DevBuf prog;
  DevBuf pool;
  DevBuf types;
};

static int32_t UploadProgram(Ctx* ctx, const pxg_program& p, const Table& t, ProgBuf* pb) {
  DevProgram dp;
  std::vector<uint8_t> pool;
  size_t off = 0;
  PXG_RETURN_IF_ERROR(CompileProgram(p, t.types.data(), t.ncols, &dp, &pool, &off));
  PXG_RETURN_IF_ERROR(pb->pool.Alloc(pool.size() + 16));
  if (!pool.empty()) PXG_HIP(hipMemcpy(pb->pool.p, pool.data(), pool.size(), hipMemcpyHostToDevice));
  dp.pool = pb->pool.as<uint8_t>() + off;
  PXG_RETURN_IF_ERROR(pb->prog.Alloc(sizeof(DevProgram)));
  PXG_HIP(hipMemcpy(pb->prog.p, &dp, sizeof(DevProgram), hipMemcpyHostToDevice));
  std::vector<int32_t> ty(kMaxCols, 0);
  for (int k = 0; k < t.ncols; ++k) ty[k] = t.types[k];
  PXG_RETURN_IF_ERROR(pb->types.Alloc(kMaxCols * 4));
  PXG_HIP(hipMemcpy(pb->types.p, ty.data(), kMaxCols * 4, hipMemcpyHostToDevice));
  (void)ctx;
  return PXG_OK;
}

__global__ void FilterFlagsKernel(const DevProgram* __restrict__ prog, const DevChunk* __restrict__ chunks, int chunk,
                                  const int32_t* __restrict__ types, int64_t lo, int64_t n, uint32_t* __restrict__ flags) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = EvalProgram(prog, chunks[chunk], lo + i, types).a != 0 ? 1u : 0u;
}

__global__ void FilterGatherFixedKernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int width,
                                        const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos, int64_t lo, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n || !flags[i]) return;
  const uint8_t* s = src + (lo + i) * width;
  uint8_t* d = dst + static_cast<int64_t>(pos[i]) * width;
  if (width == 8) *reinterpret_cast<uint64_t*>(d) = *reinterpret_cast<const uint64_t*>(s);
  else if (width == 16) { reinterpret_cast<uint64_t*>(d)[0] = reinterpret_cast<const uint64_t*>(s)[0]; reinterpret_cast<uint64_t*>(d)[1] = reinterpret_cast<const uint64_t*>(s)[1]; }
  else for (int b = 0; b < width; ++b) d[b] = s[b];
}

__global__ void FilterStrLenKernel(const int32_t* __restrict__ off, const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos,
                                   int64_t lo, int64_t n, uint32_t* __restrict__ lens, uint32_t* __restrict__ src_row) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n || !flags[i]) return;
  lens[pos[i]] = static_cast<uint32_t>(off[lo + i + 1] - off[lo + i]);
  src_row[pos[i]] = static_cast<uint32_t>(lo + i);
}

__global__ void StrCopyKernel(const int32_t* __restrict__ soff, const uint8_t* __restrict__ sdata, const uint32_t* __restrict__ src_row,
                              const uint32_t* __restrict__ doff, uint8_t* __restrict__ ddata, int64_t m) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t r = src_row[i];
  const int32_t a = soff[r], b = soff[r + 1];
  uint8_t* d = ddata + doff[i];
  for (int32_t k = a; k < b; ++k) d[k - a] = sdata[k];
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

static int32_t NewOutTable(Ctx* ctx, const std::vector<int32_t>& types, pxg_table** out) {
  return NewTable(ctx, static_cast<int32_t>(types.size()), types.data(), out);
}

}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_filter(pxg_table* inp, const pxg_program* pred, int32_t n_select, const int32_t* select, int64_t begin,
                              int64_t end, pxg_table** out) {
  if (!inp || !pred || !out || n_select < 0 || (n_select > 0 && !select)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Table& t = inp->impl;
  Ctx* ctx = t.ctx;
  PXG_RETURN_IF_ERROR(t.EnsureDeviceDescriptors());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "bad row range");
  if (pred->result_type != PXG_BOOLEAN) return SetError(PXG_INVALID_ARGUMENT, "Predicate expression must be a boolean");
  std::vector<int32_t> otypes;
  for (int i = 0; i < n_select; ++i) {
    if (select[i] < 0 || select[i] >= t.ncols) return SetError(PXG_INVALID_ARGUMENT, "selected column %d out of range", select[i]);
    otypes.push_back(t.types[select[i]]);
  }
  ProgBuf pb;
  PXG_RETURN_IF_ERROR(UploadProgram(ctx, *pred, t, &pb));
  pxg_table* ot = nullptr;
  PXG_RETURN_IF_ERROR(NewOutTable(ctx, otypes, &ot));
  std::unique_ptr<pxg_table, int32_t (*)(pxg_table*)> guard(ot, pxg_table_destroy);
  Table& o = ot->impl;
  for (size_t c = 0; c < t.chunks.size(); ++c) {
    const Chunk& ch = *t.chunks[c];
    const int64_t lo = std::max(begin, ch.row_base) - ch.row_base;
    const int64_t hi = std::min(end, ch.row_base + ch.nrows) - ch.row_base;
    if (lo >= hi) continue;
    const int64_t n = hi - lo;
    DevBuf flags, pos, scratch, total;
    PXG_RETURN_IF_ERROR(flags.Alloc(n * 4));
    PXG_RETURN_IF_ERROR(pos.Alloc(n * 4));
    PXG_RETURN_IF_ERROR(scratch.Alloc(ScanScratchBytes(n) + 64));
    PXG_RETURN_IF_ERROR(total.Alloc(16));
    PXG_RETURN_IF_ERROR(Launch(ctx, "filter_flags", FilterFlagsKernel, dim3(GridFor(n, 256, 1 << 30)), dim3(256), 0,
                               pb.prog.as<const DevProgram>(), t.d_chunks.as<const DevChunk>(), static_cast<int>(c), pb.types.as<const int32_t>(),
                               lo, n, flags.as<uint32_t>()));
    PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, flags.as<const uint32_t>(), pos.as<uint32_t>(), n, total.as<uint32_t>(), scratch.p));
    uint32_t m = 0;
    PXG_HIP(hipMemcpyAsync(&m, total.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    auto oc = std::make_unique<Chunk>();
    oc->row_base = o.nrows;
    oc->nrows = m;
    oc->rows_cap = m;
    oc->sealed = true;
    oc->cols.resize(n_select);
    for (int s = 0; s < n_select; ++s) {
      const int ci = select[s];
      const int ty = t.types[ci];
      ChunkCol& dc = oc->cols[s];
      if (ty != PXG_STRING) {
        const int w = TypeWidth(ty);
        PXG_RETURN_IF_ERROR(dc.values.Alloc(static_cast<size_t>(m) * w + 16));
        PXG_RETURN_IF_ERROR(Launch(ctx, "filter_gather", FilterGatherFixedKernel, dim3(GridFor(n, 256, 1 << 30)), dim3(256), 0,
                                   ch.cols[ci].values.as<const uint8_t>(), dc.values.as<uint8_t>(), w, flags.as<const uint32_t>(),
                                   pos.as<const uint32_t>(), lo, n));
      } else {
        DevBuf src_row;
        PXG_RETURN_IF_ERROR(dc.offsets.Alloc((static_cast<size_t>(m) + 1) * 4 + 16));
        PXG_RETURN_IF_ERROR(src_row.Alloc(static_cast<size_t>(m) * 4 + 16));
        PXG_RETURN_IF_ERROR(Launch(ctx, "filter_strlen", FilterStrLenKernel, dim3(GridFor(n, 256, 1 << 30)), dim3(256), 0,
                                   ch.cols[ci].offsets.as<const int32_t>(), flags.as<const uint32_t>(), pos.as<const uint32_t>(), lo, n,
                                   dc.offsets.as<uint32_t>(), src_row.as<uint32_t>()));
        DevBuf sc2;
        PXG_RETURN_IF_ERROR(sc2.Alloc(ScanScratchBytes(m) + 64));
        uint32_t* doff = dc.offsets.as<uint32_t>();
        PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, doff, doff, m, doff + m, sc2.p));
        uint32_t bytes = 0;
        PXG_HIP(hipMemcpyAsync(&bytes, doff + m, 4, hipMemcpyDeviceToHost, ctx->stream));
        PXG_HIP(hipStreamSynchronize(ctx->stream));
        PXG_RETURN_IF_ERROR(dc.data.Alloc(static_cast<size_t>(bytes) + 16));
        dc.data_len = bytes;
        PXG_RETURN_IF_ERROR(Launch(ctx, "str_copy", StrCopyKernel, dim3(GridFor(m, 256, 1 << 30)), dim3(256), 0,
                                   ch.cols[ci].offsets.as<const int32_t>(), ch.cols[ci].data.as<const uint8_t>(), src_row.as<const uint32_t>(),
                                   static_cast<const uint32_t*>(doff), dc.data.as<uint8_t>(), static_cast<int64_t>(m)));
        PXG_HIP(hipStreamSynchronize(ctx->stream));
      }
    }
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    o.nrows += m;
    o.chunks.push_back(std::move(oc));
    ++o.version;
  }
  *out = guard.release();
  return PXG_OK;
}

extern "C" int32_t pxg_map(pxg_table* inp, int32_t n_exprs, const pxg_program* exprs, int64_t begin, int64_t end, pxg_table** out) {
  if (!inp || !out || n_exprs < 0 || (n_exprs > 0 && !exprs)) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Table& t = inp->impl;
  Ctx* ctx = t.ctx;
  PXG_RETURN_IF_ERROR(t.EnsureDeviceDescriptors());
  if (begin < 0 || end > t.nrows || begin > end) return SetError(PXG_INVALID_ARGUMENT, "bad row range");
  std::vector<int32_t> otypes;
  std::vector<ProgBuf> pbs(n_exprs);
  for (int e = 0; e < n_exprs; ++e) {
    const pxg_program& p = exprs[e];
    const bool passthrough = p.n_insns == 1 && p.insns && p.insns[0].op == PXG_OP_COL;
    if (p.result_type == PXG_STRING && !passthrough)
      return SetError(PXG_UNIMPLEMENTED, "STRING-producing scalar UDFs are not implemented on device");
    PXG_RETURN_IF_ERROR(UploadProgram(ctx, p, t, &pbs[e]));
    otypes.push_back(p.result_type);
  }
  pxg_table* ot = nullptr;
  PXG_RETURN_IF_ERROR(NewOutTable(ctx, otypes, &ot));
  std::unique_ptr<pxg_table, int32_t (*)(pxg_table*)> guard(ot, pxg_table_destroy);
  Table& o = ot->impl;
  for (size_t c = 0; c < t.chunks.size(); ++c) {
    const Chunk& ch = *t.chunks[c];
    const int64_t lo = std::max(begin, ch.row_base) - ch.row_base;
    const int64_t hi = std::min(end, ch.row_base + ch.nrows) - ch.row_base;
    if (lo >= hi) continue;
    const int64_t n = hi - lo;
    auto oc = std::make_unique<Chunk>();
    oc->row_base = o.nrows;
    oc->nrows = n;
    oc->rows_cap = n;
    oc->sealed = true;
    oc->cols.resize(n_exprs);
    for (int e = 0; e < n_exprs; ++e) {
      const pxg_program& p = exprs[e];
      ChunkCol& dc = oc->cols[e];
      const int ty = p.result_type;
      if (p.n_insns == 1 && p.insns[0].op == PXG_OP_COL) {
        const ChunkCol& sc = ch.cols[p.insns[0].arg];
        if (ty == PXG_STRING) {
          int32_t o0 = 0, o1 = 0;
          PXG_HIP(hipMemcpy(&o0, sc.offsets.as<int32_t>() + lo, 4, hipMemcpyDeviceToHost));
          PXG_HIP(hipMemcpy(&o1, sc.offsets.as<int32_t>() + hi, 4, hipMemcpyDeviceToHost));
          PXG_RETURN_IF_ERROR(dc.offsets.Alloc((n + 1) * 4 + 16));
          PXG_RETURN_IF_ERROR(dc.data.Alloc(static_cast<size_t>(o1 - o0) + 16));
          dc.data_len = o1 - o0;
          PXG_RETURN_IF_ERROR(Launch(ctx, "map_rebase", RebaseKernel, dim3(GridFor(n + 1, 256, 1 << 30)), dim3(256), 0,
                                     dc.offsets.as<int32_t>(), sc.offsets.as<const int32_t>() + lo, n + 1));
          PXG_HIP(hipMemcpyAsync(dc.data.p, sc.data.as<uint8_t>() + o0, o1 - o0, hipMemcpyDeviceToDevice, ctx->stream));
        } else {
          const int w = TypeWidth(ty);
          PXG_RETURN_IF_ERROR(dc.values.Alloc(n * w + 16));
          PXG_HIP(hipMemcpyAsync(dc.values.p, sc.values.as<uint8_t>() + lo * w, n * w, hipMemcpyDeviceToDevice, ctx->stream));
        }
        continue;
      }
      const int w = TypeWidth(ty);
      PXG_RETURN_IF_ERROR(dc.values.Alloc(n * w + 16));
      PXG_RETURN_IF_ERROR(Launch(ctx, "map_eval", MapEvalKernel, dim3(GridFor(n, 256, 1 << 30)), dim3(256), 0,
                                 pbs[e].prog.as<const DevProgram>(), t.d_chunks.as<const DevChunk>(), static_cast<int>(c),
                                 pbs[e].types.as<const int32_t>(), lo, n, dc.values.as<uint8_t>(), w));
    }
    PXG_HIP(hipStreamSynchronize(ctx->stream));
    o.nrows += n;
    o.chunks.push_back(std::move(oc));
    ++o.version;
  }
  *out = guard.release();
  return PXG_OK;
}
