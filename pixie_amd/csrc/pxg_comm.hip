// Intra-node exchange of partial aggregation states over RCCL (xGMI), owned by libpxg so the
// C++ engine needs no torch: the Kelvin-finalize analogue of the PEM-partial split
// (src/carnot/planner/distributed/splitter/partial_op_mgr/partial_op_mgr.cc:69-83), one rank
// per GPU.
//
// pxg_agg_alltoall: export the agg's state partitioned by hash(group key) % nranks
// (exchange v2: per-group Serialize() states, raw values / centroid lists for quantiles;
// pxg_partial.hip), exchange per peer one record of {part bytes, part header} (grouped
// ncclSend / ncclRecv), exchange the parts (all-to-all(v) as grouped ncclSend / ncclRecv of
// bytes), merge what arrived (ImportPartialsV2 with the received headers).  Every RCCL call is
// enqueued on the ctx stream.  Host waits per call: the export's sizes, the export's write, the
// {bytes, header} records, the import's insert count and error flags (4; plus one when the merge
// accumulators or the group table must grow).  A high-cardinality run first moves its partition
// records into the table (SpillHc).
#include <cstddef>
#include <rccl/rccl.h>

#include "pxg_agg_host.h"

namespace pxg {

struct Comm {
  ncclComm_t nccl = nullptr;
  int32_t rank = 0, nranks = 1;
  Ctx* ctx = nullptr;
  DevBuf send, recv, counts;  // grow-only exchange buffers
};

#define PXG_NCCL(expr)                                                                                    \
  do {                                                                                                    \
    ncclResult_t r_ = (expr);                                                                             \
    if (r_ != ncclSuccess) return SetError(PXG_INTERNAL, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

// An RCCL group that is closed on every exit path: an ncclSend / ncclRecv that fails between
// ncclGroupStart and ncclGroupEnd must not leave the group open for later calls on the
// communicator.
struct NcclGroup {
  bool open = false;
  int32_t Start() {
    PXG_NCCL(ncclGroupStart());
    open = true;
    return PXG_OK;
  }
  int32_t End() {
    open = false;
    PXG_NCCL(ncclGroupEnd());
    return PXG_OK;
  }
  ~NcclGroup() {
    if (open) (void)ncclGroupEnd();
  }
};

}  // namespace pxg

struct pxg_comm {
  pxg::Comm impl;
};

using namespace pxg;

extern "C" int32_t pxg_comm_unique_id(uint8_t* id_out, int32_t id_bytes) {
  if (!id_out || id_bytes < static_cast<int32_t>(sizeof(ncclUniqueId)))
    return SetError(PXG_INVALID_ARGUMENT, "unique id buffer must hold %d bytes", static_cast<int>(sizeof(ncclUniqueId)));
  ncclUniqueId id;
  PXG_NCCL(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return PXG_OK;
}

extern "C" int32_t pxg_comm_init(pxg_ctx* ctx, int32_t rank, int32_t nranks, const uint8_t* id, int32_t id_bytes, pxg_comm** out) {
  if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks || id_bytes < static_cast<int32_t>(sizeof(ncclUniqueId)))
    return SetError(PXG_INVALID_ARGUMENT, "bad pxg_comm_init arguments");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  PXG_HIP(hipSetDevice(ctx->impl.device));
  auto c = std::make_unique<pxg_comm>();
  c->impl.ctx = &ctx->impl;
  c->impl.rank = rank;
  c->impl.nranks = nranks;
  PXG_NCCL(ncclCommInitRank(&c->impl.nccl, nranks, uid, rank));
  *out = c.release();
  return PXG_OK;
}

extern "C" int32_t pxg_comm_destroy(pxg_comm* comm) {
  if (!comm) return PXG_OK;
  if (comm->impl.ctx) (void)hipStreamSynchronize(comm->impl.ctx->stream);
  if (comm->impl.nccl) ncclCommDestroy(comm->impl.nccl);
  delete comm;
  return PXG_OK;
}

extern "C" int32_t pxg_agg_alltoall(pxg_agg* agg, pxg_comm* comm, int64_t* bytes_sent, int64_t* bytes_recv) {
  if (!agg || !comm) return SetError(PXG_INVALID_ARGUMENT, "bad pxg_agg_alltoall arguments");
  Comm& C = comm->impl;
  Agg& a = agg->impl;
  Ctx* ctx = a.ctx;
  if (ctx != C.ctx) return SetError(PXG_INVALID_ARGUMENT, "aggregation and communicator belong to different contexts");
  const int32_t n = C.nranks;
  // 1. Sizes of the n parts, then the parts themselves.
  std::vector<int64_t> offs(n), bytes(n), seg(n);
  PXG_RETURN_IF_ERROR(a.SpillHc());
  const bool v2 = ExchangeV2(a);
  auto do_export = [&](void* dst, int64_t cap) {
    return v2 ? a.ExportPartialV2(n, dst, cap, offs.data(), bytes.data()) : a.ExportPartial(n, dst, cap, offs.data(), bytes.data());
  };
  PXG_RETURN_IF_ERROR(do_export(nullptr, 0));
  int64_t total = 0;
  for (int p = 0; p < n; ++p) {
    seg[p] = p + 1 < n ? offs[p + 1] - offs[p] : ((bytes[p] + 7) & ~int64_t(7));
    total += seg[p];
  }
  PXG_RETURN_IF_ERROR(C.send.Ensure(static_cast<size_t>(total) + 64));
  PXG_RETURN_IF_ERROR(do_export(C.send.p, static_cast<int64_t>(C.send.bytes)));
  // 2. Per peer a record of {bytes, part header} (v2; the header is the part's own first bytes in
  //    the send buffer), itself included.
  const size_t hb = v2 ? XHeaderBytes() : 0;
  const size_t rec = 8 + hb;
  PXG_RETURN_IF_ERROR(C.counts.Ensure(static_cast<size_t>(2 * n) * rec + 64));
  int64_t* d_send_cnt = C.counts.as<int64_t>();
  int64_t* d_recv_cnt = d_send_cnt + n;
  uint8_t* d_recv_hdr = reinterpret_cast<uint8_t*>(d_recv_cnt + n);
  uint8_t* pin8 = static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps;
  if (static_cast<size_t>(2 * n) * 8 + static_cast<size_t>(n) * hb > Ctx::kPinnedBytes - Ctx::kPinnedOps)
    return SetError(PXG_UNIMPLEMENTED, "%d ranks", n);
  int64_t* pin = reinterpret_cast<int64_t*>(pin8);
  for (int p = 0; p < n; ++p) pin[p] = seg[p];
  PXG_HIP(hipMemcpyAsync(d_send_cnt, pin, static_cast<size_t>(n) * 8, hipMemcpyHostToDevice, ctx->stream));
  {
    NcclGroup grp;
    PXG_RETURN_IF_ERROR(grp.Start());
    for (int p = 0; p < n; ++p) {
      PXG_NCCL(ncclSend(d_send_cnt + p, 1, ncclInt64, p, C.nccl, ctx->stream));
      PXG_NCCL(ncclRecv(d_recv_cnt + p, 1, ncclInt64, p, C.nccl, ctx->stream));
      if (hb > 0) {
        PXG_NCCL(ncclSend(C.send.as<uint8_t>() + offs[p], hb, ncclUint8, p, C.nccl, ctx->stream));
        PXG_NCCL(ncclRecv(d_recv_hdr + p * hb, hb, ncclUint8, p, C.nccl, ctx->stream));
      }
    }
    PXG_RETURN_IF_ERROR(grp.End());
  }
  PXG_HIP(hipMemcpyAsync(pin + n, d_recv_cnt, static_cast<size_t>(n) * 8 + static_cast<size_t>(n) * hb, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  std::vector<int64_t> rs(pin + n, pin + 2 * n);
  std::vector<uint8_t> rhdr(pin8 + 16 * n, pin8 + 16 * n + n * hb);
  int64_t rtotal = 0;
  for (int p = 0; p < n; ++p) {
    if (rs[p] < 0) return SetError(PXG_INTERNAL, "rank %d announced %lld bytes", p, static_cast<long long>(rs[p]));
    rtotal += rs[p];
  }
  // 3. The parts: all-to-all(v) as grouped point-to-point sends over xGMI.
  PXG_RETURN_IF_ERROR(C.recv.Ensure(static_cast<size_t>(rtotal) + 64));
  {
    NcclGroup grp;
    PXG_RETURN_IF_ERROR(grp.Start());
    int64_t so = 0, ro = 0;
    for (int p = 0; p < n; ++p) {
      if (seg[p] > 0) PXG_NCCL(ncclSend(C.send.as<uint8_t>() + so, static_cast<size_t>(seg[p]), ncclUint8, p, C.nccl, ctx->stream));
      if (rs[p] > 0) PXG_NCCL(ncclRecv(C.recv.as<uint8_t>() + ro, static_cast<size_t>(rs[p]), ncclUint8, p, C.nccl, ctx->stream));
      so += seg[p];
      ro += rs[p];
    }
    PXG_RETURN_IF_ERROR(grp.End());
  }
  // 4. Every group this rank exported now lives on its owner: rebuild from the received parts
  //    (our own part included), all of them in one import.  The local state is dropped first:
  //    if the import fails, the aggregation is left empty (the caller must reset and rerun the
  //    query; the exported groups are on their owners' ranks, not here).
  PXG_RETURN_IF_ERROR(pxg_agg_reset(agg));
  std::vector<int64_t> poffs, psizes;
  std::vector<uint8_t> phdr;
  int64_t at = 0;
  for (int p = 0; p < n; ++p) {
    if (rs[p] > 0) {
      poffs.push_back(at);
      psizes.push_back(rs[p]);
      phdr.insert(phdr.end(), rhdr.begin() + p * hb, rhdr.begin() + (p + 1) * hb);
    }
    at += rs[p];
  }
  if (v2) {
    if (!poffs.empty())
      PXG_RETURN_IF_ERROR(a.ImportPartialsV2(C.recv.as<const uint8_t>(), static_cast<int32_t>(poffs.size()), poffs.data(), psizes.data(),
                                             phdr.data()));
  } else {
    PXG_RETURN_IF_ERROR(a.ImportPartials(C.recv.p, static_cast<int32_t>(poffs.size()), poffs.data(), psizes.data()));
  }
  if (bytes_sent) *bytes_sent = total;
  if (bytes_recv) *bytes_recv = rtotal;
  return PXG_OK;
}
