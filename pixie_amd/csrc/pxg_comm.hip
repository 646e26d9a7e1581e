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
// enqueued on the ctx stream.  The v2 parts are laid out on the device, so the host waits twice
// per call (AlltoallV2): once for every size and header after the {bytes, header} records have
// crossed, once for the import's insert count and error flags (plus the export finalize's
// class-count wait when the plan has quantiles, and one more when the merge accumulators or the
// group table must grow).  A high-cardinality run exports its partition groups as states
// straight from the partition pass (no spill; only the v1 row parts still spill).
#include <cstddef>
#include <rccl/rccl.h>

#include "pxg_agg_host.h"

namespace pxg {

struct Comm {
  ncclComm_t nccl = nullptr;
  // Host transport (pxg_comm_init_host): the caller's byte mover, used instead of RCCL.
  pxg_xfer_fn host_fn = nullptr;
  void* host_user = nullptr;
  int32_t rank = 0, nranks = 1;
  Ctx* ctx = nullptr;
  DevBuf send, recv, counts;  // grow-only exchange buffers
  void* hstage = nullptr;     // host transport: grow-only pinned staging of one grouped exchange
  size_t hstage_bytes = 0;
  ~Comm() {
    if (hstage) (void)hipHostFree(hstage);
  }
};

#define PXG_NCCL(expr)                                                                                    \
  do {                                                                                                    \
    ncclResult_t r_ = (expr);                                                                             \
    if (r_ != ncclSuccess) return SetError(PXG_INTERNAL, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

// One grouped exchange of point-to-point byte transfers between device buffers, the unit both
// transports share.  RCCL: ncclGroupStart, an ncclSend / ncclRecv per transfer on the ctx
// stream, ncclGroupEnd -- closed on every exit path, so a failing call between start and end
// never leaves the group open for later calls on the communicator.  Host transport: the
// transfers are collected; End() waits for the stream (the send buffers are written by earlier
// kernels), copies the send buffers to pinned staging, hands the batch to the caller's byte mover,
// and copies what arrived to the receive buffers on the stream (stream-ordered before any later
// kernel).  A rank's transfers to itself are device-to-device copies matched in issue order.
struct XferGroup {
  Comm& C;
  bool open = false;
  struct Op {
    int32_t peer;
    bool send;
    void* dev;
    size_t bytes;
  };
  std::vector<Op> ops;
  explicit XferGroup(Comm& c) : C(c) {}
  int32_t Start() {
    if (C.nccl) {
      PXG_NCCL(ncclGroupStart());
      open = true;
    }
    return PXG_OK;
  }
  int32_t Send(const void* dev, size_t bytes, int32_t peer) {
    if (C.nccl) PXG_NCCL(ncclSend(dev, bytes, ncclUint8, peer, C.nccl, C.ctx->stream));
    else if (bytes > 0) ops.push_back(Op{peer, true, const_cast<void*>(dev), bytes});
    return PXG_OK;
  }
  int32_t Recv(void* dev, size_t bytes, int32_t peer) {
    if (C.nccl) PXG_NCCL(ncclRecv(dev, bytes, ncclUint8, peer, C.nccl, C.ctx->stream));
    else if (bytes > 0) ops.push_back(Op{peer, false, dev, bytes});
    return PXG_OK;
  }
  int32_t End() {
    if (C.nccl) {
      open = false;
      PXG_NCCL(ncclGroupEnd());
      return PXG_OK;
    }
    return RunHost();
  }
  ~XferGroup() {
    if (open) (void)ncclGroupEnd();
  }

 private:
  int32_t RunHost() {
    hipStream_t s = C.ctx->stream;
    // Self transfers: the k-th send to this rank lands in the k-th receive from it.
    std::vector<const Op*> self_s, self_r;
    size_t stage = 0;
    for (const Op& o : ops) {
      if (o.peer < 0 || o.peer >= C.nranks) return SetError(PXG_INVALID_ARGUMENT, "transfer to rank %d of %d", o.peer, C.nranks);
      if (o.peer == C.rank) (o.send ? self_s : self_r).push_back(&o);
      else stage += (o.bytes + 63) & ~size_t(63);
    }
    if (self_s.size() != self_r.size()) return SetError(PXG_INTERNAL, "unmatched transfers of a rank to itself");
    for (size_t i = 0; i < self_s.size(); ++i) {
      if (self_s[i]->bytes != self_r[i]->bytes)
        return SetError(PXG_INTERNAL, "self transfer of %zu bytes into a %zu-byte receive", self_s[i]->bytes, self_r[i]->bytes);
      PXG_HIP(hipMemcpyAsync(self_r[i]->dev, self_s[i]->dev, self_s[i]->bytes, hipMemcpyDeviceToDevice, s));
    }
    if (stage == 0) return PXG_OK;
    if (stage > C.hstage_bytes) {
      const size_t want = std::max(stage, C.hstage_bytes * 2);
      if (C.hstage) PXG_HIP(hipHostFree(C.hstage));
      C.hstage = nullptr;
      C.hstage_bytes = 0;
      PXG_HIP(hipHostMalloc(&C.hstage, want, hipHostMallocDefault));
      C.hstage_bytes = want;
    }
    std::vector<pxg_xfer> x;
    x.reserve(ops.size());
    uint8_t* h = static_cast<uint8_t*>(C.hstage);
    size_t at = 0;
    for (const Op& o : ops) {
      if (o.peer == C.rank) continue;
      x.push_back(pxg_xfer{o.peer, o.send ? 1 : 0, h + at, static_cast<int64_t>(o.bytes)});
      if (o.send) PXG_HIP(hipMemcpyAsync(h + at, o.dev, o.bytes, hipMemcpyDeviceToHost, s));
      at += (o.bytes + 63) & ~size_t(63);
    }
    PXG_HIP(hipStreamSynchronize(s));
    const int32_t rc = C.host_fn(C.host_user, static_cast<int32_t>(x.size()), x.data());
    if (rc != 0) return SetError(PXG_INTERNAL, "host transport failed (%d) on a batch of %zu transfers", rc, x.size());
    at = 0;
    for (const Op& o : ops) {
      if (o.peer == C.rank) continue;
      if (!o.send) PXG_HIP(hipMemcpyAsync(o.dev, h + at, o.bytes, hipMemcpyHostToDevice, s));
      at += (o.bytes + 63) & ~size_t(63);
    }
    // The staging is reused by the next grouped exchange, which starts with a stream wait.
    return PXG_OK;
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

extern "C" int32_t pxg_comm_init_host(pxg_ctx* ctx, int32_t rank, int32_t nranks, pxg_xfer_fn fn, void* user, pxg_comm** out) {
  if (!ctx || !fn || !out || nranks < 1 || rank < 0 || rank >= nranks) return SetError(PXG_INVALID_ARGUMENT, "bad pxg_comm_init_host arguments");
  PXG_HIP(hipSetDevice(ctx->impl.device));
  auto c = std::make_unique<pxg_comm>();
  c->impl.ctx = &ctx->impl;
  c->impl.rank = rank;
  c->impl.nranks = nranks;
  c->impl.host_fn = fn;
  c->impl.host_user = user;
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

namespace pxg {

// Exchange v2 (partial states, pxg_partial.hip): the parts are laid out and written on the device
// (ExportPartialDev), so the host first learns any size after the {bytes, header} records have
// crossed: one wait for every size and header (plus the export finalize's deferred checks),
// then the parts, then the import's one wait.  (An export finalize over quantiles also waits
// once inside, for its class counts.)
static int32_t AlltoallV2(pxg_agg* agg, Comm& C, int64_t* bytes_sent, int64_t* bytes_recv) {
  Agg& a = agg->impl;
  Ctx* ctx = a.ctx;
  const int32_t n = C.nranks;
  const size_t hb = XHeaderBytes();
  // counts: [n] own part bytes, [n] received bytes, [n * hb] received headers, [n * hb] own headers
  PXG_RETURN_IF_ERROR(C.counts.Ensure(static_cast<size_t>(n) * (16 + 2 * hb) + 64));
  int64_t* d_send_cnt = C.counts.as<int64_t>();
  int64_t* d_recv_cnt = d_send_cnt + n;
  uint8_t* d_recv_hdr = reinterpret_cast<uint8_t*>(d_recv_cnt + n);
  uint8_t* d_send_hdr = d_recv_hdr + static_cast<size_t>(n) * hb;
  uint8_t* pin8 = static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps;
  const size_t back = static_cast<size_t>(n) * (16 + hb);
  if (back + 64 > Ctx::kPinnedBytes - Ctx::kPinnedOps) return SetError(PXG_UNIMPLEMENTED, "%d ranks", n);
  // A failed export still takes part in the {bytes, header} exchange, announcing -1 bytes to every
  // peer (the device layout does the same when the finalize checks fail or the parts would pass
  // the send buffer): then no rank posts the part exchange and every rank returns an error, so no
  // peer is left inside a collective this rank has dropped out of.
  const int32_t xrc = a.ExportPartialDev(n, &C.send, d_send_cnt, d_send_hdr);
  std::string xerr;
  if (xrc != PXG_OK) {
    xerr = LastErrorRef();
    PXG_HIP(hipMemsetAsync(d_send_cnt, 0xFF, static_cast<size_t>(n) * 8, ctx->stream));
    PXG_HIP(hipMemsetAsync(d_send_hdr, 0, static_cast<size_t>(n) * hb, ctx->stream));
  }
  {
    XferGroup grp(C);
    PXG_RETURN_IF_ERROR(grp.Start());
    for (int p = 0; p < n; ++p) {
      PXG_RETURN_IF_ERROR(grp.Send(d_send_cnt + p, 8, p));
      PXG_RETURN_IF_ERROR(grp.Recv(d_recv_cnt + p, 8, p));
      PXG_RETURN_IF_ERROR(grp.Send(d_send_hdr + p * hb, hb, p));
      PXG_RETURN_IF_ERROR(grp.Recv(d_recv_hdr + p * hb, hb, p));
    }
    PXG_RETURN_IF_ERROR(grp.End());
  }
  // The one wait before the parts move: own sizes, received sizes and headers, finalize checks.
  PXG_HIP(hipMemcpyAsync(pin8, d_send_cnt, back, hipMemcpyDeviceToHost, ctx->stream));
  if (xrc == PXG_OK) PXG_HIP(hipMemcpyAsync(pin8 + back, a.ws.meta.p, 24, hipMemcpyDeviceToHost, ctx->stream));
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  if (xrc != PXG_OK) return SetError(xrc, "%s", xerr.c_str());
  const int32_t crc = a.CheckExportFinalize(pin8 + back);
  const int64_t* pin = reinterpret_cast<const int64_t*>(pin8);
  std::vector<int64_t> seg(pin, pin + n), rs(pin + n, pin + 2 * n);
  std::vector<uint8_t> rhdr(pin8 + 16 * n, pin8 + 16 * n + n * hb);
  if (crc != PXG_OK) return crc;  // (the device layout announced -1 for this failure too)
  int64_t total = 0, rtotal = 0;
  for (int p = 0; p < n; ++p) {
    if (seg[p] < 0) return SetError(PXG_INTERNAL, "export parts would pass the %zu-byte send buffer; no parts moved", C.send.bytes);
    total += seg[p];
  }
  for (int p = 0; p < n; ++p) {
    if (rs[p] < 0) return SetError(PXG_INTERNAL, "rank %d failed its export; no parts moved", p);
    rtotal += rs[p];
  }
  PXG_RETURN_IF_ERROR(C.recv.Ensure(static_cast<size_t>(rtotal) + 64));
  {
    XferGroup grp(C);
    PXG_RETURN_IF_ERROR(grp.Start());
    int64_t so = 0, ro = 0;
    for (int p = 0; p < n; ++p) {
      if (seg[p] > 0) PXG_RETURN_IF_ERROR(grp.Send(C.send.as<uint8_t>() + so, static_cast<size_t>(seg[p]), p));
      if (rs[p] > 0) PXG_RETURN_IF_ERROR(grp.Recv(C.recv.as<uint8_t>() + ro, static_cast<size_t>(rs[p]), p));
      so += seg[p];
      ro += rs[p];
    }
    PXG_RETURN_IF_ERROR(grp.End());
  }
  // Every group this rank exported now lives on its owner (as in the v1 path below).
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
  if (!poffs.empty())
    PXG_RETURN_IF_ERROR(a.ImportPartialsV2(C.recv.as<const uint8_t>(), static_cast<int32_t>(poffs.size()), poffs.data(), psizes.data(), phdr.data()));
  if (bytes_sent) *bytes_sent = total;
  if (bytes_recv) *bytes_recv = rtotal;
  return PXG_OK;
}

}  // namespace pxg

extern "C" int32_t pxg_agg_alltoall(pxg_agg* agg, pxg_comm* comm, int64_t* bytes_sent, int64_t* bytes_recv) {
  if (!agg || !comm) return SetError(PXG_INVALID_ARGUMENT, "bad pxg_agg_alltoall arguments");
  Comm& C = comm->impl;
  Agg& a = agg->impl;
  Ctx* ctx = a.ctx;
  if (ctx != C.ctx) return SetError(PXG_INVALID_ARGUMENT, "aggregation and communicator belong to different contexts");
  const int32_t n = C.nranks;
  // v2 exports a high-cardinality run's partition groups directly (ExportGroupV2); the v1 row
  // parts are cut from the table state, so that path first spills the partition records.
  if (ExchangeV2(a)) return AlltoallV2(agg, C, bytes_sent, bytes_recv);
  PXG_RETURN_IF_ERROR(a.SpillHc());
  // Exchange v1 (PXG_XCHG_V1=1, row parts): sizes of the n parts, then the parts themselves.
  std::vector<int64_t> offs(n), bytes(n), seg(n);
  const bool v2 = false;
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
    XferGroup grp(C);
    PXG_RETURN_IF_ERROR(grp.Start());
    for (int p = 0; p < n; ++p) {
      PXG_RETURN_IF_ERROR(grp.Send(d_send_cnt + p, 8, p));
      PXG_RETURN_IF_ERROR(grp.Recv(d_recv_cnt + p, 8, p));
      if (hb > 0) {
        PXG_RETURN_IF_ERROR(grp.Send(C.send.as<uint8_t>() + offs[p], hb, p));
        PXG_RETURN_IF_ERROR(grp.Recv(d_recv_hdr + p * hb, hb, p));
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
    XferGroup grp(C);
    PXG_RETURN_IF_ERROR(grp.Start());
    int64_t so = 0, ro = 0;
    for (int p = 0; p < n; ++p) {
      if (seg[p] > 0) PXG_RETURN_IF_ERROR(grp.Send(C.send.as<uint8_t>() + so, static_cast<size_t>(seg[p]), p));
      if (rs[p] > 0) PXG_RETURN_IF_ERROR(grp.Recv(C.recv.as<uint8_t>() + ro, static_cast<size_t>(rs[p]), p));
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

// ---------------------------------------------------------------------------------------------
// pxg_agg_gather: the finalized rows of every rank to one rank (the Kelvin
// result stream that the reference's GRPCSink sends to the query broker, grpc_sink_node.cc:305-330).
// After pxg_agg_alltoall + pxg_agg_finalize every group lives on exactly one rank, so the global
// result is the row-wise concatenation of the ranks' results: the root's own rows first (left in
// place), then the other ranks' rows in rank order.  Per rank one 8-word header {groups, STRING
// key payload bytes} travels first; the root waits for the headers once (it sizes its buffers
// from them), the senders never wait.  STRING key offsets arrive relative to their rank's payload
// and are rebased on the device.
// ---------------------------------------------------------------------------------------------
namespace pxg {

constexpr int kGatherHdr = 1 + kMaxKeys;  // int64 words: groups, then key_data_len per key

// out[base_g[r] + 1 + j] = tmp[base_t[r] + 1 + j] - tmp[base_t[r]] + base_b[r] for the non-root
// ranks r (slot 0 = the root keeps its offsets in place); out[G] = the total payload.
__global__ void GatherRebaseKernel(const int32_t* __restrict__ tmp, const int64_t* __restrict__ bases, int32_t nr,
                                   int32_t* __restrict__ out) {
  // bases: [nr] group base, [nr] tmp base, [nr] byte base, [nr] groups (ranks in concatenation
  // order, slot 0 = the root).
  const int64_t* gb = bases;
  const int64_t* tb = bases + nr;
  const int64_t* bb = bases + 2 * nr;
  const int64_t* gn = bases + 3 * nr;
  for (int r = 1; r < nr; ++r) {
    const int32_t t0 = tmp[tb[r]];
    for (int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < gn[r]; j += static_cast<int64_t>(gridDim.x) * blockDim.x)
      out[gb[r] + 1 + j] = static_cast<int32_t>(tmp[tb[r] + 1 + j] - t0 + bb[r]);
  }
}

}  // namespace pxg

extern "C" int32_t pxg_agg_gather(pxg_agg* agg, pxg_comm* comm, int32_t root, int64_t* n_groups) {
  if (!agg || !comm) return SetError(PXG_INVALID_ARGUMENT, "bad pxg_agg_gather arguments");
  Comm& C = comm->impl;
  Agg& a = agg->impl;
  Ctx* ctx = a.ctx;
  if (ctx != C.ctx) return SetError(PXG_INVALID_ARGUMENT, "aggregation and communicator belong to different contexts");
  const int32_t n = C.nranks;
  if (root < 0 || root >= n) return SetError(PXG_INVALID_ARGUMENT, "root %d of %d ranks", root, n);
  if (!a.res.ready) return SetError(PXG_FAILED_PRECONDITION, "pxg_agg_finalize has not run since the last consume");
  if (a.n_keys == 0) return SetError(PXG_UNIMPLEMENTED, "a group-less aggregate is merged, not gathered");
  AggResult& R = a.res;
  const bool me_root = C.rank == root;
  // Per column: bytes of this rank's part (STRING keys: offsets then payload).
  auto fixed_w = [&](int k) { return static_cast<int64_t>(TypeWidth(a.key_types[k])); };
  const int64_t val_per = 8;
  auto val_bytes = [&](int u, int64_t G) -> int64_t {
    if (a.emit_states) return G * a.state_rec;
    return G * (a.uda_kind[u] == PXG_UDA_QUANTILES ? 7 * val_per : val_per);
  };
  const int n_vcols = a.emit_states ? 1 : a.n_udas;
  DevBuf* vbuf[kMaxUdas];
  for (int u = 0; u < n_vcols; ++u) vbuf[u] = a.emit_states ? &R.states : &R.uda_out[u];
  // 1. Headers: every rank's {groups, key payload bytes} to the root.
  int64_t* pin = reinterpret_cast<int64_t*>(static_cast<uint8_t*>(ctx->pinned) + Ctx::kPinnedOps);
  if (static_cast<size_t>(n + 1) * kGatherHdr * 8 > Ctx::kPinnedBytes - Ctx::kPinnedOps) return SetError(PXG_UNIMPLEMENTED, "%d ranks", n);
  PXG_RETURN_IF_ERROR(C.counts.Ensure(static_cast<size_t>(n + 1) * kGatherHdr * 8 + 64));
  int64_t* d_hdr = C.counts.as<int64_t>();  // [0] mine, [1 + r] rank r's (root)
  // The stream may still be writing pinned scratch of an earlier call (the finalize's readbacks
  // are synchronous, so it is idle here); write this rank's header.
  pin[0] = R.n_groups;
  for (int k = 0; k < kMaxKeys; ++k) pin[1 + k] = k < a.n_keys && a.key_types[k] == PXG_STRING ? R.key_data_len[k] : 0;
  std::vector<int64_t> hdr(static_cast<size_t>(n) * kGatherHdr, 0);
  if (!me_root) {
    PXG_HIP(hipMemcpyAsync(d_hdr, pin, kGatherHdr * 8, hipMemcpyHostToDevice, ctx->stream));
    XferGroup grp(C);
    PXG_RETURN_IF_ERROR(grp.Start());
    PXG_RETURN_IF_ERROR(grp.Send(d_hdr, (kGatherHdr) * 8, root));
    PXG_RETURN_IF_ERROR(grp.End());
  } else {
    std::copy(pin, pin + kGatherHdr, hdr.begin() + static_cast<size_t>(root) * kGatherHdr);
    if (n > 1) {
      XferGroup grp(C);
      PXG_RETURN_IF_ERROR(grp.Start());
      for (int r = 0; r < n; ++r)
        if (r != root) PXG_RETURN_IF_ERROR(grp.Recv(d_hdr + static_cast<size_t>(1 + r) * kGatherHdr, (kGatherHdr) * 8, r));
      PXG_RETURN_IF_ERROR(grp.End());
      PXG_HIP(hipMemcpyAsync(pin + kGatherHdr, d_hdr + kGatherHdr, static_cast<size_t>(n) * kGatherHdr * 8, hipMemcpyDeviceToHost, ctx->stream));
      PXG_HIP(hipStreamSynchronize(ctx->stream));
      for (int r = 0; r < n; ++r)
        if (r != root) std::copy(pin + (1 + r) * kGatherHdr, pin + (2 + r) * kGatherHdr, hdr.begin() + static_cast<size_t>(r) * kGatherHdr);
    }
  }
  // 2. Senders: every column to the root, in column order (zero-length columns skipped on both
  //    sides by the same rule).
  if (!me_root) {
    const int64_t G = R.n_groups;
    if (G > 0) {
      XferGroup grp(C);
      PXG_RETURN_IF_ERROR(grp.Start());
      for (int k = 0; k < a.n_keys; ++k) {
        if (a.key_types[k] == PXG_STRING) {
          PXG_RETURN_IF_ERROR(grp.Send(R.key_offsets[k].p, (static_cast<size_t>(G + 1)) * 4, root));
          if (R.key_data_len[k] > 0) PXG_RETURN_IF_ERROR(grp.Send(R.key_data[k].p, static_cast<size_t>(R.key_data_len[k]), root));
        } else {
          PXG_RETURN_IF_ERROR(grp.Send(R.key_fixed[k].p, static_cast<size_t>(G * fixed_w(k)), root));
        }
      }
      for (int u = 0; u < n_vcols; ++u) {
        const int64_t b = val_bytes(u, G);
        if (b > 0) PXG_RETURN_IF_ERROR(grp.Send(vbuf[u]->p, static_cast<size_t>(b), root));
      }
      PXG_RETURN_IF_ERROR(grp.End());
    }
    // The rows now belong to the root's result; this rank keeps its (already sent) copy until
    // the next finalize.  The sends are stream-ordered before any later write of these buffers.
    if (n_groups) *n_groups = 0;
    return PXG_OK;
  }
  // 3. Root: concatenation order = the root, then the other ranks by rank.
  std::vector<int> order{root};
  for (int r = 0; r < n; ++r)
    if (r != root) order.push_back(r);
  const int nr = static_cast<int>(order.size());
  std::vector<int64_t> gbase(nr), tbase(nr), gcnt(nr);
  std::vector<std::vector<int64_t>> bbase(a.n_keys, std::vector<int64_t>(nr, 0));
  int64_t Gt = 0, Tt = 0;
  std::vector<int64_t> btot(a.n_keys, 0);
  for (int i = 0; i < nr; ++i) {
    const int64_t* h = hdr.data() + static_cast<size_t>(order[i]) * kGatherHdr;
    if (h[0] < 0) return SetError(PXG_INTERNAL, "rank %d announced %lld groups", order[i], static_cast<long long>(h[0]));
    gbase[i] = Gt;
    gcnt[i] = h[0];
    tbase[i] = Tt;
    Gt += h[0];
    Tt += h[0] + 1;
    for (int k = 0; k < a.n_keys; ++k) {
      bbase[k][i] = btot[k];
      btot[k] += h[1 + k];
    }
  }
  for (int k = 0; k < a.n_keys; ++k)
    if (btot[k] >= (int64_t(1) << 31)) return SetError(PXG_UNIMPLEMENTED, "gathered key payload of %lld bytes needs 64-bit offsets", static_cast<long long>(btot[k]));
  const int64_t G0 = R.n_groups;  // the root's own rows stay at the front of its buffers
  for (int k = 0; k < a.n_keys; ++k) {
    if (a.key_types[k] == PXG_STRING) {
      PXG_RETURN_IF_ERROR(R.key_offsets[k].Reserve(static_cast<size_t>(Gt + 1) * 4 + 16, static_cast<size_t>(G0 + 1) * 4, ctx->stream));
      PXG_RETURN_IF_ERROR(R.key_data[k].Reserve(static_cast<size_t>(btot[k]) + 16, static_cast<size_t>(R.key_data_len[k]), ctx->stream));
    } else {
      PXG_RETURN_IF_ERROR(R.key_fixed[k].Reserve(static_cast<size_t>(Gt * fixed_w(k)) + 16, static_cast<size_t>(G0 * fixed_w(k)), ctx->stream));
    }
  }
  for (int u = 0; u < n_vcols; ++u)
    PXG_RETURN_IF_ERROR(vbuf[u]->Reserve(static_cast<size_t>(val_bytes(u, Gt)) + 16, static_cast<size_t>(val_bytes(u, G0)), ctx->stream));
  // Other ranks' STRING offsets land in scratch (C.recv), rebased below.
  bool any_str = false;
  for (int k = 0; k < a.n_keys; ++k) any_str |= a.key_types[k] == PXG_STRING;
  const size_t tmp_words = static_cast<size_t>(Tt);
  if (any_str) PXG_RETURN_IF_ERROR(C.recv.Ensure(static_cast<size_t>(a.n_keys) * tmp_words * 4 + static_cast<size_t>(4 * nr) * 8 + 128));
  int32_t* tmp = C.recv.as<int32_t>();
  if (Gt > G0) {
    XferGroup grp(C);
    PXG_RETURN_IF_ERROR(grp.Start());
    for (int i = 1; i < nr; ++i) {
      const int64_t G = gcnt[i];
      if (G == 0) continue;
      const int src = order[i];
      for (int k = 0; k < a.n_keys; ++k) {
        if (a.key_types[k] == PXG_STRING) {
          PXG_RETURN_IF_ERROR(grp.Recv(tmp + static_cast<size_t>(k) * tmp_words + tbase[i], (static_cast<size_t>(G + 1)) * 4, src));
          const int64_t len = hdr[static_cast<size_t>(src) * kGatherHdr + 1 + k];
          if (len > 0) PXG_RETURN_IF_ERROR(grp.Recv(R.key_data[k].as<uint8_t>() + bbase[k][i], static_cast<size_t>(len), src));
        } else {
          PXG_RETURN_IF_ERROR(grp.Recv(R.key_fixed[k].as<uint8_t>() + gbase[i] * fixed_w(k), static_cast<size_t>(G * fixed_w(k)), src));
        }
      }
      for (int u = 0; u < n_vcols; ++u) {
        const int64_t b = val_bytes(u, G);
        if (b > 0) PXG_RETURN_IF_ERROR(grp.Recv(vbuf[u]->as<uint8_t>() + val_bytes(u, gbase[i]), static_cast<size_t>(b), src));
      }
    }
    PXG_RETURN_IF_ERROR(grp.End());
    if (any_str) {
      int64_t* d_bases = reinterpret_cast<int64_t*>(tmp + static_cast<size_t>(a.n_keys) * tmp_words + 16);
      d_bases = reinterpret_cast<int64_t*>((reinterpret_cast<uintptr_t>(d_bases) + 7) & ~uintptr_t(7));
      for (int k = 0; k < a.n_keys; ++k) {
        if (a.key_types[k] != PXG_STRING) continue;
        // Host table of bases, staged through pinned memory one key at a time (stream-ordered).
        int64_t* hb = pin + kGatherHdr * (n + 1);
        if (static_cast<size_t>(kGatherHdr * (n + 1) + 4 * nr + 1) * 8 > Ctx::kPinnedBytes - Ctx::kPinnedOps)
          return SetError(PXG_UNIMPLEMENTED, "%d ranks", n);
        for (int i = 0; i < nr; ++i) {
          hb[i] = gbase[i];
          hb[nr + i] = tbase[i] + static_cast<int64_t>(k) * static_cast<int64_t>(tmp_words);
          hb[2 * nr + i] = bbase[k][i];
          hb[3 * nr + i] = gcnt[i];
        }
        PXG_HIP(hipMemcpyAsync(d_bases, hb, static_cast<size_t>(4 * nr) * 8, hipMemcpyHostToDevice, ctx->stream));
        PXG_RETURN_IF_ERROR(Launch(ctx, "gather_rebase", GatherRebaseKernel, dim3(GridFor(Gt, 256, 1024)), dim3(256), 0,
                                   static_cast<const int32_t*>(tmp), static_cast<const int64_t*>(d_bases), nr, R.key_offsets[k].as<int32_t>()));
        // The pinned base table is reused by the next key: wait for this copy first.
        PXG_HIP(hipStreamSynchronize(ctx->stream));
      }
    }
  }
  for (int k = 0; k < a.n_keys; ++k)
    if (a.key_types[k] == PXG_STRING) {
      if (G0 == 0) {
        // The root had no rows: its offsets start at 0 (the other ranks' rows follow).
        PXG_HIP(hipMemsetAsync(R.key_offsets[k].p, 0, 4, ctx->stream));
      }
      R.key_data_len[k] = btot[k];
    }
  R.n_groups = Gt;
  PXG_HIP(hipStreamSynchronize(ctx->stream));
  if (n_groups) *n_groups = Gt;
  return PXG_OK;
}
