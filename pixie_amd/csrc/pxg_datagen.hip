// Device generator of the synthetic http_events table (SURVEY.md §8d spec,
// pxg_datagen_spec.h): rows are generated straight into HBM, bit-identical to the host generator
// (pxg_datagen_http_events), so a 1B-row table is resident in well under a second instead of
// ~100 s of host generation and PCIe upload.  Bench / test input only: not a reference path.
#include <algorithm>

#include "pxg_datagen_spec.h"
#include "pxg_internal.h"
#include "pxg_scan.h"

namespace pxg {

using gen::Row;
using gen::Tables;

struct GenCols {
  int64_t* time;
  uint64_t* upid;
  int64_t* status;
  int64_t* latency;
  int64_t* req_body;
  int64_t* resp_body;
  uint32_t* off[4];  // service, req_path, remote_addr, pod: lengths, scanned in place to offsets
  uint8_t* data[4];
};

constexpr int kGenBlock = 256;

__global__ void __launch_bounds__(kGenBlock) GenFixedKernel(uint64_t seed, int64_t row0, int64_t n, int64_t n_pair_keys,
                                                            const Tables* __restrict__ T, GenCols o) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kGenBlock + threadIdx.x;
  if (r > n) return;
  if (r == n) {  // the scans' last element: offsets[n] = total
    for (int s = 0; s < 4; ++s) o.off[s][n] = 0;
    return;
  }
  const Row w = gen::MakeRow(seed, row0 + r, n_pair_keys, T->svc_cdf, T->path_cdf, T->lat_grid);
  o.time[r] = w.time;
  o.upid[2 * r] = w.upid_lo;
  o.upid[2 * r + 1] = w.upid_hi;
  o.status[r] = w.status;
  o.latency[r] = w.latency;
  o.req_body[r] = w.req_body;
  o.resp_body[r] = w.resp_body;
  o.off[0][r] = static_cast<uint32_t>(T->svc_off[w.svc + 1] - T->svc_off[w.svc]);
  o.off[1][r] = static_cast<uint32_t>(T->path_off[w.path + 1] - T->path_off[w.path]);
  o.off[2][r] = static_cast<uint32_t>(gen::AddrLen(w.addr_idx));
  o.off[3][r] = gen::kPodLen;
}

__global__ void __launch_bounds__(kGenBlock) GenStringsKernel(uint64_t seed, int64_t row0, int64_t n, int64_t n_pair_keys,
                                                              const Tables* __restrict__ T, GenCols o) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kGenBlock + threadIdx.x;
  if (r >= n) return;
  const Row w = gen::MakeRow(seed, row0 + r, n_pair_keys, T->svc_cdf, T->path_cdf, T->lat_grid);
  {
    const int32_t a = T->svc_off[w.svc], l = T->svc_off[w.svc + 1] - a;
    uint8_t* d = o.data[0] + o.off[0][r];
    for (int i = 0; i < l; ++i) d[i] = static_cast<uint8_t>(T->svc_bytes[a + i]);
  }
  {
    const int32_t a = T->path_off[w.path], l = T->path_off[w.path + 1] - a;
    uint8_t* d = o.data[1] + o.off[1][r];
    for (int i = 0; i < l; ++i) d[i] = static_cast<uint8_t>(T->path_bytes[a + i]);
  }
  char buf[24];
  const int la = gen::FormatAddr(w.addr_idx, buf);
  uint8_t* d = o.data[2] + o.off[2][r];
  for (int i = 0; i < la; ++i) d[i] = static_cast<uint8_t>(buf[i]);
  gen::FormatPod(w.pod, buf);
  d = o.data[3] + o.off[3][r];
  for (int i = 0; i < gen::kPodLen; ++i) d[i] = static_cast<uint8_t>(buf[i]);
}

}  // namespace pxg

using namespace pxg;

extern "C" int32_t pxg_table_append_http_events(pxg_table* tp, uint64_t seed, int64_t row_begin, int64_t nrows,
                                                int64_t n_pair_keys) {
  if (!tp || nrows < 0) return SetError(PXG_INVALID_ARGUMENT, "bad arguments");
  Table& t = tp->impl;
  static const int32_t kTypes[PXG_HTTP_EVENTS_NCOLS] = {PXG_TIME64NS, PXG_UINT128, PXG_STRING, PXG_STRING, PXG_STRING,
                                                        PXG_INT64,    PXG_INT64,   PXG_INT64,  PXG_INT64,  PXG_STRING};
  if (t.ncols != PXG_HTTP_EVENTS_NCOLS) return SetError(PXG_INVALID_ARGUMENT, "table is not http_events-shaped");
  for (int c = 0; c < PXG_HTTP_EVENTS_NCOLS; ++c)
    if (t.types[c] != kTypes[c]) return SetError(PXG_INVALID_ARGUMENT, "column %d has type %d, http_events needs %d", c, t.types[c], kTypes[c]);
  if (n_pair_keys <= 0) n_pair_keys = 10000000;
  if (nrows == 0) return PXG_OK;
  PXG_RETURN_IF_ERROR(t.FlushStage());
  Ctx* ctx = t.ctx;
  const Tables& T = gen::GetTables();
  DevBuf d_tables;
  PXG_RETURN_IF_ERROR(d_tables.Alloc(sizeof(Tables)));
  PXG_HIP(hipMemcpyAsync(d_tables.p, &T, sizeof(Tables), hipMemcpyHostToDevice, ctx->stream));
  const int64_t S = std::min<int64_t>(nrows, kChunkRows);
  // Per-row upper bounds of the payload: service 16 B, req_path 48 B, remote_addr 15 B, pod 17 B.
  static const size_t kMaxLen[4] = {16, 48, 15, static_cast<size_t>(gen::kPodLen)};
  DevBuf fixed[6], off[4], data[4], scan_tmp;
  for (int i = 0; i < 6; ++i) PXG_RETURN_IF_ERROR(fixed[i].Alloc(static_cast<size_t>(S) * (i == 1 ? 16 : 8) + 16));
  for (int s = 0; s < 4; ++s) {
    PXG_RETURN_IF_ERROR(off[s].Alloc(static_cast<size_t>(S + 1) * 4 + 16));
    PXG_RETURN_IF_ERROR(data[s].Alloc(static_cast<size_t>(S) * kMaxLen[s] + 16));
  }
  PXG_RETURN_IF_ERROR(scan_tmp.Alloc(ScanScratchBytes(S + 1) + 64));
  GenCols o;
  o.time = fixed[0].as<int64_t>();
  o.upid = fixed[1].as<uint64_t>();
  o.status = fixed[2].as<int64_t>();
  o.latency = fixed[3].as<int64_t>();
  o.req_body = fixed[4].as<int64_t>();
  o.resp_body = fixed[5].as<int64_t>();
  for (int s = 0; s < 4; ++s) {
    o.off[s] = off[s].as<uint32_t>();
    o.data[s] = data[s].as<uint8_t>();
  }
  for (int64_t done = 0; done < nrows;) {
    const int64_t n = std::min<int64_t>(S, nrows - done);
    const int64_t g0 = row_begin + done;
    PXG_RETURN_IF_ERROR(Launch(ctx, "gen_fixed", GenFixedKernel, dim3(static_cast<unsigned>((n + 1 + kGenBlock - 1) / kGenBlock)),
                               dim3(kGenBlock), 0, seed, g0, n, n_pair_keys, d_tables.as<const Tables>(), o));
    for (int s = 0; s < 4; ++s)
      PXG_RETURN_IF_ERROR(ScanExclusiveU32(ctx, o.off[s], o.off[s], n + 1, nullptr, scan_tmp.p));
    PXG_RETURN_IF_ERROR(Launch(ctx, "gen_strings", GenStringsKernel, dim3(static_cast<unsigned>((n + kGenBlock - 1) / kGenBlock)),
                               dim3(kGenBlock), 0, seed, g0, n, n_pair_keys, d_tables.as<const Tables>(), o));
    pxg_column_view v[PXG_HTTP_EVENTS_NCOLS];
    std::memset(v, 0, sizeof(v));
    const int fixed_col[6] = {0, 1, 5, 6, 7, 8};
    for (int i = 0; i < 6; ++i) v[fixed_col[i]].values = fixed[i].p;
    const int str_col[4] = {2, 3, 4, 9};
    for (int s = 0; s < 4; ++s) {
      v[str_col[s]].offsets = reinterpret_cast<const int32_t*>(o.off[s]);
      v[str_col[s]].data = o.data[s];
    }
    for (int c = 0; c < PXG_HTTP_EVENTS_NCOLS; ++c) {
      v[c].type = kTypes[c];
      v[c].length = n;
    }
    PXG_RETURN_IF_ERROR(t.AppendRows(v, n, hipMemcpyDeviceToDevice));  // synchronises
    done += n;
  }
  return PXG_OK;
}
