"""Multi-GPU exchange of partial aggregation states (PEM-partial / Kelvin-finalize on one node).

The reference splits a distributed aggregate into a partial agg on every PEM and a finalize
agg on Kelvin (src/carnot/planner/distributed/splitter/partial_op_mgr/partial_op_mgr.cc:69-83;
planpb AggregateOperator.partial_agg / finalize_results, src/carnot/planpb/plan.proto:250-257),
joined by GRPCSink -> GRPCSource.  On one MI355X node every rank is both: it aggregates its
row shard, exports its state partitioned by hash(group key) % world, exchanges the parts with
ONE all-to-all(v) and merges what it receives.  Afterwards every group lives on exactly one
rank, so finalize runs locally and the union over ranks is the result.

The production path is libpxg's own communicator (pxg_comm_init over RCCL / xGMI,
pxg_agg_alltoall + pxg_agg_gather).  Where RCCL cannot run -- ranks sharing one GPU, CPU
process groups -- GlooTransport is the byte mover of a host communicator (Comm.host,
pxg_comm_init_host): the SAME libpxg exchange code runs (device part layout, {bytes, header}
records, import with the received headers, gather rebase), only the bytes travel through
torch.distributed gloo.  exchange_partials / gather_device_results are that path.

exchange_partials also keeps a host protocol for objects without a device aggregation (the CPU
stand-ins of tests/test_dist_cpu.py): two all-to-alls, the per-destination byte counts and the
parts themselves.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def _align8(x: int) -> int:
    return (x + 7) & ~7


def segments(offsets: Sequence[int], nbytes: Sequence[int]) -> List[int]:
    """Byte length of each part's segment in the export buffer (parts are 8-byte aligned and
    laid out back to back, include/pxg.h pxg_agg_export_partial)."""
    n = len(offsets)
    return [(offsets[p + 1] - offsets[p]) if p + 1 < n else _align8(nbytes[p]) for p in range(n)]


class GlooTransport:
    """The byte mover of a host communicator (pixie_amd.device.Comm.host): one batch of
    point-to-point transfers between host buffers over a torch.distributed process group
    (gloo: CPU tensors).  The k-th transfer of a rank to a peer carries tag k, so it meets the
    peer's k-th transfer from that rank, the grouped ncclSend / ncclRecv matching rule."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.batches = 0
        self.bytes_moved = 0

    def _global(self, peer: int) -> int:
        return peer if self.group is None else dist.get_global_rank(self.group, peer)

    def __call__(self, ops) -> None:
        reqs = []
        seq = {}
        for peer, is_send, buf in ops:
            k = seq.get((peer, is_send), 0)
            seq[(peer, is_send)] = k + 1
            t = torch.frombuffer(buf, dtype=torch.uint8)
            if is_send:
                reqs.append(dist.isend(t, dst=self._global(peer), group=self.group, tag=k))
            else:
                reqs.append(dist.irecv(t, src=self._global(peer), group=self.group, tag=k))
            self.bytes_moved += len(buf)
        for r in reqs:
            r.wait()
        self.batches += 1


_HOST_COMMS = {}


def host_comm(ctx, group: Optional[dist.ProcessGroup] = None):
    """The host communicator of `ctx` over `group` (created once, collective-free: the ranks
    meet in their first transfer)."""
    from .device import Comm
    key = (id(ctx), id(group))
    c = _HOST_COMMS.get(key)
    if c is None or not c.h:
        c = Comm.host(ctx, dist.get_rank(group), dist.get_world_size(group), GlooTransport(group))
        _HOST_COMMS[key] = c
    return c


def close_host_comms() -> None:
    for c in _HOST_COMMS.values():
        c.close()
    _HOST_COMMS.clear()


def exchange_partials(agg, group: Optional[dist.ProcessGroup] = None) -> Tuple[int, int]:
    """Re-partition `agg`'s state across the ranks of `group` by group-key hash.

    A pixie_amd.device.Agg runs pxg_agg_alltoall over a host communicator on `group` (the RCCL
    path's device code, bytes over gloo).  Any other object with export_partial / import_partial
    / reset / device (the CPU stand-ins) takes the host protocol below.  Returns (bytes sent,
    bytes received)."""
    if hasattr(agg, "alltoall") and getattr(agg, "ctx", None) is not None:
        return agg.alltoall(host_comm(agg.ctx, group))
    world = dist.get_world_size(group)
    comm_dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    agg_dev = torch.device(agg.device)
    offs, nbytes = agg.export_partial(world)
    seg = segments(offs, nbytes)
    total = sum(seg)
    send = torch.empty(max(total, 8), dtype=torch.uint8, device=agg_dev)
    agg.export_partial(world, send)
    send_sizes = torch.tensor(seg, dtype=torch.int64, device=comm_dev)
    recv_sizes = torch.empty(world, dtype=torch.int64, device=comm_dev)
    dist.all_to_all_single(recv_sizes, send_sizes, group=group)
    rs = [int(x) for x in recv_sizes.tolist()]
    recv = torch.empty(max(sum(rs), 8), dtype=torch.uint8, device=comm_dev)
    send_c = send if send.device == comm_dev else send.to(comm_dev)
    dist.all_to_all_single(recv[:sum(rs)], send_c[:total], output_split_sizes=rs, input_split_sizes=seg, group=group)
    if comm_dev.type == "cuda":
        torch.cuda.current_stream(comm_dev).synchronize()
    if recv.device != agg_dev:
        recv = recv.to(agg_dev)
    # Every group this rank exported now lives on its owner; rebuild from the received parts
    # (our own part included: it travelled rank -> rank through the same buffer), all of them in
    # one import call.
    agg.reset()
    offs, sizes, at = [], [], 0
    for src in range(world):
        if rs[src] > 0:
            offs.append(at)
            sizes.append(rs[src])
        at += rs[src]
    if hasattr(agg, "import_partials"):
        agg.import_partials(recv, offs, sizes)
    else:
        for o, z in zip(offs, sizes):
            agg.import_partial(recv[o:o + z])
    return total, sum(rs)


def gather_device_results(agg, group: Optional[dist.ProcessGroup] = None, dst: int = 0) -> int:
    """Every rank's finalized rows to rank `dst` with pxg_agg_gather over the host communicator
    (device-side rebase of the STRING offsets, as on RCCL).  Returns the gathered groups on
    `dst` (0 elsewhere); `agg.result()` on `dst` is then the whole result."""
    return agg.gather(host_comm(agg.ctx, group), dst)


def gather_results(cols: list, group: Optional[dist.ProcessGroup] = None, dst: int = 0) -> Optional[list]:
    """Gather every rank's finalized result columns (host numpy Columns) on rank `dst`
    (the GRPCSink -> Kelvin result stream analogue; sizes are G rows, not N)."""
    world = dist.get_world_size(group)
    objs = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(cols, objs, dst=dst, group=group)
    return objs
