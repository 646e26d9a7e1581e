"""Multi-GPU exchange of partial aggregation states (PEM-partial / Kelvin-finalize on one node).

The reference splits a distributed aggregate into a partial agg on every PEM and a finalize
agg on Kelvin (src/carnot/planner/distributed/splitter/partial_op_mgr/partial_op_mgr.cc:69-83;
planpb AggregateOperator.partial_agg / finalize_results, src/carnot/planpb/plan.proto:250-257),
joined by GRPCSink -> GRPCSource.  On one MI355X node every rank is both: it aggregates its
row shard, exports its state partitioned by hash(group key) % world (pxg_agg_export_partial),
exchanges the parts with ONE all-to-all(v) -- torch.distributed over RCCL/xGMI on GPU ("nccl"),
gloo on CPU -- and merges what it receives (pxg_agg_import_partial).  Afterwards every group
lives on exactly one rank, so finalize runs locally and the union over ranks is the result.

Two collectives per exchange: an all-to-all of the per-destination byte counts (world int64s)
and the all-to-all(v) of the parts themselves.  No other collective is on the data path.
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


def exchange_partials(agg, group: Optional[dist.ProcessGroup] = None) -> Tuple[int, int]:
    """Re-partition `agg`'s state across the ranks of `group` by group-key hash.

    `agg` is a pixie_amd.device.Agg (or any object with the same export_partial /
    import_partial / reset / device interface).  Returns (bytes sent, bytes received)."""
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


def gather_results(cols: list, group: Optional[dist.ProcessGroup] = None, dst: int = 0) -> Optional[list]:
    """Gather every rank's finalized result columns (host numpy Columns) on rank `dst`
    (the GRPCSink -> Kelvin result stream analogue; sizes are G rows, not N)."""
    world = dist.get_world_size(group)
    objs = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(cols, objs, dst=dst, group=group)
    return objs
