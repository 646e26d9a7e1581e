"""Multi-GPU exchange of partial aggregation states (PEM-partial / Kelvin-finalize on one node).

Each rank aggregates its row shard into partial UDA states, exports them partitioned by
hash(group key) % world (pxg_agg_export_partial), exchanges them with one all-to-all(v)
(torch.distributed over RCCL/xGMI on GPU, gloo on CPU), and merges what it receives
(pxg_agg_import_partial).  After the exchange every group lives on exactly one rank.
"""
from __future__ import annotations


def exchange_partials(agg, world: int, rank: int, ctx) -> None:
    raise NotImplementedError("partial-state exchange lands with pxg_agg_export_partial")
