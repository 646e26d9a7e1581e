"""Run a linear planpb fragment on the device with the same batch / eow / eos structure the
reference's nodes produce, so results compare batch-for-batch with the oracle."""
from __future__ import annotations

from typing import Dict, List

from pixie_amd.device import Column, Table
from pixie_amd.pipeline import LinearQuery


def _upload(ctx, types, batches) -> Table:
    t = Table(ctx, types)
    for b in batches:
        if len(b) and len(b[0]) > 0:
            t.append(b)
    t.flush()
    return t


def run_plan(ctx, plan, tables: Dict[str, dict], expected_groups: int = 0) -> List[dict]:
    src = plan.nodes[0].nodes[0].op.mem_source_op
    tin = tables[src.name]
    types = tin["types"]
    batches = tin["batches"]
    flags = tin.get("flags") or [(i == len(batches) - 1, i == len(batches) - 1) for i in range(len(batches))]
    q = LinearQuery(plan, types, expected_groups=expected_groups)
    out = []
    if q.agg_op is None:
        for b, (eow, eos) in zip(batches, flags):
            t = _upload(ctx, types, [b])
            cols = q.run(ctx, t)
            t.close()
            out.append({"rows": len(cols[0]) if cols else 0, "eow": eow, "eos": eos, "cols": cols})
        return out
    agg = q.make_agg(ctx)
    window: List = []
    if not batches:
        flags = [(True, True)]
        batches = [[]]
    for b, (eow, eos) in zip(batches, flags):
        window.append(b)
        ready = eos or (eow and q.windowed)   # ReadyToEmitBatches (agg_node.cc:169-171)
        if not ready:
            continue
        t = _upload(ctx, types, [w for w in window if w])
        agg.consume(t)
        agg.finalize()
        cols = q.emit(agg.result())
        out.append({"rows": len(cols[0]) if cols else 0, "eow": eow, "eos": eos, "cols": cols})
        agg.reset()
        t.close()
        window = []
    agg.close()
    return out


def _empty_cols(q):
    return [Column.from_values(t, []) for t in q.out_types]
