"""ExecNodeStats through the C++ engine (exec_node.h:41-125, carnot.cc:379-420): per-node rows /
bytes / batches in and out (bytes as RowBatch::NumBytes: fixed widths, STRING lengths), total
and self time, extra metrics, and the query's bytes_processed / rows_processed."""
import numpy as np
import pytest

from pixie_amd import host_engine as H
from pixie_amd import plans as P
from pixie_amd.device import Column, datagen_http_events

pytestmark = pytest.mark.gpu


def _num_bytes(cols, lo, hi):
    b = 0
    for c in cols:
        if c.type == 5:
            b += int(c.offsets[hi]) - int(c.offsets[lo])
        elif c.type == 1:
            b += hi - lo
        else:
            b += 8 * (hi - lo)
    return b


def test_filter_map_node_stats():
    rng = np.random.default_rng(1)
    n = 30_000
    a = rng.integers(0, 10, n)
    s = [f"s{x}" * int(x % 3 + 1) for x in rng.integers(0, 1000, n)]
    f = rng.normal(size=n)
    cols = [Column(2, values=a.astype(np.int64)), Column.from_values(5, s), Column(4, values=f)]
    bounds = [0, 7000, 19_000, n]
    batches = [[Column(2, values=cols[0].values[lo:hi]), Column.from_values(5, s[lo:hi]), Column(4, values=f[lo:hi])]
               for lo, hi in zip(bounds, bounds[1:])]
    pred = P.func("greaterThan", [P.col(0), P.const(2, 5)], [2, 2])
    plan = P.linear_plan([P.source_op("t", [2, 5, 4], ["a", "s", "f"], [0, 1, 2]),
                          P.filter_op(pred, [0, 1, 2]),
                          P.map_op([P.func("multiply", [P.col(2), P.const(4, 2.0)], [4, 4]), P.col(1)], ["f2", "s"]),
                          P.sink_op("out")])
    e = H.Engine(0)
    try:
        e.set_analyze(True)
        out = e.execute(plan, {"t": {"types": [2, 5, 4], "batches": batches}})["out"]
        st = e.last_stats()
    finally:
        e.close()
    kept = int((a > 5).sum())
    assert sum(b["rows"] for b in out) == kept
    nodes = {x["node_id"]: x for x in st["nodes"]}
    src, flt, mp, snk = nodes[1], nodes[2], nodes[3], nodes[4]
    assert st["rows_processed"] == n and src["records_output"] == n
    assert st["bytes_processed"] == src["bytes_output"] == _num_bytes(cols, 0, n)
    assert src["batches_output"] == 3 and flt["batches_input"] == 3
    assert flt["records_input"] == n and flt["bytes_input"] == src["bytes_output"]
    assert flt["records_output"] == kept == mp["records_input"] == mp["records_output"] == snk["records_input"]
    sel = a > 5
    kept_bytes = 8 * kept + sum(len(x) for x, k in zip(s, sel) if k)
    assert mp["bytes_output"] == kept_bytes  # f2 (8 B) + s
    for x in (src, flt, mp, snk):
        assert x["total_execution_time_ns"] >= x["self_execution_time_ns"] >= 0
        assert x["extra_metrics"]["batches_output"] == x["batches_output"]
    assert src["total_execution_time_ns"] > 0


def test_fused_c2_over_the_store_reports_the_table_and_groups():
    n = 500_000
    cols = datagen_http_events(20250117, 0, n, n_pair_keys=10_000_000, threads=8)
    e = H.Engine(0)
    try:
        e.create_table("http_events", P.HTTP_TYPES, P.HTTP_NAMES)
        e.append("http_events", cols)
        e.set_analyze(False)
        out = e.execute(P.c2_plan(with_pluck=True))["output"]
        st0 = e.last_stats()
        e.set_analyze(True)
        e.execute(P.c2_plan(with_pluck=True))
        st = e.last_stats()
    finally:
        e.close()
    groups = sum(b["rows"] for b in out)
    for s in (st0, st):
        assert s["rows_processed"] == n
        # the stored columns the plan reads: service, req_path, resp_status, latency
        need = [P.HE[c] for c in ("service", "req_path", "resp_status", "latency")]
        assert s["bytes_processed"] == _num_bytes([cols[i] for i in need], 0, n)
    agg = [x for x in st["nodes"] if x["name"].startswith("GpuAggNode")][0]
    assert len(agg["fused_node_ids"]) == 2  # the Filter and the Map
    assert agg["records_output"] == groups and agg["extra_metrics"]["groups"] == groups
    assert agg["extra_metrics"]["rows_aggregated"] == int((cols[P.HE["resp_status"]].values >= 400).sum())
    assert st0["nodes"][0]["total_execution_time_ns"] == 0  # timers only under analyze
