"""Streaming MemorySource (memory_source_node.cc:58-124): an infinite_stream cursor has no stop
(unless stop_time is set), its RowBatches never carry eow / eos, and the exec loop keeps pulling
it while a batch is ready (exec_graph.cc:205-224).  Inside one engine call no data can arrive
after the call starts (appends go through the same engine), so the query runs until the source
has sent what the table holds -- or until a Limit aborts it, which is what ends a streaming
query in the reference -- and then returns, like a streaming query cancelled at that point.  A
blocking agg under a stream never sees eos and so emits nothing; the engine does not fuse it."""
import numpy as np
import pytest

from pixie_amd import host_engine as H
from pixie_amd import plans as P
from pixie_amd.device import Column

I, T, S = P.INT64, P.TIME64NS, P.STRING
TYPES, NAMES = [T, S, I], ["time_", "svc", "lat"]


def _cols(n, seed=1):
    rng = np.random.default_rng(seed)
    t = 1_000_000 + np.arange(n, dtype=np.int64) * 10
    return [Column(T, values=t), Column.from_values(S, [f"s{x}" for x in rng.integers(0, 20, n)]),
            Column(I, values=rng.integers(0, 1000, n).astype(np.int64))]


def _rows(cols):
    out = []
    for r in range(len(cols[0].values) if cols[0].values is not None else len(cols[0].offsets) - 1):
        row = []
        for c in cols:
            row.append(bytes(c.data[c.offsets[r]:c.offsets[r + 1]]).decode() if c.type == S else int(c.values[r]))
        out.append(tuple(row))
    return out


def _agg_plan(streaming):
    return P.linear_plan([P.source_op("t", TYPES, NAMES, [1, 2], streaming=streaming),
                          P.filter_op(P.func("greaterThan", [P.col(1), P.const(I, 10)], [I, I]), [0, 1]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [I])], ["svc"], ["n"]), P.sink_op("out")])


def test_streaming_agg_is_not_fused_on_cpu():
    host = {"t": {"types": TYPES, "names": NAMES, "batches": []}}
    assert "fused" in H.explain(_agg_plan(False), host)
    assert "fused" not in H.explain(_agg_plan(True), host)


@pytest.fixture
def engine():
    e = H.Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
def test_stored_stream_sends_the_table_without_eos(engine):
    n = 150_000
    cols = _cols(n)
    engine.create_table("t", TYPES, NAMES)
    for a in range(0, n, 20_000):
        engine.append("t", [c.slice(a, min(n, a + 20_000)) for c in cols])
    start = 1_000_000 + 10 * 4321
    plan = P.linear_plan([P.source_op("t", TYPES, NAMES, [0, 1, 2], start_time=start, streaming=True),
                          P.filter_op(P.func("greaterThan", [P.col(2), P.const(I, 500)], [I, I]), [0, 1, 2]),
                          P.sink_op("out")])
    out = engine.execute(plan)["out"]
    assert out and not any(b["eow"] or b["eos"] for b in out)
    got = [r for b in out for r in _rows(b["cols"])]
    want = [r for r in _rows(cols) if r[0] >= start and r[2] > 500]
    assert got == want
    # the same source, bounded by stop_time: the cursor stops there, still without eos
    stop = 1_000_000 + 10 * 90_000
    plan = P.linear_plan([P.source_op("t", TYPES, NAMES, [0, 2], start_time=start, stop_time=stop, streaming=True),
                          P.sink_op("out")])
    out = engine.execute(plan)["out"]
    assert not any(b["eos"] for b in out)
    assert [r[0] for b in out for r in _rows(b["cols"])] == [r[0] for r in _rows(cols) if start <= r[0] <= stop]
    # a blocking agg under the stream never sees eos: nothing comes out
    assert engine.execute(_agg_plan(True))["out"] == []
    assert len(engine.execute(_agg_plan(False))["out"]) == 1


@pytest.mark.gpu
def test_limit_ends_the_stream(engine):
    n = 100_000
    cols = _cols(n, seed=2)
    engine.create_table("t", TYPES, NAMES)
    engine.append("t", cols)
    plan = P.linear_plan([P.source_op("t", TYPES, NAMES, [0, 1, 2], streaming=True),
                          P.limit_op(70_000, [0, 1, 2], abortable_srcs=[1]), P.sink_op("out")])
    out = engine.execute(plan)["out"]
    assert sum(b["rows"] for b in out) == 70_000
    assert out[-1]["eos"] and out[-1]["eow"] and not any(b["eos"] for b in out[:-1])
    assert [r for b in out for r in _rows(b["cols"])] == _rows(cols)[:70_000]


@pytest.mark.gpu
def test_host_table_stream_clears_the_batch_flags(engine):
    cols = _cols(9_000, seed=3)
    batches = [[c.slice(a, a + 3000) for c in cols] for a in range(0, 9000, 3000)]
    plan = P.linear_plan([P.source_op("t", TYPES, NAMES, [0, 2], streaming=True), P.sink_op("out")])
    out = engine.execute(plan, {"t": {"types": TYPES, "names": NAMES, "batches": batches}})["out"]
    assert [(b["rows"], b["eow"], b["eos"]) for b in out] == [(3000, False, False)] * 3
    empty = engine.execute(plan, {"t": {"types": TYPES, "names": NAMES, "batches": []}})["out"]
    assert empty == []
