"""Parity at BASELINE sizes (VERDICT r1 "next" #1): the device generator against the host one,
C3 with 10M distinct (pod, remote_addr) keys against the oracle on 20M rows and through
size-independent properties at 100M rows, and the 8-way sharded C2 exchange at 10M rows.
Bars: tests/parity.py."""
import numpy as np
import pytest

import oracle_client as oc
import parity
from golden.make_datagen_hash import digests
from pixie_amd import plans as P
from pixie_amd.device import Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
SEED = 20250117


def _device_table(ctx, row0, n, n_pair_keys=10_000_000):
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, row0, n, n_pair_keys)
    return t


def test_device_generator_matches_host_generator(ctx):
    for row0, n in ((0, 1_000_000), (123_456_789, 300_000)):
        t = _device_table(ctx, row0, n)
        dev = t.fetch_all()
        host = datagen_http_events(SEED, row0, n, n_pair_keys=10_000_000, threads=8)
        assert digests(dev) == digests(host), row0
        t.close()


def _tables(cols):
    return {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}


def test_c3_10m_keys_matches_oracle_on_20m_rows(ctx):
    n = 20_000_000
    cols = datagen_http_events(SEED, 0, n, n_pair_keys=10_000_000, threads=16)
    need = {P.HE[c] for c in ("pod", "remote_addr", "resp_status", "latency", "resp_body_size")}
    ocols = [c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)]
    ref = oc.execute_plan(P.c3_plan(), _tables(ocols))["output"][0]["cols"]
    t = _device_table(ctx, 0, n)
    q = LinearQuery(P.c3_plan(), P.HTTP_TYPES, expected_groups=2_000_000)
    dev = q.run(ctx, t)
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "exact"])
    assert rep["ok"], rep
    assert rep["groups_ref"] > 1_500_000
    t.close()


def test_c3_100m_rows_properties_and_table_growth_without_hint(ctx):
    """100M rows, ~7M groups, no expected_groups hint: the table must grow by groups, not rows
    (ADVICE r1), and sum(count) / #groups / sum(sum) / sum(mean*count) must match numpy."""
    n = 100_000_000
    t = _device_table(ctx, 0, n)
    q = LinearQuery(P.c3_plan(), P.HTTP_TYPES)   # no hint
    agg = q.make_agg(ctx)
    agg.consume(t)
    G = agg.finalize()
    info = agg.info()
    out = agg.result()
    status = t.fetch(P.HE["resp_status"]).values
    sel = np.flatnonzero(status >= 400)
    del status
    assert info["rows_selected"] == len(sel)
    cnt = out[2].values
    assert int(cnt.sum()) == len(sel)
    assert info["table_capacity"] <= 16 * G, info
    pod, addr = t.fetch(P.HE["pod"]), t.fetch(P.HE["remote_addr"])
    h = parity.row_hash64([pod, addr], sel)
    del pod, addr
    assert len(np.unique(h)) == G
    # device group keys are distinct and hash into exactly the same set
    hd = parity.row_hash64(out[:2])
    assert len(np.unique(hd)) == G and np.array_equal(np.unique(hd), np.unique(h))
    body = t.fetch(P.HE["resp_body_size"]).values[sel]
    assert int(out[4].values.sum()) == int(body.sum())
    lat = t.fetch(P.HE["latency"]).values[sel]
    tot = float(np.sum(lat.astype(np.float64)))
    assert abs(float(np.sum(out[3].values * cnt)) - tot) <= 1e-9 * tot
    agg.close()
    t.close()


def test_sharded_c2_8_parts_10m_rows_matches_single_node(ctx):
    import torch
    from pixie_amd.dist import segments
    n, shards = 10_000_000, 8
    cols = datagen_http_events(SEED, 0, n, n_pair_keys=10_000_000, threads=16)
    plan = P.c2_plan(with_pluck=False)
    need = {P.HE[c] for c in ("service", "req_path", "resp_status", "latency")}
    ocols = [c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)]
    ref = oc.execute_plan(plan, _tables(ocols))["output"][0]["cols"]
    q = LinearQuery(plan, P.HTTP_TYPES, expected_groups=65536)
    bounds = [n * s // shards for s in range(shards + 1)]
    tabs, aggs, bufs = [], [], []
    for s in range(shards):
        t = _device_table(ctx, bounds[s], bounds[s + 1] - bounds[s])
        a = q.make_agg(ctx)
        a.consume(t)
        offs, nb = a.export_partial(shards)
        buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
        a.export_partial(shards, buf)
        tabs.append(t)
        aggs.append(a)
        bufs.append((buf, offs, nb))
    parts = []
    for p in range(shards):
        d = q.make_agg(ctx)
        for buf, offs, nb in bufs:
            d.import_partial(buf[offs[p]:offs[p] + nb[p]])
        d.finalize()
        parts.append(d.result())
        d.close()
    dev = parity.concat_columns(parts)
    gv = parity.GroupValues([[cols[2], cols[3]]], [cols[5].values >= 400], [cols[6].values / 1e6])
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep
    assert rep["v2_quantiles"]["groups_rank"] > 0
    for x in aggs + tabs:
        x.close()


def test_c3_full_cardinality_matches_oracle_on_20m_rows(ctx):
    """BASELINE configs[2] without the filter (plans.c3_full_plan): every row aggregated, ~8.6M
    groups of the 10M pairs in 20M rows, through the partitioned high-cardinality path."""
    n = 20_000_000
    cols = datagen_http_events(SEED, 0, n, n_pair_keys=10_000_000, threads=16)
    need = {P.HE[c] for c in ("pod", "remote_addr", "latency", "resp_body_size")}
    ocols = [c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)]
    ref = oc.execute_plan(P.c3_full_plan(), _tables(ocols))["output"][0]["cols"]
    t = _device_table(ctx, 0, n)
    q = LinearQuery(P.c3_full_plan(), P.HTTP_TYPES, expected_groups=n // 2)
    a = q.make_agg(ctx)
    a.consume(t)
    assert a.info()["hc_mode"] == 1
    a.finalize()
    dev = a.result()
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "exact"])
    assert rep["ok"], rep
    assert rep["groups_ref"] > 5_000_000
    a.close()
    t.close()
