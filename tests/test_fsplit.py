"""The fused split (pixie_amd/csrc/pxg_finalize.hip FsHistKernel / FsScatterKernel): the largest
groups by a sample get their own bucket in a 9-bit first radix pass, the rest records are
sorted by their low digit in the same pass and by the higher digits after it.  Both this and the
plain radix sort are stable sorts of the same staging, so the grouped value streams -- and every
result, means and big-group quantiles included -- are bit-identical between them (forced on and
off with PXG_FSPLIT on one consume's staging).  Also checked against the CPU restatement."""
import numpy as np
import pytest

import oracle_client as oc
import parity
from pixie_amd import plans as P
from pixie_amd.device import Column, Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
SEED = 20250117


def _finalize_with(monkeypatch, agg, on):
    monkeypatch.setenv("PXG_FSPLIT", "1" if on else "0")
    agg.finalize()
    return agg.result()


def _same(a, b, nk):
    """Identical rows (group order differs: designated groups take the last ids)."""
    assert len(a) == len(b) and len(a[0]) == len(b[0])
    w = [max(int(np.diff(c.offsets).max()), 1) if c.offsets is not None else 0 for c in a[:nk]]
    ka, kb = parity.key_rows(a[:nk], w), parity.key_rows(b[:nk], w)
    oa, ob = np.argsort(ka, kind="stable"), np.argsort(kb, kind="stable")
    assert np.array_equal(ka[oa], kb[ob])
    for x, y in zip(a[nk:], b[nk:]):
        assert np.array_equal(np.asarray(x.values)[oa].view(np.uint8), np.asarray(y.values)[ob].view(np.uint8))


@pytest.mark.parametrize("rows", [6_000_000, 25_000_000])
def test_fused_split_bit_identical_to_radix(ctx, monkeypatch, rows):
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, rows, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(t)
    R = _finalize_with(monkeypatch, a, False)
    D = _finalize_with(monkeypatch, a, True)
    _same(R, D, 2)
    a.close()
    t.close()


def test_fused_split_every_group_designated_or_rest(ctx, monkeypatch):
    """1024 groups (group by req_path): up to 255 designated, the rest needs one more pass."""
    cols = datagen_http_events(SEED, 0, 2_000_000, threads=8)
    types = P.HTTP_TYPES
    plan = P.linear_plan([P.source_op("http_events", types, P.HTTP_NAMES, list(range(len(types)))),
                          P.agg_op([P.HE["req_path"]], [P.agg_expr("count", [P.col(P.HE["latency"])], [2]),
                                                        P.agg_expr("sum", [P.col(P.HE["latency"])], [2], fid=1),
                                                        P.agg_expr("quantiles", [P.col(P.HE["latency"])], [2], fid=2)]),
                          P.sink_op("out")])
    t = Table(ctx, types)
    t.append(cols)
    q = LinearQuery(plan, types, expected_groups=4096)
    a = q.make_agg(ctx)
    a.consume(t)
    R = _finalize_with(monkeypatch, a, False)
    D = _finalize_with(monkeypatch, a, True)
    _same(R, D, 1)
    assert len(R[0]) > 767  # more groups than designated buckets (~1015 distinct paths)
    a.close()
    t.close()


def test_fused_split_c2_matches_oracle(ctx, monkeypatch):
    monkeypatch.setenv("PXG_FSPLIT", "1")
    cols = datagen_http_events(SEED, 0, 4_000_000, threads=8)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    plan = P.c2_plan(with_pluck=False)
    ref = oc.execute_plan(plan, tables)["output"][0]["cols"]
    t = Table(ctx, P.HTTP_TYPES)
    t.append(cols)
    q = LinearQuery(plan, P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(t)
    a.finalize()
    gv = parity.GroupValues([[cols[2], cols[3]]], [cols[5].values >= 400], [cols[6].values / 1e6])
    rep = parity.compare_agg(a.result(), ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep
    a.close()
    t.close()
