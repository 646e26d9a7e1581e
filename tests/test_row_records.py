"""In-launch probe records (pixie_amd/csrc/pxg_agg.hip WriteRowRecord; PXG_NO_PREC=1 turns records off): the consume
writes a group's probe record as soon as its inserting lane (or a lane that confirmed the group
against its representative row) has the key in registers, and later probes trust a record only
when it equals their key.  Checked against the CPU restatement on single consumes, on several
consumes into one run (published + in-launch records side by side) and through table growth."""
import numpy as np
import pytest

import oracle_client as oc
import parity
from pixie_amd import plans as P
from pixie_amd.device import Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
SEED = 20250117


def _check(dev, cols_list):
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": cols_list, "names": P.HTTP_NAMES}}
    ref = oc.execute_plan(P.c2_plan(with_pluck=False), tables)["output"][0]["cols"]
    gv = parity.GroupValues([[c[2], c[3]] for c in cols_list], [c[5].values >= 400 for c in cols_list],
                            [c[6].values / 1e6 for c in cols_list])
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep


@pytest.mark.parametrize("expected_groups", [65536, 16])
def test_row_records_single_consume_matches_oracle(ctx, monkeypatch, expected_groups):
    cols = datagen_http_events(SEED, 0, 3_000_000, threads=8)
    t = Table(ctx, P.HTTP_TYPES)
    t.append(cols)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=expected_groups)
    a = q.make_agg(ctx)
    for _ in range(2):  # the second run starts from cleared records
        a.reset()
        a.consume(t)
        a.finalize()
        _check(a.result(), [cols])
    a.close()
    t.close()


def test_row_records_across_consumes_of_two_tables(ctx, monkeypatch):
    """Rows of table B probe groups published from table A (arena records) and groups B inserts
    itself (in-launch records); the same row references name different keys in A and B."""
    ca = datagen_http_events(SEED, 0, 1_500_000, threads=8)
    cb = datagen_http_events(SEED + 1, 5_000_000, 1_500_000, threads=8)
    ta, tb = Table(ctx, P.HTTP_TYPES), Table(ctx, P.HTTP_TYPES)
    ta.append(ca)
    tb.append(cb)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(ta)
    a.consume(tb)
    a.finalize()
    _check(a.result(), [ca, cb])
    a.close()
    ta.close()
    tb.close()


def test_row_records_same_result_as_without(ctx, monkeypatch):
    """Group set and counts identical with and without in-launch records on the same table."""
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, 20_000_000, 10_000_000)
    out = []
    for on in ("0", "1"):
        if on == "0":
            monkeypatch.setenv("PXG_NO_PREC", "1")
        else:
            monkeypatch.delenv("PXG_NO_PREC", raising=False)
        q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
        a = q.make_agg(ctx)
        a.consume(t)
        a.finalize()
        r = a.result()
        keys = parity.key_rows(r[:2], [max(int(np.diff(c.offsets).max()), 1) for c in r[:2]])
        o = np.argsort(keys, kind="stable")
        out.append((keys[o], np.asarray(r[2].values)[o], np.asarray(r[3].values)[o]))
        a.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert np.allclose(out[0][2], out[1][2], rtol=1e-12, atol=0)
    t.close()
