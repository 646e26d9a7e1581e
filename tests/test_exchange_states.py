"""The multi-GPU exchange carries partial UDA states (partial_op_mgr.cc:69-83):
per group and rank one Serialize() state record (count / sum / min / max, MeanInfo for mean),
and for quantiles the raw values when the rank holds <= 8 * delta of them, else the rank's
single-pass centroid list (<= 2 * delta centroids).  The owner merges the states and builds each
group's digest as tdigest's batch add (math_sketches.h:38).

Checked against the CPU restatement: keys, counts, integer sums and min / max bit-exact; float
sums and means 1e-9 relative; quantiles of groups that arrived as raw values only as on one node
(<= 4 ULP up to 8000 values); quantiles of groups that received centroid lists equal to
oracle/tdigest.h merge_batch over the same contributions (1e-12 relative) and inside the rank bound
of the exact quantile."""
import json
import math

import numpy as np
import pytest

import oracle_client as oc
from kat import rows, ulp_diff
from pixie_amd import plans as P
from pixie_amd.device import Column, Table
from pixie_amd.dist import segments
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
NAMES = ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]
QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]
TYPES = [5, 4, 2]


def _plan():
    return P.linear_plan([P.source_op("t", TYPES, ["k", "v", "i"], [0, 1, 2]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [4]), P.agg_expr("mean", [P.col(1)], [4], fid=1),
                                         P.agg_expr("quantiles", [P.col(1)], [4], fid=2), P.agg_expr("sum", [P.col(2)], [2], fid=3),
                                         P.agg_expr("min", [P.col(1)], [4], fid=4), P.agg_expr("max", [P.col(2)], [2], fid=5),
                                         P.agg_expr("sum", [P.col(1)], [4], fid=6)]),
                          P.sink_op("out")])


def _shards(seed=42):
    """3 shards; groups: 'big' (large everywhere), 'lop' (large on shard 0 only), 'mid' (9000
    values, <= 8000 on every shard), and 400 small groups."""
    rng = np.random.default_rng(seed)
    spec = {"big": (40_000, 25_000, 30_000), "lop": (20_000, 900, 0), "mid": (3000, 3000, 3000), "edge": (8000, 8001, 10)}
    shards = []
    for s in range(3):
        keys, vals = [], []
        for k, counts in spec.items():
            keys += [k] * counts[s]
            vals.append(rng.lognormal(1.5, 1.0, counts[s]))
        n_small = 20_000
        keys += [f"s{int(x):03d}" for x in rng.integers(0, 400, n_small)]
        vals.append(rng.normal(0, 10, n_small))
        v = np.concatenate(vals)
        perm = rng.permutation(len(keys))
        keys = [keys[i] for i in perm]
        v = v[perm]
        ints = rng.integers(-(1 << 40), 1 << 40, len(keys))
        shards.append((keys, v, ints))
    return shards


def _by_key(cols):
    return {t[0]: t[1:] for t in rows(cols)}


def test_states_and_digests_merge_like_the_oracle(ctx):
    import torch
    shards = _shards()
    plan = _plan()
    q = LinearQuery(plan, TYPES)
    aggs, tabs, bufs = [], [], []
    for keys, v, ints in shards:
        t = Table(ctx, TYPES)
        t.append([Column.from_values(5, keys), Column(4, values=v), Column.from_values(2, ints.tolist())])
        a = q.make_agg(ctx)
        a.consume(t)
        offs, nb = a.export_partial(2)
        buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
        a.export_partial(2, buf)
        aggs.append(a)
        tabs.append(t)
        bufs.append((buf, offs, nb))
    D = {}
    for p in range(2):
        d = q.make_agg(ctx)
        for buf, offs, nb in bufs:
            d.import_partial(buf[offs[p]:offs[p] + nb[p]])
        d.finalize()
        part = _by_key(q.emit(d.result()))
        assert not (set(part) & set(D))
        D.update(part)
        d.close()
    # single-node oracle over the union
    allk = sum((s[0] for s in shards), [])
    allv = np.concatenate([s[1] for s in shards])
    alli = np.concatenate([s[2] for s in shards])
    tables = {"t": {"types": TYPES, "batches": [[Column.from_values(5, allk), Column(4, values=allv),
                                                 Column.from_values(2, alli.tolist())]]}}
    R = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"])
    assert set(R) == set(D)
    per_shard = []
    for keys, v, _ in shards:
        g = {}
        for k, x in zip(keys, v):
            g.setdefault(k, []).append(x)
        per_shard.append({k: np.asarray(x) for k, x in g.items()})
    n_digest = 0
    for k in R:
        rc, rm, rq, rs, rmin, rmax, rfs = R[k]
        dc, dm, dq, ds, dmin, dmax, dfs = D[k]
        assert (rc, rs, rmin, rmax) == (dc, ds, dmin, dmax), k
        assert abs(rm - dm) <= 1e-9 * abs(rm) and abs(rfs - dfs) <= 1e-9 * abs(rfs), k
        rq, dq = json.loads(rq), json.loads(dq)
        contrib = [per_shard[s][k] for s in range(3) if k in per_shard[s]]
        if all(len(c) <= 8000 for c in contrib):
            if rc <= 8000:
                for name in NAMES:
                    assert ulp_diff(rq[name], dq[name]) <= 4, (k, name)
            continue
        n_digest += 1
        parts = [("raw", c) if len(c) <= 8000 else ("centroids", oc.tdigest_centroids(c)) for c in contrib]
        ref = oc.tdigest_batch_quantiles(parts)
        exact = np.sort(np.concatenate(contrib))
        for name, qv, r in zip(NAMES, QS, ref):
            assert abs(dq[name] - r) <= 1e-12 * max(1.0, abs(r)), (k, name, dq[name], r)
            rank = (np.searchsorted(exact, dq[name], "left") + np.searchsorted(exact, dq[name], "right")) / 2 / len(exact)
            assert abs(rank - qv) <= 2 * math.pi * math.sqrt(qv * (1 - qv)) / 1000 + 1e-3, (k, name)
    assert n_digest == 3  # big, lop, edge
    for x in aggs + tabs:
        x.close()


def test_exchange_ships_fewer_bytes_than_rows(ctx):
    """A shard of 400K rows in few groups: the state parts are a small fraction of the v1 row
    parts (values of groups above 8000 travel as <= 2000 centroids)."""
    import os
    import torch
    keys, v, ints = _shards(7)[0]
    t = Table(ctx, TYPES)
    t.append([Column.from_values(5, keys), Column(4, values=v), Column.from_values(2, ints.tolist())])
    q = LinearQuery(_plan(), TYPES)
    a = q.make_agg(ctx)
    a.consume(t)
    _, nb2 = a.export_partial(4)
    os.environ["PXG_XCHG_V1"] = "1"
    try:
        a.reset()
        a.consume(t)
        _, nb1 = a.export_partial(4)
    finally:
        del os.environ["PXG_XCHG_V1"]
    assert sum(nb2) < 0.6 * sum(nb1), (sum(nb2), sum(nb1))
    a.close()
    t.close()


def test_merged_aggregation_refuses_rows_and_reexport(ctx):
    import torch
    from pixie_amd._lib import PxgError
    keys, v, ints = _shards(9)[1]
    t = Table(ctx, TYPES)
    t.append([Column.from_values(5, keys), Column(4, values=v), Column.from_values(2, ints.tolist())])
    q = LinearQuery(_plan(), TYPES)
    a = q.make_agg(ctx)
    a.consume(t)
    offs, nb = a.export_partial(1)
    buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
    a.export_partial(1, buf)
    with pytest.raises(PxgError):
        a.import_partial(buf[:nb[0]])  # rows already consumed here
    d = q.make_agg(ctx)
    d.import_partial(buf[:nb[0]])
    with pytest.raises(PxgError):
        d.consume(t)
    d.reset()
    d.consume(t)  # after a reset it is an ordinary aggregation again
    assert d.finalize() == a.finalize()
    for x in (a, d, t):
        x.close()
