"""Partial aggregation export / import (the PEM-partial -> Kelvin-finalize split of
src/carnot/planner/distributed/splitter/partial_op_mgr/partial_op_mgr.cc:69-83 on one node):
shards aggregated separately, re-partitioned by group-key hash and merged must give exactly
the single-node aggregate (the oracle of SURVEY.md §8e).  Bars as in test_gpu_parity.py."""
import json
import math

import numpy as np
import pytest

import oracle_client as oc
from kat import rows, ulp_diff
from pixie_amd import plans as P
from pixie_amd.device import Table, datagen_http_events
from pixie_amd.dist import segments
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu


def _by_key(cols, nkeys):
    return {t[:nkeys]: t[nkeys:] for t in rows(cols)}


def _sharded_run(ctx, plan, cols, n_shards, n_parts):
    """Aggregate n_shards row shards separately, export each into n_parts, import part p of
    every shard into destination agg p, finalize every destination; return the union."""
    import torch
    q = LinearQuery(plan, P.HTTP_TYPES)
    n = len(cols[0])
    bounds = [n * s // n_shards for s in range(n_shards + 1)]
    tables, shards = [], []
    for s in range(n_shards):
        t = Table(ctx, P.HTTP_TYPES)
        t.append([c.slice(bounds[s], bounds[s + 1]) for c in cols])
        a = q.make_agg(ctx)
        a.consume(t)
        tables.append(t)
        shards.append(a)
    bufs = []
    for a in shards:
        offs, nb = a.export_partial(n_parts)
        seg = segments(offs, nb)
        buf = torch.empty(max(sum(seg), 8), dtype=torch.uint8, device="cuda")
        offs2, nb2 = a.export_partial(n_parts, buf)
        assert (offs2, nb2) == (offs, nb)
        bufs.append((buf, offs, nb))
    out = []
    total_groups = 0
    for p in range(n_parts):
        d = q.make_agg(ctx)
        for buf, offs, nb in bufs:
            d.import_partial(buf[offs[p]:offs[p] + nb[p]])
        total_groups += d.finalize()
        out.append(q.emit(d.result()))
        d.close()
    for a in shards:
        a.close()
    for t in tables:
        t.close()
    return out, total_groups


@pytest.mark.parametrize("n_shards,n_parts", [(2, 2), (3, 4), (1, 1), (4, 8)])
def test_sharded_c2_matches_single_node(ctx, n_shards, n_parts):
    cols = datagen_http_events(20250117, 0, 240_000, threads=8)
    plan = P.c2_plan(with_pluck=False)
    ref = oc.execute_plan(plan, {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}})["output"][0]["cols"]
    R = _by_key(ref, 2)
    out, ng = _sharded_run(ctx, plan, cols, n_shards, n_parts)
    assert ng == len(R)
    D = {}
    for part in out:
        d = _by_key(part, 2)
        assert not (set(d) & set(D)), "a group landed on two ranks"
        D.update(d)
    assert set(D) == set(R)
    for k in R:
        rc, rm, rq = R[k]
        dc, dm, dq = D[k]
        assert rc == dc, k
        assert abs(rm - dm) <= 1e-6 * abs(rm), (k, rm, dm)
        if rc <= 8000:   # t-digest of <= 8000 values is order independent: exact
            rq, dq = json.loads(rq), json.loads(dq)
            for name in rq:
                assert ulp_diff(rq[name], dq[name]) <= 4, (k, name)


def test_sharded_high_cardinality_string_keys(ctx):
    """C3 shape: (pod, remote_addr) with ~1 row per key, count/mean/sum; also exercises the
    import-side table growth."""
    cols = datagen_http_events(7, 0, 300_000, n_pair_keys=100_000, threads=8)
    plan = P.c3_plan()
    ref = oc.execute_plan(plan, {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}})["output"][0]["cols"]
    R = _by_key(ref, 2)
    out, ng = _sharded_run(ctx, plan, cols, 3, 5)
    D = {}
    for part in out:
        D.update(_by_key(part, 2))
    assert ng == len(R) and set(D) == set(R)
    for k in R:
        assert R[k][0] == D[k][0] and R[k][2] == D[k][2], k
        assert abs(R[k][1] - D[k][1]) <= 1e-6 * abs(R[k][1]), k


def test_import_rejects_foreign_and_truncated_buffers(ctx):
    import torch
    from pixie_amd._lib import PxgError
    cols = datagen_http_events(1, 0, 20_000, threads=4)
    t = Table(ctx, P.HTTP_TYPES)
    t.append(cols)
    a = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES).make_agg(ctx)
    a.consume(t)
    offs, nb = a.export_partial(1)
    buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
    a.export_partial(1, buf)
    other = LinearQuery(P.c1_plan(), P.HTTP_TYPES).make_agg(ctx)   # different key/value types
    with pytest.raises(PxgError):
        other.import_partial(buf[:nb[0]])
    with pytest.raises(PxgError):
        a.import_partial(buf[:nb[0] - 8])
    junk = torch.zeros(128, dtype=torch.uint8, device="cuda")
    with pytest.raises(PxgError):
        a.import_partial(junk)
    for x in (a, other):
        x.close()
    t.close()


def test_batched_import_equals_part_by_part(ctx):
    """pxg_agg_import_partials (every received part in one buffer, one pass) must give exactly
    what importing the parts one by one gives."""
    import torch
    cols = datagen_http_events(99, 0, 300_000, threads=8)
    plan = P.c2_plan(with_pluck=False)
    q = LinearQuery(plan, P.HTTP_TYPES)
    bounds = [0, 80_000, 190_000, 300_000]
    shards, tabs = [], []
    for s in range(3):
        t = Table(ctx, P.HTTP_TYPES)
        t.append([c.slice(bounds[s], bounds[s + 1]) for c in cols])
        a = q.make_agg(ctx)
        a.consume(t)
        shards.append(a)
        tabs.append(t)
    parts = []
    for a in shards:
        offs, nb = a.export_partial(2)
        buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
        a.export_partial(2, buf)
        parts.append((buf, offs, nb))
    for p in range(2):
        one = q.make_agg(ctx)
        for buf, offs, nb in parts:
            one.import_partial(buf[offs[p]:offs[p] + nb[p]])
        one.finalize()
        A = _by_key(q.emit(one.result()), 2)
        segs = [buf[offs[p]:offs[p] + nb[p]] for buf, offs, nb in parts]
        pad = [(len(x) + 7) // 8 * 8 for x in segs]
        cat = torch.zeros(sum(pad), dtype=torch.uint8, device="cuda")
        at, o = 0, []
        for x, w in zip(segs, pad):
            cat[at:at + len(x)] = x
            o.append(at)
            at += w
        batched = q.make_agg(ctx)
        batched.import_partials(cat, o, [len(x) for x in segs])
        batched.finalize()
        B = _by_key(q.emit(batched.result()), 2)
        assert A == B
        one.close()
        batched.close()
    for x in shards + tabs:
        x.close()
