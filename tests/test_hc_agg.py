"""High-cardinality mode (pixie_amd/csrc/pxg_hc.hip): partition records + per-partition LDS
tables instead of the global table.  Forced at small sizes with PXG_HC_MIN_GROUPS=1 and a
group-count hint; every case is checked against the oracle (keys and integer results
bit-exact, means 1e-6 relative: the mode divides the exact integer sum)."""
import numpy as np
import pytest

import oracle_client as oc
from device_runner import run_plan
from kat import rows, rows_match
from pixie_amd import plans as P
from pixie_amd.device import Column, Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
SEED = 20250117


@pytest.fixture
def hc_env(monkeypatch):
    monkeypatch.setenv("PXG_HC_MIN_GROUPS", "1")
    monkeypatch.delenv("PXG_HC_PBITS", raising=False)
    return monkeypatch


def _http(nrows, n_pair_keys):
    cols = datagen_http_events(SEED, 0, nrows, n_pair_keys=n_pair_keys, threads=8)
    return {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}, cols


def _by_key(cols, nkeys):
    return {t[:nkeys]: t[nkeys:] for t in rows(cols)}


def _check_c3(R, D):
    assert set(R) == set(D)
    for k in R:
        assert R[k][0] == D[k][0] and R[k][2] == D[k][2], k
        assert abs(R[k][1] - D[k][1]) <= 1e-6 * abs(R[k][1]), k


def _c3_agg(ctx, t, hint):
    q = LinearQuery(P.c3_plan(), P.HTTP_TYPES, expected_groups=hint)
    a = q.make_agg(ctx)
    a.consume(t)
    return q, a


def test_c3_partitioned_matches_oracle(ctx, hc_env):
    tables, cols = _http(600_000, 200_000)
    ref = _by_key(oc.execute_plan(P.c3_plan(), tables)["output"][0]["cols"], 2)
    t = Table(ctx, P.HTTP_TYPES)
    t.append(cols)
    q, a = _c3_agg(ctx, t, 100_000)
    info = a.info()
    assert info["hc_mode"] == 1 and info["table_capacity"] <= 1 << 16, info
    g = a.finalize()
    assert a.info()["hc_partition_bits"] > 0
    dev = _by_key(q.emit(a.result()), 2)
    assert g == len(ref) > 40_000
    _check_c3(ref, dev)
    # the same agg again after a reset (decided per run; workspaces reused)
    a.reset()
    a.consume(t)
    assert a.info()["hc_mode"] == 1
    a.finalize()
    _check_c3(ref, _by_key(q.emit(a.result()), 2))
    a.close()
    t.close()


def test_partition_overflow_reruns_with_more_partitions(ctx, hc_env):
    """Two partitions for ~6K groups overflow the 1024-entry LDS tables: the pass reruns with
    4x the partitions until every partition fits, and the result is unchanged."""
    tables, cols = _http(60_000, 20_000)
    ref = _by_key(oc.execute_plan(P.c3_plan(), tables)["output"][0]["cols"], 2)
    hc_env.setenv("PXG_HC_PBITS", "1")
    t = Table(ctx, P.HTTP_TYPES)
    t.append(cols)
    q, a = _c3_agg(ctx, t, 10_000)
    a.finalize()
    assert a.info()["hc_partition_bits"] >= 3
    _check_c3(ref, _by_key(q.emit(a.result()), 2))
    a.close()
    t.close()


def test_long_keys_take_the_table_path_alongside(ctx, hc_env):
    """Keys over 24 bytes leave holes in the partition records and go through the table path;
    both halves are emitted together and stay disjoint (a key is long or it is not)."""
    rng = np.random.default_rng(3)
    n = 80_000
    short = [f"s{i:05d}" for i in range(3000)]
    long_ = ["L" * 25 + f"{i:04d}" for i in range(500)] + ["x" * 24, "y" * 23 + "z", ""]
    pool = short + long_
    k1 = [pool[i] for i in rng.integers(0, len(pool), n)]
    k2 = [("q" * int(l)) for l in rng.integers(0, 30, n)]
    v = rng.integers(-1000, 1000, n)
    plan = P.linear_plan([P.source_op("t", [5, 5, 2], ["k", "k2", "v"], [0, 1, 2]),
                          P.filter_op(P.func("greaterThan", [P.col(2), P.const(2, -900)], [2, 2]), [0, 1, 2]),
                          P.agg_op([0, 1], [P.agg_expr("count", [P.col(2)], [2]), P.agg_expr("sum", [P.col(2)], [2], fid=1),
                                            P.agg_expr("min", [P.col(2)], [2], fid=2), P.agg_expr("max", [P.col(2)], [2], fid=3),
                                            P.agg_expr("mean", [P.col(2)], [2], fid=4)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 5, 2], "batches": [[Column.from_values(5, k1), Column.from_values(5, k2),
                                                     Column.from_values(2, v.tolist())]]}}
    ref = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 2)
    dev = _by_key(run_plan(ctx, plan, tables, expected_groups=50_000)[0]["cols"], 2)
    assert len(ref) > 20_000 and set(ref) == set(dev)
    for k in ref:
        assert ref[k][:4] == dev[k][:4], k
        assert abs(ref[k][4] - dev[k][4]) <= 1e-9 * abs(ref[k][4]) + 1e-12, k


def test_fixed_width_keys_and_integer_udas(ctx, hc_env):
    """INT64 / BOOLEAN / UINT128 / TIME64NS keys with count, sum, min, max, mean over INT64 and
    BOOLEAN arguments (every accumulator kind the LDS tables hold)."""
    rng = np.random.default_rng(8)
    n = 50_000
    ik = rng.integers(0, 4000, n)
    bk = rng.integers(0, 2, n).astype(bool)
    uk = [int(x) << 64 | int(y) for x, y in zip(rng.integers(0, 3, n), rng.integers(0, 5, n))]
    tk = rng.integers(0, 7, n) * 1_000_000_000
    v = rng.integers(-(1 << 40), 1 << 40, n)
    bv = rng.integers(0, 2, n).astype(bool)
    types = [2, 1, 3, 6, 2, 1]
    batch = [Column.from_values(2, ik.tolist()), Column.from_values(1, bk.tolist()), Column.from_values(3, uk),
             Column.from_values(6, tk.tolist()), Column.from_values(2, v.tolist()), Column.from_values(1, bv.tolist())]
    tables = {"t": {"types": types, "batches": [batch]}}
    for gcols in ([0, 1], [2, 3], [0, 2, 1]):
        plan = P.linear_plan([P.source_op("t", types, [f"c{i}" for i in range(6)], list(range(6))),
                              P.agg_op(gcols, [P.agg_expr("count", [P.col(4)], [2]), P.agg_expr("sum", [P.col(4)], [2], fid=1),
                                               P.agg_expr("min", [P.col(4)], [2], fid=2), P.agg_expr("max", [P.col(4)], [2], fid=3),
                                               P.agg_expr("sum", [P.col(5)], [1], fid=4)]),
                              P.sink_op("out")])
        ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
        dev = run_plan(ctx, plan, tables, expected_groups=10_000)[0]["cols"]
        assert rows_match(rows(dev), rows(ref), ordered=False, tol_ulp=0), gcols
        plan = P.linear_plan([P.source_op("t", types, [f"c{i}" for i in range(6)], list(range(6))),
                              P.agg_op(gcols, [P.agg_expr("mean", [P.col(4)], [2]), P.agg_expr("mean", [P.col(5)], [1], fid=1)]),
                              P.sink_op("out")])
        R = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], len(gcols))
        D = _by_key(run_plan(ctx, plan, tables, expected_groups=10_000)[0]["cols"], len(gcols))
        assert set(R) == set(D)
        for k in R:
            for a, b in zip(R[k], D[k]):
                assert abs(a - b) <= 1e-9 * abs(a) + 1e-12, (gcols, k, a, b)


def test_empty_selection_and_multiple_consumes(ctx, hc_env):
    tables, cols = _http(200_000, 50_000)
    ref = _by_key(oc.execute_plan(P.c3_plan(), tables)["output"][0]["cols"], 2)
    t1, t2 = Table(ctx, P.HTTP_TYPES), Table(ctx, P.HTTP_TYPES)
    t1.append([c.slice(0, 70_000) for c in cols])
    t2.append([c.slice(70_000, 200_000) for c in cols])
    q = LinearQuery(P.c3_plan(), P.HTTP_TYPES, expected_groups=20_000)
    a = q.make_agg(ctx)
    a.consume(t1, 0, 0)  # an empty range first
    a.consume(t1)
    a.consume(t2)
    assert a.info()["hc_mode"] == 1 and a.rows_selected() == sum(c for c, _, _ in ref.values())
    a.finalize()
    _check_c3(ref, _by_key(q.emit(a.result()), 2))
    # nothing selected: zero groups
    empty = P.linear_plan([P.source_op("http_events", P.HTTP_TYPES, P.HTTP_NAMES, list(range(10))),
                           P.filter_op(P.func("greaterThan", [P.col(5), P.const(2, 10_000)], [2, 2]), list(range(10))),
                           P.agg_op([8, 9], [P.agg_expr("count", [P.col(6)], [2])]), P.sink_op("out")])
    qe = LinearQuery(empty, P.HTTP_TYPES, expected_groups=20_000)
    ae = qe.make_agg(ctx)
    ae.consume(t1)
    assert ae.finalize() == 0
    for x in (a, ae, t1, t2):
        x.close()


def test_export_partition_groups_without_spill(ctx, hc_env):
    """export_partial on a high-cardinality run sends the partition pass's groups as states (no
    spill into the table: the run stays in partition mode); the parts merged on 4 importers
    equal the single-agg result."""
    import torch
    from pixie_amd.dist import segments
    tables, cols = _http(300_000, 100_000)
    ref = _by_key(oc.execute_plan(P.c3_plan(), tables)["output"][0]["cols"], 2)
    q = LinearQuery(P.c3_plan(), P.HTTP_TYPES, expected_groups=50_000)
    shards, parts = 3, 4
    bounds = [300_000 * s // shards for s in range(shards + 1)]
    tabs, bufs, aggs = [], [], []
    for s in range(shards):
        t = Table(ctx, P.HTTP_TYPES)
        t.append([c.slice(bounds[s], bounds[s + 1]) for c in cols])
        a = q.make_agg(ctx)
        a.consume(t)
        assert a.info()["hc_mode"] == 1
        offs, nb = a.export_partial(parts)
        assert a.info()["hc_mode"] == 1
        buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
        a.export_partial(parts, buf)
        tabs.append(t)
        aggs.append(a)
        bufs.append((buf, offs, nb))
    out = {}
    for p in range(parts):
        d = q.make_agg(ctx)
        for buf, offs, nb in bufs:
            d.import_partial(buf[offs[p]:offs[p] + nb[p]])
        d.finalize()
        part = _by_key(q.emit(d.result()), 2)
        assert not (set(part) & set(out))
        out.update(part)
        d.close()
    _check_c3(ref, out)
    for x in aggs + tabs:
        x.close()


def test_export_mixes_table_and_partition_groups(ctx, hc_env):
    """A run whose long keys took the table path exports both halves: table groups (states from
    the export finalize) and partition groups (states from the partition pass) share the parts,
    and 3 importers merging 2 shards each reproduce the oracle."""
    import torch
    from pixie_amd.dist import segments
    rng = np.random.default_rng(5)
    n = 90_000
    short = [f"s{i:05d}" for i in range(4000)]
    long_ = ["L" * 25 + f"{i:04d}" for i in range(400)]
    pool = short + long_
    k1 = [pool[i] for i in rng.integers(0, len(pool), n)]
    k2 = [("q" * int(l)) for l in rng.integers(0, 8, n)]
    v = rng.integers(-1000, 1000, n)
    types = [5, 5, 2]
    plan = P.linear_plan([P.source_op("t", types, ["k", "k2", "v"], [0, 1, 2]),
                          P.agg_op([0, 1], [P.agg_expr("count", [P.col(2)], [2]), P.agg_expr("sum", [P.col(2)], [2], fid=1),
                                            P.agg_expr("min", [P.col(2)], [2], fid=2), P.agg_expr("max", [P.col(2)], [2], fid=3),
                                            P.agg_expr("mean", [P.col(2)], [2], fid=4)]),
                          P.sink_op("out")])
    cols = [Column.from_values(5, k1), Column.from_values(5, k2), Column.from_values(2, v.tolist())]
    tables = {"t": {"types": types, "batches": [cols], "names": ["k", "k2", "v"]}}
    ref = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 2)
    q = LinearQuery(plan, types, expected_groups=30_000)
    parts, bufs, keep = 3, [], []
    for lo, hi in ((0, n // 2), (n // 2, n)):
        t = Table(ctx, types)
        t.append([c.slice(lo, hi) for c in cols])
        a = q.make_agg(ctx)
        a.consume(t)
        assert a.info()["hc_mode"] == 1
        offs, nb = a.export_partial(parts)
        buf = torch.empty(max(sum(segments(offs, nb)), 8), dtype=torch.uint8, device="cuda")
        a.export_partial(parts, buf)
        bufs.append((buf, offs, nb))
        keep += [a, t]
    out = {}
    for p in range(parts):
        d = q.make_agg(ctx)
        for buf, offs, nb in bufs:
            d.import_partial(buf[offs[p]:offs[p] + nb[p]])
        d.finalize()
        part = _by_key(q.emit(d.result()), 2)
        assert not (set(part) & set(out))
        out.update(part)
        d.close()
    assert len(ref) > 10_000 and set(ref) == set(out)
    assert any(len(k[0]) > 24 for k in ref)
    for k in ref:
        assert ref[k][:4] == out[k][:4], k
        assert abs(ref[k][4] - out[k][4]) <= 1e-9 * abs(ref[k][4]) + 1e-12, k
    for x in keep:
        x.close()


def test_partitions_of_many_batches(ctx, hc_env):
    """Two partitions of ~25K records (a few hundred groups each): every partition takes many
    record batches, and the representative keys are re-read at emit (the multi-batch path)."""
    hc_env.setenv("PXG_HC_PBITS", "1")
    rng = np.random.default_rng(21)
    n = 50_000
    keys = [f"k{int(i)}" for i in rng.integers(0, 600, n)]
    ik = rng.integers(0, 3, n)
    v = rng.integers(-50, 50, n)
    types = [5, 2, 2]
    plan = P.linear_plan([P.source_op("t", types, ["k", "i", "v"], [0, 1, 2]),
                          P.agg_op([0, 1], [P.agg_expr("count", [P.col(2)], [2]), P.agg_expr("sum", [P.col(2)], [2], fid=1),
                                            P.agg_expr("max", [P.col(2)], [2], fid=2)]),
                          P.sink_op("out")])
    tables = {"t": {"types": types, "batches": [[Column.from_values(5, keys), Column.from_values(2, ik.tolist()),
                                                 Column.from_values(2, v.tolist())]]}}
    ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
    dev = run_plan(ctx, plan, tables, expected_groups=1000)[0]["cols"]
    assert len(rows(ref)) > 1500
    assert rows_match(rows(dev), rows(ref), ordered=False, tol_ulp=0)


def test_all_empty_and_short_string_keys(ctx, hc_env):
    """The partition pass keeps only the words the longest staged key needs: a key column of
    empty strings keeps none (the record is the lengths word alone), short keys keep one."""
    rng = np.random.default_rng(9)
    n = 30_000
    ints = rng.integers(0, 2000, n)
    short = [f"{int(i) % 97:x}" for i in rng.integers(0, 1 << 30, n)]
    v = rng.integers(0, 100, n)
    types = [5, 2, 5, 2]
    batch = [Column.from_values(5, [""] * n), Column.from_values(2, ints.tolist()), Column.from_values(5, short),
             Column.from_values(2, v.tolist())]
    tables = {"t": {"types": types, "batches": [batch]}}
    for gcols in ([0], [0, 1], [2, 0], [2, 1]):
        plan = P.linear_plan([P.source_op("t", types, ["e", "i", "s", "v"], [0, 1, 2, 3]),
                              P.agg_op(gcols, [P.agg_expr("count", [P.col(3)], [2]), P.agg_expr("sum", [P.col(3)], [2], fid=1)]),
                              P.sink_op("out")])
        ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
        dev = run_plan(ctx, plan, tables, expected_groups=5000)[0]["cols"]
        assert rows_match(rows(dev), rows(ref), ordered=False, tol_ulp=0), gcols


def _agg_hc(ctx, plan, tables, hint):
    """run_plan through one agg, returning (cols, info) so a test can see which mode ran."""
    src = plan.nodes[0].nodes[0].op.mem_source_op
    tin = tables[src.name]
    q = LinearQuery(plan, tin["types"], expected_groups=hint)
    t = Table(ctx, tin["types"])
    for b in tin["batches"]:
        t.append(b)
    t.flush()
    a = q.make_agg(ctx)
    a.consume(t)
    info = a.info()
    a.finalize()
    cols = q.emit(a.result())
    a.close()
    t.close()
    return cols, info


def test_int64_mean_past_2_63_does_not_wrap(ctx, hc_env):
    """MeanUDA accumulates `double sum += arg` (math_ops.h:586-589), so a group whose INT64 sum
    passes 2^63 still has the right mean.  The partition tables sum MEAN arguments as exact
    128-bit integers; the table path sums doubles: both must match the oracle, and each other.
    (SUM over INT64 wraps in the reference, and here, bit-exactly.)"""
    rng = np.random.default_rng(62)
    ngroups = 6000
    sizes = rng.integers(2, 9, ngroups)
    gid = np.repeat(np.arange(ngroups), sizes)
    rng.shuffle(gid)
    n = len(gid)
    sign = np.where(np.arange(ngroups) % 3 == 0, -1, 1)  # a third of the groups all negative
    mag = (1 << 62) - rng.integers(0, 1 << 40, n)
    v = [int(sign[g]) * int(m) for g, m in zip(gid, mag)]
    keys = [f"g{int(g):05d}" for g in gid]
    types = [5, 2]
    plan = P.linear_plan([P.source_op("t", types, ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("mean", [P.col(1)], [2]), P.agg_expr("sum", [P.col(1)], [2], fid=1),
                                         P.agg_expr("count", [P.col(1)], [2], fid=2)]),
                          P.sink_op("out")])
    tables = {"t": {"types": types, "batches": [[Column.from_values(5, keys), Column.from_values(2, v)]]}}
    R = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 1)
    hc_cols, hc_info = _agg_hc(ctx, plan, tables, 5000)
    assert hc_info["hc_mode"] == 1, hc_info
    H = _by_key(hc_cols, 1)
    hc_env.setenv("PXG_NO_HC", "1")
    tb_cols, tb_info = _agg_hc(ctx, plan, tables, 5000)
    assert tb_info["hc_mode"] == 0, tb_info
    T = _by_key(tb_cols, 1)
    assert set(R) == set(H) == set(T) and len(R) == ngroups
    wrapped = 0
    for k, (mean, s, c) in R.items():
        assert H[k][1:] == (s, c) and T[k][1:] == (s, c), k  # sum wraps identically, counts exact
        assert abs(H[k][0] - mean) <= 1e-9 * abs(mean), (k, H[k][0], mean)
        assert abs(T[k][0] - mean) <= 1e-9 * abs(mean), (k, T[k][0], mean)
        assert abs(H[k][0] - T[k][0]) <= 1e-12 * abs(mean), k
        wrapped += (mean > 0) != (s > 0)
    assert wrapped > 1000  # most groups' 64-bit sums wrapped; the means did not


def test_every_key_long_leaves_no_partition_groups(ctx, hc_env):
    """All STRING keys longer than the records hold: every staged record is a hole, the
    partition pass finds no group, and the table path's groups and key offsets stand alone."""
    rng = np.random.default_rng(24)
    n = 20_000
    pool = ["K" * 30 + f"{i:05d}" for i in range(700)]
    keys = [pool[i] for i in rng.integers(0, len(pool), n)]
    v = rng.integers(-1000, 1000, n)
    types = [5, 2]
    plan = P.linear_plan([P.source_op("t", types, ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [2]), P.agg_expr("sum", [P.col(1)], [2], fid=1)]),
                          P.sink_op("out")])
    tables = {"t": {"types": types, "batches": [[Column.from_values(5, keys), Column.from_values(2, v.tolist())]]}}
    ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
    cols, info = _agg_hc(ctx, plan, tables, 5000)
    assert info["hc_mode"] == 1, info
    off = cols[0].offsets if hasattr(cols[0], "offsets") else None
    if off is not None:
        assert list(off)[-1] == sum(len(s) for s in cols[0].to_list())
    assert rows_match(rows(cols), rows(ref), ordered=False, tol_ulp=0)


@pytest.mark.parametrize("kinds", [["mean", "mean", "mean", "mean"], ["mean", "mean", "mean", "sum"]])
def test_four_accumulators_with_wide_means_fit_lds(ctx, hc_env, kinds):
    """The widest high-cardinality plans: 4 INT64 MEANs (each with a 128-bit LDS sum: 77,824 B of
    LDS per hc_agg workgroup) and 3 MEANs + 1 SUM run partitioned and match the oracle."""
    rng = np.random.default_rng(11)
    n = 80_000
    types = [2, 2, 2, 2]
    batch = [Column.from_values(2, rng.integers(0, 9000, n).tolist())] + \
            [Column.from_values(2, rng.integers(-(1 << 50), 1 << 50, n).tolist()) for _ in range(3)]
    tables = {"t": {"types": types, "batches": [batch]}}
    plan = P.linear_plan([P.source_op("t", types, [f"c{i}" for i in range(4)], list(range(4))),
                          P.agg_op([0], [P.agg_expr(k, [P.col(1 + (i % 3))], [2], fid=i) for i, k in enumerate(kinds)]),
                          P.sink_op("out")])
    R = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 1)
    t = Table(ctx, types)
    t.append(batch)
    q = LinearQuery(plan, types, expected_groups=10_000)
    a = q.make_agg(ctx)
    a.consume(t)
    assert a.info()["hc_mode"] == 1
    a.finalize()
    D = _by_key(q.emit(a.result()), 1)
    assert set(R) == set(D)
    for k in R:
        for kind, x, y in zip(kinds, R[k], D[k]):
            if kind == "sum":
                assert x == y, k
            else:
                assert abs(x - y) <= 1e-9 * abs(x) + 1e-12, (k, x, y)
    a.close()
    t.close()
