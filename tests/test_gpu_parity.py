"""Device parity: the HIP path (through the libpxg C ABI) against the CPU Carnot restatement
and the reference's golden vectors.  Bars: keys / counts / filters / integer results
bit-exact; float sum/mean 1e-6 relative; quantiles bit-exact (<= 4 ULP) for groups of
<= 8000 values, within the t-digest rank bound above that."""
import bisect
import math

import numpy as np
import pytest

import oracle_client as oc
from device_runner import run_plan
from kat import case_plan, case_tables, expected_rows, load_kat, rows, rows_match, ulp_diff
from pixie_amd import _lib
from pixie_amd import plans as P
from pixie_amd.device import Agg, Column, Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
KAT = load_kat()
QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]


@pytest.mark.parametrize("case", KAT["cases"], ids=[c["name"] for c in KAT["cases"]])
def test_device_matches_reference_kat(ctx, case):
    out = run_plan(ctx, case_plan(case), case_tables(case))
    want = case["output"]["batches"]
    assert len(out) == len(want)
    for bi, (g, w) in enumerate(zip(out, want)):
        assert (g["eow"], g["eos"]) == (w["eow"], w["eos"])
        assert [c.type for c in g["cols"]] == case["output"]["types"]
        assert rows_match(rows(g["cols"]), expected_rows(case, bi), case["ordered"], case["tol_ulp"]), \
            f"{case['name']} batch {bi}: {rows(g['cols'])} != {expected_rows(case, bi)}"


@pytest.mark.parametrize("q", KAT["quantiles"], ids=["floats", "ints"])
def test_device_quantiles_known_answers(ctx, q):
    plan = P.linear_plan([P.source_op("t", [4], ["v"], [0]),
                          P.agg_op([], [P.agg_expr("quantiles", [P.col(0)], [4])]), P.sink_op("out")])
    vals = [float(x) for x in q["input"]]
    out = run_plan(ctx, plan, {"t": {"types": [4], "batches": [[Column.from_values(4, vals)]]}})
    import json
    got = json.loads(out[0]["cols"][0].to_list()[0])
    for k, v in q["expected"].items():
        assert ulp_diff(got[k], float(v)) <= 4, (k, got[k], v)


def _http_tables(nrows, batch_rows=None, n_pair_keys=10_000_000, seed=20250117):
    cols = datagen_http_events(seed, 0, nrows, n_pair_keys=n_pair_keys, threads=8)
    if batch_rows is None:
        batches = [cols]
    else:
        batches = [[c.slice(a, min(a + batch_rows, nrows)) for c in cols] for a in range(0, nrows, batch_rows)]
    return {"http_events": {"types": P.HTTP_TYPES, "batches": batches, "names": P.HTTP_NAMES}}, cols


def _by_key(cols, nkeys):
    r = rows(cols)
    return {t[:nkeys]: t[nkeys:] for t in r}


def _rank(sorted_vals, v):
    n = len(sorted_vals)
    return (bisect.bisect_left(sorted_vals, v) + bisect.bisect_right(sorted_vals, v)) / 2 / n


def test_c2_query_parity(ctx):
    tables, cols = _http_tables(400_000, batch_rows=50_000)
    plan = P.c2_plan(with_pluck=False)
    ref = oc.execute_plan(plan, tables)["output"]
    dev = run_plan(ctx, plan, tables)
    assert len(ref) == len(dev) == 1
    R = _by_key(ref[0]["cols"], 2)
    D = _by_key(dev[0]["cols"], 2)
    assert set(R) == set(D)
    import json
    # group values for the rank checks
    sel = cols[5].values >= 400
    svc = np.array(cols[2].to_list(), dtype=object)[sel]
    path = np.array(cols[3].to_list(), dtype=object)[sel]
    lat = cols[6].values[sel] / 1e6
    groups = {}
    for s, p, v in zip(svc, path, lat):
        groups.setdefault((s, p), []).append(v)
    n_exact = 0
    for k in R:
        rc, rm, rq = R[k]
        dc, dm, dq = D[k]
        assert rc == dc, k
        assert abs(rm - dm) <= 1e-6 * abs(rm), (k, rm, dm)
        rq, dq = json.loads(rq), json.loads(dq)
        n = rc
        if n <= 8000:
            for name in rq:
                assert ulp_diff(rq[name], dq[name]) <= 4, (k, name, rq[name], dq[name])
            n_exact += 1
        else:
            s = sorted(groups[k])
            for q, name in zip(QS, ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]):
                bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / n
                assert abs(_rank(s, dq[name]) - _rank(s, rq[name])) <= bound, (k, name)
    assert n_exact > 100


def test_c2_with_pluck_matches(ctx):
    tables, _ = _http_tables(100_000)
    plan = P.c2_plan(with_pluck=True)
    ref = oc.execute_plan(plan, tables)["output"][0]
    dev = run_plan(ctx, plan, tables)[0]
    R = _by_key(ref["cols"], 2)
    D = _by_key(dev["cols"], 2)
    assert set(R) == set(D)
    for k in R:
        assert R[k][0] == D[k][0]
        for a, b in zip(R[k][2:], D[k][2:]):   # p50, p99 through pluck_float64
            assert ulp_diff(a, b) <= 4, (k, a, b)


def test_c1_groupby_service(ctx):
    tables, _ = _http_tables(200_000, batch_rows=100)
    plan = P.c1_plan()
    ref = oc.execute_plan(plan, tables)["output"][0]
    dev = run_plan(ctx, plan, tables)[0]
    R, D = _by_key(ref["cols"], 1), _by_key(dev["cols"], 1)
    assert set(R) == set(D)
    for k in R:
        assert R[k][0] == D[k][0]
        assert abs(R[k][1] - D[k][1]) <= 1e-6 * abs(R[k][1])


def test_c3_high_cardinality_with_table_growth(ctx):
    tables, _ = _http_tables(600_000, n_pair_keys=200_000)
    plan = P.c3_plan()
    ref = oc.execute_plan(plan, tables)["output"][0]
    dev = run_plan(ctx, plan, tables, expected_groups=16)[0]  # forces deferral + rehash growth
    R, D = _by_key(ref["cols"], 2), _by_key(dev["cols"], 2)
    assert len(R) > 40_000
    assert set(R) == set(D)
    for k in R:
        assert R[k][0] == D[k][0] and R[k][2] == D[k][2]
        assert abs(R[k][1] - D[k][1]) <= 1e-6 * abs(R[k][1])


def test_big_group_quantiles_rank_bound_and_exact_small(ctx):
    rng = np.random.default_rng(5)
    n_big = 150_000
    keys = ["big"] * n_big + ["g8000"] * 8000 + ["g1500"] * 1500 + ["g3"] * 3
    vals = np.concatenate([rng.lognormal(1.6, 1.0, n_big), rng.lognormal(1.0, 0.5, 8000), rng.normal(0, 1, 1500),
                           np.array([3.0, -0.0, 0.0])])
    perm = rng.permutation(len(keys))
    keys = [keys[i] for i in perm]
    vals = vals[perm]
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [4]), P.agg_expr("count", [P.col(1)], [4], fid=1)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 4], "batches": [[Column.from_values(5, keys), Column(4, values=vals)]]}}
    ref = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 1)
    dev = _by_key(run_plan(ctx, plan, tables)[0]["cols"], 1)
    import json
    for k in ref:
        rq, dq = json.loads(ref[k][0]), json.loads(dev[k][0])
        assert ref[k][1] == dev[k][1]
        if ref[k][1] <= 8000:
            for name in rq:
                assert ulp_diff(rq[name], dq[name]) <= 4, (k, name, rq[name], dq[name])
        else:
            s = sorted(vals[[i for i, kk in enumerate(keys) if kk == k[0]]])
            n = len(s)
            for q, name in zip(QS, ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]):
                bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / n
                assert abs(_rank(s, dq[name]) - _rank(s, rq[name])) <= bound, (k, name, dq[name], rq[name])


def test_nan_and_signed_zero_and_key_types(ctx):
    nan = float("nan")
    f = [1.5, nan, -0.0, 0.0, 2.5, nan, 7.0, -3.0]
    bkey = [True, False, True, False, True, False, True, False]
    fkey = [0.0, -0.0, 0.0, -0.0, 1.5, 1.5, nan, nan]
    ukey = [1, 1 << 70, 1, 1 << 70, 5, 5, 5, 1]
    skey = ["", "", "a" * 70, "a" * 70, "a" * 69 + "b", "x", "", "x"]
    types = [1, 4, 3, 5, 4]
    batch = [Column.from_values(1, bkey), Column.from_values(4, fkey), Column.from_values(3, ukey),
             Column.from_values(5, skey), Column.from_values(4, f)]
    for gcols in ([0], [1], [2], [3], [0, 3], [1, 2, 3]):
        plan = P.linear_plan([P.source_op("t", types, [f"c{i}" for i in range(5)], list(range(5))),
                              P.agg_op(gcols, [P.agg_expr("count", [P.col(4)], [4]), P.agg_expr("sum", [P.col(4)], [4], fid=1),
                                               P.agg_expr("min", [P.col(4)], [4], fid=2), P.agg_expr("max", [P.col(4)], [4], fid=3),
                                               P.agg_expr("quantiles", [P.col(4)], [4], fid=4)]),
                              P.sink_op("out")])
        tables = {"t": {"types": types, "batches": [batch]}}
        ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
        dev = run_plan(ctx, plan, tables)[0]["cols"]
        assert rows_match(rows(dev), rows(ref), ordered=False, tol_ulp=4), (gcols, rows(dev), rows(ref))


def test_int64_sum_wraps_and_minmax_init(ctx):
    big = 2**62
    vals = [big, big, big, -5]
    plan = P.linear_plan([P.source_op("t", [2], ["a"], [0]),
                          P.agg_op([], [P.agg_expr("sum", [P.col(0)], [2]), P.agg_expr("max", [P.col(0)], [2], fid=1),
                                        P.agg_expr("min", [P.col(0)], [2], fid=2)]), P.sink_op("out")])
    tables = {"t": {"types": [2], "batches": [[Column.from_values(2, vals)]]}}
    ref = rows(oc.execute_plan(plan, tables)["out"][0]["cols"])
    dev = rows(run_plan(ctx, plan, tables)[0]["cols"])
    assert ref == dev
    # MaxUDA<FLOAT64> init is numeric_limits<double>::min() (math_ops.h:699)
    plan = P.linear_plan([P.source_op("t", [4], ["a"], [0]),
                          P.agg_op([], [P.agg_expr("max", [P.col(0)], [4])]), P.sink_op("out")])
    tables = {"t": {"types": [4], "batches": [[Column.from_values(4, [-1.0, -2.0])]]}}
    assert rows(run_plan(ctx, plan, tables)[0]["cols"]) == rows(oc.execute_plan(plan, tables)["out"][0]["cols"])


def test_standalone_filter_map_random(ctx):
    tables, _ = _http_tables(150_000, batch_rows=40_000)
    plan = P.linear_plan([P.source_op("http_events", P.HTTP_TYPES, P.HTTP_NAMES, list(range(10))),
                          P.filter_op(P.func("logicalAnd", [P.func("greaterThanEqual", [P.col(5), P.const(2, 400)], [2, 2]),
                                                            P.func("notEqual", [P.col(2), P.const(5, "ns01/svc-037")], [5, 5])],
                                             [1, 1]), [0, 2, 3, 5, 6, 9, 1]),
                          P.map_op([P.col(1), P.col(2), P.func("divide", [P.col(4), P.const(4, 1e6)], [2, 4]),
                                    P.func("bin", [P.col(0), P.const(2, 10_000_000)], [6, 2]), P.col(6), P.col(5)],
                                   ["svc", "path", "lat_ms", "t10", "upid", "pod"]),
                          P.sink_op("out")])
    ref = oc.execute_plan(plan, tables)["out"]
    dev = run_plan(ctx, plan, tables)
    assert len(ref) == len(dev)
    for a, b in zip(ref, dev):
        assert (a["eow"], a["eos"]) == (b["eow"], b["eos"])
        assert rows(a["cols"]) == rows(b["cols"])   # bit-exact, order preserved


def test_multiple_consumes_and_small_batch_coalescing(ctx):
    cols = datagen_http_events(77, 0, 60_000, threads=4)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES)
    t1 = Table(ctx, P.HTTP_TYPES)
    for a in range(0, 30_000, 100):      # reference-sized 100-row RowBatches
        t1.append([c.slice(a, a + 100) for c in cols])
    t1.flush()
    assert t1.num_rows == 30_000
    t2 = Table(ctx, P.HTTP_TYPES)
    t2.append([c.slice(30_000, 60_000) for c in cols])
    agg = q.make_agg(ctx)
    agg.consume(t1)
    agg.consume(t2)
    agg.finalize()
    two = _by_key(q.emit(agg.result()), 2)
    t3 = Table(ctx, P.HTTP_TYPES)
    t3.append(cols)
    one = _by_key(q.run(ctx, t3), 2)
    assert set(one) == set(two)
    for k in one:
        assert one[k][0] == two[k][0] and one[k][2] == two[k][2]
        assert abs(one[k][1] - two[k][1]) <= 1e-9 * abs(one[k][1])
    for c in range(10):
        assert t1.fetch(c).to_list() == cols[c].slice(0, 30_000).to_list()


def test_unsupported_signature_fails_loudly(ctx):
    from pixie_amd.compile import UnsupportedError
    plan = P.linear_plan([P.source_op("t", [5], ["s"], [0]), P.agg_op([], [P.agg_expr("max", [P.col(0)], [5])]),
                          P.sink_op("out")])
    with pytest.raises(UnsupportedError):
        LinearQuery(plan, [5])


def test_long_and_empty_string_keys_take_the_deferred_path(ctx):
    """Group keys longer than the fast path's register budget (48 B) are deferred to the generic
    kernel; empty strings and keys differing only past byte 48 must stay distinct groups."""
    rng = np.random.default_rng(11)
    n = 60_000
    base = "x" * 48
    pool = ["", "a", base, base + "1", base + "2", "y" * 100, "y" * 99 + "z", "k" * 47, "k" * 49]
    keys = [pool[i] for i in rng.integers(0, len(pool), n)]
    keys2 = [("p" * int(l)) for l in rng.integers(0, 60, n)]
    vals = rng.integers(0, 1000, n)
    plan = P.linear_plan([P.source_op("t", [5, 5, 2], ["k", "k2", "v"], [0, 1, 2]),
                          P.filter_op(P.func("greaterThan", [P.col(2), P.const(2, 100)], [2, 2]), [0, 1, 2]),
                          P.agg_op([0, 1], [P.agg_expr("count", [P.col(2)], [2]), P.agg_expr("sum", [P.col(2)], [2], fid=1)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 5, 2], "batches": [[Column.from_values(5, keys), Column.from_values(5, keys2),
                                                     Column.from_values(2, vals.tolist())]]}}
    ref = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 2)
    dev = _by_key(run_plan(ctx, plan, tables)[0]["cols"], 2)
    assert len(ref) > 400 and set(ref) == set(dev)
    for k in ref:
        assert ref[k] == dev[k], k


@pytest.mark.gpu
def test_device_join_hot_key_and_scale(ctx):
    """pxg_join at scale against numpy: 2M probe rows x 50K build rows with one hot key holding
    20K build rows (one probe row fans out to 20K outputs), UINT128 keys, unmatched rows on both
    sides.  Checks the row count, per-row match counts, the probe-order / build-order layout and
    an order-independent checksum of the gathered payloads."""
    import numpy as np
    from pixie_amd.device import Column, Table
    rng = np.random.default_rng(5)
    nb, npb = 50_000, 2_000_000
    bkey = rng.integers(0, 40_000, nb).astype(np.uint64)
    bkey[:20_000] = 7                                  # hot key
    bpay = rng.integers(0, 1 << 40, nb).astype(np.int64)
    pkey = rng.integers(0, 45_000, npb).astype(np.uint64)
    pkey[rng.integers(0, npb, 20)] = 7                 # a few probe rows hit the hot key
    ppay = np.arange(npb, dtype=np.int64)
    u128 = lambda k: Column(_lib.UINT128, values=np.ascontiguousarray(np.stack([k, k ^ np.uint64(0xABCDEF)], axis=1)))  # noqa: E731
    B = Table(ctx, [_lib.UINT128, _lib.INT64]); B.append([u128(bkey), Column(_lib.INT64, values=bpay)]); B.flush()
    Pt = Table(ctx, [_lib.UINT128, _lib.INT64]); Pt.append([u128(pkey), Column(_lib.INT64, values=ppay)]); Pt.flush()
    out, nprobe = B.join(Pt, [0], [0], [(0, 1), (1, 1)])
    cnt = np.bincount(bkey.astype(np.int64), minlength=50_000)
    per = cnt[pkey.astype(np.int64)]
    assert out.num_rows == nprobe == int(per.sum())
    pp = out.fetch(0).values
    bp = out.fetch(1).values
    # probe rows appear in table order, each repeated per match
    assert np.array_equal(pp, np.repeat(ppay, per))
    # within one probe row, build rows follow build-table order
    order = np.argsort(bkey, kind="stable")
    starts = np.concatenate([[0], np.cumsum(cnt)])
    first = np.flatnonzero(pkey == 7)[0]
    o0 = int(per[:first].sum())
    assert np.array_equal(bp[o0:o0 + cnt[7]], bpay[order[starts[7]:starts[8]]])
    # checksum of build payloads over all output rows
    sums = np.bincount(bkey.astype(np.int64), weights=bpay.astype(np.float64), minlength=50_000)
    assert abs(float(bp.astype(np.float64).sum()) - float(sums[pkey.astype(np.int64)].sum())) < 1e-3 * float(bp.sum())
    out.close(); B.close(); Pt.close()


def test_standalone_filter_string_lengths(ctx):
    """Filter compaction of STRING columns whose lengths cover every copy path of the payload
    gather (0..3 bytes, 4..7, 8..15, 16..48, > 48) next to INT64 / BOOLEAN / UINT128 columns,
    bit-exact and in order against the CPU restatement (FilterNode, filter_node.cc:78-171)."""
    rng = np.random.default_rng(41)
    n = 70_000
    lens = np.concatenate([np.arange(0, 130), rng.integers(0, 130, n - 130)])
    alphabet = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789/-_.", dtype=np.uint8)
    strs = [alphabet[rng.integers(0, len(alphabet), L)].tobytes().decode() for L in lens]
    keep = rng.integers(0, 2, n)
    cols = [Column(2, values=keep.astype(np.int64)), Column.from_values(5, strs),
            Column(1, values=(rng.integers(0, 2, n)).astype(np.uint8)),
            Column.from_values(3, [(int(a) << 64) | int(b) for a, b in zip(rng.integers(0, 2**62, n), rng.integers(0, 2**62, n))])]
    tables = {"t": {"types": [2, 5, 1, 3], "batches": [cols]}}
    plan = P.linear_plan([P.source_op("t", [2, 5, 1, 3], ["k", "s", "b", "u"], [0, 1, 2, 3]),
                          P.filter_op(P.func("equal", [P.col(0), P.const(2, 1)], [2, 2]), [1, 2, 3, 0]),
                          P.sink_op("out")])
    ref = oc.execute_plan(plan, tables)["out"]
    dev = run_plan(ctx, plan, tables)
    assert len(ref) == len(dev) == 1
    assert rows(ref[0]["cols"]) == rows(dev[0]["cols"])
    assert dev[0]["rows"] == int(keep.sum())


@pytest.mark.gpu
def test_standalone_filter_across_chunks_and_launches(ctx, monkeypatch):
    """pxg_filter over a device-generated table of two chunks (2^24 + 300_001 rows), with one
    chunk per launch (PXG_FILTER_BATCH=1) and with both in one launch: the selected rows of
    resp_status >= 400 (service, req_path, latency, resp_status) equal numpy's filter of the
    fetched input columns, in order, bit for bit; a range [begin, end) crossing the chunk
    boundary keeps the same rows."""
    from pixie_amd.compile import ExprCompiler
    n = (1 << 24) + 300_001
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, n, 10_000_000)
    assert t.num_chunks == 2
    comp = ExprCompiler(P.HTTP_TYPES)
    pred = comp.compile(P.func("greaterThanEqual", [P.col(P.HE["resp_status"]), P.const(2, 400)], [2, 2]))
    sel = [P.HE["service"], P.HE["req_path"], P.HE["latency"], P.HE["resp_status"]]
    status = t.fetch(P.HE["resp_status"]).values
    inp = {c: t.fetch(c) for c in sel}

    def want(begin, end):
        keep = np.flatnonzero(status[begin:end] >= 400) + begin
        out = []
        for c in sel:
            col = inp[c]
            if col.type == 5:
                o = col.offsets.astype(np.int64)
                lens = o[keep + 1] - o[keep]
                starts = np.repeat(o[keep], lens)
                within = np.arange(int(lens.sum())) - np.repeat(np.cumsum(lens) - lens, lens)
                out.append((np.concatenate([[0], np.cumsum(lens)]), col.data[starts + within]))
            else:
                out.append(col.values[keep])
        return keep.size, out

    for batch, (begin, end) in [("1", (0, n)), ("8", (0, n)), ("1", ((1 << 24) - 77_777, n - 5))]:
        monkeypatch.setenv("PXG_FILTER_BATCH", batch)
        f = t.filter(pred, sel, begin, end)
        m, exp = want(begin, end)
        assert f.num_rows == m
        for j, c in enumerate(sel):
            got = f.fetch(j)
            if got.type == 5:
                assert np.array_equal(got.offsets.astype(np.int64), exp[j][0])
                assert np.array_equal(got.data[:got.offsets[-1]], exp[j][1])
            else:
                assert np.array_equal(got.values, exp[j])
        f.close()
    t.close()


@pytest.mark.gpu
def test_probe_records_match_plain_consume(ctx, monkeypatch):
    """The probe-record path (records written inside the consume launch by inserting and
    confirming lanes, WriteRowRecord; published groups' records from publication) gives the same
    groups, counts, means and quantiles as the plain consume (PXG_NO_PREC=1), with a second
    consume into the same run (records of published groups, new groups inserted beside them)."""
    from pixie_amd.pipeline import LinearQuery
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, 12_000_000, 10_000_000)
    t2 = Table(ctx, P.HTTP_TYPES)
    t2.append_http_events(20250117, 12_000_000, 3_000_000, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)

    def run(records):
        if not records:
            monkeypatch.setenv("PXG_NO_PREC", "1")
        a = q.make_agg(ctx)
        a.consume(t)
        a.consume(t2)
        a.finalize()
        out = sorted(map(tuple, zip(*[c.to_list() for c in a.result()])))
        a.close()
        monkeypatch.delenv("PXG_NO_PREC", raising=False)
        return out

    plain, rec = run(False), run(True)
    assert len(plain) == len(rec) > 40_000
    for x, y in zip(plain, rec):
        assert x[:3] == y[:3], (x, y)
        assert abs(x[3] - y[3]) <= 1e-9 * abs(x[3])
        if x[2] <= 8000:
            assert x[4] == y[4], (x, y)
    t.close()
    t2.close()
