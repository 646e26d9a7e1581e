"""The C++ host engine (libpxcarnot: planpb wire decoder -> ExecNode graph with the GPU nodes at
the operator switch, include/pxcarnot.h).  CPU tests check the lowering (no device); GPU tests
run whole binary plans through it and compare with the reference's golden vectors and with
the CPU Carnot restatement, batch for batch."""
import json
import math

import pytest

import oracle_client as oc
from kat import case_plan, case_tables, expected_rows, load_kat, rows, rows_match, ulp_diff
from pixie_amd import host_engine as H
from pixie_amd import planpb
from pixie_amd import plans as P

KAT = load_kat()
HTTP = {"http_events": {"types": P.HTTP_TYPES, "batches": []}}


def test_library_exports_engine_symbols():
    lib = H.load()
    for s in ["pxc_engine_create", "pxc_engine_destroy", "pxc_execute_plan", "pxc_explain_plan", "pxc_free", "pxc_last_error"]:
        assert hasattr(lib, s), s


def test_c2_plan_lowers_to_one_fused_agg_node():
    txt = H.explain(P.c2_plan(with_pluck=True), HTTP)
    lines = txt.splitlines()
    assert lines[0] == "MemorySourceNode(http_events)"
    assert "GpuAggNode(fused filter/map chain)" in lines[1]
    assert "GpuFilterNode" not in txt and "GpuMapNode" not in txt
    # greaterThanEqual(resp_status INT64, 400) -> COL(INT64) CONST(400) GE_I
    filt = [l for l in lines if l.strip().startswith("filter:")][0].split()[1:]
    assert filt[0].startswith("1:2:") and filt[1] == "2:2:0:400" and filt[2].startswith("35:1:")
    # the substituted Map expression divide(latency, 1e6) is the quantiles / mean argument
    udas = [l for l in lines if "uda kind=" in l]
    assert [u.split()[1] for u in udas] == ["kind=1", "kind=3", "kind=6"]
    assert all(" 23:4:0:0" in u for u in udas[1:])
    assert "PostAggMapNode" in txt and "SinkNode" in txt


def test_filter_map_plan_without_agg_uses_standalone_nodes():
    plan = P.linear_plan([P.source_op("t", [2, 4], ["a", "b"], [0, 1]),
                          P.filter_op(P.func("greaterThan", [P.col(0), P.const(2, 3)], [2, 2]), [0, 1]),
                          P.map_op([P.func("multiply", [P.col(1), P.const(4, 2.0)], [4, 4])], ["m"]), P.sink_op("out")])
    txt = H.explain(plan, {"t": {"types": [2, 4], "batches": []}})
    assert "GpuFilterNode" in txt and "GpuMapNode" in txt and "GpuAggNode" not in txt


def test_unknown_udf_is_not_found_and_bad_bytes_invalid():
    plan = P.linear_plan([P.source_op("t", [2], ["a"], [0]),
                          P.filter_op(P.func("frobnicate", [P.col(0)], [2]), [0]), P.sink_op("out")])
    with pytest.raises(H.PxcError) as e:
        H.explain(plan, {"t": {"types": [2], "batches": []}})
    assert e.value.code == 5 and "frobnicate" in str(e.value)
    lib = H.load()
    import ctypes as C
    out = C.c_void_p()
    t = H._Tables({})
    assert lib.pxc_explain_plan(b"\x12\xff\xff\xff", 4, 0, t.arr, C.byref(out)) == 3


def test_windowed_agg_is_not_fused():
    plan = P.linear_plan([P.source_op("t", [2, 2], ["a", "b"], [0, 1]),
                          P.filter_op(P.func("greaterThan", [P.col(0), P.const(2, 0)], [2, 2]), [0, 1]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [2])], windowed=True), P.sink_op("out")])
    txt = H.explain(plan, {"t": {"types": [2, 2], "batches": []}})
    assert "GpuFilterNode" in txt and "GpuAggNode out=" in txt and "fused" not in txt


@pytest.fixture(scope="module")
def engine():
    e = H.Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", KAT["cases"], ids=[c["name"] for c in KAT["cases"]])
def test_engine_matches_reference_kat(engine, case):
    out = engine.execute(case_plan(case), case_tables(case))["out"]
    want = case["output"]["batches"]
    assert len(out) == len(want)
    for bi, (g, w) in enumerate(zip(out, want)):
        assert (g["eow"], g["eos"]) == (w["eow"], w["eos"])
        assert [c.type for c in g["cols"]] == case["output"]["types"]
        assert rows_match(rows(g["cols"]), expected_rows(case, bi), case["ordered"], case["tol_ulp"]), case["name"]


@pytest.mark.gpu
def test_engine_c2_with_pluck_matches_oracle(engine):
    from pixie_amd.device import datagen_http_events
    cols = datagen_http_events(20250117, 0, 300_000, threads=8)
    batches = [[c.slice(a, min(a + 1024, 300_000)) for c in cols] for a in range(0, 300_000, 1024)]
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": batches, "names": P.HTTP_NAMES}}
    plan = P.c2_plan(with_pluck=True)
    ref = oc.execute_plan(plan, tables)["output"]
    dev = engine.execute(plan, tables)["output"]
    assert len(ref) == len(dev) == 1 and dev[0]["eos"]
    R = {r[:2]: r[2:] for r in rows(ref[0]["cols"])}
    D = {r[:2]: r[2:] for r in rows(dev[0]["cols"])}
    assert set(R) == set(D) and len(R) > 1000
    for k in R:
        assert R[k][0] == D[k][0]                                   # count: exact
        assert abs(R[k][1] - D[k][1]) <= 1e-6 * abs(R[k][1])        # mean: 1e-6 relative
        if R[k][0] <= 8000:
            for a, b in zip(R[k][2:], D[k][2:]):                    # p50 / p99 via pluck_float64
                assert ulp_diff(a, b) <= 4, (k, a, b)


@pytest.mark.gpu
def test_engine_quantiles_json_keys_and_values(engine):
    q = KAT["quantiles"][1]
    plan = P.linear_plan([P.source_op("t", [4], ["v"], [0]),
                          P.agg_op([], [P.agg_expr("quantiles", [P.col(0)], [4])]), P.sink_op("out")])
    from pixie_amd.device import Column
    out = engine.execute(plan, {"t": {"types": [4], "batches": [[Column.from_values(4, [float(x) for x in q["input"]])]]}})
    s = out["out"][0]["cols"][0].to_list()[0]
    got = json.loads(s)
    assert list(got) == ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]
    for k, v in q["expected"].items():
        assert ulp_diff(got[k], float(v)) <= 4
