"""Pin the CPU restatement (oracle/) to the reference's own known answers (CPU only)."""
import math

import pytest

import oracle_client as oc
from kat import case_plan, case_tables, check_case_output, expected_rows, load_kat, rows, rows_match, ulp_diff

KAT = load_kat()


@pytest.mark.parametrize("case", KAT["cases"], ids=[c["name"] for c in KAT["cases"]])
def test_oracle_matches_reference_kat(case):
    out = oc.execute_plan(case_plan(case), case_tables(case))["out"]
    want = case["output"]["batches"]
    assert len(out) == len(want), f"{case['name']}: {len(out)} batches, want {len(want)}"
    for bi, (g, w) in enumerate(zip(out, want)):
        assert (g["eow"], g["eos"]) == (w["eow"], w["eos"]), f"batch {bi} flags"
        assert [c.type for c in g["cols"]] == case["output"]["types"]
        assert rows_match(rows(g["cols"]), expected_rows(case, bi), case["ordered"], case["tol_ulp"]), \
            f"{case['name']} batch {bi}: {rows(g['cols'])} != {expected_rows(case, bi)}"


@pytest.mark.parametrize("case", KAT["join_cases"], ids=[c["name"] for c in KAT["join_cases"]])
def test_oracle_matches_reference_join_kat(case):
    check_case_output(oc.execute_plan(case_plan(case), case_tables(case))["out"], case)


@pytest.mark.parametrize("q", KAT["quantiles"], ids=["floats", "ints"])
def test_oracle_tdigest_known_answers(q):
    got = oc.tdigest_quantiles(q["input"])
    names = ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]
    for k, v in q["expected"].items():
        assert ulp_diff(got[names.index(k)], float(v)) <= 4, (k, got[names.index(k)], v)


def test_quantiles_json_and_pluck_roundtrip():
    js = oc.quantiles_json([1, 2, 2, 1, 1, 5, 6])
    assert js.startswith('{"p01":') and '"p99":' in js
    assert oc.pluck_float64(js, "p90") == pytest.approx(5.8)
    assert oc.pluck_float64(js, "p50") == 2.0       # rendered "2.0" so rapidjson reads a double
    assert oc.pluck_float64(js, "nope") == 0.0
    assert oc.pluck_float64("not json", "p50") == 0.0


def test_tdigest_single_process_is_order_independent():
    import random
    r = random.Random(7)
    vals = [r.lognormvariate(1.6, 1.0) for _ in range(5000)]
    a = oc.tdigest_quantiles(vals)
    r.shuffle(vals)
    b = oc.tdigest_quantiles(vals)
    assert a == b  # n <= 8000: one process() over the sorted multiset


def test_tdigest_rank_error_large_group():
    import random
    r = random.Random(11)
    vals = [r.lognormvariate(1.6, 1.0) for _ in range(200_000)]
    got = oc.tdigest_quantiles(vals)
    s = sorted(vals)
    n = len(s)
    import bisect
    for q, v in zip([0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99], got):
        rank = (bisect.bisect_left(s, v) + bisect.bisect_right(s, v)) / 2 / n
        assert abs(rank - q) <= math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / n


def test_empty_table_no_groups_agg_emits_one_row():
    from pixie_amd import plans as P
    from pixie_amd.device import Column
    plan = P.linear_plan([P.source_op("t", [2], ["a"], [0]),
                          P.agg_op([], [P.agg_expr("count", [P.col(0)], [2]), P.agg_expr("mean", [P.col(0)], [2], fid=1),
                                        P.agg_expr("sum", [P.col(0)], [2], fid=2)]),
                          P.sink_op("out")])
    out = oc.execute_plan(plan, {"t": {"types": [2], "batches": []}})["out"]
    assert len(out) == 1 and out[0]["rows"] == 1 and out[0]["eos"]
    cnt, mean, s = [c.to_list()[0] for c in out[0]["cols"]]
    assert cnt == 0 and math.isnan(mean) and s == 0


def test_empty_table_group_by_emits_zero_rows():
    from pixie_amd import plans as P
    plan = P.linear_plan([P.source_op("t", [2, 2], ["a", "b"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("sum", [P.col(1)], [2])]), P.sink_op("out")])
    out = oc.execute_plan(plan, {"t": {"types": [2, 2], "batches": []}})["out"]
    assert len(out) == 1 and out[0]["rows"] == 0 and out[0]["eos"]


def test_unknown_udf_is_not_found():
    from pixie_amd import plans as P
    plan = P.linear_plan([P.source_op("t", [2], ["a"], [0]),
                          P.map_op([P.func("frobnicate", [P.col(0)], [2])], ["x"]), P.sink_op("out")])
    with pytest.raises(oc.OracleError) as e:
        oc.execute_plan(plan, {"t": {"types": [2], "batches": []}})
    assert e.value.code == 5


@pytest.mark.parametrize("case", KAT["limit_cases"], ids=[c["name"] for c in KAT["limit_cases"]])
def test_oracle_limit_node_kat(case):
    check_case_output(oc.execute_plan(case_plan(case), case_tables(case))["out"], case)
