"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/pxg.h declares,
and the host-only pieces (datagen, expression compiler) behave.  No GPU compute here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from pixie_amd import _lib, planpb
from pixie_amd import compile as pc
from pixie_amd import plans as P
from pixie_amd.device import HTTP_EVENTS_SCHEMA, datagen_http_events

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "pxg.h")).read()
    return sorted(set(re.findall(r"\b(pxg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    declared = header_functions()
    assert declared, "no functions parsed from include/pxg.h"
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(_lib.EXPORTED) == declared


def test_abi_version_and_errors():
    lib = _lib.load()
    assert lib.pxg_abi_version() == 1
    # a call that fails before touching the device
    rc = lib.pxg_ctx_create(0, None)
    assert rc == 3  # INVALID_ARGUMENT
    assert b"null" in lib.pxg_last_error()


def test_status_codes_match_reference_numbering():
    src = open(os.path.join(REPO, "include", "pxg.h")).read()
    want = {"OK": 0, "CANCELLED": 1, "UNKNOWN": 2, "INVALID_ARGUMENT": 3, "DEADLINE_EXCEEDED": 4, "NOT_FOUND": 5,
            "ALREADY_EXISTS": 6, "INTERNAL": 9, "UNIMPLEMENTED": 10, "RESOURCE_UNAVAILABLE": 11}
    for k, v in want.items():
        assert re.search(rf"PXG_{k} = {v}\b", src), k


def test_datagen_deterministic_and_shardable():
    a = datagen_http_events(20250117, 0, 20000, threads=3)
    b = datagen_http_events(20250117, 0, 20000, threads=5)
    s1 = datagen_http_events(20250117, 0, 7000, threads=2)
    s2 = datagen_http_events(20250117, 7000, 13000, threads=2)
    for i, (name, t) in enumerate(HTTP_EVENTS_SCHEMA):
        assert a[i].to_list() == b[i].to_list(), name
        assert s1[i].to_list() + s2[i].to_list() == a[i].to_list(), name


def test_datagen_distribution_matches_spec():
    cols = datagen_http_events(20250117, 0, 200_000, threads=8)
    status = cols[5].values
    sel = (status >= 400).mean()
    assert 0.11 < sel < 0.13
    lat = cols[6].values
    assert lat.min() >= 1000 and lat.max() <= 2_000_000_000
    assert 4.5e6 < np.median(lat) < 5.5e6
    svc_len = np.diff(cols[2].offsets)
    assert (svc_len == 12).all()
    path_len = np.diff(cols[3].offsets).mean()
    assert 15 < path_len < 35
    assert len(set(cols[2].to_list())) <= 64
    assert len(set(cols[3].to_list())) <= 1024


def test_compile_registry_resolution():
    types = [t for _, t in HTTP_EVENTS_SCHEMA]
    comp = pc.ExprCompiler(types)
    ge = comp.compile(P.func("greaterThanEqual", [P.col(5), P.const(2, 400)], [2, 2]))
    assert ge.result_type == 1 and [i[0] for i in ge.insns_py] == [1, 2, 35]
    div = comp.compile(P.func("divide", [P.col(6), P.const(4, 1e6)], [2, 4]))
    assert div.result_type == 4 and [i[0] for i in div.insns_py] == [1, 3, 2, 23]
    eq = comp.compile(P.func("equal", [P.col(2), P.const(5, "x")], [5, 5]))
    assert eq.insns_py[-1][0] == _lib.OP["EQ_S"] and eq.pool.startswith(b"x")
    feq = pc.ExprCompiler([4, 4]).compile(P.func("equal", [P.col(0), P.col(1)], [4, 4]))
    assert feq.insns_py[-1][0] == _lib.OP["APPROX_EQ_F"]   # ApproxEqualUDF registration
    with pytest.raises(pc.UnsupportedError):
        comp.compile(P.func("greaterThan", [P.col(5), P.const(4, 1.0)], [2, 4]))  # not registered
    with pytest.raises(pc.UnsupportedError):
        comp.compile(P.func("regex_match", [P.col(2)], [5]))


def test_compile_uda_registry():
    comp = pc.ExprCompiler([2, 4, 5])
    u = pc.compile_uda(P.agg_expr("quantiles", [P.col(1)], [4]), comp)
    assert u.kind == _lib.UDA_QUANTILES and u.out_type == 5
    u = pc.compile_uda(P.agg_expr("count", [P.col(2)], [5]), comp)
    assert u.kind == _lib.UDA_COUNT and u.out_type == 2
    u = pc.compile_uda(P.agg_expr("sum", [P.col(0)], [2]), comp)
    assert u.kind == _lib.UDA_SUM and u.out_type == 2
    with pytest.raises(pc.UnsupportedError):
        pc.compile_uda(P.agg_expr("max", [P.col(2)], [5]), comp)


def test_pipeline_lowering_of_c2_plan():
    from pixie_amd.pipeline import LinearQuery
    q = LinearQuery(P.c2_plan(), P.HTTP_TYPES)
    assert q.filter is not None and q.filter.result_type == 1
    assert [k.insns_py[0][2] for k in q.keys] == [P.HE["service"], P.HE["req_path"]]
    # latency_ms = divide(latency, 1e6) substituted into every UDA argument
    assert all(u.arg.insns_py[0][2] == P.HE["latency"] for u in q.udas)
    assert [u.kind for u in q.udas] == [_lib.UDA_COUNT, _lib.UDA_MEAN, _lib.UDA_QUANTILES]
    assert q.post_map is not None


def test_plan_binary_roundtrip():
    plan = P.c2_plan()
    blob = plan.SerializeToString()
    again = planpb.Plan()
    again.ParseFromString(blob)
    assert again == plan
