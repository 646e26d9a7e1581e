"""Byte-level pinning of the quantiles JSON (QuantilesUDA::Finalize, math_sketches.h:40-54,
written by rapidjson::Writer at Tencent/rapidjson@f56928de, bazel/repository_locations.bzl:
153-157).  The engine's renderer (pixie_amd/host/json_double.h) is pinned against strings fixed
by rapidjson's published Grisu2 + Prettify rules and the reference's own test expectations
(math_sketches_test.cc:30-70), and against the oracle's separate restatement
(oracle/json_number.h: cached powers computed by exact multi-precision arithmetic, its own digit
generation and Prettify) byte for byte over ~10^6 doubles."""
import json
import math
import struct

import numpy as np
import pytest

import oracle_client as oc
from pixie_amd.pipeline import quantiles_json, quantiles_json_column

# value -> rapidjson Writer::Double output
KNOWN = [
    (100000.0, "100000.0"), (3e6, "3000000.0"), (1e-4, "0.0001"), (1e-7, "1e-7"), (1e21, "1e21"),
    (1e20, "100000000000000000000.0"), (1e-6, "0.000001"), (1.5e-6, "0.0000015"), (1.2345e-7, "1.2345e-7"),
    (0.1, "0.1"), (1 / 3, "0.3333333333333333"), (5.8, "5.8"), (2.442, "2.442"), (1.04, "1.04"), (6.333, "6.333"),
    (0.0, "0.0"), (-0.0, "-0.0"), (-2.5, "-2.5"), (123456789012345678901234.0, "1.2345678901234569e23"),
    (5e-324, "5e-324"), (1.7976931348623157e308, "1.7976931348623157e308"), (12.0, "12.0"), (-1e-300, "-1e-300"),
    (1e100, "1e100"), (2.5e-10, "2.5e-10"),
    # GrisuRound after the 10th fractional digit (rapidjson's 20-entry uint64 kPow10; a 10-entry
    # table left the upper boundary's "...97" here)
    (2419999.9999999995, "2419999.9999999995"),
]


def _one(v):
    s = quantiles_json([v] * 7)
    body = s[len('{"p01":'):].split(",")[0]
    return body


@pytest.mark.parametrize("v,want", KNOWN, ids=[w for _, w in KNOWN])
def test_rapidjson_number_forms(v, want):
    assert _one(v) == want


def test_full_object_bytes_and_reference_kat():
    # math_sketches_test.cc:30-70 expectations, rendered in key order p01..p99
    s = quantiles_json([1.04, 1.04, 1.142, 2.442, 5.322, 6.333, 6.333])
    assert s == '{"p01":1.04,"p10":1.04,"p25":1.142,"p50":2.442,"p75":5.322,"p90":6.333,"p99":6.333}'
    assert quantiles_json([1.0, 1.0, 1.0, 2.0, 2.0, 5.8, 6.0]) == \
        '{"p01":1.0,"p10":1.0,"p25":1.0,"p50":2.0,"p75":2.0,"p90":5.8,"p99":6.0}'


def test_nan_truncates_like_document_accept():
    # Writer::Double(NaN) fails with the default write flags; Document::Accept stops after the key.
    nan = float("nan")
    assert quantiles_json([nan] * 7) == '{"p01":'
    assert quantiles_json([1.0, 2.0, float("inf"), 3.0, 4.0, 5.0, 6.0]) == '{"p01":1.0,"p10":2.0,"p25":'


def test_round_trip_and_shape_random():
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 2**63 - 1, 20000, dtype=np.int64).view(np.float64)
    vals = bits[np.isfinite(bits)][:7 * 2000]
    vals = np.concatenate([vals, rng.lognormal(1, 3, 7 * 500), np.round(rng.normal(0, 1e6, 7 * 500))])
    vals = vals[:len(vals) // 7 * 7]
    col = quantiles_json_column(vals.reshape(-1, 7)).to_list()
    for s, row in zip(col, vals.reshape(-1, 7)):
        d = json.loads(s)
        for k, v in zip(["p01", "p10", "p25", "p50", "p75", "p90", "p99"], row):
            assert d[k] == v  # Grisu2 output always round-trips
        for tok in s[1:-1].split(","):
            num = tok.split(":")[1]
            assert "+" not in num and "e0" not in num and "e-0" not in num  # no '+', no zero padding
            mant = num.split("e")[0].lstrip("-")
            assert "e" in num or "." in mant  # rapidjson emits a '.' or an exponent


def test_oracle_renders_the_same_bytes():
    vals = [1.0, 2.0, 3.0, 4.0, 1e5, 3e6, 7.0]
    assert oc.quantiles_json(vals) == quantiles_json(oc.tdigest_quantiles(vals))


def _oracle_render(q7: np.ndarray) -> bytes:
    import ctypes as C
    lib = oc.load()
    f = lib.oracle_quantiles_json_render
    f.restype = C.c_int64
    f.argtypes = [C.POINTER(C.c_double), C.c_int64, C.c_char_p, C.c_int64]
    q = np.ascontiguousarray(q7, dtype=np.float64).reshape(-1, 7)
    need = f(q.ctypes.data_as(C.POINTER(C.c_double)), q.shape[0], None, 0)
    buf = C.create_string_buffer(int(need))
    f(q.ctypes.data_as(C.POINTER(C.c_double)), q.shape[0], buf, need)
    return buf.raw[:need]


def _engine_render(q7: np.ndarray) -> bytes:
    import ctypes as C
    from pixie_amd import host_engine
    lib = host_engine.load()
    q = np.ascontiguousarray(q7, dtype=np.float64).reshape(-1, 7)
    out, n = C.c_void_p(), C.c_int64()
    assert lib.pxc_quantiles_json(q.ctypes.data_as(C.POINTER(C.c_double)), q.shape[0], C.byref(out), C.byref(n)) == 0
    try:
        return C.string_at(out.value, n.value)
    finally:
        lib.pxc_free(out)


def _doubles(n, seed):
    """Every kind of finite double: uniform bit patterns (all exponents, subnormals), values
    near powers of ten and two, integers, short decimals, and the Prettify boundaries."""
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2**63 - 1, n, dtype=np.int64).view(np.float64)
    bits = bits[np.isfinite(bits)]
    k = rng.integers(-330, 309, n)
    near10 = np.power(10.0, k.astype(np.float64)) * (1 + rng.integers(-3, 4, n) * np.finfo(np.float64).eps)
    near2 = np.ldexp(1.0, rng.integers(-1074, 1024, n)) * (1 + rng.integers(-2, 3, n) * np.finfo(np.float64).eps)
    ints = rng.integers(-10**17, 10**17, n).astype(np.float64)
    short = np.round(rng.uniform(-1e4, 1e4, n), rng.integers(0, 7))
    edges = np.array([1e21, 1e21 * (1 - 2**-52), 1e-6, 1e-6 * (1 - 2**-52), 1e-7, 9.999999999999999e20, 2**53, 2**53 + 2.0,
                      5e-324, 1e-323, 2.2250738585072014e-308, 2.2250738585072009e-308, 1.7976931348623157e308, 0.0, -0.0])
    v = np.concatenate([bits, near10, near2, ints, short, edges, -edges])
    v = v[np.isfinite(v)]
    rng.shuffle(v)
    return v[:len(v) // 7 * 7]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_engine_and_oracle_renderers_agree_bytewise(seed):
    """The engine's json_double.h and the oracle's json_number.h, written separately, produce the
    same bytes for ~340K doubles per seed (~10^6 over the three seeds), and every number
    round-trips."""
    v = _doubles(50_000, seed)
    q = v.reshape(-1, 7)
    a, b = _engine_render(q), _oracle_render(q)
    if a != b:
        sa, sb = a.split(b"\0"), b.split(b"\0")
        bad = [(i, x, y) for i, (x, y) in enumerate(zip(sa, sb)) if x != y][:5]
        raise AssertionError(f"renderers differ: {bad}")
    for s, row in zip(a.split(b"\0")[:200], q[:200]):
        d = json.loads(s)
        assert [d[k] for k in ("p01", "p10", "p25", "p50", "p75", "p90", "p99")] == list(row)


def test_oracle_renderer_known_forms_and_truncation():
    for v, want in KNOWN:
        got = _oracle_render(np.full((1, 7), v)).split(b"\0")[0].decode()
        assert got.split(",")[0] == '{"p01":' + want, (v, got)
    nan = float("nan")
    assert _oracle_render(np.array([[1.0, 2.0, float("inf"), 3.0, 4.0, 5.0, 6.0]])) == b'{"p01":1.0,"p10":2.0,"p25":\0'
    assert _oracle_render(np.full((1, 7), nan)) == b'{"p01":\0'
